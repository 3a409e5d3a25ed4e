"""The nested walker's per-word UTF-8 check (kx_nested.h) against its byte-wise restatement of utf8.Valid,
compiled for the host with g++ (tests/native/utf8_check.cpp): every 3-byte sequence at three alignments
around the 8-byte word boundary plus 2 M seeded random strings must agree."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_utf8_word_check_matches_bytewise(tmp_path):
    exe = str(tmp_path / "utf8_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "include"),
                    "-I", os.path.join(ROOT, "kitex_amd", "csrc"), os.path.join(ROOT, "tests", "native", "utf8_check.cpp"),
                    "-o", exe], check=True)
    out = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout
    assert out.stdout.strip().endswith("bad=0")
