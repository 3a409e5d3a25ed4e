"""Host sanitizers over the device code's CPU builds (SURVEY.md §5 "race detection / sanitizers"; the GPU pool
has no GPU AddressSanitizer): the decode kernels' CPU SIMT emulation (tests/emu), the nested walker's host
build (tests/emu/nested_host.cpp), the schema compilers and the oracle, all built with ASan + UBSan
(`-fsanitize=address,undefined`, UBSan non-recovering), run in a child pytest with the ASan runtime preloaded.
Any out-of-bounds read or write, use after free or undefined behaviour aborts the child and fails here.

The emulator reads each input dword that holds the batch's last bytes through emu_gdword (input bytes only,
the rest poisoned): on the device that aligned dword read never crosses a page (kx_decode.hip gdword), so a
byte-granular ASan report there would be a false positive, and a caller depending on those bytes still shows
up as a parity failure."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLANG = "/opt/rocm/lib/llvm/bin/clang++"

# the emulator and host-walker suites and the oracle suites closest to them; the emulator's long-running
# cases (large persistent-loop and look-back batches, the chunked / combined experiments, the 25 000-frame
# batch) and the gloo shard suite are left to the full sanitizer runs recorded in
# profiles/r4_sanitizers_*.log (about 5x slower under ASan)
SUITES = ["tests/test_emu_decode.py", "tests/test_nested.py", "tests/test_pbn.py", "tests/test_oracle_list_struct.py",
          "tests/test_oracle_crc.py", "tests/test_oracle_kat.py"]
SLOW = ("persistent_loop", "slotcap_64", "deep_lookback", "25000", "chunked", "combo", "index_prefetch", "many")


def _asan_runtime():
    if not os.path.exists(CLANG):
        return None
    r = subprocess.run([CLANG, "-print-file-name=libclang_rt.asan-x86_64.so"], capture_output=True, text=True)
    p = r.stdout.strip()
    return p if r.returncode == 0 and os.path.isabs(p) and os.path.exists(p) else None


def test_device_code_host_builds_under_asan_ubsan():
    rt = _asan_runtime()
    if rt is None:
        pytest.skip("no ASan runtime for the ROCm clang")
    env = dict(os.environ, LD_PRELOAD=rt, KX_EMU_SAN="1", KX_ORACLE_SAN="1",
               ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:abort_on_error=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    probe = ("from tests.emu import emu as E; from oracle import oracle as O; import ctypes; "
             "E.lib(); O.lib(); assert E.SAN and O.SAN; ctypes.CDLL(None).__asan_init")
    r = subprocess.run([sys.executable, "-c", probe], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=900)
    assert r.returncode == 0, r.stderr[-4000:]
    r = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-m", "not gpu", "-p", "no:cacheprovider",
                        "-n", "4", "-k", " and ".join(f"not {k}" for k in SLOW), *SUITES],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=1500)
    assert r.returncode == 0, (r.stdout[-3000:] + r.stderr[-6000:])
