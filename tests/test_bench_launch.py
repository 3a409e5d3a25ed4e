"""bench.py --gpus N launches N ranks (one process per GPU) when no launcher is around it, and every
rank sees WORLD_SIZE == --gpus (checked on CPU: --dry-run meets over gloo and makes no GPU call)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                       timeout=240, cwd=ROOT)
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    return r.returncode, [json.loads(l) for l in lines], r.stderr


def test_bench_gpus2_launches_two_ranks():
    rc, out, err = _run("--gpus", "2", "--dry-run")
    assert rc == 0, err[-2000:]
    assert len(out) == 1, out                # rank 0 alone prints
    assert out[0]["n_gpus"] == 2 and out[0]["ranks_seen"] == 2


def test_bench_default_is_one_rank():
    rc, out, err = _run("--dry-run")
    assert rc == 0, err[-2000:]
    assert out == [{"metric": "dry-run", "n_gpus": 1, "ranks_seen": 1, "gpus_flag": 1, "dry_run": True}]


def test_bench_world_mismatch_refused():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run"],
                       capture_output=True, text=True, timeout=120, cwd=ROOT, env=env)
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr
