"""Decode-call time of one config under values of one environment knob (each in its own process; the
decoded columns of the last call are verified against the generator).
  python scripts/env_sweep.py <cfg> <n> <mode> <VAR> <v1,v2,...> [VAR2=val ...]"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import os, sys
sys.path.insert(0, %r)
import torch
import bench
cfg, n, mode = sys.argv[1], int(sys.argv[2]), sys.argv[3]
dev = torch.device("cuda", 0)
views = mode.endswith("views")
b = bench.Batch(cfg, n, dev, 0, mode.replace("_views", ""), 0, views=views)
for _ in range(3):
    b.step()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(10):
    b.step()
e1.record()
torch.cuda.synchronize()
print("%%.3f ms verified=%%s" %% (e0.elapsed_time(e1) / 10, b.verify()))
''' % ROOT
cfg, n, mode, var, vals = sys.argv[1:6]
extra = dict(kv.split("=", 1) for kv in sys.argv[6:])
for v in vals.split(","):
    env = dict(os.environ, **extra)
    env[var] = v
    r = subprocess.run([sys.executable, "-c", CHILD, cfg, n, mode], env=env, capture_output=True, text=True,
                       timeout=240)
    print(f"{cfg} {mode} {var}={v} {extra}: {r.stdout.strip()} {r.stderr.strip()[-400:] if r.returncode else ''}",
          flush=True)
