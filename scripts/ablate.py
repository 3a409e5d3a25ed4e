"""Diagnostic: decode-call time under KX_DIAG variants (each in its own process; output not checked)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import os, sys
sys.path.insert(0, %r)
import torch
from kitex_amd import _abi as A, schema as S, synth
from kitex_amd.codec import ThriftCodec, status_tensor
from kitex_amd.columns import alloc_device
cfg, n, mode = sys.argv[1], int(sys.argv[2]), sys.argv[3]
dev = torch.device("cuda", 0)
cdc = ThriftCodec(S.SCHEMAS[cfg]())
src = synth.TORCH_GENERATORS[cfg](n, dev)
wire, offs = cdc.Marshal(src)
infos = cdc.dschema.infos
caps = [0 if ci.kind == A.COL_FIXED else int(src.cols[c][0][-1].item()) for c, ci in enumerate(infos)]
out = alloc_device(infos, n, caps, cdc.dschema.npresence, dev)
st = status_tensor(dev)
o = offs if mode == "offsets" else None
for _ in range(2):
    cdc.Unmarshal(wire, n, offsets=o, out=out, var_caps=caps, raise_on_error=False, status=st)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(5):
    cdc.Unmarshal(wire, n, offsets=o, out=out, var_caps=caps, raise_on_error=False, status=st)
e1.record()
torch.cuda.synchronize()
print("%%.3f" %% (e0.elapsed_time(e1) / 5))
''' % ROOT
cfg = sys.argv[1] if len(sys.argv) > 1 else "r2"
n = sys.argv[2] if len(sys.argv) > 2 else str(16 << 20)
variants = sys.argv[3].split(",") if len(sys.argv) > 3 else ["0", "256", "257", "258", "262", "263"]
for mode in ("concat",):
    for ab in variants:
        env = dict(os.environ, KX_DIAG=ab)
        r = subprocess.run([sys.executable, "-c", CHILD, cfg, n, mode], env=env, capture_output=True, text=True,
                           timeout=240)
        print(f"{cfg} {mode} KX_DIAG={ab}: {r.stdout.strip()} ms {r.stderr.strip()[-300:] if r.returncode else ''}",
              flush=True)
