"""Diagnostic: shader-clock cycles per index-pass phase (KX_DIAG=64+256: index pass only)."""
import ctypes as C
import os
import sys

os.environ["KX_DIAG"] = os.environ.get("KX_DIAG", "320")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from kitex_amd import _abi as A  # noqa: E402
from kitex_amd import schema as S, synth  # noqa: E402
from kitex_amd._lib import lib  # noqa: E402
from kitex_amd.codec import ThriftCodec, status_tensor  # noqa: E402
from kitex_amd.columns import alloc_device  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "r2"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 16 << 20
dev = torch.device("cuda", 0)
cdc = ThriftCodec(S.SCHEMAS[cfg]())
src = synth.TORCH_GENERATORS[cfg](n, dev)
wire, offs = cdc.Marshal(src)
infos = cdc.dschema.infos
caps = [0 if ci.kind == A.COL_FIXED else int(src.cols[c][0][-1].item()) for c, ci in enumerate(infos)]
out = alloc_device(infos, n, caps, cdc.dschema.npresence, dev)
st = status_tensor(dev)
L = lib()
L.kx_debug_phase_cycles.argtypes = [C.c_void_p, C.c_int]
buf = (C.c_ulonglong * 8)()
cdc.Unmarshal(wire, n, out=out, var_caps=caps, raise_on_error=False, status=st)
torch.cuda.synchronize()
L.kx_debug_phase_cycles(buf, 8)
reps = 3
for _ in range(reps):
    cdc.Unmarshal(wire, n, out=out, var_caps=caps, raise_on_error=False, status=st)
torch.cuda.synchronize()
L.kx_debug_phase_cycles(buf, 8)
tiles = (wire.numel() + 8191) // 8192
names = ["window DMA", "sig scan", "walk round 1", "repair+agg", "starts", "total wave", "-", "-"]
for i in range(6):
    print(f"  {names[i]:14s} {buf[i] / reps / tiles:10.0f} cycles/tile")
