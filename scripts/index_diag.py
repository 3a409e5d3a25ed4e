"""Diagnostic: time one decode configuration of 16 M R2 records under the current KX_DIAG bits
(256: index pass only; +1: no walk (DMA + tile words only); +64: per-phase cycles of the fast path).
  KX_DIAG=256 python scripts/index_diag.py [cfg] [n] [mode]"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from kitex_amd import _abi as A  # noqa: E402
from kitex_amd import schema as S, synth  # noqa: E402
from kitex_amd._lib import lib  # noqa: E402
from kitex_amd.codec import ProtobufCodec, ThriftCodec, status_tensor  # noqa: E402
from kitex_amd.columns import alloc_device  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "r2"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 16 << 20
mode = sys.argv[3] if len(sys.argv) > 3 else "concat"
dev = torch.device("cuda", 0)
cdc = ProtobufCodec(S.SCHEMAS[cfg]()) if cfg == "pf" else ThriftCodec(S.SCHEMAS[cfg]())  # pf: Kitex-Protobuf, as bench.py
src = synth.TORCH_GENERATORS[cfg](n, dev)
wire, offs = cdc.Marshal(src, with_offsets=True)
infos = cdc.dschema.infos
caps = [0 if ci.kind == A.COL_FIXED else int(src.cols[c][0][-1].item()) & 0xFFFFFFFF for c, ci in enumerate(infos)]
out = alloc_device(infos, n, caps, cdc.dschema.npresence, dev)
st = status_tensor(dev)
L = lib()
L.kx_debug_phase_cycles.argtypes = [C.c_void_p, C.c_int]
buf = (C.c_ulonglong * 8)()
o = offs if mode == "offsets" else None


def call():
    cdc.Unmarshal(wire, n, offsets=o, out=out, var_caps=caps, raise_on_error=False, status=st)


for _ in range(3):
    call()
torch.cuda.synchronize()
L.kx_debug_phase_cycles(buf, 8)
reps = 10
evs = [torch.cuda.Event(enable_timing=True) for _ in range(reps + 1)]
evs[0].record()
for k in range(reps):
    call()
    evs[k + 1].record()
torch.cuda.synchronize()
ms = sorted(evs[k].elapsed_time(evs[k + 1]) for k in range(reps))
L.kx_debug_phase_cycles(buf, 8)
tiles = (wire.numel() + 8191) // 8192
print(f"KX_DIAG={os.environ.get('KX_DIAG', '0')} {cfg} {mode} n={n}: median {ms[reps // 2]:.4f} ms "
      f"min {ms[0]:.4f} ms ({wire.numel() / ms[reps // 2] / 1e6:.0f} GB/s of input)", flush=True)
if int(os.environ.get("KX_DIAG", "0")) & 64:
    names = ["window DMA", "scan", "candidates", "walk", "agg+starts", "total wave", "-", "-"]
    for i in range(6):
        print(f"  {names[i]:14s} {buf[i] / reps / tiles:10.0f} cycles/tile", flush=True)
