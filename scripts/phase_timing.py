"""Diagnostic: per-phase cycles of the decode kernel (KX_PHASE_TIMING=1 build path)."""
import ctypes as C
import os
import sys

os.environ["KX_PHASE_TIMING"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from kitex_amd import _abi as A  # noqa: E402
from kitex_amd import schema as S, synth  # noqa: E402
from kitex_amd._lib import lib  # noqa: E402
from kitex_amd.codec import ThriftCodec, read_status, status_tensor  # noqa: E402
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
buf = (C.c_ulonglong * 10)()
for mode in ("concat", "offsets"):
    o = offs if mode == "offsets" else None
    cdc.Unmarshal(wire, n, offsets=o, out=out, var_caps=caps, raise_on_error=False, status=st)
    torch.cuda.synchronize()
    L.kx_debug_phase_cycles(buf, 10)
    reps = 3
    for _ in range(reps):
        cdc.Unmarshal(wire, n, offsets=o, out=out, var_caps=caps, raise_on_error=False, status=st)
    torch.cuda.synchronize()
    L.kx_debug_phase_cycles(buf, 10)
    s = read_status(st)
    # one wave per tile: 8 KiB (concatenated) or krec records (offsets mode)
    krec = max(1, min(64, 8192 // max(1, -(-wire.numel() // n))))
    tiles = (wire.numel() + 8191) // 8192 if o is None else (n + krec - 1) // krec
    names = ["claim+window", "scan+walk1", "scans+AGG", "lookback", "repair+INCL", "walk2"]
    tot = sum(buf[:6])
    print(f"{cfg} {mode}: code={s.code} tiles={tiles}")
    for i, nm in enumerate(names):
        print(f"  {nm:12s} {buf[i] / reps / tiles:10.0f} cycles/tile  {100 * buf[i] / max(1, tot):5.1f}%")
