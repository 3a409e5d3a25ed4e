"""Encode A/B inside one process: python scripts/enc_wcu.py [cfg] [n] [values]; the write pass's queued
payload copy with KX_ENC_WCU = each of values (output dwords per lane in flight; 1 = one payload at a
time), outputs compared byte for byte; event-timed median of 7 calls."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kitex_amd import schema as S, synth  # noqa: E402
from kitex_amd.codec import ThriftCodec, status_tensor  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "r3"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 4 << 20
vals = (sys.argv[3] if len(sys.argv) > 3 else "1,8,1,8").split(",")
dev = torch.device("cuda", 0)
cdc = ThriftCodec(S.SCHEMAS[cfg]())
src = synth.TORCH_GENERATORS[cfg](n, dev)
total = int(cdc.BLength(src).sum().item())
ref = None
for v in vals:
    os.environ["KX_ENC_WCU"] = v
    out = torch.empty(total, dtype=torch.uint8, device=dev)
    st = status_tensor(dev)
    for _ in range(2):
        cdc.Marshal(src, with_offsets=False, out=out, status=st, check_status=False)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(8)]
    ev[0].record()
    for k in range(7):
        cdc.Marshal(src, with_offsets=False, out=out, status=st, check_status=False)
        ev[k + 1].record()
    torch.cuda.synchronize()
    ms = sorted(ev[k].elapsed_time(ev[k + 1]) for k in range(7))
    same = True if ref is None else bool(torch.equal(ref, out))
    if ref is None:
        ref = out.clone()
    print(f"{cfg} n={n} KX_ENC_WCU={v} direct={os.environ.get('KX_ENC_DIRECT', '0')}: median {ms[3]:.3f} ms "
          f"min {ms[0]:.3f} ms code={int(st[0].item())} same={same}", flush=True)
