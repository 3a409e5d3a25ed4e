"""Encode timing A/B inside one process: python scripts/enc_time.py [cfg] [n]; the write pass's image path
(default) against KX_ENC_DIRECT=1 (every record straight to HBM, list payloads by wave_copy), outputs
compared byte for byte."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kitex_amd import schema as S, synth  # noqa: E402
from kitex_amd.codec import ThriftCodec, status_tensor  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "r3"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 4 << 20
dev = torch.device("cuda", 0)
cdc = ThriftCodec(S.SCHEMAS[cfg]())
src = synth.TORCH_GENERATORS[cfg](n, dev)
total = int(cdc.BLength(src).sum().item())
outs = {}
for direct in ("0", "1", "0", "1"):
    os.environ["KX_ENC_DIRECT"] = direct
    out = torch.empty(total, dtype=torch.uint8, device=dev)
    st = status_tensor(dev)
    for _ in range(2):
        cdc.Marshal(src, with_offsets=False, out=out, status=st, check_status=False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        cdc.Marshal(src, with_offsets=False, out=out, status=st, check_status=False)
    torch.cuda.synchronize()
    outs[direct] = out
    print(f"{cfg} encode n={n} KX_ENC_DIRECT={direct}: {(time.perf_counter() - t0) / 5 * 1e3:.3f} ms", flush=True)
print("identical:", bool(torch.equal(outs["0"], outs["1"])))
