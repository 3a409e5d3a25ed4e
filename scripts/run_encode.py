"""Profiler driver: a few encode calls (fastMarshal: size pass + scan + write pass) of one config.
  python scripts/run_encode.py [cfg] [n] [calls]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from kitex_amd import schema as S, synth  # noqa: E402
from kitex_amd.codec import ProtobufCodec, ThriftCodec, status_tensor  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "r2"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 16 << 20
calls = int(sys.argv[3]) if len(sys.argv) > 3 else 3
dev = torch.device("cuda", 0)
cdc = (ProtobufCodec if cfg == "pf" else ThriftCodec)(S.SCHEMAS[cfg]())
src = synth.TORCH_GENERATORS[cfg](n, dev)
total = int(cdc.BLength(src).sum().item())
out = torch.empty(total, dtype=torch.uint8, device=dev)
st = status_tensor(dev)
for _ in range(calls):
    cdc.Marshal(src, with_offsets=False, out=out, status=st, check_status=False)
torch.cuda.synchronize()
print("ok", cfg, n, calls)
