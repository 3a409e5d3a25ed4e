"""Round 5: a few known-offsets decode calls of one config, timed, for a kernel trace:
python scripts/run_decode_offsets.py [cfg] [n] [calls]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from kitex_amd import _abi as A, schema as S, synth  # noqa: E402
from kitex_amd.codec import ThriftCodec, status_tensor  # noqa: E402
from kitex_amd.columns import alloc_device  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "r2"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 16 << 20
calls = int(sys.argv[3]) if len(sys.argv) > 3 else 5
dev = torch.device("cuda", 0)
cdc = ThriftCodec(S.SCHEMAS[cfg]())
src = synth.TORCH_GENERATORS[cfg](n, dev)
wire, offs = cdc.Marshal(src)
infos = cdc.dschema.infos
caps = [0 if ci.kind == A.COL_FIXED else int(src.cols[c][0][-1].item()) for c, ci in enumerate(infos)]
out = alloc_device(infos, n, caps, cdc.dschema.npresence, dev)
st = status_tensor(dev)
for _ in range(2):
    cdc.Unmarshal(wire, n, offsets=offs, out=out, var_caps=caps, raise_on_error=False, status=st)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(calls):
    cdc.Unmarshal(wire, n, offsets=offs, out=out, var_caps=caps, raise_on_error=False, status=st)
torch.cuda.synchronize()
print(f"{cfg} offsets n={n}: {(time.perf_counter() - t0) / calls * 1e3:.3f} ms", flush=True)
