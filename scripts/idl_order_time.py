"""Round 5: the IDL-order producer batch of tests/test_gpu_adversarial.py decoded 5 times (for a kernel trace)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kitex_amd import _abi as A  # noqa: E402
from kitex_amd import schema as S  # noqa: E402
from kitex_amd.codec import ThriftCodec, read_status, status_tensor  # noqa: E402
from tests.test_gpu_adversarial import N, _idl_order_r2  # noqa: E402

dev = torch.device("cuda", 0)
fs = [S.Field(1, A.T_STRING, "s1")] + [S.Field(i, A.T_I64, f"a{i}") for i in range(2, 10)]
fs += [S.Field(10, A.T_STRING, "s10")]
cdc = ThriftCodec(S.Schema(S.Struct("R2idl", fs)))
_, wire = _idl_order_r2(torch, dev, N)
res = cdc.Unmarshal(wire, N)
st = status_tensor(dev)
for _ in range(3):
    cdc.Unmarshal(wire, N, out=res.columns, raise_on_error=False, status=st)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(5):
    cdc.Unmarshal(wire, N, out=res.columns, raise_on_error=False, status=st)
torch.cuda.synchronize()
print(f"idl-order n={N}: {(time.perf_counter() - t0) / 5 * 1e3:.3f} ms code={read_status(st).code}", flush=True)
