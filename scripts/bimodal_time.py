"""Round 5: the bimodal batch of tests/test_gpu_adversarial.py (1 % of the records at 64 KiB, the rest 50 B),
decoded 5 times for a kernel trace: python scripts/bimodal_time.py"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kitex_amd import _abi as A  # noqa: E402
from kitex_amd import schema as S  # noqa: E402
from kitex_amd.codec import ThriftCodec, read_status, status_tensor  # noqa: E402
from tests.test_gpu_adversarial import _bimodal_batch  # noqa: E402

n = 1 << 18
dev = torch.device("cuda", 0)
sch = S.Schema(S.Struct("Bi", [S.Field(1, A.T_I64, "id"), S.Field(2, A.T_STRING, "s")]))
cdc = ThriftCodec(sch)
_, _, _, wire_np = _bimodal_batch(n)
wire = torch.from_numpy(wire_np).to(dev)
res = cdc.Unmarshal(wire, n)
st = status_tensor(dev)
for _ in range(3):
    cdc.Unmarshal(wire, n, out=res.columns, raise_on_error=False, status=st)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(5):
    cdc.Unmarshal(wire, n, out=res.columns, raise_on_error=False, status=st)
torch.cuda.synchronize()
s = read_status(st)
print(f"bimodal n={n} bytes={wire.numel()}: {(time.perf_counter() - t0) / 5 * 1e3:.3f} ms code={s.code} "
      f"diag={list(s.diag)}", flush=True)
