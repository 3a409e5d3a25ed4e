"""Round 5: time the nested walker in proto mode (tests/pbn_cases.py PN, Batch-framed, 1 M records)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kitex_amd.codec import ProtobufCodec, read_status, status_tensor  # noqa: E402
from kitex_amd.columns import alloc_device  # noqa: E402
from tests import pbn_cases as PB  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
k = 4096
dev = torch.device("cuda", 0)
sch = PB.schema_pn()
cdc = ProtobufCodec(sch)
_, bodies, boffs = PB.batch(k, seed=7, name="PN")
lens = np.diff(boffs).astype(np.int64)
recs = [b"\x0a" + PB.uvarint(int(lens[i])) + bodies[int(boffs[i]):int(boffs[i + 1])].tobytes() for i in range(k)]
one = np.frombuffer(b"".join(recs), dtype=np.uint8).copy()
wire = torch.from_numpy(one).to(dev).repeat(n // k)
units = cdc.DecodeSizes(wire, n)
vc, ec, sc = units[0::3], units[1::3], units[2::3]
ds = cdc.dschema
out = alloc_device(ds.infos, n, vc, ds.npresence, dev, elem_caps=ec, sub_caps=sc)
st = status_tensor(dev)
for _ in range(2):
    cdc.Unmarshal(wire, n, out=out, var_caps=vc, raise_on_error=False, status=st)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(5):
    cdc.Unmarshal(wire, n, out=out, var_caps=vc, raise_on_error=False, status=st)
torch.cuda.synchronize()
s = read_status(st)
print(f"pn decode n={n}: {(time.perf_counter() - t0) / 5 * 1e3:.2f} ms code={s.code} n_records={s.n_records}", flush=True)
