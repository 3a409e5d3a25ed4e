"""Round 4: time the nested walker (baseline.thrift Nesting, decode + encode) alone: python scripts/nested_time.py [n]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kitex_amd import idl, synth  # noqa: E402
from kitex_amd.codec import ThriftCodec, read_status, status_tensor  # noqa: E402
from kitex_amd.columns import alloc_device  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
k = int(sys.argv[2]) if len(sys.argv) > 2 else 4096   # distinct records (1: every lane walks the same shape)
dev = torch.device("cuda", 0)
doc = idl.parse_idl(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden",
                                 "idl", "baseline.thrift"))
sch = idl.to_schema(doc.struct("Nesting"))
cdc = ThriftCodec(sch)
ds = cdc.dschema
if os.environ.get("NEST_FILE"):   # n distinct records from a file (scripts/r5sort_gpu.sh)
    wire = torch.from_numpy(np.fromfile(os.environ["NEST_FILE"], dtype=np.uint8)).to(dev)
    k = n
else:
    one = np.frombuffer(b"".join(synth.thrift_records(sch, k, seed=7)), dtype=np.uint8).copy()
    wire = torch.from_numpy(one).to(dev).repeat(n // k)
offs = None
units = cdc.DecodeSizes(wire, n)
vc, ec, sc = units[0::3], units[1::3], units[2::3]
out = alloc_device(ds.infos, n, vc, ds.npresence, dev, elem_caps=ec, sub_caps=sc)
st = status_tensor(dev)
for mode in ("concat", "offsets"):
    if mode == "offsets":
        offs = cdc.Skip(wire, n)
    for _ in range(2):
        cdc.Unmarshal(wire, n, offsets=offs, out=out, var_caps=vc, raise_on_error=False, status=st)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        cdc.Unmarshal(wire, n, offsets=offs, out=out, var_caps=vc, raise_on_error=False, status=st)
    torch.cuda.synchronize()
    s = read_status(st)
    print(f"k={k} decode {mode} n={n}: "
          f"{(time.perf_counter() - t0) / 5 * 1e3:.2f} ms code={s.code} n_records={s.n_records}", flush=True)
w2, _ = cdc.Marshal(out)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(5):
    cdc.Marshal(out)
torch.cuda.synchronize()
print(f"encode n={n}: {(time.perf_counter() - t0) / 5 * 1e3:.2f} ms bytes={w2.numel()}", flush=True)
