"""Diagnostic: decode concatenated batches and print the decode diagnostics (tile re-walks, group
re-scans, fast-path fallbacks) and the first records that differ from the oracle.
  python scripts/fast_diag.py cfg n [streams]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from kitex_amd import schema as S, synth  # noqa: E402
from kitex_amd.codec import ThriftCodec  # noqa: E402
from oracle import oracle  # noqa: E402

cfg, n = sys.argv[1], int(sys.argv[2])
streams = int(sys.argv[3]) if len(sys.argv) > 3 else 1
sch = S.SCHEMAS[cfg]()
cdc = ThriftCodec(sch)
dev = torch.device("cuda", 0)
cs = synth.GENERATORS[cfg](n)
rc, wire, offs = oracle.encode(sch, cs)
_, exp, est, _ = oracle.decode(sch, wire, n)
buf = torch.from_numpy(wire).to(dev)
ss = [torch.cuda.Stream() for _ in range(streams)] if streams > 1 else [None]
for rep in range(3):
    res = [cdc.Unmarshal(buf, n, stream=s, raise_on_error=False) for s in ss]
    for r in res:
        st = r.read_status()
        got = r.columns.cols[0].cpu().numpy()
        bad = np.nonzero(got != exp.cols[0])[0]
        print(f"rep {rep}: code {st.code} n {st.n_records} diag {list(st.diag)} bad {bad.size} first {bad[:5]}",
              flush=True)
        if bad.size:
            r0 = int(bad[0])
            print("  record", r0, "at", int(offs[r0]), "tile", int(offs[r0]) // 8192, "got", got[r0:r0 + 3],
                  "want", exp.cols[0][r0:r0 + 3])
