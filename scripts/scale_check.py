"""Diagnostic: decode R2 at growing sizes on cuda:0, report status / diag and a column check."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from kitex_amd import _abi as A  # noqa: E402
from kitex_amd import schema as S, synth  # noqa: E402
from kitex_amd.codec import ThriftCodec, read_status, status_tensor  # noqa: E402
from kitex_amd.columns import alloc_device  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "r2"
dev = torch.device("cuda", 0)
cdc = ThriftCodec(S.SCHEMAS[cfg]())
infos = cdc.dschema.infos
for lg in range(int(os.environ.get("LG0", "12")), int(os.environ.get("LG1", "25"))):
    n = 1 << lg
    src = synth.TORCH_GENERATORS[cfg](n, dev)
    wire, offs = cdc.Marshal(src)
    caps = [0 if ci.kind == A.COL_FIXED else int(src.cols[c][0][-1].item()) for c, ci in enumerate(infos)]
    for mode in ("concat", "offsets"):
        out = alloc_device(infos, n, caps, cdc.dschema.npresence, dev)
        st = status_tensor(dev)
        o = offs if mode == "offsets" else None
        torch.cuda.synchronize()
        t0 = time.time()
        cdc.Unmarshal(wire, n, offsets=o, out=out, var_caps=caps, raise_on_error=False, status=st)
        torch.cuda.synchronize()
        dt = time.time() - t0
        s = read_status(st)
        good = True
        for c, ci in enumerate(infos):
            a, b = out.cols[c], src.cols[c]
            if ci.kind == A.COL_FIXED:
                good &= bool(torch.equal(a[0][:n], b[0][:n]))
            else:
                good &= bool(torch.equal(a[1][: n + 1], b[1][: n + 1]))
        print(f"n=2^{lg} {mode:7s} code={s.code} n_rec={s.n_records} consumed={s.consumed}/{wire.numel()} "
              f"diag={list(s.diag)} equal={good} {dt * 1e3:.2f} ms", flush=True)
