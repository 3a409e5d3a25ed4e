"""R3 decode at several sizes: time per call and the re-walk diagnostics (tile re-walks, group re-scans).
  python scripts/r3_probe.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from kitex_amd import _abi as A, schema as S, synth  # noqa: E402
from kitex_amd.codec import ThriftCodec, read_status, status_tensor  # noqa: E402
from kitex_amd.columns import alloc_device  # noqa: E402

dev = torch.device("cuda", 0)
cdc = ThriftCodec(S.schema_r3())
for n in [int(x) for x in (sys.argv[1:] or ["262144", "1048576", "2097152", "4194304"])]:
    src = synth.gen_r3_torch(n, dev, maxlist=int(os.environ.get("MAXLIST", "128")))
    wire, offs = cdc.Marshal(src)
    infos = cdc.dschema.infos
    caps = [0 if ci.kind == A.COL_FIXED else int(src.cols[c][0][-1].item()) & 0xFFFFFFFF for c, ci in enumerate(infos)]
    out = alloc_device(infos, n, caps, cdc.dschema.npresence, dev)
    st = status_tensor(dev)
    for _ in range(2):
        cdc.Unmarshal(wire, n, out=out, var_caps=caps, raise_on_error=False, status=st)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        cdc.Unmarshal(wire, n, out=out, var_caps=caps, raise_on_error=False, status=st)
    e1.record()
    torch.cuda.synchronize()
    s = read_status(st)
    ms = e0.elapsed_time(e1) / 5
    print(f"n={n} bytes={wire.numel()} ms={ms:.3f} GB/s={wire.numel() / ms / 1e6:.0f} code={s.code} "
          f"diag={s.diag[0]},{s.diag[1]}", flush=True)
    if s.diag[1]:
        os.environ["KX_DIAG_DUMP"] = "1"
    del src, wire, offs, out
    torch.cuda.empty_cache()
