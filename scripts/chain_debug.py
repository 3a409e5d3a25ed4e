"""Diagnostic: decode a concatenated R2 batch, then compare every tile's published look-back words
(AGG / INCL, epoch-tagged) with the truth computed from the record offsets."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from kitex_amd import _abi as A  # noqa: E402
from kitex_amd import schema as S, synth  # noqa: E402
from kitex_amd._lib import lib  # noqa: E402
from kitex_amd.codec import ThriftCodec, read_status, status_tensor  # noqa: E402
from kitex_amd.columns import alloc_device  # noqa: E402

TILE, DSTRIDE, V48 = 8192, 24, (1 << 48) - 1
names = {V48: "ERR", V48 - 1: "DONE", V48 - 2: "NONE"}
cfg = sys.argv[1] if len(sys.argv) > 1 else "r2"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 24
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 2
dev = torch.device("cuda", 0)
cdc = ThriftCodec(S.SCHEMAS[cfg]())
infos = cdc.dschema.infos
src = synth.TORCH_GENERATORS[cfg](n, dev)
wire, offs = cdc.Marshal(src)
caps = [0 if ci.kind == A.COL_FIXED else int(src.cols[c][0][-1].item()) for c, ci in enumerate(infos)]
out = alloc_device(infos, n, caps, cdc.dschema.npresence, dev)
st = status_tensor(dev)
L = lib()
L.kx_debug_workspace.argtypes = [C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t), C.POINTER(C.c_uint64)]
starts = offs[:n].cpu().numpy().astype(np.int64)
in_len = wire.numel()
ntiles = (in_len + TILE - 1) // TILE
tlo = np.arange(ntiles, dtype=np.int64) * TILE
thi = np.minimum(tlo + TILE, in_len)
true_cnt = np.searchsorted(starts, thi, "left")           # records starting before thi
idx = np.minimum(true_cnt, n - 1)
true_exit = np.where(true_cnt < n, starts[idx], in_len)
for r in range(reps):
    cdc.Unmarshal(wire, n, out=out, var_caps=caps, raise_on_error=False, status=st)
    torch.cuda.synchronize()
    s = read_status(st)
    p, sz, ep = C.c_void_p(), C.c_size_t(), C.c_uint64()
    L.kx_debug_workspace(cdc.ctx.handle, C.byref(p), C.byref(sz), C.byref(ep))
    host = np.empty(sz.value // 8, dtype=np.uint64)
    hip = C.CDLL("libamdhip64.so")
    rc = hip.hipMemcpy(C.c_void_p(host.ctypes.data), p, C.c_size_t(sz.value), 2)  # device -> host
    assert rc == 0, rc
    words = host[32:32 + 21 * ntiles].reshape(21, ntiles).T  # structure of arrays: word f of tile t at f*ntiles+t
    tag = (words >> np.uint64(48)).astype(np.int64)
    val = (words & np.uint64(V48)).astype(np.int64)
    inc_ok = tag[:, 11] == ep.value
    agg_ok = tag[:, 0] == ep.value
    print(f"rep {r}: epoch={ep.value} code={s.code} n_rec={s.n_records}/{n} consumed={s.consumed}/{in_len} "
          f"diag={list(s.diag)} tiles={ntiles} incl={inc_ok.sum()} agg={agg_ok.sum()}")
    bad_cnt = np.nonzero(inc_ok & (val[:, 11] != np.minimum(true_cnt, n)) & (val[:, 12] != V48 - 1))[0]
    bad_exit = np.nonzero(inc_ok & (val[:, 12] != true_exit) & (val[:, 12] != V48 - 1) & (true_cnt < n))[0]
    print(f"  INCL cnt mismatches: {len(bad_cnt)}  INCL exit mismatches: {len(bad_exit)}")
    done = np.nonzero(inc_ok & (val[:, 12] == V48 - 1))[0]
    print(f"  first DONE tile: {done[:3]} (true tile of record n-1: {np.searchsorted(thi, starts[-1], 'right')})")
    for t in list(bad_cnt[:5]) + list(bad_exit[:5]):
        ag = agg_ok[t]
        fmt = lambda x: names.get(int(x), int(x))  # noqa: E731
        print(f"  tile {t}: INCL cnt={val[t, 11]} exit={fmt(val[t, 12])} | true cnt={true_cnt[t]} exit={true_exit[t]} | "
              f"AGG{'' if ag else '(none)'} cnt={val[t, 0]} ent={fmt(val[t, 1])} exit={fmt(val[t, 2])} | "
              f"true entry={true_exit[t - 1] if t else 0}")
