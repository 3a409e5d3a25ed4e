"""Record-range sharding over the GPUs of one node.

Records are independent, so a batch of N records is split into contiguous ranges, one per rank
(one process per GPU); every rank decodes its range with no collective in the data path. The only
exchange is the final concatenation of the decoded columns into one rank's HBM (RCCL point-to-point
over xGMI with backend "nccl", or gloo on CPU for tests):

  1. all_gather of each rank's (record count, arena units per var column)   -- a few int64s
  2. root allocates the concatenated ColumnSet; every other rank sends its column slices
     (fixed columns, var offsets, var arenas, presence) with batched isend/irecv
  3. root rebases the received var offsets by the arena units of the ranks before it, on the device
     (one add per rank slice, no host round trips); the concatenated offsets are int64, so a
     concatenated arena of 2^32 units or more (8 x 16M R2 strings) never wraps

The reference has no multi-device path; this is the MI355X-side answer to config 5 of
BASELINE.json (112M R2 + 16M R3 records sharded across the GPUs, concatenation over xGMI):
`concat_batches_to_root` concatenates several same-schema batches (one per schema) in one go.
"""
from __future__ import annotations

import ctypes as C
from typing import List, Optional, Sequence, Tuple

from . import _abi as A
from .synth import ColumnSet


def shard_range(n_total: int, world: int, rank: int) -> Tuple[int, int]:
    """(first record, record count) of `rank`'s contiguous shard; shards differ by at most 1."""
    base, extra = divmod(n_total, world)
    start = rank * base + min(rank, extra)
    return start, base + (1 if rank < extra else 0)


def _unsigned(t):
    """offsets as int64 values: 4-byte offset columns hold uint32 in int32 tensors"""
    import torch
    return t if t.dtype == torch.int64 else t.to(torch.int64) & 0xFFFFFFFF


# offsets arrays above the data array, per column kind (kitex_amd.columns): a column is a chain
# o_0[n + 1] -> o_1 -> ... -> o_{k-1} -> data, where o_j indexes o_{j+1} (the last one indexes data)
_DEPTH = {A.COL_BYTES: 1, A.COL_LIST: 1, A.COL_LIST_BYTES: 2, A.COL_LIST2: 2, A.COL_LIST2_BYTES: 3}


def _kind(col, ci):
    """how a decoded column is laid out: 'fixed' values[n]; 'view' (offset, length) pairs into the decode
    input; else the depth k of its offsets chain (1: strings / numeric lists / a map's fixed side as
    (offsets[n+1], arena); 2: list/set<string>, a map's string side, list<list<scalar>> as (record
    offsets, element offsets, data); 3: two container levels over strings as (record offsets, element
    offsets, inner element byte offsets, bytes)). Decided by the column's kind, checked against the tuple."""
    from ._lib import KxError
    from .columns import Views
    if isinstance(col, Views):
        return "view"
    if ci.kind == A.COL_FIXED:
        return "fixed"
    k = _DEPTH.get(ci.kind)
    if k is None or not isinstance(col, tuple) or len(col) != k + 1:
        raise KxError(A.ERR_INVALID_ARG, f"concat: column kind {ci.kind} does not match its layout")
    return k


def _depth(ci) -> int:
    return 0 if ci.kind == A.COL_FIXED else _DEPTH[ci.kind]


def _meta(cols: ColumnSet, n: int, infos, in_len: int, dev):
    """this rank's exchange header (include/kxcodec.h kx_shard_meta): n, input bytes, then per non-FIXED
    column and per level j of its offsets chain the first entry f_j and the units u_j it spans (f_0 =
    o_0[0], u_0 = o_0[n] - f_0; f_{j+1} = o_{j+1}[f_j], u_{j+1} = o_{j+1}[f_j + u_j] - f_{j+1}); a view
    column's words are 0. Device columns: kx_shard_meta (one wave on the device); host tensors (the gloo
    test harness): the same words with torch ops."""
    import torch
    if dev.type == "cuda":
        from .codec import _ctx_for
        from .columns import to_kx_columns
        from ._lib import check, lib
        L = lib()
        cinfos = (A.ColumnInfo * max(1, len(infos)))(*infos)
        words = L.kx_shard_meta_words(cinfos, len(infos))
        meta = torch.empty(words, dtype=torch.int64, device=dev)
        kc = to_kx_columns(cols, infos)
        s = torch.cuda.current_stream(dev)
        check(L.kx_shard_meta(_ctx_for(dev.index or 0, s).handle, cinfos, len(infos), C.byref(kc), n, in_len,
                              meta.data_ptr(), int(s.cuda_stream)), "kx_shard_meta")
        return meta
    parts = [torch.tensor([n, in_len], dtype=torch.int64, device=dev)]
    for c, ci in enumerate(infos):
        k = _kind(cols.cols[c], ci)
        if k == "view":
            parts.append(torch.zeros(2 * _depth(ci), dtype=torch.int64, device=dev))
        elif isinstance(k, int):
            col = cols.cols[c]
            f, l = _unsigned(col[0][0:1]), _unsigned(col[0][n:n + 1])
            parts += [f, l - f]
            for j in range(1, k):
                f, l = _unsigned(col[j].index_select(0, f)), _unsigned(col[j].index_select(0, l))
                parts += [f, l - f]
    return torch.cat(parts)


def rebase(dst, src, delta: int):
    """dst[:] = src (uint32 values in int32, or int64) + delta, as int64 (host tensors; device columns
    go through kx_concat_rebase)"""
    if dst.numel():
        dst.copy_(_unsigned(src) + delta)


def rebase_views(dst, src, delta: int):
    """(offset, length) pairs moved by `delta` input bytes; empty views stay (0, 0) (put_view)"""
    import torch
    if not dst.numel():
        return
    s = _unsigned(src)
    dst[:, 1] = s[:, 1]
    dst[:, 0] = torch.where(s[:, 1] != 0, s[:, 0] + delta, torch.zeros_like(s[:, 0]))


def _arrays(col, k):
    """a column's arrays by KX_PIECE_* index (offsets, elem_offsets, sub_offsets, data)"""
    if k == "fixed":
        return [None, None, None, col]
    if k == "view":
        return [col.pairs, None, None, None]
    return list(col[:k]) + [None] * (3 - k) + [col[k]]


class _Plan:
    """Where every rank's slice lands in the concatenation: kx_concat_plan (libkxcodec, host code) over
    the ranks' exchange headers. A piece of an offsets array (or a view column's pairs) lands in a
    staging array in the sender's width, which kx_concat_rebase (device) or rebase / rebase_views (host
    tensors) turn into the output's int64 entries plus the ranks' bases, closing every level."""

    def __init__(self, metas, kinds, infos, like: ColumnSet):
        import numpy as np

        from .columns import to_kx_columns
        from ._lib import KxError, check, lib
        self.kinds, self.infos = kinds, infos
        self.world = len(metas)
        self.cinfos = (A.ColumnInfo * max(1, len(infos)))(*infos)
        L = lib()
        m = np.ascontiguousarray(np.array(metas, dtype=np.int64).view(np.uint64))
        if m.shape[1] != L.kx_shard_meta_words(self.cinfos, len(infos)):
            raise KxError(A.ERR_INVALID_ARG, "concat: exchange header size")
        layout = to_kx_columns(like, infos)
        mp = m.ctypes.data_as(C.POINTER(C.c_uint64))
        cnt, sizes = C.c_uint32(0), A.ConcatSizes()
        rc = L.kx_concat_plan(self.cinfos, len(infos), C.byref(layout), mp, self.world, None, C.byref(cnt),
                              C.byref(sizes))
        if rc not in (0, A.ERR_SIZE_LIMIT):
            check(rc, "kx_concat_plan")
        self.pieces = (A.ConcatPiece * max(1, cnt.value))()
        check(L.kx_concat_plan(self.cinfos, len(infos), C.byref(layout), mp, self.world, self.pieces,
                               C.byref(cnt), C.byref(sizes)), "kx_concat_plan")
        self.npieces, self.sizes = cnt.value, sizes
        self.N = int(sizes.n)
        self.counts = [int(x[0]) for x in metas]
        self.rec0 = [sum(self.counts[:r]) for r in range(self.world)]
        self.by_rank = [[self.pieces[i] for i in range(self.npieces) if self.pieces[i].rank == r]
                        for r in range(self.world)]

    def _src(self, cs: ColumnSet, p):
        if p.column == A.MAX_COLUMNS:
            return cs.presence
        return _arrays(cs.cols[p.column], self.kinds[p.column])[p.array]

    def local_parts(self, cs: ColumnSet, r: int, n: int):
        """what rank r contributes, in piece order"""
        assert n == self.counts[r]
        return [self._src(cs, p)[p.src_first:p.src_first + p.count] for p in self.by_rank[r]]

    def alloc(self, like: ColumnSet, dev):
        """the concatenated batch (int64 offsets / views) and the staging arrays of the received offsets
        (in the senders' dtypes)"""
        import torch

        from .columns import Views
        N, U = self.N, self.sizes.units
        out_cols, stage_cols = [], []
        for c, k in enumerate(self.kinds):
            col = like.cols[c]
            if k == "fixed":
                out_cols.append(torch.empty(N, dtype=col.dtype, device=dev))
                stage_cols.append(None)
            elif k == "view":
                out_cols.append(Views(torch.empty((max(1, N), 2), dtype=torch.int64, device=dev)))
                stage_cols.append(Views(torch.empty((max(1, N), 2), dtype=col.pairs.dtype, device=dev)))
            else:
                parts = [torch.empty(int(U[c][j]) + 1, dtype=torch.int64, device=dev) for j in range(k)]
                parts.append(torch.empty(max(1, int(U[c][A.PIECE_DATA])), dtype=col[k].dtype, device=dev))
                out_cols.append(tuple(parts))
                stage_cols.append(tuple(torch.empty(max(1, int(U[c][j])), dtype=col[j].dtype, device=dev)
                                        for j in range(k)) + (parts[k],))
        pres = torch.empty(N, dtype=like.presence.dtype, device=dev) if like.presence is not None else None
        self.out = ColumnSet(out_cols, pres, N)
        self.stage = ColumnSet([s if s is not None else o for s, o in zip(stage_cols, out_cols)], pres, N)
        return self.out

    def dest_parts(self, r: int):
        """where rank r's pieces (local_parts order) are received"""
        out = []
        for p in self.by_rank[r]:
            if p.column == A.MAX_COLUMNS:
                dst = self.out.presence
            elif p.array == A.PIECE_DATA:
                dst = _arrays(self.out.cols[p.column], self.kinds[p.column])[A.PIECE_DATA]
            else:
                dst = _arrays(self.stage.cols[p.column], self.kinds[p.column])[p.array]
            out.append(dst[p.dst_first:p.dst_first + p.count])
        return out

    def rebase_all(self):
        """staging offsets + each piece's base -> output, closing entries: kx_concat_rebase on the device"""
        import torch
        dev = _device_of(self.out)
        if dev.type == "cuda":
            from .codec import _ctx_for
            from .columns import to_kx_columns
            from ._lib import check, lib
            s = torch.cuda.current_stream(dev)
            ks, ko = to_kx_columns(self.stage, self.infos), to_kx_columns(self.out, self.infos)
            check(lib().kx_concat_rebase(_ctx_for(dev.index or 0, s).handle, self.cinfos, len(self.infos),
                                         self.pieces, self.npieces, C.byref(ks), C.byref(ko), C.byref(self.sizes),
                                         int(s.cuda_stream)), "kx_concat_rebase")
            return
        # host tensors (the gloo test harness): the same arithmetic with torch ops
        for i in range(self.npieces):
            p = self.pieces[i]
            if p.column == A.MAX_COLUMNS or p.array == A.PIECE_DATA:
                continue
            k = self.kinds[p.column]
            a, b = p.dst_first, p.dst_first + p.count
            if k == "view":
                rebase_views(self.out.cols[p.column].pairs[a:b], self.stage.cols[p.column].pairs[a:b], p.rebase)
            else:
                rebase(self.out.cols[p.column][p.array][a:b], self.stage.cols[p.column][p.array][a:b], p.rebase)
        for c, k in enumerate(self.kinds):
            if not isinstance(k, int):
                continue
            for j in range(k):
                nxt = self.sizes.units[c][j + 1 if j + 1 < k else A.PIECE_DATA]
                self.out.cols[c][j][int(self.sizes.units[c][j])] = int(nxt)


def _check_views(kinds, in_len):
    from ._lib import KxError
    if "view" in kinds and in_len is None:
        raise KxError(A.ERR_NOT_IMPLEMENTED, "concat: view columns need in_len (the shard's input bytes)")


def _device_of(cols: ColumnSet):
    from .columns import Views
    t = cols.cols[0]
    return (t.pairs if isinstance(t, Views) else t[0] if isinstance(t, tuple) else t).device


def concat_to_root(cols: ColumnSet, n_local: int, infos: Sequence[A.ColumnInfo], root: int = 0,
                   group=None, in_len: Optional[int] = None) -> Optional[ColumnSet]:
    """Concatenate every rank's decoded shard (records in rank order) into `root`.

    `cols` holds this rank's decoded columns (torch tensors on this rank's device, or CPU for gloo),
    as the decoder writes them (kitex_amd.columns): FIXED -> tensor[>= n_local]; BYTES / LIST / a map's
    fixed side -> (offsets[>= n_local + 1], arena); LIST_BYTES (list/set<string>, a map's string side)
    -> (record offsets in elements, element byte offsets, bytes); offsets int32 (uint32 values) or
    int64; zero-copy string views -> Views(pairs[n, 2]). Views point into this rank's decode input: they
    are rebased into the concatenation of the ranks' inputs in rank order, so `in_len` (this rank's input
    bytes) is required for them. Returns the concatenated ColumnSet on root (int64 offsets and views),
    None elsewhere."""
    import torch
    import torch.distributed as dist

    kinds = [_kind(cols.cols[c], ci) for c, ci in enumerate(infos)]
    _check_views(kinds, in_len)
    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    dev = _device_of(cols)
    meta = _meta(cols, n_local, infos, int(in_len or 0), dev)
    metas = [torch.empty_like(meta) for _ in range(world)]
    dist.all_gather(metas, meta, group=group)
    plan = _Plan(torch.stack(metas).cpu().tolist(), kinds, infos, cols)
    if rank != root:
        ops = [dist.P2POp(dist.isend, t.contiguous(), root, group) for t in plan.local_parts(cols, rank, n_local)
               if t.numel()]
        for req in dist.batch_isend_irecv(ops) if ops else []:
            req.wait()
        return None
    out = plan.alloc(cols, dev)
    ops = []
    for r in range(world):
        if r == root:
            for d, s_ in zip(plan.dest_parts(r), plan.local_parts(cols, r, n_local)):
                d.copy_(s_)
        else:
            ops += [dist.P2POp(dist.irecv, d, r, group) for d in plan.dest_parts(r) if d.numel()]
    for req in dist.batch_isend_irecv(ops) if ops else []:
        req.wait()
    plan.rebase_all()
    return out


def concat_local(shards, infos: Sequence[A.ColumnInfo]) -> ColumnSet:
    """The same concatenation of decoded shards that live in one process (one device): shards =
    [(ColumnSet, n, in_len or None)] in record order. What concat_to_root does on the root, with the
    exchange replaced by device copies (single-GPU tests of config 5, several ctxs / streams)."""
    kinds = [_kind(shards[0][0].cols[c], ci) for c, ci in enumerate(infos)]
    for s_ in shards:
        _check_views(kinds, s_[2] if len(s_) > 2 else None)
    dev = _device_of(shards[0][0])
    metas = [_meta(cs, n, infos, int((rest[0] if rest else 0) or 0), dev).cpu().tolist()
             for cs, n, *rest in shards]
    plan = _Plan(metas, kinds, infos, shards[0][0])
    plan.alloc(shards[0][0], dev)
    for r, (cs, n, *_) in enumerate(shards):
        for d, s_ in zip(plan.dest_parts(r), plan.local_parts(cs, r, n)):
            if d.numel():
                d.copy_(s_)
    plan.rebase_all()
    return plan.out


def concat_batches_to_root(batches, root: int = 0, group=None):
    """Config 5: several decoded batches per rank (one per schema, e.g. R2 and R3), each
    concatenated across the ranks into root. batches: [(ColumnSet, n_local, infos[, in_len])]."""
    return [concat_to_root(b[0], b[1], b[2], root, group, *(b[3:4])) for b in batches]
