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


def _meta(cols: ColumnSet, n: int, infos, in_len: int, dev):
    """this rank's exchange header, built on the device: n, input bytes, then per var column and per
    level j of its offsets chain the first entry f_j and the units u_j it spans (f_0 = o_0[0],
    u_0 = o_0[n] - f_0; f_{j+1} = o_{j+1}[f_j], u_{j+1} = o_{j+1}[f_j + u_j] - f_{j+1})"""
    import torch
    parts = [torch.tensor([n, in_len], dtype=torch.int64, device=dev)]
    for c, ci in enumerate(infos):
        k = _kind(cols.cols[c], ci)
        if isinstance(k, int):
            col = cols.cols[c]
            f, l = _unsigned(col[0][0:1]), _unsigned(col[0][n:n + 1])
            parts += [f, l - f]
            for j in range(1, k):
                f, l = _unsigned(col[j].index_select(0, f)), _unsigned(col[j].index_select(0, l))
                parts += [f, l - f]
    return torch.cat(parts)


def rebase(dst, src, delta: int):
    """dst[:] = src (uint32 values in int32, or int64) + delta, as int64, on src's device: the offset
    rebase of the concatenation (one add per rank slice, no host round trip)"""
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


class _Plan:
    """Where every rank's slice lands in the concatenation, from the ranks' exchange headers (_meta).
    For a column of depth k, rank r sends o_0[:n] and, for j = 1 .. k-1, the o_j entries its o_{j-1}
    slice spans, then its data; the root rebases its o_j slice by (the units of o_{j+1} (or data) the
    ranks before it hold) - f_{j+1}(r), and closes every level with the total."""

    def __init__(self, metas, kinds):
        self.kinds = kinds
        self.world = world = len(metas)
        self.counts = [m[0] for m in metas]
        inl = [m[1] for m in metas]
        self.info = []  # per rank, per var column: [(f_j, u_j) for each level j]
        for m in metas:
            i, d = 2, {}
            for c, k in enumerate(kinds):
                if isinstance(k, int):
                    d[c] = [(m[i + 2 * j], m[i + 2 * j + 1]) for j in range(k)]
                    i += 2 * k
            self.info.append(d)
        self.N = sum(self.counts)
        self.rec0 = [sum(self.counts[:r]) for r in range(world)]
        self.in0 = [sum(inl[:r]) for r in range(world)]
        # base[c][j][r]: units of level j held by the ranks before r (r = world: the total)
        self.base = {c: [[sum(self.info[q][c][j][1] for q in range(r)) for r in range(world + 1)]
                         for j in range(k)]
                     for c, k in enumerate(kinds) if isinstance(k, int)}

    def _slices(self, c, k, r, n):
        """(start, length) of rank r's piece of each array o_0 .. o_{k-1}, data, in its own column"""
        info = self.info[r][c]
        out = [(0, n)]
        for j in range(1, k):
            out.append(info[j - 1])       # o_j entries spanned by the o_{j-1} slice
        out.append(info[k - 1])           # data units spanned by o_{k-1}
        return out

    def local_parts(self, cs: ColumnSet, r: int, n: int):
        """what rank r contributes, in a fixed order: per column its pieces, then presence"""
        out = []
        for c, k in enumerate(self.kinds):
            col = cs.cols[c]
            if k == "fixed":
                out.append(col[:n])
            elif k == "view":
                out.append(col.pairs[:n])
            else:
                for j, (a, u) in enumerate(self._slices(c, k, r, n)):
                    out.append(col[j][a:a + u])
        if cs.presence is not None:
            out.append(cs.presence[:n])
        return out

    def alloc(self, like: ColumnSet, dev):
        """the concatenated batch (int64 offsets / views) and the staging of the ranks' offsets / views
        (in the senders' dtypes) that the rebase reads"""
        import torch

        from .columns import Views
        N, W = self.N, self.world
        out_cols, self.recv = [], {}
        for c, k in enumerate(self.kinds):
            col = like.cols[c]
            if k == "fixed":
                out_cols.append(torch.empty(N, dtype=col.dtype, device=dev))
            elif k == "view":
                out_cols.append(Views(torch.empty((max(1, N), 2), dtype=torch.int64, device=dev)))
                self.recv[c] = (torch.empty((max(1, N), 2), dtype=col.pairs.dtype, device=dev),)
            else:
                sizes = [N] + [self.base[c][j - 1][W] for j in range(1, k)]   # entries of o_j before closing
                parts = [torch.empty(s + 1, dtype=torch.int64, device=dev) for s in sizes]
                parts.append(torch.empty(max(1, self.base[c][k - 1][W]), dtype=col[k].dtype, device=dev))
                out_cols.append(tuple(parts))
                self.recv[c] = tuple(torch.empty(max(1, s), dtype=col[j].dtype, device=dev)
                                     for j, s in enumerate(sizes))
        pres = torch.empty(N, dtype=like.presence.dtype, device=dev) if like.presence is not None else None
        self.out = ColumnSet(out_cols, pres, N)
        return self.out

    def _dest_off(self, c, j, r):
        """where rank r's piece of o_j (j >= 1: entries of level j - 1) or data (j = k) starts"""
        return self.rec0[r] if j == 0 else self.base[c][j - 1][r]

    def dest_parts(self, r: int):
        """where rank r's pieces (local_parts order) are received"""
        out, d = self.out, []
        a, b = self.rec0[r], self.rec0[r] + self.counts[r]
        for c, k in enumerate(self.kinds):
            if k == "fixed":
                d.append(out.cols[c][a:b])
            elif k == "view":
                d.append(self.recv[c][0][a:b])
            else:
                for j, (_, u) in enumerate(self._slices(c, k, r, self.counts[r])):
                    s0 = self._dest_off(c, j, r)
                    d.append((self.recv[c][j] if j < k else out.cols[c][k])[s0:s0 + u])
        if out.presence is not None:
            d.append(out.presence[a:b])
        return d

    def rebase_all(self):
        """every rank's slice, on the device: level j's entries by the units of level j + 1 (or data)
        before it, views by the input bytes before it; then the closing entry of every level"""
        out, W = self.out, self.world
        for c, k in enumerate(self.kinds):
            if k == "fixed":
                continue
            for r in range(W):
                a, b = self.rec0[r], self.rec0[r] + self.counts[r]
                if k == "view":
                    rebase_views(out.cols[c].pairs[a:b], self.recv[c][0][a:b], self.in0[r])
                    continue
                for j, (_, u) in enumerate(self._slices(c, k, r, self.counts[r])[:k]):
                    s0 = self._dest_off(c, j, r)
                    f_next = self.info[r][c][j][0]
                    rebase(out.cols[c][j][s0:s0 + u], self.recv[c][j][s0:s0 + u], self.base[c][j][r] - f_next)
            if k == "view":
                continue
            for j in range(k):
                end = self.N if j == 0 else self.base[c][j - 1][W]
                out.cols[c][j][end] = self.base[c][j][W]


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
    plan = _Plan(torch.stack(metas).cpu().tolist(), kinds)
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
    plan = _Plan(metas, kinds)
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
