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


def concat_to_root(cols: ColumnSet, n_local: int, infos: Sequence[A.ColumnInfo], root: int = 0,
                   group=None) -> Optional[ColumnSet]:
    """Concatenate every rank's decoded shard (records in rank order) into `root`.

    `cols` holds this rank's decoded columns (torch tensors on this rank's device, or CPU for
    gloo): FIXED -> tensor[>= n_local], BYTES/LIST -> (offsets[>= n_local + 1] int32 (uint32 values)
    or int64, arena). Returns the concatenated ColumnSet on root (int64 offsets), None elsewhere."""
    import torch
    import torch.distributed as dist

    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    dev = cols.cols[0][0].device if isinstance(cols.cols[0], tuple) else cols.cols[0].device
    var = [c for c, ci in enumerate(infos) if ci.kind != A.COL_FIXED]
    # meta: n, then per var column (first offset, units); built on the device, one exchange
    firsts = [_unsigned(cols.cols[c][0][0:1]) for c in var]
    lasts = [_unsigned(cols.cols[c][0][n_local:n_local + 1]) for c in var]
    parts = [torch.tensor([n_local], dtype=torch.int64, device=dev)]
    for f, l in zip(firsts, lasts):
        parts += [f, l - f]
    meta = torch.cat(parts)
    metas = [torch.empty_like(meta) for _ in range(world)]
    dist.all_gather(metas, meta, group=group)
    metas = torch.stack(metas).cpu().tolist()
    counts = [m[0] for m in metas]
    first = [m[1::2] for m in metas]
    units = [m[2::2] for m in metas]
    N = sum(counts)
    rec0 = [sum(counts[:r]) for r in range(world)]
    arena0 = [[sum(units[q][j] for q in range(r)) for j in range(len(var))] for r in range(world)]

    # what this rank sends / root receives, in a fixed order: per column then presence
    def local_parts(cs: ColumnSet, r: int, n: int):
        out = []
        for c, ci in enumerate(infos):
            if ci.kind == A.COL_FIXED:
                out.append(cs.cols[c][:n])
            else:
                j = var.index(c)
                off, data = cs.cols[c]
                o0 = first[r][j]
                out.append(off[:n])
                out.append(data[o0:o0 + units[r][j]])
        if cs.presence is not None:
            out.append(cs.presence[:n])
        return out

    if rank != root:
        ops = [dist.P2POp(dist.isend, t.contiguous(), root, group) for t in local_parts(cols, rank, n_local)
               if t.numel()]
        for req in dist.batch_isend_irecv(ops) if ops else []:
            req.wait()
        return None

    # root: receive buffers (offsets in the senders' dtype), the concatenated batch (int64 offsets)
    out_cols: List[object] = []
    recv_off = {}
    for c, ci in enumerate(infos):
        if ci.kind == A.COL_FIXED:
            t = cols.cols[c]
            out_cols.append(torch.empty(N, dtype=t.dtype, device=dev))
        else:
            j = var.index(c)
            off, data = cols.cols[c]
            tot = sum(units[r][j] for r in range(world))
            out_cols.append((torch.empty(N + 1, dtype=torch.int64, device=dev),
                             torch.empty(max(1, tot), dtype=data.dtype, device=dev)))
            recv_off[c] = torch.empty(max(1, N), dtype=off.dtype, device=dev)
    out_pres = torch.empty(N, dtype=cols.presence.dtype, device=dev) if cols.presence is not None else None
    out = ColumnSet(out_cols, out_pres, N)

    def dest_parts(r: int):
        d = []
        a, b = rec0[r], rec0[r] + counts[r]
        for c, ci in enumerate(infos):
            if ci.kind == A.COL_FIXED:
                d.append(out.cols[c][a:b])
            else:
                j = var.index(c)
                _, data = out.cols[c]
                d.append(recv_off[c][a:b])
                d.append(data[arena0[r][j]:arena0[r][j] + units[r][j]])
        if out.presence is not None:
            d.append(out.presence[a:b])
        return d

    ops = []
    for r in range(world):
        if r == root:
            for d, s_ in zip(dest_parts(r), local_parts(cols, r, n_local)):
                d.copy_(s_)
        else:
            ops += [dist.P2POp(dist.irecv, d, r, group) for d in dest_parts(r) if d.numel()]
    for req in dist.batch_isend_irecv(ops) if ops else []:
        req.wait()
    # rebase: rank r's offsets start at its own first offset, move them to arena0[r] (device adds)
    for c in var:
        j = var.index(c)
        off, _ = out.cols[c]
        for r in range(world):
            a, b = rec0[r], rec0[r] + counts[r]
            if b > a:
                off[a:b] = _unsigned(recv_off[c][a:b]) + (arena0[r][j] - first[r][j])
        off[N] = sum(units[r][j] for r in range(world))
    return out


def concat_batches_to_root(batches, root: int = 0, group=None):
    """Config 5: several decoded batches per rank (one per schema, e.g. R2 and R3), each
    concatenated across the ranks into root. batches: [(ColumnSet, n_local, infos)]."""
    return [concat_to_root(cs, n, infos, root, group) for cs, n, infos in batches]
