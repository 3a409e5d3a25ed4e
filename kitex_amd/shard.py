"""Record-range sharding over the GPUs of one node.

Records are independent, so a batch of N records is split into contiguous ranges, one per rank
(one process per GPU); every rank decodes its range with no collective in the data path. The only
exchange is the final concatenation of the decoded columns into one rank's HBM (RCCL point-to-point
over xGMI with backend "nccl", or gloo on CPU for tests):

  1. all_gather of each rank's (record count, arena units per var column)   -- a few int64s
  2. root allocates the concatenated ColumnSet; every other rank sends its column slices
     (fixed columns, var offsets, var arenas, presence) with batched isend/irecv
  3. root rebases the received var offsets by the arena units of the ranks before it
     (uint32 arithmetic, same wrap as a single decode's offsets)

The reference has no multi-device path; this is the MI355X-side answer to config 5 of
BASELINE.json (records sharded across 8 GPUs, concatenation over xGMI).
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


def _var_units(cols: ColumnSet, infos, n: int, c: int) -> int:
    off = cols.cols[c][0]
    return (int(off[n].item()) - int(off[0].item())) & 0xFFFFFFFF


def concat_to_root(cols: ColumnSet, n_local: int, infos: Sequence[A.ColumnInfo], root: int = 0,
                   group=None) -> Optional[ColumnSet]:
    """Concatenate every rank's decoded shard (records in rank order) into `root`.

    `cols` holds this rank's decoded columns (torch tensors on this rank's device, or CPU for
    gloo): FIXED -> tensor[>= n_local], BYTES/LIST -> (int32 offsets[>= n_local + 1], arena).
    Returns the concatenated ColumnSet on root, None elsewhere."""
    import torch
    import torch.distributed as dist

    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    dev = cols.cols[0][0].device if isinstance(cols.cols[0], tuple) else cols.cols[0].device
    var = [c for c, ci in enumerate(infos) if ci.kind != A.COL_FIXED]
    meta = torch.tensor([n_local] + [_var_units(cols, infos, n_local, c) for c in var], dtype=torch.int64,
                        device=dev)
    metas = [torch.empty_like(meta) for _ in range(world)]
    dist.all_gather(metas, meta, group=group)
    metas = [m.cpu().tolist() for m in metas]
    counts = [m[0] for m in metas]
    units = [m[1:] for m in metas]
    N = sum(counts)
    rec0 = [sum(counts[:r]) for r in range(world)]
    arena0 = [[sum(units[q][j] for q in range(r)) for j in range(len(var))] for r in range(world)]

    # what this rank sends / root receives, in a fixed order: per column then presence
    def local_parts(cs: ColumnSet, r: int, n: int):
        parts = []
        for c, ci in enumerate(infos):
            if ci.kind == A.COL_FIXED:
                parts.append(cs.cols[c][:n])
            else:
                j = var.index(c)
                off, data = cs.cols[c]
                o0 = int(off[0].item()) if r == rank else 0
                parts.append(off[:n])
                parts.append(data[o0:o0 + units[r][j]])
        if cs.presence is not None:
            parts.append(cs.presence[:n])
        return parts

    if rank != root:
        ops = [dist.P2POp(dist.isend, t.contiguous(), root, group) for t in local_parts(cols, rank, n_local)
               if t.numel()]
        for req in dist.batch_isend_irecv(ops) if ops else []:
            req.wait()
        return None

    # root: allocate the concatenated batch and post every receive
    out_cols: List[object] = []
    for c, ci in enumerate(infos):
        if ci.kind == A.COL_FIXED:
            t = cols.cols[c]
            out_cols.append(torch.empty(N, dtype=t.dtype, device=dev))
        else:
            j = var.index(c)
            off, data = cols.cols[c]
            tot = sum(units[r][j] for r in range(world))
            out_cols.append((torch.empty(N + 1, dtype=off.dtype, device=dev),
                             torch.empty(max(1, tot), dtype=data.dtype, device=dev)))
    out_pres = torch.empty(N, dtype=cols.presence.dtype, device=dev) if cols.presence is not None else None
    out = ColumnSet(out_cols, out_pres, N)

    def dest_parts(r: int):
        parts = []
        a, b = rec0[r], rec0[r] + counts[r]
        for c, ci in enumerate(infos):
            if ci.kind == A.COL_FIXED:
                parts.append(out.cols[c][a:b])
            else:
                j = var.index(c)
                off, data = out.cols[c]
                parts.append(off[a:b])
                parts.append(data[arena0[r][j]:arena0[r][j] + units[r][j]])
        if out.presence is not None:
            parts.append(out.presence[a:b])
        return parts

    ops = []
    for r in range(world):
        if r == root:
            for d, s in zip(dest_parts(r), local_parts(cols, r, n_local)):
                d.copy_(s)
        else:
            ops += [dist.P2POp(dist.irecv, d, r, group) for d in dest_parts(r) if d.numel()]
    for req in dist.batch_isend_irecv(ops) if ops else []:
        req.wait()
    # rebase var offsets: rank r's offsets start at its own arena origin, move them to arena0[r]
    for c, ci in enumerate(infos):
        if ci.kind == A.COL_FIXED:
            continue
        j = var.index(c)
        off, _ = out.cols[c]
        for r in range(world):
            a, b = rec0[r], rec0[r] + counts[r]
            if b > a:
                first = int(off[a].item())
                delta = (arena0[r][j] - first) & 0xFFFFFFFF
                if delta:
                    d = delta - (1 << 32) if delta >= 1 << 31 else delta
                    off[a:b] += d          # int32 wraps like the uint32 offsets of one decode
        tot = sum(units[r][j] for r in range(world)) & 0xFFFFFFFF
        off[N] = tot - (1 << 32) if tot >= 1 << 31 else tot
    return out
