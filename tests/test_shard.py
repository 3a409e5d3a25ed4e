"""Multi-rank path on CPU (gloo, world_size 2 and 3): record-range shards and the concatenation of
decoded shards into rank 0 (kitex_amd/shard.py). The same code runs over RCCL/xGMI on GPUs."""
import os
import socket

import numpy as np
import pytest

from kitex_amd import schema as S
from kitex_amd import synth
from kitex_amd.shard import shard_range


def test_shard_range_covers_all():
    for n in (0, 1, 7, 1000, 16 << 20):
        for world in (1, 2, 3, 8):
            got = [shard_range(n, world, r) for r in range(world)]
            assert sum(c for _, c in got) == n
            pos = 0
            for s, c in got:
                assert s == pos
                pos += c
            assert max(c for _, c in got) - min(c for _, c in got) <= 1


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _to_torch(cs):
    import torch

    from kitex_amd.columns import Views

    def t(a):
        a = np.ascontiguousarray(a)
        if a.dtype == np.uint32:
            a = a.view(np.int32)
        elif a.dtype == np.uint64:
            a = a.view(np.int64)
        return torch.from_numpy(a.copy())
    cols = []
    for c in cs.cols:
        if isinstance(c, Views):
            cols.append(Views(t(c.pairs)))
        elif isinstance(c, tuple):
            cols.append(tuple(t(x) for x in c))
        else:
            cols.append(t(c))
    pres = torch.from_numpy(cs.presence.view(np.int64).copy()) if cs.presence is not None else None
    return synth.ColumnSet(cols, pres, cs.n)


def _shift_arena(cs, shift):
    """a decoded shard whose arenas do not start at 0 (offsets[0] = shift), as a sliced decode gives"""
    cols = []
    for c in cs.cols:
        if isinstance(c, tuple):
            off = c[0].astype(np.uint64) + shift
            data = np.concatenate([np.zeros(shift * (c[1].itemsize and 1), dtype=c[1].dtype), c[1]])
            cols.append((off.astype(np.uint32), data))
        else:
            cols.append(c)
    return synth.ColumnSet(cols, cs.presence, cs.n)


def _worker(rank, world, port, name, n, q):
    import torch.distributed as dist

    from kitex_amd.shard import concat_to_root
    from oracle import oracle
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sch = S.SCHEMAS[name]()
        _, infos, _ = oracle.flatten(sch)
        s0, cnt = shard_range(n, world, rank)
        local = synth.GENERATORS[name](cnt, start=s0)
        if rank == 1:
            local = _shift_arena(local, 5)
        out = concat_to_root(_to_torch(local), cnt, infos)
        if rank == 0:
            from tests.helpers import assert_columns_equal, offsets_u64
            full = synth.GENERATORS[name](n)
            assert out.n == n
            assert_columns_equal(out, full, infos, n)
            for c, ci in enumerate(infos):
                if isinstance(full.cols[c], tuple):
                    assert int(out.cols[c][0][n]) == int(offsets_u64(full.cols[c][0])[n])
        q.put((rank, "ok"))
    except Exception as e:  # report to the parent
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,name,n", [(2, "r2", 5001), (3, "r3", 2000), (2, "r1", 1)])
def test_concat_to_root_gloo(world, name, n):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, name, n, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
    assert all(v == "ok" for v in res.values()), res


def _mixed_worker(rank, world, port, n2, n3, q):
    """config 5 in miniature: every rank decodes its R2 and R3 record ranges with the decode KERNEL
    SOURCE under the SIMT emulator, then both decoded batches are concatenated into rank 0 and
    compared with the oracle's decode of the whole batches"""
    import torch.distributed as dist

    from kitex_amd.shard import concat_batches_to_root
    from oracle import oracle
    from tests.emu import emu
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        batches, wholes = [], []
        for name, n in (("r2", n2), ("r3", n3)):
            sch = S.SCHEMAS[name]()
            _, infos, npres = oracle.flatten(sch)
            s0, cnt = shard_range(n, world, rank)
            rc, wire, _ = oracle.encode(sch, synth.GENERATORS[name](cnt, start=s0))
            assert rc == 0
            erc, cols, st, _ = emu.decode(sch, infos, npres, wire, cnt, threads=4)
            assert erc == 0 and st.code == 0 and st.n_records == cnt, (erc, st.code, st.n_records)
            batches.append((_to_torch(cols), cnt, infos))
            if rank == 0:
                rc, whole, _ = oracle.encode(sch, synth.GENERATORS[name](n))
                wholes.append((sch, whole, n, infos))
        outs = concat_batches_to_root(batches)
        if rank == 0:
            from tests.helpers import assert_columns_equal, offsets_u64
            for out, (sch, whole, n, infos) in zip(outs, wholes):
                rc, exp, est, _ = oracle.decode(sch, whole, n)
                assert est.code == 0 and out.n == n
                assert_columns_equal(out, exp, infos, n)
                for c, ci in enumerate(infos):
                    if isinstance(exp.cols[c], tuple):
                        assert int(offsets_u64(out.cols[c][0])[n]) == int(offsets_u64(exp.cols[c][0])[n])
        q.put((rank, "ok"))
    except Exception as e:  # report to the parent
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


def test_concat_mixed_emulator_decoded_shards_gloo():
    import torch.multiprocessing as mp
    from tests.emu import emu
    emu.lib()                                  # build once, before the ranks start
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world = 2
    ps = [ctx.Process(target=_mixed_worker, args=(r, world, port, 7001, 1500, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
    assert all(v == "ok" for v in res.values()), res


_CX = {"cx1": (S.schema_cx1, synth.gen_cx1), "cx2": (S.schema_cx2, synth.gen_cx2)}


def _oracle_worker(rank, world, port, name, n, views, q):
    """every rank holds the oracle decode of its own shard (containers: list<string>, set<string>,
    maps; or R2 with zero-copy string views); rank 0 compares the concatenation with the oracle's decode
    of the ranks' wires concatenated"""
    import torch.distributed as dist

    from kitex_amd.shard import concat_to_root
    from oracle import oracle
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mk_s, gen = _CX.get(name, (S.SCHEMAS.get(name), synth.GENERATORS.get(name)))
        sch = mk_s()
        _, infos, _ = oracle.flatten(sch)
        shards = [shard_range(n, world, r) for r in range(world)]
        wires = []
        for s0, cnt in shards:
            rc, w, _ = oracle.encode(sch, gen(cnt, start=s0))
            assert rc == 0
            wires.append(w)
        s0, cnt = shards[rank]
        rc, local, st, _ = oracle.decode(sch, wires[rank], cnt, views=views)
        assert rc == 0 and st.code == 0
        out = concat_to_root(_to_torch(local), cnt, infos, in_len=wires[rank].size)
        if rank == 0:
            from tests.helpers import assert_columns_equal, offsets_u64
            whole = np.concatenate(wires)
            rc, exp, est, _ = oracle.decode(sch, whole, n, views=views)
            assert rc == 0 and est.code == 0 and out.n == n
            assert_columns_equal(out, exp, infos, n)
            for c, ci in enumerate(infos):
                if isinstance(exp.cols[c], tuple):
                    assert int(offsets_u64(out.cols[c][0])[n]) == int(offsets_u64(exp.cols[c][0])[n])
        q.put((rank, "ok"))
    except Exception as e:  # report to the parent
        import traceback
        q.put((rank, repr(e) + traceback.format_exc()[-800:]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,name,n,views", [(2, "cx1", 3001, False), (3, "cx2", 2500, False),
                                                 (2, "r2", 4001, True), (3, "r3", 1200, False)])
def test_concat_containers_and_views_gloo(world, name, n, views):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_oracle_worker, args=(r, world, port, name, n, views, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=180) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
    assert all(v == "ok" for v in res.values()), res


def test_concat_views_need_in_len():
    """views point into the rank's own input: without its length they cannot be rebased"""
    from kitex_amd import _abi as A
    from kitex_amd._lib import KxError
    from kitex_amd.columns import Views
    from kitex_amd.shard import concat_to_root
    import torch
    cs = synth.ColumnSet([Views(torch.zeros((4, 2), dtype=torch.int32))], None, 4)
    ci = A.ColumnInfo()
    ci.kind = A.COL_BYTES
    with pytest.raises(KxError):
        concat_to_root(cs, 4, [ci])


@pytest.mark.parametrize("name,views", [("cx1", False), ("r2", True), ("r3", False)])
def test_concat_local_matches_whole(oracle, name, views):
    """concat_local (one process, several shards): same plan and rebase as concat_to_root"""
    from kitex_amd.shard import concat_local
    from tests.helpers import assert_columns_equal
    mk_s, gen = _CX.get(name, (S.SCHEMAS.get(name), synth.GENERATORS.get(name)))
    sch = mk_s()
    _, infos, _ = oracle.flatten(sch)
    n, parts = 2003, 3
    shards, wires = [], []
    for r in range(parts):
        s0, cnt = shard_range(n, parts, r)
        rc, w, _ = oracle.encode(sch, gen(cnt, start=s0))
        rc, local, st, _ = oracle.decode(sch, w, cnt, views=views)
        assert rc == 0 and st.code == 0
        shards.append((_to_torch(local), cnt, w.size))
        wires.append(w)
    out = concat_local(shards, infos)
    rc, exp, est, _ = oracle.decode(sch, np.concatenate(wires), n, views=views)
    assert est.code == 0
    assert_columns_equal(out, exp, infos, n)


@pytest.mark.parametrize("name", ["nesting", "nx"])
def test_concat_local_nested(oracle, name):
    """nested schemas: LIST2 (record -> element -> value) and LIST2_BYTES (record -> element -> inner
    element -> bytes) columns keep every level of their offsets chain through the concatenation"""
    from kitex_amd import _abi as A
    from kitex_amd.shard import concat_local
    from tests import nested_cases as NC
    from tests.helpers import assert_columns_equal
    sch = {"nesting": S.schema_nesting, "nx": S.schema_nx}[name]()
    rc, infos, _ = oracle.flatten(sch)
    assert rc == 0
    kinds = {ci.kind for ci in infos}
    assert A.COL_LIST2_BYTES in kinds or name == "nesting"
    n, parts = 700, 3
    _, wire, offs = NC.batch(sch, n, seed=3)
    shards = []
    for r in range(parts):
        s0, cnt = shard_range(n, parts, r)
        w = wire[int(offs[s0]):int(offs[s0 + cnt])]
        rc, local, st, _ = oracle.decode(sch, w, cnt)
        assert rc == 0 and st.code == 0
        shards.append((_to_torch(local), cnt, w.size))
    out = concat_local(shards, infos)
    rc, exp, est, _ = oracle.decode(sch, wire, n)
    assert est.code == 0
    assert_columns_equal(out, exp, infos, n)


def test_concat_kind_layout_mismatch():
    """a column whose tuple does not match its kind is refused (was: silently mis-concatenated)"""
    import torch

    from kitex_amd import _abi as A
    from kitex_amd._lib import KxError
    from kitex_amd.shard import concat_local
    ci = A.ColumnInfo()
    ci.kind = A.COL_LIST2_BYTES
    cs = synth.ColumnSet([(torch.zeros(5, dtype=torch.int32), torch.zeros(1, dtype=torch.int32),
                           torch.zeros(1, dtype=torch.uint8))], None, 4)
    with pytest.raises(KxError):
        concat_local([(cs, 4, 0)], [ci])
