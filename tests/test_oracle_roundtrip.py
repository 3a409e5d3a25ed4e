"""Oracle self-consistency on the benchmark schemas + the independent protobuf fixture."""
import os

import numpy as np
import pytest

from kitex_amd import _abi as A
from kitex_amd import schema as S
from kitex_amd import synth
from tests.helpers import assert_columns_equal

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_flatten_r2(oracle):
    rc, infos, npres = oracle.flatten(S.schema_r2())
    assert rc == 0 and npres == 0 and len(infos) == 10
    assert [ci.kind for ci in infos] == [A.COL_FIXED] * 8 + [A.COL_BYTES] * 2
    assert all(ci.width == 8 for ci in infos[:8])


def test_flatten_r3(oracle):
    rc, infos, npres = oracle.flatten(S.schema_r3())
    assert rc == 0 and npres == 2
    assert [(ci.kind, ci.width, ci.depth) for ci in infos] == [
        (A.COL_FIXED, 8, 0), (A.COL_LIST, 8, 0), (A.COL_FIXED, 8, 1), (A.COL_FIXED, 4, 1),
        (A.COL_BYTES, 1, 1), (A.COL_FIXED, 4, 0)]
    assert [ci.presence_bit for ci in infos] == [-1, 0, -1, -1, -1, -1]
    assert list(infos[4].path[:2]) == [3, 3]


def test_flatten_rejects_recursive_and_map(oracle):
    node = S.Struct("Node", [S.Field(1, A.T_I64)])
    node.fields.append(S.Field(2, A.T_STRUCT, child=node))
    rc, infos, _ = oracle.flatten(S.Schema(node))     # a recursive field keeps its bytes (nested schema)
    assert rc == 0 and infos[1].kind == A.COL_BYTES and infos[1].ttype == A.T_STRUCT
    m = S.Struct("M", [S.Field(1, A.T_MAP)])
    assert oracle.flatten(S.Schema(m))[0] == A.ERR_NOT_IMPLEMENTED


@pytest.mark.parametrize("name,per_rec", [("r1", 89), ("r2", 167)])
def test_wire_sizes(oracle, name, per_rec):
    cs = synth.GENERATORS[name](100)
    rc, wire, offs = oracle.encode(S.SCHEMAS[name](), cs)
    assert rc == 0 and wire.size == 100 * per_rec
    assert np.all(np.diff(offs) == per_rec)


@pytest.mark.parametrize("name", ["r1", "r2", "r3"])
def test_thrift_roundtrip(oracle, name):
    sch = S.SCHEMAS[name]()
    cs = synth.GENERATORS[name](500)
    rc, wire, offs = oracle.encode(sch, cs)
    assert rc == 0
    _, infos, _ = oracle.flatten(sch)
    # concatenated (list<Struct>) mode
    rc, out, st, _ = oracle.decode(sch, wire, cs.n)
    assert rc == 0 and st.n_records == cs.n and st.consumed == wire.size
    assert_columns_equal(out, cs, infos, cs.n)
    # known-offsets mode, multi-threaded
    rc, out2, st2, _ = oracle.decode(sch, wire, cs.n, offsets=offs, threads=4)
    assert rc == 0
    assert_columns_equal(out2, cs, infos, cs.n)
    # skip decoder finds the same boundaries
    rc, soffs, done = oracle.skip_batch(wire, cs.n)
    assert rc == 0 and np.array_equal(soffs, offs)


def test_r3_encoder_field_order(oracle):
    """reorderStructFields: fixed-length fields first (id, kind), then vals, inner (patcher.go:503-522)."""
    cs = synth.gen_r3(1)
    rc, wire, _ = oracle.encode(S.schema_r3(), cs)
    w = bytes(wire)
    assert w[0:3] == bytes([A.T_I64, 0, 1])
    assert w[11:14] == bytes([A.T_I32, 0, 4])
    assert w[18:21] == bytes([A.T_LIST, 0, 2]) and w[21] == A.T_I64


def test_pb_golden_fixture(oracle):
    """oracle proto3 encode == google.protobuf (upb) serialization; decode inverts it."""
    golden = np.fromfile(os.path.join(GOLDEN, "pf_batch_64.bin"), dtype=np.uint8)
    cs = synth.gen_pf(64)
    sch = S.schema_pf()
    rc, wire, offs = oracle.encode(sch, cs, pb=True)
    assert rc == 0 and np.array_equal(wire, golden)
    _, infos, _ = oracle.flatten(sch)
    rc, out, st, _ = oracle.decode(sch, golden, 64, pb=True)
    assert rc == 0 and st.n_records == 64 and st.consumed == golden.size
    assert_columns_equal(out, cs, infos, 64)


def test_pf_varint_lengths_cover_1_to_10(oracle):
    cs = synth.gen_pf(4000)
    v = np.concatenate([cs.cols[i] for i in range(8)]).view(np.uint64)
    nz = v[v != 0]
    lens = np.ceil(np.maximum(1, np.floor(np.log2(nz.astype(np.float64))) + 1) / 7).astype(int)
    assert set(np.unique(lens)) >= set(range(2, 11))
    assert 0.03 < np.mean(v == 0) < 0.1


def test_synth_numpy_matches_splitmix(oracle):
    seed = synth.seed_for("r1")
    cs = synth.gen_r1(3)
    for r in range(3):
        for f in range(1, 9):
            assert int(cs.cols[f - 1][r]) & ((1 << 64) - 1) == oracle.splitmix64(seed + r * 16 + f)


@pytest.mark.parametrize("name", ["r1", "r2", "r3", "pf"])
def test_synth_torch_matches_numpy(name):
    torch = pytest.importorskip("torch")
    a = synth.GENERATORS[name](257, start=1000)
    b = synth.TORCH_GENERATORS[name](257, torch.device("cpu"), start=1000)
    for ca, cb in zip(a.cols, b.cols):
        if isinstance(ca, tuple):
            assert np.array_equal(ca[0].view(np.uint32) - ca[0].view(np.uint32)[0],
                                  cb[0].numpy().view(np.uint32) - cb[0].numpy().view(np.uint32)[0])
            assert np.array_equal(ca[1].view(np.uint8), cb[1].numpy().view(np.uint8))
        else:
            assert np.array_equal(ca.view(np.uint8), cb.numpy().view(np.uint8))
