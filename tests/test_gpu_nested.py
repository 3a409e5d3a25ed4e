"""GPU parity of nested schemas (include/kxcodec.h "Nested schemas"; kitex_amd/csrc/kx_nested.hip): decode and
encode through libkxcodec's C-ABI against the oracle (oracle/kx_oracle_nested.c) on the reference's own IDL
methods (baseline.thrift NestingMethod, example.thrift ExampleMethod and Foo) and containers of containers,
canonical and noisy batches (shuffled / repeated / unknown / mistyped fields), known offsets and
concatenated records (skip-decoder boundaries), per-record errors, exact arena sizing (kx_thrift_decode_sizes)."""
import time

import numpy as np
import pytest

from kitex_amd import _abi as A
from tests import nested_cases as NC
from tests.helpers import assert_columns_equal, to_np
from tests.test_nested import SCHEMAS, _err_wire

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as t
    if not t.cuda.is_available():
        pytest.skip("no GPU")
    return t


@pytest.fixture(scope="module")
def dev(torch):
    return torch.device("cuda", 0)


_codecs = {}


def codec(name):
    from kitex_amd.codec import ThriftCodec
    if name not in _codecs:
        _codecs[name] = ThriftCodec(SCHEMAS[name])
    return _codecs[name]


def to_dev(torch, dev, cs):
    from kitex_amd.synth import ColumnSet
    cols = []
    for c in cs.cols:
        if isinstance(c, tuple):
            cols.append(tuple(torch.from_numpy(x.view(np.int32).copy() if x.dtype == np.uint32 else x.copy()).to(dev)
                              for x in c[:-1]) + (torch.from_numpy(c[-1].copy()).to(dev),))
        else:
            cols.append(torch.from_numpy(c.copy()).to(dev))
    pres = torch.from_numpy(cs.presence.view(np.int64).copy()).to(dev) if cs.presence is not None else None
    return ColumnSet(cols, pres, cs.n)


@pytest.mark.parametrize("name", sorted(SCHEMAS))
@pytest.mark.parametrize("noise", [False, True])
@pytest.mark.parametrize("known", [True, False])
def test_decode_matches_oracle(torch, dev, oracle, name, noise, known):
    cdc = codec(name)
    sch = SCHEMAS[name]
    assert cdc.dschema.nested
    n = 3000                                      # three 1024-record blocks of the scan
    _, wire, offs = NC.batch(sch, n, seed=21, noise=noise)
    rc, exp, est, _ = oracle.decode(sch, wire, n, offsets=offs if known else None)
    assert rc == 0
    buf = torch.from_numpy(wire).to(dev)
    o = torch.from_numpy(offs.view(np.int64)).to(dev) if known else None
    res = cdc.Unmarshal(buf, n, offsets=o)
    st = res.read_status()
    assert st.code == 0 and st.n_records == n and st.consumed == wire.size
    _, infos, _ = oracle.flatten(sch)
    assert_columns_equal(res.columns, exp, infos, n)


@pytest.mark.parametrize("name", sorted(SCHEMAS))
def test_encode_matches_oracle(torch, dev, oracle, name):
    cdc = codec(name)
    sch = SCHEMAS[name]
    n = 2500
    _, wire, offs = NC.batch(sch, n, seed=8, noise=True)
    rc, cols, _, _ = oracle.decode(sch, wire, n, offsets=offs)
    assert rc == 0
    rc, exp, eoffs = oracle.encode(sch, cols)
    assert rc == 0
    dcols = to_dev(torch, dev, cols)
    sizes = cdc.BLength(dcols)
    assert np.array_equal(to_np(sizes), np.diff(eoffs).astype(np.int64))
    got, goffs = cdc.Marshal(dcols)
    assert np.array_equal(to_np(got), exp)
    assert np.array_equal(to_np(goffs).astype(np.uint64), eoffs)


def test_decode_sizes_exact(torch, dev, oracle):
    """kx_thrift_decode_sizes: the units a decode fills, per column (data, elem_offsets, sub_offsets)"""
    cdc = codec("nx")
    sch = SCHEMAS["nx"]
    n = 1500
    _, wire, offs = NC.batch(sch, n, seed=3)
    rc, exp, _, _ = oracle.decode(sch, wire, n, offsets=offs)
    buf = torch.from_numpy(wire).to(dev)
    units = cdc.DecodeSizes(buf, n, torch.from_numpy(offs.view(np.int64)).to(dev))
    _, infos, _ = oracle.flatten(sch)
    for c, ci in enumerate(infos):
        if ci.kind == A.COL_FIXED:
            assert units[3 * c] == n
            continue
        parts = exp.cols[c]
        arrays = [np.asarray(p).view(np.uint32 if np.asarray(p).itemsize == 4 else np.uint64) for p in parts[:-1]]
        # each array's closing entry is the size of the level below
        hi, sizes = n, []
        for a in arrays:
            hi = int(a[hi])
            sizes.append(hi)
        assert units[3 * c] == sizes[-1], f"column {c}"
        if len(arrays) >= 2:
            assert units[3 * c + 1] == sizes[0]
        if len(arrays) >= 3:
            assert units[3 * c + 2] == sizes[1]


@pytest.mark.parametrize("kind,code", [("truncated", A.ERR_EOF), ("negative_list", A.ERR_NEGATIVE_SIZE),
                                       ("bad_type_unknown", A.ERR_INVALID_DATA)])
@pytest.mark.parametrize("known", [True, False])
def test_errors_match_oracle(torch, dev, oracle, kind, code, known):
    cdc = codec("nesting")
    sch = SCHEMAS["nesting"]
    wire, offs = _err_wire(sch, kind)
    rc, exp, est, ers = oracle.decode(sch, wire, 5, offsets=offs if known else None)
    buf = torch.from_numpy(wire).to(dev)
    o = torch.from_numpy(offs.view(np.int64)).to(dev) if known else None
    res = cdc.Unmarshal(buf, 5, offsets=o, record_status=True, raise_on_error=False)
    st = res.read_status()
    assert st.code == est.code != 0 and (not known or st.code == code)
    assert (st.record, st.offset, st.n_records) == (est.record, est.offset, est.n_records)
    _, infos, _ = oracle.flatten(sch)
    if known:
        assert list(to_np(res.record_status)[:5]) == list(ers)
        assert_columns_equal(res.columns, exp, infos, 5)
    else:
        assert_columns_equal(res.columns, exp, infos, est.n_records)


def test_large_batch_timed(torch, dev, oracle):
    """100k NestingMethod records (≈55 MB): decode + encode on the GPU, bit-exact on a slice and round-tripped"""
    cdc = codec("idl_nesting")
    sch = SCHEMAS["idl_nesting"]
    n = 100_000
    _, wire, offs = NC.batch(sch, n, seed=77, max_elems=3, max_str=16)
    buf = torch.from_numpy(wire).to(dev)
    res = cdc.Unmarshal(buf, n)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = cdc.Unmarshal(buf, n)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    got, _ = cdc.Marshal(res.columns)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"nested decode {n} NestingMethod records ({wire.size / 1e6:.1f} MB): {(t1 - t0) * 1e3:.2f} ms, "
          f"encode {(t2 - t1) * 1e3:.2f} ms")
    k = 2000
    rc, exp, _, _ = oracle.decode(sch, wire[:int(offs[k])], k)
    _, infos, _ = oracle.flatten(sch)
    assert_columns_equal(res.columns, exp, infos, k)
    rc, back, _ = oracle.encode(sch, oracle.decode(sch, wire, n)[1])
    assert np.array_equal(to_np(got), back)


def test_unmarshal_extents_sized_exactly(torch, dev, oracle):
    """UnmarshalExtents of a nested schema without var_caps sizes its arenas with the measure pass over
    the same extents (kx_thrift_decode_sizes_extents) instead of one buf-sized arena per column; the
    bodies sit at gaps (ttstream frames between them) and decode as the oracle does"""
    cdc = codec("nx")
    sch = SCHEMAS["nx"]
    n = 900
    _, wire, offs = NC.batch(sch, n, seed=8)
    gap = 5
    buf_np = np.zeros(wire.size + gap * (n + 1), dtype=np.uint8)
    starts = np.zeros(n, dtype=np.int64)
    ends = np.zeros(n, dtype=np.int64)
    for i in range(n):
        a, b = int(offs[i]), int(offs[i + 1])
        s0 = a + gap * (i + 1)
        buf_np[s0:s0 + b - a] = wire[a:b]
        starts[i], ends[i] = s0, s0 + b - a
    buf = torch.from_numpy(buf_np).to(dev)
    res = cdc.UnmarshalExtents(buf, torch.from_numpy(starts).to(dev), torch.from_numpy(ends).to(dev))
    rc, exp, _, _ = oracle.decode(sch, wire, n, offsets=offs)
    _, infos, _ = oracle.flatten(sch)
    for c, ci in enumerate(infos):
        col = res.columns.cols[c]
        if isinstance(col, tuple):   # arenas sized to the decoded units, not to the buffer
            assert col[-1].numel() <= max(1, wire.size)
    assert_columns_equal(res.columns, exp, infos, n)
