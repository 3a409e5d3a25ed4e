"""GPU parity of Kitex-Protobuf nested messages (include/kxcodec.h, KX_STRUCT_PROTOBUF; the nested walker of
kitex_amd/csrc/kx_nested.h in proto mode) through libkxcodec's C-ABI against the oracle
(oracle/kx_oracle_nested.c, pinned by google.protobuf in tests/test_pbn.py): every proto3 shape of the test
message (zig-zag, fixed32/64, float, uint32/64, bool, double, string/bytes, packed and unpacked repeated
scalars, repeated strings, nested and repeated messages, maps with scalar, string and message values,
proto3 optional), canonical and noisy bytes, known offsets, explicit extents and Batch-framed batches,
errors, and bit-exact encode. Also the committed upb fixture (tests/golden/pbn_batch_*.bin)."""
import os

import numpy as np
import pytest

from tests import pbn_cases as P
from tests.helpers import assert_columns_equal, to_np

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


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
    from kitex_amd.codec import ProtobufCodec
    if name not in _codecs:
        _codecs[name] = ProtobufCodec(P.SCHEMAS[name]())
    return _codecs[name]


def _gpu_decode(torch, dev, name, wire, n, offs=None):
    cdc = codec(name)
    buf = torch.from_numpy(wire.copy()).to(dev) if wire.size else torch.empty(0, dtype=torch.uint8, device=dev)
    o = torch.from_numpy(offs.astype(np.int64)).to(dev) if offs is not None else None
    res = cdc.Unmarshal(buf, n, offsets=o, record_status=offs is not None, raise_on_error=False)
    return res


@pytest.mark.parametrize("name", ["PN", "PK"])
@pytest.mark.parametrize("noise", [False, True])
@pytest.mark.parametrize("mode", ["offsets", "framed"])
@pytest.mark.parametrize("n", [1, 257, 5000])
def test_decode_matches_oracle(torch, dev, oracle, name, noise, mode, n):
    sch = P.SCHEMAS[name]()
    framed = mode == "framed"
    _, wire, offs = P.batch(n, seed=n + (7 if noise else 0), noise=noise, name=name, framed=framed)
    o = None if framed else offs
    rc, exp, est, _ = oracle.decode(sch, wire, n, offsets=o, pb=True)
    assert est.code == 0
    res = _gpu_decode(torch, dev, name, wire, n, o)
    st = res.read_status()
    _, infos, _ = oracle.flatten(sch)
    assert st.code == 0 and st.n_records == n and st.consumed == est.consumed
    assert_columns_equal(res.columns, exp, infos, n)


def test_extents_match_oracle(torch, dev, oracle):
    """bare bodies at explicit extents with gaps (ttstream ProtobufStruct payloads), sized exactly"""
    sch = P.schema_pn()
    n = 700
    _, wire, offs = P.batch(n, seed=3, noise=True)
    gap = 3
    buf_np = np.zeros(wire.size + gap * (n + 1), dtype=np.uint8)
    starts, ends = np.zeros(n, np.int64), np.zeros(n, np.int64)
    for i in range(n):
        a, b = int(offs[i]), int(offs[i + 1])
        s0 = a + gap * (i + 1)
        buf_np[s0:s0 + b - a] = wire[a:b]
        starts[i], ends[i] = s0, s0 + b - a
    res = codec("PN").UnmarshalExtents(torch.from_numpy(buf_np).to(dev), torch.from_numpy(starts).to(dev),
                                       torch.from_numpy(ends).to(dev))
    rc, exp, _, _ = oracle.decode(sch, wire, n, offsets=offs, pb=True)
    _, infos, _ = oracle.flatten(sch)
    assert_columns_equal(res.columns, exp, infos, n)


@pytest.mark.parametrize("case", ["truncated_varint", "bad_utf8", "group", "field0", "sub_overrun",
                                  "packed_trunc"])
def test_errors_match_oracle(torch, dev, oracle, case):
    from tests.test_pbn import ERRS
    sch = P.schema_pn()
    _, good, goffs = P.batch(5, seed=2)
    bodies = [good[int(goffs[i]):int(goffs[i + 1])].tobytes() for i in range(5)]
    bodies[3] = ERRS[case]
    wire = np.frombuffer(b"".join(bodies), dtype=np.uint8).copy()
    offs = np.zeros(6, dtype=np.uint64)
    offs[1:] = np.cumsum([len(b) for b in bodies])
    rc, exp, est, ers = oracle.decode(sch, wire, 5, offsets=offs, pb=True)
    res = _gpu_decode(torch, dev, "PN", wire, 5, offs)
    st = res.read_status()
    _, infos, _ = oracle.flatten(sch)
    assert est.code != 0 and (st.code, st.record) == (est.code, est.record) == (est.code, 3)
    assert list(to_np(res.record_status)[:5]) == list(ers)
    assert_columns_equal(res.columns, exp, infos, 5)


def test_framed_error_ends_batch(torch, dev, oracle):
    sch = P.schema_pn()
    _, wire, offs = P.batch(400, seed=9, framed=True)
    b = bytearray(wire.tobytes())
    b[int(offs[250])] = 0x00                      # record 250's first tag: field number 0
    w2 = np.frombuffer(bytes(b), dtype=np.uint8).copy()
    for data in (w2, wire[:int(offs[300]) - 2]):
        rc, exp, est, _ = oracle.decode(sch, data, 400, pb=True)
        res = _gpu_decode(torch, dev, "PN", data, 400)
        st = res.read_status()
        _, infos, _ = oracle.flatten(sch)
        assert (st.code, st.record, st.offset, st.n_records, st.consumed) == \
            (est.code, est.record, est.offset, est.n_records, est.consumed)
        assert_columns_equal(res.columns, exp, infos, est.n_records)


@pytest.mark.parametrize("name", ["PN", "PK"])
@pytest.mark.parametrize("n", [1, 3000])
def test_encode_bit_exact(torch, dev, oracle, name, n):
    """proto.Marshal on the device == the oracle's (field-number order, packed, zero omission, maps)"""
    sch = P.SCHEMAS[name]()
    _, wire, offs = P.batch(n, seed=40 + n, name=name)
    rc, cols, st, _ = oracle.decode(sch, wire, n, offsets=offs, pb=True)
    rc, ow, _ = oracle.encode(sch, cols, pb=True)
    from tests.test_gpu_nested import to_dev
    got, _ = codec(name).Marshal(to_dev(torch, dev, cols))
    assert np.array_equal(to_np(got), ow)


def test_golden_fixture(torch, dev, oracle):
    """the committed upb-serialized Batch (tests/golden/make_pbn_golden.py) decodes like the oracle and
    re-encodes to upb's bytes (its maps hold at most one entry)"""
    path = os.path.join(GOLDEN, "pbn_batch_64.bin")
    wire = np.fromfile(path, dtype=np.uint8)
    sch = P.schema_pn()
    rc, exp, est, _ = oracle.decode(sch, wire, 64, pb=True)
    assert est.code == 0 and est.consumed == wire.size
    res = _gpu_decode(torch, dev, "PN", wire, 64)
    _, infos, _ = oracle.flatten(sch)
    assert_columns_equal(res.columns, exp, infos, 64)
    got, _ = codec("PN").Marshal(res.columns)
    assert np.array_equal(to_np(got), wire)
