"""Kitex-Protobuf nested messages on the CPU (include/kxcodec.h, KX_STRUCT_PROTOBUF): the oracle's proto3
restatement (oracle/kx_oracle_nested.c) pinned by google.protobuf (upb, third-party, in this image) on the
writer's canonical and noisy bytes, and the device walker's source (kitex_amd/csrc/kx_nested.h, proto mode,
run on the host by tests/emu/nested_host.cpp) against the oracle: columns, codes, bit-exact encode.

The reference calls proto.Unmarshal / proto.Marshal (pkg/remote/codec/protobuf/protobuf.go:64-134,209-216)
from google.golang.org/protobuf, which is not vendored; upb implements the same published wire format and
message semantics (last singular wins, messages merge, repeated append, packed and unpacked scalars, maps
from entries). Map entry order is not fixed by proto.Marshal (Go maps iterate in random order): byte
comparisons with upb are made on records whose maps hold at most one entry, semantic ones on the rest."""
import numpy as np
import pytest

from kitex_amd import _abi as A
from tests import pbn_cases as P
from tests.helpers import assert_columns_equal

pytest.importorskip("google.protobuf")


@pytest.fixture(scope="module")
def upb():
    return P.upb_classes()


@pytest.fixture(scope="module")
def emu():
    from tests.emu import emu as E
    E.lib()
    return E


def _small_maps(v, name="PN"):
    for num, fname, ty, label in P.MESSAGES[name]:
        if label == "map" and len(v.get(fname, {})) > 1:
            return False
        if ty in P.MESSAGES and label == "repeated":
            if not all(_small_maps(e, ty) for e in v.get(fname, [])):
                return False
        elif ty in P.MESSAGES and fname in v:
            if not _small_maps(v[fname], ty):
                return False
    return True


def _bodies(wire, offs, n):
    return [wire[int(offs[i]):int(offs[i + 1])].tobytes() for i in range(n)]


@pytest.mark.parametrize("name", ["PN", "PK"])
def test_writer_matches_upb(upb, name):
    """the independent writer's canonical bytes are proto.Marshal's (upb, deterministic)"""
    vals, wire, offs = P.batch(200, seed=5, name=name)
    exact = 0
    for v, body in zip(vals, _bodies(wire, offs, len(vals))):
        m = upb[name]()
        P.fill(upb, name, m, v)
        if _small_maps(v, name):
            assert m.SerializeToString(deterministic=True) == body
            exact += 1
        m2 = upb[name]()
        m2.ParseFromString(body)
        assert m2 == m
    assert exact > 20


@pytest.mark.parametrize("name", ["PN", "PK"])
@pytest.mark.parametrize("noise", [False, True])
def test_oracle_roundtrip_pinned_by_upb(oracle, upb, name, noise):
    """oracle decode -> oracle encode reproduces the message upb reads from the same bytes; on canonical
    bytes the re-encode is byte-identical (encoder order, packing, zero omission, map entries)"""
    sch = P.SCHEMAS[name]()
    n = 300
    vals, wire, offs = P.batch(n, seed=11, noise=noise, name=name)
    rc, cols, st, _ = oracle.decode(sch, wire, n, offsets=offs, pb=True)
    assert rc == 0 and st.code == 0
    rc, wire2, offs2 = oracle.encode(sch, cols, pb=True)
    assert rc == 0
    from tests.pb_cases import split_frames
    bodies2 = split_frames(wire2)
    assert len(bodies2) == n
    for i, (b0, b2) in enumerate(zip(_bodies(wire, offs, n), bodies2)):
        m0, m2 = upb[name](), upb[name]()
        m0.ParseFromString(b0)
        m2.ParseFromString(b2)
        m0.DiscardUnknownFields()   # upb keeps unknown fields; proto.Unmarshal into a Go struct drops them here
        assert m0 == m2, f"record {i}"
        if not noise:
            assert b0 == b2, f"record {i}"


def test_oracle_map_duplicates_and_absent_entry_parts(oracle, upb):
    """map entries in wire order (a later duplicate key wins when inserted into a map, as upb's parse);
    an entry without key or value decodes as the zero key / value"""
    sch = P.schema_pn()
    u, t = P.uvarint, P.tag
    ent = lambda kb, vb: t(17, 2) + u(len(kb + vb)) + kb + vb  # noqa: E731  map<string,int64> counts = 17
    body = (ent(t(1, 2) + u(1) + b"a", t(2, 0) + u(5)) + ent(t(1, 2) + u(1) + b"a", t(2, 0) + u(7)) +
            ent(b"", t(2, 0) + u(9)) + ent(t(1, 2) + u(1) + b"b", b""))
    wire = np.frombuffer(body, dtype=np.uint8).copy()
    offs = np.array([0, wire.size], dtype=np.uint64)
    rc, cols, st, _ = oracle.decode(sch, wire, 1, offsets=offs, pb=True)
    assert rc == 0
    rc, wire2, _ = oracle.encode(sch, cols, pb=True)
    from tests.pb_cases import split_frames
    m0, m2 = upb["PN"](), upb["PN"]()
    m0.ParseFromString(body)
    m2.ParseFromString(split_frames(wire2)[0])
    assert m0 == m2 and dict(m0.counts) == {"a": 7, "": 9, "b": 0}


ERRS = {
    "truncated_varint": b"\x08\xff",
    "truncated_len": b"\x5a\x05ab",
    "bad_utf8": b"\x5a\x02\xc3\x28",
    "group": b"\x0b\x0c",
    "field0": b"\x00\x01",
    "long_varint": b"\x08" + b"\xff" * 10 + b"\x01",
    "sub_overrun": b"\x7a\x02\x08",            # inner (15): length 2, then a truncated field inside
    "packed_trunc": b"\x6a\x03\x01\x02\xff",   # vals (13): packed, last varint cut at the run's end
}


@pytest.mark.parametrize("case", sorted(ERRS))
def test_errors_host_walker_matches_oracle(oracle, emu, case):
    sch = P.schema_pn()
    _, infos, npres = oracle.flatten(sch)
    _, good, goffs = P.batch(3, seed=2)
    bodies = _bodies(good, goffs, 3)
    bodies[1] = ERRS[case]
    wire = np.frombuffer(b"".join(bodies), dtype=np.uint8).copy()
    offs = np.zeros(4, dtype=np.uint64)
    offs[1:] = np.cumsum([len(b) for b in bodies])
    rc, exp, est, ers = oracle.decode(sch, wire, 3, offsets=offs, pb=True)
    rc2, got, gst, grs = emu.nested_decode(sch, infos, npres, wire, 3, offsets=offs)
    assert est.code != 0 and gst.code == est.code and gst.record == est.record == 1
    assert list(grs) == list(ers)
    assert_columns_equal(got, exp, infos, 3)


@pytest.mark.parametrize("name", ["PN", "PK"])
@pytest.mark.parametrize("noise", [False, True])
@pytest.mark.parametrize("framed", [False, True])
def test_host_walker_decode_matches_oracle(oracle, emu, name, noise, framed):
    sch = P.SCHEMAS[name]()
    _, infos, npres = oracle.flatten(sch)
    n = 400
    _, wire, offs = P.batch(n, seed=21, noise=noise, name=name, framed=framed)
    o = None if framed else offs
    rc, exp, est, _ = oracle.decode(sch, wire, n, offsets=o, pb=True)
    rc2, got, gst, _ = emu.nested_decode(sch, infos, npres, wire, n, offsets=o)
    assert est.code == 0 and gst.code == 0 and gst.n_records == n and gst.consumed == est.consumed
    assert_columns_equal(got, exp, infos, n)


def test_host_walker_framed_errors_match_oracle(oracle, emu):
    """Batch frames: the first failing record ends the batch (its frame start is the status offset)"""
    sch = P.schema_pn()
    _, infos, npres = oracle.flatten(sch)
    _, wire, offs = P.batch(50, seed=4, framed=True)
    b = bytearray(wire.tobytes())
    cut = int(offs[30])                          # body of record 30: corrupt its first tag into field 0
    b[cut] = 0x00
    w2 = np.frombuffer(bytes(b), dtype=np.uint8).copy()
    for data in (w2, wire[:int(offs[40]) - 3]):  # a bad body; a truncated frame
        rc, exp, est, _ = oracle.decode(sch, data, 50, pb=True)
        rc2, got, gst, _ = emu.nested_decode(sch, infos, npres, data, 50)
        assert est.code != 0 and (gst.code, gst.record, gst.offset, gst.n_records, gst.consumed) == \
            (est.code, est.record, est.offset, est.n_records, est.consumed)
        assert_columns_equal(got, exp, infos, est.n_records)


@pytest.mark.parametrize("name", ["PN", "PK"])
def test_host_walker_encode_bit_exact(oracle, emu, name):
    sch = P.SCHEMAS[name]()
    _, infos, _ = oracle.flatten(sch)
    n = 300
    _, wire, offs = P.batch(n, seed=31, name=name)
    rc, cols, st, _ = oracle.decode(sch, wire, n, offsets=offs, pb=True)
    assert rc == 0
    rc, ow, _ = oracle.encode(sch, cols, pb=True)
    rc2, ew, _ = emu.nested_encode(sch, infos, cols)
    assert rc == 0 and rc2 == 0
    assert np.array_equal(ow, ew)


def test_flat_proto_schema_stays_flat():
    """a flat proto3 message of natural kinds keeps the tile pipeline (and its layout)"""
    from kitex_amd import schema as S
    from kitex_amd.codec import DeviceSchema
    assert not DeviceSchema(S.schema_pf()).nested
    assert DeviceSchema(P.schema_pk()).nested


def test_proto_schema_refusals():
    """proto3 has no required fields, 8/16-bit scalars or containers of containers"""
    from kitex_amd._lib import KxError
    from kitex_amd.codec import DeviceSchema
    from kitex_amd.schema import Field, Schema, Struct
    bad = [Schema(Struct("R", [Field(1, A.T_I64, "a", req=A.REQ_REQUIRED), Field(2, A.T_LIST, "l", elem=A.T_I64)]),
                  protobuf=True),
           Schema(Struct("B", [Field(1, A.T_I16, "a"), Field(2, A.T_LIST, "l", elem=A.T_I64)]), protobuf=True),
           Schema(Struct("C", [Field(1, A.T_LIST, "l", elem=Field(0, A.T_LIST, elem=A.T_I64))]), protobuf=True)]
    for sch in bad:
        with pytest.raises(KxError):
            DeviceSchema(sch)


def test_golden_fixture_oracle_and_host_walker(oracle, emu):
    """the committed upb-serialized Batch of 64 PN records (tests/golden/make_pbn_golden.py): the oracle
    and the host walker decode it alike and both re-encode upb's bytes exactly"""
    import os
    wire = np.fromfile(os.path.join(os.path.dirname(__file__), "golden", "pbn_batch_64.bin"), dtype=np.uint8)
    sch = P.schema_pn()
    _, infos, npres = oracle.flatten(sch)
    rc, exp, est, _ = oracle.decode(sch, wire, 64, pb=True)
    assert rc == 0 and est.code == 0 and est.consumed == wire.size
    rc2, got, gst, _ = emu.nested_decode(sch, infos, npres, wire, 64)
    assert gst.code == 0
    assert_columns_equal(got, exp, infos, 64)
    rc, ow, _ = oracle.encode(sch, exp, pb=True)
    rc2, ew, _ = emu.nested_encode(sch, infos, exp)
    assert np.array_equal(ow, wire) and np.array_equal(ew, wire)
