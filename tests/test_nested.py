"""Nested schemas on the CPU (include/kxcodec.h "Nested schemas"): the library's column layout against the
oracle's (oracle/kx_oracle_nested.c), and the device walker's source (kitex_amd/csrc/kx_nested.h, run on the
host by tests/emu/nested_host.cpp with the device pipeline's steps) against the oracle, on batches written by
the independent writer of tests/nested_cases.py: canonical and noisy records (shuffled fields, unknown ids,
mistyped ids, repeated fields), known offsets and concatenated, errors, capacities, round trips.

Parity of these shapes is pinned by construction only (no reference fixture holds a nested record): the
writer, the oracle and the walker are three independent implementations of the reference's field loop
(struct_tpl.go:41-149, 405-625) and FastWriteNocopy (:225-391)."""
import os

import numpy as np
import pytest

from kitex_amd import _abi as A
from kitex_amd import idl
from kitex_amd import schema as S
from kitex_amd.schema import Field
from tests import nested_cases as NC
from tests.helpers import assert_columns_equal

IDL = os.path.join(os.path.dirname(__file__), "golden", "idl")


def _schemas():
    doc_b = idl.parse_idl(os.path.join(IDL, "baseline.thrift"))
    doc_e = idl.parse_idl(os.path.join(IDL, "example.thrift"))
    return {
        "nesting": S.schema_nesting(),
        "nx": S.schema_nx(),
        "idl_nesting": idl.request_schema(doc_b, "NestingMethod"),
        "idl_example": idl.request_schema(doc_e, "ExampleMethod"),
        "idl_foo": idl.request_schema(doc_e, "Foo"),
    }


SCHEMAS = _schemas()


@pytest.fixture(scope="module")
def emu():
    from tests.emu import emu as E
    E.lib()
    return E


def _raw_cols(infos):
    return {c for c, ci in enumerate(infos) if ci.kind in A.STRING_KINDS and (ci.elem_ttype & 15 if ci.level else
                                                                              ci.ttype) == A.T_STRUCT}


@pytest.mark.parametrize("name", sorted(SCHEMAS))
def test_layout_lib_equals_oracle(oracle, name):
    from kitex_amd.codec import DeviceSchema
    sch = SCHEMAS[name]
    ds = DeviceSchema(sch)
    rc, infos, npres = oracle.flatten(sch)
    assert rc == 0 and ds.nested
    assert ds.ncols == len(infos) and ds.npresence == npres

    def key(ci):
        return (ci.kind, ci.width, ci.ttype, ci.elem_ttype, ci.field_id, ci.presence_bit, ci.depth,
                tuple(ci.path)[:ci.depth + 1], ci.level)
    assert [key(a) for a in ds.infos] == [key(b) for b in infos]


def test_nesting_layout_is_the_idl_one(oracle):
    """baseline.thrift Nesting built by hand equals the IDL compiler's"""
    a = oracle.flatten(SCHEMAS["nesting"])
    b = oracle.flatten(SCHEMAS["idl_nesting"])
    assert a[0] == b[0] == 0 and len(a[1]) == len(b[1]) == 34
    assert [(x.kind, x.width, x.level, x.elem_ttype) for x in a[1]] == [(x.kind, x.width, x.level, x.elem_ttype)
                                                                         for x in b[1]]


@pytest.mark.parametrize("name", sorted(SCHEMAS))
@pytest.mark.parametrize("noise", [False, True])
@pytest.mark.parametrize("known", [True, False])
def test_walker_decode_matches_oracle(oracle, emu, name, noise, known):
    sch = SCHEMAS[name]
    _, infos, npres = oracle.flatten(sch)
    n = 150
    _, wire, offs = NC.batch(sch, n, seed=11, noise=noise)
    o = offs if known else None
    rc1, exp, st1, rs1 = oracle.decode(sch, wire, n, offsets=o)
    rc2, got, st2, rs2 = emu.nested_decode(sch, infos, npres, wire, n, offsets=o)
    assert rc1 == 0 and rc2 == 0
    assert (st2.n_records, st2.consumed) == (st1.n_records, st1.consumed) == (n, wire.size)
    assert_columns_equal(got, exp, infos, n)


@pytest.mark.parametrize("name", sorted(SCHEMAS))
def test_noise_decodes_like_canonical(oracle, name):
    """shuffled, repeated (last wins), unknown and mistyped fields decode to the same columns"""
    sch = SCHEMAS[name]
    _, infos, _ = oracle.flatten(sch)
    n = 120
    _, cw, co = NC.batch(sch, n, seed=5)
    _, nw, no = NC.batch(sch, n, seed=5, noise=True)
    rc1, a, _, _ = oracle.decode(sch, cw, n, offsets=co)
    rc2, b, _, _ = oracle.decode(sch, nw, n, offsets=no)
    assert rc1 == rc2 == 0
    raw = _raw_cols(infos)   # a recursive struct keeps its (noisy) bytes
    keep = [c for c in range(len(infos)) if c not in raw]
    from kitex_amd.synth import ColumnSet
    sub = lambda cs: ColumnSet([cs.cols[c] for c in keep], cs.presence, n)  # noqa: E731
    assert_columns_equal(sub(b), sub(a), [infos[c] for c in keep], n)


@pytest.mark.parametrize("name", sorted(SCHEMAS))
def test_encode_matches_oracle_and_round_trips(oracle, emu, name):
    sch = SCHEMAS[name]
    _, infos, _ = oracle.flatten(sch)
    n = 150
    _, wire, offs = NC.batch(sch, n, seed=2, noise=True)
    rc, cols, _, _ = oracle.decode(sch, wire, n, offsets=offs)
    assert rc == 0
    rc1, w1, o1 = oracle.encode(sch, cols)
    rc2, w2, o2 = emu.nested_encode(sch, infos, cols)
    assert rc1 == rc2 == 0
    assert np.array_equal(w1, w2) and np.array_equal(o1, o2)
    # encode(decode(.)) reaches a fixed point: each round may turn a nil struct field written as STOP into
    # an empty struct (Go's decode allocates it), whose default fields the next FastWrite writes
    w = w1
    for _ in range(4):
        rc3, c3, st3, _ = oracle.decode(sch, w, n)
        assert rc3 == 0 and st3.consumed == w.size
        rc4, w4, _ = oracle.encode(sch, c3)
        if np.array_equal(w4, w):
            break
        w = w4
    else:
        pytest.fail("no fixed point")


def test_canonical_writer_equals_fastwrite(oracle):
    """records without nil struct fields: the independent writer's canonical bytes == encode(decode)"""
    sch = SCHEMAS["nesting"]
    g = NC.Gen(9)
    w = NC.Writer()
    recs = []
    for _ in range(100):
        v = g.struct(sch.root)
        v.setdefault(8, g.struct(sch.root.fields[7].child))   # SimpleStruct never nil
        recs.append(w.struct(sch.root, v))
    wire = np.frombuffer(b"".join(recs), dtype=np.uint8).copy()
    rc, cols, st, _ = oracle.decode(sch, wire, 100)
    assert rc == 0
    rc, back, _ = oracle.encode(sch, cols)
    assert rc == 0 and np.array_equal(back, wire)


def _err_wire(sch, kind):
    """one bad record between good ones"""
    _, good, offs = NC.batch(sch, 5, seed=1)
    recs = [good[int(offs[i]):int(offs[i + 1])].tobytes() for i in range(5)]
    if kind == "truncated":
        bad = recs[2][:len(recs[2]) // 2]
    elif kind == "negative_list":  # field 2 (ListSimple) with a negative count
        bad = bytes([A.T_LIST, 0, 2, A.T_STRUCT]) + (-3 & 0xFFFFFFFF).to_bytes(4, "big") + b"\x00"
    elif kind == "bad_type_unknown":  # an unknown field of an invalid wire type: skip fails
        bad = bytes([A.T_I64, 0, 99]) + b"\x00" * 8 + bytes([7, 0, 98, 0])
    else:
        raise ValueError(kind)
    recs[2] = bad
    wire = np.frombuffer(b"".join(recs), dtype=np.uint8).copy()
    o = np.zeros(6, dtype=np.uint64)
    o[1:] = np.cumsum([len(r) for r in recs])
    return wire, o


@pytest.mark.parametrize("kind,code", [("truncated", A.ERR_EOF), ("negative_list", A.ERR_NEGATIVE_SIZE),
                                       ("bad_type_unknown", A.ERR_INVALID_DATA)])
@pytest.mark.parametrize("known", [True, False])
def test_errors_match_oracle(oracle, emu, kind, code, known):
    sch = SCHEMAS["nesting"]
    _, infos, npres = oracle.flatten(sch)
    wire, offs = _err_wire(sch, kind)
    o = offs if known else None
    rc1, exp, st1, rs1 = oracle.decode(sch, wire, 5, offsets=o)
    rc2, got, st2, rs2 = emu.nested_decode(sch, infos, npres, wire, 5, offsets=o)
    # concatenated: the bytes after a cut record are read on as its continuation, so only the record and the
    # oracle's code are pinned; with offsets the record fails on its own with `code`
    assert st1.code == st2.code != 0 and (not known or st1.code == code)
    assert (st2.record, st2.offset, st2.n_records) == (st1.record, st1.offset, st1.n_records)
    if known:
        assert list(rs2) == list(rs1) and rs1[2] == code
        assert_columns_equal(got, exp, infos, 5)       # the failing record reads as defaults
    else:
        assert st1.n_records == 2
        assert_columns_equal(got, exp, infos, 2)


def test_required_missing_in_element_struct(oracle, emu):
    """NX.byid is map<i32, Leaf>, Leaf.k required: an entry whose Leaf lacks k fails the record"""
    sch = SCHEMAS["nx"]
    _, infos, npres = oracle.flatten(sch)
    rec = bytes([A.T_MAP, 0, 8, A.T_I32, A.T_STRUCT]) + (1).to_bytes(4, "big") + (5).to_bytes(4, "big") + \
        bytes([A.T_STRING, 0, 2]) + (1).to_bytes(4, "big") + b"q" + b"\x00" + b"\x00"
    wire = np.frombuffer(rec, dtype=np.uint8).copy()
    offs = np.array([0, wire.size], dtype=np.uint64)
    rc1, _, st1, _ = oracle.decode(sch, wire, 1, offsets=offs)
    rc2, _, st2, _ = emu.nested_decode(sch, infos, npres, wire, 1, offsets=offs)
    assert st1.code == st2.code == A.ERR_INVALID_DATA


def test_string_defaults_and_absent_fields(oracle, emu):
    """NX.title = "untitled" and Leaf.v = "none": absent -> the default string; an empty record decodes"""
    sch = SCHEMAS["nx"]
    _, infos, npres = oracle.flatten(sch)
    wire = np.zeros(1, dtype=np.uint8)    # STOP only
    caps = [0 if ci.kind == A.COL_FIXED else 64 for ci in infos]
    rc1, exp, st1, _ = oracle.decode(sch, wire, 1, var_caps=caps)
    rc2, got, st2, _ = emu.nested_decode(sch, infos, npres, wire, 1, var_caps=caps)
    assert rc1 == rc2 == 0
    assert_columns_equal(got, exp, infos, 1)
    title = [c for c, ci in enumerate(infos) if ci.field_id == 2 and ci.level == 0 and ci.kind == A.COL_BYTES][0]
    o, d = exp.cols[title]
    assert bytes(d[int(o[0]):int(o[1])]) == b"untitled"


def test_capacity_refused(oracle, emu):
    sch = SCHEMAS["nesting"]
    _, infos, npres = oracle.flatten(sch)
    _, wire, offs = NC.batch(sch, 40, seed=4)
    caps = [0 if ci.kind == A.COL_FIXED else 1 for ci in infos]
    rc, _, st, _ = emu.nested_decode(sch, infos, npres, wire, 40, offsets=offs, var_caps=caps, elem_caps=caps,
                                     sub_caps=caps)
    assert rc == A.ERR_SIZE_LIMIT


def test_idl_example_method_columns(oracle):
    """ExampleMethod (example.thrift): InnerBase.Base and Base (base.thrift) with Extra map<string,string>,
    Test.aaa = "aaaaaaa" (optional string default), optional scalars"""
    sch = SCHEMAS["idl_example"]
    rc, infos, npres = oracle.flatten(sch)
    assert rc == 0 and len(infos) == 25 and npres == 14
    assert sum(1 for ci in infos if ci.kind == A.COL_LIST_BYTES) == 4    # two Extra maps: keys, values


def test_device_limits_enforced_at_schema_create():
    """a nested program needing more cursors than the device walker holds per lane (KXN_MAX_CUR) is
    refused when the schema is created, not at its first decode"""
    from kitex_amd._lib import KxError
    from kitex_amd.codec import DeviceSchema

    def wide(k):
        return S.Schema(S.Struct("W", [Field(i + 1, A.T_MAP, f"f{i}", elem=A.T_STRING, val=A.T_STRING)
                                       for i in range(k)]))
    ds = DeviceSchema(wide(12))       # 12 x (entry domain + key bytes + value bytes) cursors: fine
    assert ds.nested
    with pytest.raises(KxError) as e:
        DeviceSchema(wide(30))        # 90 cursors > 64, 60 columns
    assert e.value.code == A.ERR_NOT_IMPLEMENTED
