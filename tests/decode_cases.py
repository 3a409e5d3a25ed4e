"""Decode parity cases shared by the GPU suite (tests/test_gpu_thrift.py, the HIP library through
the C-ABI) and the CPU emulation suite (tests/test_emu_decode.py, the same kernel source under the
SIMT emulator). Every case compares against the CPU oracle on the same input, bit-exact: decoded
columns field-for-field, error code / failing record / byte offset identical."""
import numpy as np

from kitex_amd import _abi as A
from kitex_amd import schema as S
from kitex_amd import synth
from tests.helpers import assert_columns_equal, offsets_u64, to_np


def check_decode(dec, oracle, sch, wire, n, offsets=None):
    rc, exp, est, ers = oracle.decode(sch, wire, n, offsets=offsets)
    cols, st, rs = dec.decode(sch, wire, n, offsets)
    assert st.code == est.code, (st.code, est.code)
    if est.code:
        assert (st.record, st.offset) == (est.record, est.offset)
    nrec = est.n_records
    assert st.n_records == nrec
    if offsets is None:
        assert st.consumed == est.consumed
    else:
        assert np.array_equal(to_np(rs)[:n], ers[:n])
    _, infos, _ = oracle.flatten(sch)
    ok_rows = nrec if offsets is None else n
    assert_columns_equal(cols, exp, infos, ok_rows)
    for k in range(min(8, sum(ci.kind != A.COL_FIXED for ci in infos))):
        assert st.var_total[k] == est.var_total[k]
    return cols, st


def case_concat(dec, oracle, name, n):
    sch = S.SCHEMAS[name]()
    cs = synth.GENERATORS[name](n)
    rc, wire, offs = oracle.encode(sch, cs)
    assert rc == 0
    cols, st = check_decode(dec, oracle, sch, wire, n)
    assert st.code == 0 and st.consumed == wire.size


def case_offsets(dec, oracle, name, n):
    sch = S.SCHEMAS[name]()
    cs = synth.GENERATORS[name](n, start=777)
    rc, wire, offs = oracle.encode(sch, cs)
    check_decode(dec, oracle, sch, wire, n, offsets=offs)


def case_roundtrip(dec, oracle):
    sch = S.schema_r2()
    cs = synth.gen_r2(4096)
    rc, wire, _ = oracle.encode(sch, cs)
    cols, st, _ = dec.decode(sch, wire, cs.n, None)
    assert st.code == 0
    _, infos, _ = oracle.flatten(sch)
    assert_columns_equal(cols, cs, infos, cs.n)


# ---- hand-built records: non-canonical order, unknown fields, duplicates, ragged strings ----
def rec_bytes(oracle, fields):
    """fields: list of (ttype, id, payload bytes) in wire order; appends STOP."""
    out = b""
    for t, fid, payload in fields:
        out += oracle.prim("kxo_write_field_begin", t, fid) + payload
    return out + b"\x00"


def i64(oracle, v):
    return oracle.prim("kxo_write_i64", v)


def sbytes(oracle, s: bytes):
    return oracle.prim("kxo_write_string", s, len(s))


def r2_record(oracle, rng, order=None, strlens=(32, 32), extra=None, dup=False):
    fields = [(A.T_I64, f, i64(oracle, int(rng.integers(-2**63, 2**63 - 1)))) for f in range(1, 9)]
    for j, f in enumerate((9, 10)):
        s = bytes(rng.integers(97, 123, size=strlens[j], dtype=np.uint8))
        fields.append((A.T_STRING, f, sbytes(oracle, s)))
    if order is not None:
        fields = [fields[k] for k in order]
    if extra:
        fields = fields[:3] + extra + fields[3:]
    if dup:
        fields.append((A.T_I64, 2, i64(oracle, 12345)))
        fields.append((A.T_STRING, 9, sbytes(oracle, b"dup")))
    return rec_bytes(oracle, fields)


def concat(records):
    wire = np.frombuffer(b"".join(records), dtype=np.uint8).copy()
    offs = np.zeros(len(records) + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(r) for r in records])
    return wire, offs


def case_noncanonical(dec, oracle, mode):
    """reordered fields, unknown fields (skipped), mistyped known ids (skipped), duplicates
    (last wins) — mixed with canonical ones so some tiles validate and some fall back."""
    sch = S.schema_r2()
    rng = np.random.default_rng(1)
    unknown = [(A.T_STRUCT, 77, rec_bytes(oracle, [(A.T_LIST, 1, oracle.prim("kxo_write_list_begin", A.T_STRING, 2)
                                                    + sbytes(oracle, b"a") + sbytes(oracle, b"bc"))])),
               (A.T_I32, 3, oracle.prim("kxo_write_i32", 5)),          # field 3 with the wrong type
               (A.T_MAP, 300, oracle.prim("kxo_write_map_begin", A.T_I64, A.T_DOUBLE, 2) + bytes(32))]
    recs = []
    for i in range(3000):
        k = i % 10
        if k == 3:
            recs.append(r2_record(oracle, rng, order=list(rng.permutation(10))))
        elif k == 5:
            recs.append(r2_record(oracle, rng, extra=unknown))
        elif k == 7:
            recs.append(r2_record(oracle, rng, dup=True))
        else:
            recs.append(r2_record(oracle, rng))
    wire, offs = concat(recs)
    check_decode(dec, oracle, sch, wire, len(recs), offsets=offs if mode == "offsets" else None)


def case_ragged(dec, oracle, mode):
    """empty strings, strings crossing tile/halo boundaries, one string larger than a tile."""
    sch = S.schema_r2()
    rng = np.random.default_rng(2)
    recs = []
    lens = [0, 1, 3, 4, 5, 31, 32, 33, 127, 128, 129, 511, 513, 4097, 40000, 70000, 0, 2]
    for i in range(600):
        a = lens[i % len(lens)] if i % 3 == 0 else int(rng.integers(0, 64))
        b = lens[(i * 7) % len(lens)] if i % 5 == 0 else int(rng.integers(0, 40))
        recs.append(r2_record(oracle, rng, strlens=(a, b)))
    wire, offs = concat(recs)
    check_decode(dec, oracle, sch, wire, len(recs), offsets=offs if mode == "offsets" else None)


def case_empty(dec, oracle):
    """records with no fields at all (just STOP) decode to defaults; 1-byte records pack a tile."""
    sch = S.Schema(S.Struct("D", [S.Field(1, A.T_I64, default=42), S.Field(2, A.T_I32, default=-7),
                                  S.Field(3, A.T_BOOL), S.Field(4, A.T_STRING)]))
    recs = []
    for i in range(70000):
        if i % 4 == 0:
            recs.append(rec_bytes(oracle, [(A.T_I64, 1, i64(oracle, i)), (A.T_BOOL, 3, bytes([i % 3]))]))
        else:
            recs.append(b"\x00")
    wire, offs = concat(recs)
    check_decode(dec, oracle, sch, wire, len(recs))
    check_decode(dec, oracle, sch, wire, len(recs), offsets=offs)


def case_slot_overflow(dec, oracle):
    """tiles holding far more records than the batch's mean size predicts (large records, then a run of
    1-byte records): the first slotcap record starts of such a tile are kept, the rest are emitted one per
    round from the previous record's end (kx_decode.hip ws_layout / emit_tile)"""
    sch = S.Schema(S.Struct("D", [S.Field(1, A.T_I64, default=42), S.Field(2, A.T_I32, default=-7),
                                  S.Field(3, A.T_BOOL), S.Field(4, A.T_STRING)]))
    recs = []
    for i in range(24):
        recs.append(rec_bytes(oracle, [(A.T_I64, 1, i64(oracle, i)), (A.T_STRING, 4, sbytes(oracle, b"x" * 30000))]))
    for i in range(30000):
        recs.append(rec_bytes(oracle, [(A.T_BOOL, 3, bytes([1]))]) if i % 1000 == 7 else b"\x00")
    for i in range(24):
        recs.append(rec_bytes(oracle, [(A.T_STRING, 4, sbytes(oracle, b"y" * (i * 37)))]))
    wire, offs = concat(recs)
    assert wire.size / len(recs) > 20          # the mean-size slot estimate is far below the 1-byte run's
    check_decode(dec, oracle, sch, wire, len(recs))
    check_decode(dec, oracle, sch, wire, len(recs), offsets=offs)


def case_long_strings(dec, oracle, n=400, seed=3):
    """strings at and past the wave-copy threshold (1024 B, kx_decode.hip wave_copy_one) among short ones,
    random bytes at every destination alignment: the ones inside a tile's window (the fast emit form copies
    from LDS) and the ones that leave it (the general form copies from global memory)"""
    rng = np.random.default_rng(seed)
    sch = S.Schema(S.Struct("L", [S.Field(1, A.T_I64), S.Field(2, A.T_STRING), S.Field(3, A.T_STRING, binary=True)]))
    kinds = rng.integers(0, 6, size=n)
    recs = []
    for i in range(n):
        k = kinds[i]
        ln = [int(rng.integers(0, 40)), 1023, 1024, int(rng.integers(1025, 3000)),
              int(rng.integers(3000, 40000)), int(rng.integers(0, 8))][k]
        s = rng.integers(0, 256, size=ln, dtype=np.uint8).tobytes()
        b = rng.integers(0, 256, size=int(rng.integers(0, 1200 if i % 7 == 0 else 20)), dtype=np.uint8).tobytes()
        recs.append(rec_bytes(oracle, [(A.T_I64, 1, i64(oracle, i * 7919)), (A.T_STRING, 2, sbytes(oracle, s)),
                                       (A.T_STRING, 3, sbytes(oracle, b))]))
    wire, offs = concat(recs)
    check_decode(dec, oracle, sch, wire, n)
    check_decode(dec, oracle, sch, wire, n, offsets=offs)


def case_nested(dec, oracle):
    inner = S.Struct("In", [S.Field(1, A.T_I64, req=A.REQ_REQUIRED), S.Field(2, A.T_STRING, req=A.REQ_OPTIONAL),
                            S.Field(3, A.T_I16, default=9)])
    sch = S.Schema(S.Struct("Out", [S.Field(1, A.T_I32), S.Field(2, A.T_STRUCT, child=inner),
                                    S.Field(3, A.T_LIST, elem=A.T_I16), S.Field(4, A.T_DOUBLE, req=A.REQ_OPTIONAL)]))
    P = oracle.prim
    good_inner = rec_bytes(oracle, [(A.T_I64, 1, i64(oracle, 5)), (A.T_STRING, 2, sbytes(oracle, b"xy")),
                                    (A.T_I16, 3, P("kxo_write_i16", 3))])
    inner2 = rec_bytes(oracle, [(A.T_I64, 1, i64(oracle, 6))])                 # second occurrence resets
    recs = []
    for i in range(2000):
        f = [(A.T_I32, 1, P("kxo_write_i32", i)), (A.T_STRUCT, 2, good_inner),
             (A.T_LIST, 3, P("kxo_write_list_begin", A.T_I16, 3) + P("kxo_write_i16", 1) * 3)]
        if i % 3 == 0:
            f.append((A.T_STRUCT, 2, inner2))
        if i % 4 == 0:
            f.append((A.T_DOUBLE, 4, P("kxo_write_double", 1.5)))
        if i % 11 == 0:
            f.append((A.T_LIST, 3, P("kxo_write_list_begin", A.T_STRING, 1) + P("kxo_write_i16", 7)))  # elem type ignored
        recs.append(rec_bytes(oracle, f))
    wire, offs = concat(recs)
    check_decode(dec, oracle, sch, wire, len(recs), offsets=offs)
    check_decode(dec, oracle, sch, wire, len(recs))
    # a record whose nested struct misses its required field fails with INVALID_DATA
    bad = rec_bytes(oracle, [(A.T_I32, 1, P("kxo_write_i32", 1)),
                             (A.T_STRUCT, 2, rec_bytes(oracle, [(A.T_I16, 3, P("kxo_write_i16", 3))]))])
    wire2, offs2 = concat(recs[:500] + [bad] + recs[500:900])
    cols, st = check_decode(dec, oracle, sch, wire2, 901)
    assert st.code == A.ERR_INVALID_DATA and st.record == 500
    cols, st = check_decode(dec, oracle, sch, wire2, 901, offsets=offs2)
    assert st.code == A.ERR_INVALID_DATA and st.record == 500


ERROR_CASES = ["truncated", "negative", "unknown_type", "depth", "short_input"]


def case_error(dec, oracle, case):
    sch = S.schema_r2()
    rng = np.random.default_rng(4)
    recs = [r2_record(oracle, rng) for _ in range(900)]
    n = len(recs)
    if case == "truncated":
        wire, offs = concat(recs)
        wire = wire[:-7]
    elif case == "negative":
        recs[400] = rec_bytes(oracle, [(A.T_STRING, 9, bytes.fromhex("fffffff0"))])
        wire, offs = concat(recs)
    elif case == "unknown_type":
        recs[123] = rec_bytes(oracle, [(A.T_I64, 1, i64(oracle, 1)), (99, 50, b"")])
        wire, offs = concat(recs)
    elif case == "depth":
        deep = rec_bytes(oracle, [(A.T_STRING, 1, sbytes(oracle, b"x"))])
        for _ in range(63):
            deep = rec_bytes(oracle, [(A.T_STRUCT, 1, deep)])
        recs[77] = rec_bytes(oracle, [(A.T_STRUCT, 99, deep)])
        wire, offs = concat(recs)
    else:
        wire, offs = concat(recs)
        n = n + 5                                     # ask for more records than the input holds
    check_decode(dec, oracle, sch, wire, n)
    if case != "short_input":
        o = offs.copy()
        if case == "truncated":
            o[-1] = wire.size
        check_decode(dec, oracle, sch, wire, len(recs), offsets=o)


def case_skip(skipper, oracle):
    sch = S.schema_r3()
    cs = synth.gen_r3(3000)
    rc, wire, offs = oracle.encode(sch, cs)
    got = skipper(wire, cs.n)
    assert np.array_equal(to_np(got).astype(np.uint64), offs)


# ---- R2 + base.Base (pkg/generic/json_test/idl/base.thrift:10-17): 11 var slots on the flat pipeline ----
R2BASE_IDL = """include "base.thrift"
struct R2Base {
  1: i64 a1, 2: i64 a2, 3: i64 a3, 4: i64 a4, 5: i64 a5, 6: i64 a6, 7: i64 a7, 8: i64 a8,
  9: string s9, 10: string s10,
  255: base.Base Base,
}
"""


def schema_r2_base():
    import os

    from kitex_amd import idl
    d = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "idl")
    return idl.to_schema(idl.parse_idl(R2BASE_IDL, include_dirs=[d]).struct("R2Base"))


def r2_base_record(oracle, rng, i, repeat=False):
    P = oracle.prim
    fields = [(A.T_I64, f, i64(oracle, int(rng.integers(-2**63, 2**63 - 1)))) for f in range(1, 9)]
    fields += [(A.T_STRING, f, sbytes(oracle, bytes(rng.integers(97, 123, size=int(rng.integers(0, 40)),
                                                                 dtype=np.uint8)))) for f in (9, 10)]
    base = [(A.T_STRING, 1, sbytes(oracle, b"log-%d" % i)), (A.T_STRING, 2, sbytes(oracle, b"caller.svc")),
            (A.T_STRING, 3, sbytes(oracle, b"10.0.%d.%d:8888" % (i % 256, i % 7))),
            (A.T_STRING, 4, sbytes(oracle, b"" if i % 3 else b"client"))]
    if i % 2:
        base.append((A.T_STRUCT, 5, rec_bytes(oracle, [(A.T_BOOL, 1, P("kxo_write_bool", i % 4 == 1)),
                                                       (A.T_STRING, 2, sbytes(oracle, b"env%d" % (i % 5)))])))
    k = i % 4
    if k:
        m = P("kxo_write_map_begin", A.T_STRING, A.T_STRING, k)
        for j in range(k):
            m += sbytes(oracle, b"k%d" % j) + sbytes(oracle, b"v%d-%d" % (i, j))
        base.append((A.T_MAP, 6, m))
    if i % 5 == 0:
        base = base[::-1]                     # some records off the canonical order: the walk path
    fields.append((A.T_STRUCT, 255, rec_bytes(oracle, base)))
    if repeat and i % 3 == 1:
        # 255:Base again without its Extra map: the struct is replaced wholesale (NewX() + FastRead,
        # struct_tpl.go:79-101), so the first copy's Extra entries (var slots 7..10) must not survive
        fields.append((A.T_STRUCT, 255, rec_bytes(oracle, [(A.T_STRING, 1, sbytes(oracle, b"again-%d" % i))])))
    return rec_bytes(oracle, fields)


def case_r2_base(dec, oracle, mode, n=3000, repeat=False):
    sch = schema_r2_base()
    rng = np.random.default_rng(8)
    wire, offs = concat([r2_base_record(oracle, rng, i, repeat) for i in range(n)])
    check_decode(dec, oracle, sch, wire, n, offsets=offs if mode == "offsets" else None)


# ---- split points (kx_thrift_split_points: SURVEY.md §8e pass A) ------------------------------------
def expected_points(offs, n, parts):
    return np.array([int(offs[(k * n) // parts]) if k < parts else int(offs[n]) for k in range(parts + 1)],
                    dtype=np.uint64)


SPLIT_CASES = ["r2", "r3", "r1", "noncanonical", "slot_overflow", "ragged", "tiny"]


def split_input(oracle, case):
    """(schema, wire, offs) of one split-point case"""
    if case in ("r2", "r3", "r1"):
        sch = S.SCHEMAS[case]()
        n = {"r2": 20000, "r3": 3000, "r1": 30000}[case]
        cs = synth.GENERATORS[case](n)
        rc, wire, offs = oracle.encode(sch, cs)
        return sch, wire, offs
    if case == "tiny":
        sch = S.schema_r2()
        rc, wire, offs = oracle.encode(sch, synth.gen_r2(5))
        return sch, wire, offs
    rng = np.random.default_rng(11)
    if case == "noncanonical":       # every 3rd record reordered: the walk path, not the fast path
        recs = [r2_record(oracle, rng, order=list(rng.permutation(10)) if i % 3 == 0 else None)
                for i in range(4000)]
        return (S.schema_r2(),) + concat(recs)
    if case == "ragged":             # records larger than a tile between small ones
        recs = [r2_record(oracle, rng, strlens=((20000 if i % 97 == 0 else int(rng.integers(0, 64))), 3))
                for i in range(2000)]
        return (S.schema_r2(),) + concat(recs)
    sch = S.Schema(S.Struct("D", [S.Field(1, A.T_I64, default=42), S.Field(2, A.T_I32, default=-7),
                                  S.Field(3, A.T_BOOL), S.Field(4, A.T_STRING)]))
    recs = [rec_bytes(oracle, [(A.T_I64, 1, i64(oracle, i)), (A.T_STRING, 4, sbytes(oracle, b"x" * 30000))])
            for i in range(24)]
    recs += [b"\x00"] * 30000          # tiles of 1-byte records: past the record-start slots
    recs += [rec_bytes(oracle, [(A.T_STRING, 4, sbytes(oracle, b"y" * 100))]) for i in range(24)]
    return (sch,) + concat(recs)


def case_split(splitter, oracle, case, parts_list=(1, 2, 3, 8, 64)):
    """splitter(schema, wire, n, parts) -> (points, status): record floor(k n / parts)'s start per k, the
    batch end last, and the status of a clean pass"""
    sch, wire, offs = split_input(oracle, case)
    n = len(offs) - 1
    for parts in parts_list:
        pts, st = splitter(sch, wire, n, parts)
        assert st.code == 0 and st.n_records == n and st.consumed == wire.size, (parts, st.code)
        assert np.array_equal(to_np(pts).astype(np.uint64), expected_points(offs, n, parts)), parts


def case_split_errors(splitter, oracle):
    """a decode error or EOF before n records: the decode's status; n == 0: zero points"""
    sch = S.schema_r2()
    rng = np.random.default_rng(4)
    recs = [r2_record(oracle, rng) for _ in range(900)]
    wire, offs = concat(recs)
    for data, n in ((wire[:-7], 900), (wire, 905)):
        rc, exp, est, _ = oracle.decode(sch, data, n)
        pts, st = splitter(sch, data, n, 4)
        assert est.code != 0 and (st.code, st.record, st.offset) == (est.code, est.record, est.offset)
    recs[400] = rec_bytes(oracle, [(A.T_STRING, 9, bytes.fromhex("fffffff0"))])
    wire2, _ = concat(recs)
    rc, exp, est, _ = oracle.decode(sch, wire2, 900)
    pts, st = splitter(sch, wire2, 900, 4)
    assert est.code != 0 and (st.code, st.record, st.offset) == (est.code, est.record, est.offset)


# ---- containers beyond list<scalar>: list<string>, set<string>, map<K,V> (FieldFastReadList/Map,
#      struct_tpl.go:466-625) -------------------------------------------------------------------
CONTAINER_SCHEMAS = {"cx1": (S.schema_cx1, synth.gen_cx1), "cx2": (S.schema_cx2, synth.gen_cx2)}


def case_containers(dec, oracle, name, n, mode):
    mk, gen = CONTAINER_SCHEMAS[name]
    sch = mk()
    cs = gen(n, start=5)
    rc, wire, offs = oracle.encode(sch, cs)
    assert rc == 0
    cols, st = check_decode(dec, oracle, sch, wire, n, offsets=offs if mode == "offsets" else None)
    assert st.code == 0
    _, infos, _ = oracle.flatten(sch)
    assert_columns_equal(cols, cs, infos, n)


def case_mock_req_fault(dec, oracle):
    """thrift_data_test.go:100-118: list<i16> bytes where MockReq declares list<string> -> EOF on the
    device exactly as in the oracle (the reference asserts err != nil); the golden MockReq bytes
    (thrift_data_test.go:35-40, empty map and list) decode"""
    from tests.test_oracle_kat import FAULT_MOCK_REQ_THRIFT, MOCK_REQ_THRIFT
    sch = S.schema_mockreq()
    for raw, code in ((FAULT_MOCK_REQ_THRIFT, A.ERR_EOF), (MOCK_REQ_THRIFT, 0)):
        data = np.frombuffer(raw * 3, dtype=np.uint8).copy()
        offs = np.arange(4, dtype=np.uint64) * len(raw)
        cols, st = check_decode(dec, oracle, sch, data, 3, offsets=offs)
        assert st.code == code
        cols, st = check_decode(dec, oracle, sch, data, 3)
        assert st.code == code


# ---- chunked pipeline (launch_t): the batch is cut into whole groups of tiles; index + group of
#      chunk k overlap chain + emit of chunk k - ahead, the chain state is carried between chunks ----
CHUNK_CASES = ["r2", "r3", "r2_offsets", "error", "error_offsets", "truncated", "short_input", "fewer",
               "noncanonical", "pb", "pb_offsets", "containers"]


def case_chunked(dec, oracle, case):
    """each batch spans >= 4 chunks of 64 tiles (512 KiB); errors / the end of the chain fall in a
    middle chunk"""
    n = 15000
    if case in ("r2", "r3", "r2_offsets"):
        name = case.split("_")[0]
        n = 5000 if name == "r3" else n
        sch = S.SCHEMAS[name]()
        rc, wire, offs = oracle.encode(sch, synth.GENERATORS[name](n, start=3))
        check_decode(dec, oracle, sch, wire, n, offsets=offs if case.endswith("offsets") else None)
        return
    if case in ("pb", "pb_offsets"):
        from tests import pb_cases as PC
        PC.case_pb_concat(dec, oracle, 20000) if case == "pb" else PC.case_pb_offsets(dec, oracle, 20000)
        return
    if case == "containers":
        case_containers(dec, oracle, "cx1", 6000, "concat")
        return
    sch = S.schema_r2()
    rng = np.random.default_rng(9)
    if case == "noncanonical":
        recs = []
        for i in range(n):
            k = i % 97
            recs.append(r2_record(oracle, rng, order=list(rng.permutation(10))) if k == 3 else
                        r2_record(oracle, rng, dup=True) if k == 50 else r2_record(oracle, rng))
        wire, offs = concat(recs)
        check_decode(dec, oracle, sch, wire, n)
        check_decode(dec, oracle, sch, wire, n, offsets=offs)
        return
    cs = synth.gen_r2(n, start=11)
    rc, wire, offs = oracle.encode(sch, cs)
    if case in ("error", "error_offsets"):
        # record 9001 gets an unknown wire type in place of field 1's header
        p = int(offs[9001])
        wire = wire.copy()
        wire[p] = 99
        check_decode(dec, oracle, sch, wire, n, offsets=offs if case == "error_offsets" else None)
    elif case == "truncated":
        check_decode(dec, oracle, sch, wire[:int(offs[11000]) + 40].copy(), n)
    elif case == "short_input":
        check_decode(dec, oracle, sch, wire, n + 3)
    elif case == "fewer":
        cols, st = check_decode(dec, oracle, sch, wire, 6000)   # the chain ends in chunk 1 of 5
        assert st.consumed == int(offs[6000])


# ---- zero-copy string views (KX_COLF_VIEW): (offset, length) into the input instead of copies ----
VIEW_CASES = ["r2_concat", "r2_offsets", "r3_concat", "noncanonical", "errors", "wide", "pb"]


def case_views(dec, oracle, case):
    """the view pairs equal the oracle's, and every view names exactly the bytes the copy mode copies"""
    if case == "pb":
        sch = S.schema_pf()
        rc, wire, _ = oracle.encode(sch, synth.gen_pf(3000, start=4), pb=True)
        _check_views(dec, oracle, sch, wire, 3000, None, pb=True)
        return
    if case in ("r2_concat", "r2_offsets", "r3_concat", "wide"):
        name = case.split("_")[0] if case != "wide" else "r2"
        n = 4000 if name == "r3" else 20000
        sch = S.SCHEMAS[name]()
        rc, wire, offs = oracle.encode(sch, synth.GENERATORS[name](n, start=21))
        _check_views(dec, oracle, sch, wire, n, offs if case == "r2_offsets" else None, wide=case == "wide")
        return
    sch = S.schema_r2()
    rng = np.random.default_rng(12)
    recs = [r2_record(oracle, rng, order=list(rng.permutation(10)) if i % 7 == 3 else None,
                      strlens=(int(rng.integers(0, 50)), 0 if i % 5 == 0 else 32), dup=i % 11 == 4)
            for i in range(3000)]
    if case == "errors":   # a failing record in offsets mode reads as defaults: empty views (0, 0)
        recs[1234] = rec_bytes(oracle, [(A.T_STRING, 9, bytes.fromhex("fffffff0"))])
    wire, offs = concat(recs)
    _check_views(dec, oracle, sch, wire, len(recs), offs)
    if case == "noncanonical":
        _check_views(dec, oracle, sch, wire, len(recs), None)


def _check_views(dec, oracle, sch, wire, n, offsets, pb=False, wide=False):
    rc, exp, est, ers = oracle.decode(sch, wire, n, offsets=offsets, pb=pb, views=True, wide=wide)
    cols, st = dec.decode_views(sch, wire, n, offsets, pb=pb, wide=wide)
    assert st.code == est.code, (st.code, est.code)
    _, infos, _ = oracle.flatten(sch)
    ok = est.n_records if offsets is None else n
    assert_columns_equal(cols, exp, infos, ok)
    # each view covers exactly the bytes the copy mode copies
    rc2, cp, _, _ = oracle.decode(sch, wire, n, offsets=offsets, pb=pb)
    from kitex_amd.columns import Views
    for c, ci in enumerate(infos):
        if not isinstance(exp.cols[c], Views):
            continue
        pairs = to_np(cols.cols[c].pairs)[:ok].astype(np.int64)
        co = offsets_u64(to_np(cp.cols[c][0]))[:ok + 1].astype(np.int64)
        data = to_np(cp.cols[c][1])
        for r in range(0, ok, max(1, ok // 200)):
            o, ln = pairs[r]
            assert ln == co[r + 1] - co[r]
            assert bytes(wire[o:o + ln]) == bytes(data[co[r]:co[r + 1]])


# ---- the wave-cooperative numeric list emit (kx_decode.hip COOP): edge cases ----
COOP_TYPES = [(A.T_I16, 2), (A.T_I32, 4), (A.T_I64, 8), (A.T_DOUBLE, 8)]


def coop_schema(et):
    return S.Schema(S.Struct("CL", [S.Field(1, A.T_I64, "id"), S.Field(2, A.T_LIST, "v", elem=et),
                                    S.Field(3, A.T_LIST, "u", elem=A.T_I64)]))


def coop_columns(et, w, n, seed=0):
    """lists mostly empty, a few of 1..70 elements, one of 1500 elements (a list longer than a wave),
    records inactive lanes of a partial last wave"""
    from kitex_amd.synth import ColumnSet
    rng = np.random.default_rng(seed)
    dt = {2: np.int16, 4: np.int32, 8: np.int64}[w]
    l1 = np.where(rng.random(n) < 0.7, 0, rng.integers(1, 71, size=n))
    l1[n // 3] = 1500
    o1 = np.zeros(n + 1, np.uint32)
    o1[1:] = np.cumsum(l1)
    v1 = rng.integers(-(1 << 62), 1 << 62, size=max(1, int(o1[-1]))).astype(dt)
    l2 = np.where(rng.random(n) < 0.5, 0, rng.integers(1, 5, size=n))
    o2 = np.zeros(n + 1, np.uint32)
    o2[1:] = np.cumsum(l2)
    v2 = rng.integers(-(1 << 62), 1 << 62, size=max(1, int(o2[-1]))).astype(np.int64)
    ids = rng.integers(-(1 << 62), 1 << 62, size=n).astype(np.int64)
    return ColumnSet([ids, (o1, v1), (o2, v2)], np.zeros(n, np.uint64), n)


def case_coop_lists(dec, oracle, et, w, mode, n=1000):
    sch = coop_schema(et)
    cs = coop_columns(et, w, n, seed=w)
    rc, wire, offs = oracle.encode(sch, cs)
    assert rc == 0
    cols, st = check_decode(dec, oracle, sch, wire, n, offsets=offs if mode == "offsets" else None)
    assert st.code == 0
    _, infos, _ = oracle.flatten(sch)
    assert_columns_equal(cols, cs, infos, n, check_presence=False)


