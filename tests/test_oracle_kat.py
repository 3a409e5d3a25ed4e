"""Pin the CPU oracle against the reference's own known-answer tests.

Every expected value below is copied (as data) from the reference test it cites; the oracle must
reproduce it before any GPU result is compared with the oracle.
"""
import struct

import numpy as np

from kitex_amd import schema as S
from kitex_amd import synth
import pytest

from kitex_amd import _abi as A
from kitex_amd.schema import Field, Schema, Struct


# ---- pkg/protocol/bthrift/binary_test.go ------------------------------------------------------
@pytest.mark.parametrize("fn,args,hexs", [
    ("kxo_write_field_begin", (A.T_I32, 32), "080020"),               # :56-75
    ("kxo_write_map_begin", (A.T_MAP, 32, 1), "0d2000000001"),        # :90-109
    ("kxo_write_list_begin", (A.T_LIST, 32), "0f00000020"),           # :118-136
    ("kxo_write_set_begin", (A.T_SET, 32), "0e00000020"),             # :145-163
    ("kxo_write_bool", (1,), "01"),                                   # :172-196
    ("kxo_write_bool", (0,), "00"),
    ("kxo_write_byte", (ord("1"),), "31"),                            # :199-212
    ("kxo_write_i16", (1,), "0001"),                                  # :215-228
    ("kxo_write_i32", (1,), "00000001"),                              # :231-244
    ("kxo_write_i64", (1,), "0000000000000001"),                      # :247-260
    ("kxo_write_double", (1.0,), "3ff0000000000000"),                 # :263-276
    ("kxo_write_field_stop", (), "00"),                               # :83-87
])
def test_primitive_kat(oracle, fn, args, hexs):
    assert oracle.prim(fn, *args).hex() == hexs


def test_string_kat(oracle):
    assert oracle.prim("kxo_write_string", b"kitex", 5).hex() == "000000056b69746578"       # :279-292
    assert oracle.prim("kxo_write_string", b"messageBegin", 12).hex() == \
        "0000000c6d657373616765426567696e"                                                   # :314-322


def test_lengths(oracle):                                                                    # :336-384
    L = oracle.lib()
    assert L.kxo_message_begin_length(len(b"kitex")) == 17
    assert len(oracle.prim("kxo_write_field_begin", A.T_I32, 1)) == 3
    assert len(oracle.prim("kxo_write_field_stop")) == 1
    assert len(oracle.prim("kxo_write_map_begin", A.T_MAP, A.T_MAP, 4)) == 6
    assert len(oracle.prim("kxo_write_list_begin", A.T_LIST, 4)) == 5
    assert len(oracle.prim("kxo_write_set_begin", A.T_SET, 4)) == 5
    assert len(oracle.prim("kxo_write_string", b"1", 1)) == 5


@pytest.mark.parametrize("mtype,hexs", [                                                     # :387-457
    (A.MSG_CALL, "800100010000000c6d657373616765426567696e00000001"),
    (A.MSG_REPLY, "800100020000000c6d657373616765426567696e00000001"),
    (A.MSG_EXCEPTION, "800100030000000c6d657373616765426567696e00000001"),
    (A.MSG_ONEWAY, "800100040000000c6d657373616765426567696e00000001"),
])
def test_message_begin_kat(oracle, mtype, hexs):
    b = oracle.prim("kxo_write_message_begin", b"messageBegin", 12, mtype, 1)
    assert b.hex() == hexs and len(b) == 24
    rc, (name, t, seq, used) = oracle.read_message_begin(b)
    assert rc == 0 and name == "messageBegin" and t == mtype and seq == 1 and used == 24


def test_message_begin_bad_version(oracle):
    rc, _ = oracle.read_message_begin(bytes.fromhex("000000050000000c"))
    assert rc == A.ERR_BAD_VERSION


def test_skip_kat(oracle):
    """TestSkip (binary_test.go:460-529): a 46-byte sequence and Skip's consumed lengths,
    including the test's offset arithmetic that skips from inside a header."""
    P = oracle.prim
    b = (P("kxo_write_byte", ord("1")) + P("kxo_write_string", b"2", 1) + P("kxo_write_double", 3.0)
         + P("kxo_write_byte", ord("4")) + P("kxo_write_bool", 1) + P("kxo_write_i16", 6)
         + P("kxo_write_i32", 7) + P("kxo_write_i64", 8) + P("kxo_write_list_begin", A.T_LIST, 9)
         + P("kxo_write_map_begin", A.T_MAP, A.T_STRING, 10) + P("kxo_write_set_begin", A.T_STRING, 11))
    assert len(b) == 46
    buf = b + bytes(1024 - 46)
    off = 0
    for t, nxt in [(A.T_BYTE, 1), (A.T_STRING, 5), (A.T_DOUBLE, 8), (A.T_BYTE, 1), (A.T_BOOL, 1),
                   (A.T_I16, 2), (A.T_I32, 4), (A.T_I64, 8)]:
        rc, n = oracle.skip(buf[off:], t)
        assert rc == 0 and n == nxt
        off += n
    assert struct.unpack(">i", buf[off + 1:off + 5])[0] == 9                 # ReadListBegin == 9
    rc, n = oracle.skip(buf[off + 9:], A.T_LIST)                             # Skip(buf[offset+valList:])
    off += n                                                                 # error ignored by the test
    assert struct.unpack(">i", buf[off + 2:off + 6])[0] == 10                # ReadMapBegin == 10
    rc, n = oracle.skip(buf[off + 10 + 9:], A.T_MAP)
    assert rc == 0
    off += n
    assert struct.unpack(">i", buf[off + 1:off + 5])[0] == 11                # ReadSetBegin == 11


# ---- pkg/remote/codec/thrift/thrift_data_test.go -----------------------------------------------
MOCK_REQ_THRIFT = bytes([                                                     # :35-40
    11, 0, 1, 0, 0, 0, 5, 104, 101, 108, 108, 111,
    13, 0, 2, 11, 11, 0, 0, 0, 0,
    15, 0, 3, 11, 0, 0, 0, 0,
    0,
])
FAULT_MOCK_REQ_THRIFT = bytes([                                               # :107-112
    11, 0, 1, 0, 0, 0, 5, 104, 101, 108, 108, 111,
    13, 0, 2, 11, 11, 0, 0, 0, 0,
    15, 0, 3, 6, 0, 0, 0, 1, 0, 1,
    0,
])


def test_mock_req_bytes_from_primitives(oracle):
    """MockReq{Msg:"hello"}: FastWriteNocopy writes field1, empty map, empty list, STOP (30 B)."""
    P = oracle.prim
    b = (P("kxo_write_field_begin", A.T_STRING, 1) + P("kxo_write_string", b"hello", 5)
         + P("kxo_write_field_begin", A.T_MAP, 2) + P("kxo_write_map_begin", A.T_STRING, A.T_STRING, 0)
         + P("kxo_write_field_begin", A.T_LIST, 3) + P("kxo_write_list_begin", A.T_STRING, 0)
         + P("kxo_write_field_stop"))
    assert b == MOCK_REQ_THRIFT and len(b) == 30


def test_mock_req_skip_and_decode(oracle):
    assert oracle.skip(MOCK_REQ_THRIFT, A.T_STRUCT) == (0, 30)
    # FastRead: field 1 decoded, the container fields skipped when not in the schema
    sch = Schema(Struct("MockReqMsg", [Field(1, A.T_STRING, "Msg")]))
    data = np.frombuffer(MOCK_REQ_THRIFT, dtype=np.uint8).copy()
    rc, out, st, rs = oracle.decode(sch, data, 1, offsets=np.array([0, 30], dtype=np.uint64))
    assert rc == 0
    offs, blob = out.cols[0]
    assert bytes(blob[offs[0]:offs[1]]) == b"hello"


def test_fault_vector_skip(oracle):
    """The skip decoder accepts the fault vector (its list<i16> is well formed); only the typed
    FastRead of list<string> rejects it (thrift_data_test.go:100-118)."""
    assert oracle.skip(FAULT_MOCK_REQ_THRIFT, A.T_STRUCT) == (0, len(FAULT_MOCK_REQ_THRIFT))


def test_fault_vector_fails_as_mock_req(oracle):
    """thrift_data_test.go:100-118: the fault vector sends field 3 as list<i16> where MockReq declares
    list<string>; FastRead reads the element as a string (i32 length from the i16 bytes) and runs
    past the end -> the decode FAILS (EOF), exactly where the reference's test asserts err != nil."""
    sch = S.schema_mockreq()
    data = np.frombuffer(FAULT_MOCK_REQ_THRIFT, dtype=np.uint8).copy()
    rc, out, st, rs = oracle.decode(sch, data, 1, offsets=np.array([0, data.size], dtype=np.uint64))
    assert rc == A.ERR_EOF and st.code == A.ERR_EOF and st.record == 0 and rs[0] == A.ERR_EOF
    # declared as list<i16> instead, the same bytes decode
    ok = Schema(Struct("M", [Field(1, A.T_STRING), Field(3, A.T_LIST, elem=A.T_I16)]))
    rc, out, st, _ = oracle.decode(ok, data, 1, offsets=np.array([0, data.size], dtype=np.uint64))
    assert rc == 0
    lo, le = out.cols[1]
    assert list(le[lo[0]:lo[1]]) == [1]


def test_mock_req_encode_decode_golden(oracle):
    """MockReq{Msg:"hello"} (empty strMap / strList still written, thrift_data_test.go:35-40): the
    oracle's FastWriteNocopy gives the golden 30 bytes and FastRead gives the struct back"""
    sch = S.schema_mockreq()
    _, infos, npres = oracle.flatten(sch)
    u32 = lambda *v: np.array(v, dtype=np.uint32)  # noqa: E731
    cs = synth.ColumnSet([(u32(0, 5), np.frombuffer(b"hello", np.uint8).copy()),
                          (u32(0, 0), u32(0), np.zeros(1, np.uint8)),
                          (u32(0, 0), u32(0), np.zeros(1, np.uint8)),
                          (u32(0, 0), u32(0), np.zeros(1, np.uint8))], np.zeros(1, np.uint64), 1)
    rc, wire, offs = oracle.encode(sch, cs)
    assert rc == 0 and bytes(wire) == MOCK_REQ_THRIFT
    data = np.frombuffer(MOCK_REQ_THRIFT, dtype=np.uint8).copy()
    rc, out, st, _ = oracle.decode(sch, data, 1)
    assert rc == 0 and st.consumed == 30
    o, b = out.cols[0]
    assert bytes(b[o[0]:o[1]]) == b"hello"
    for c in (1, 2, 3):
        assert out.cols[c][0][1] - out.cols[c][0][0] == 0
    # one entry each: map<string,string>{"k": "vv"}, list<string>["a", "", "bcd"]
    P = oracle.prim
    one = (P("kxo_write_field_begin", A.T_STRING, 1) + P("kxo_write_string", b"hi", 2)
           + P("kxo_write_field_begin", A.T_MAP, 2) + P("kxo_write_map_begin", A.T_STRING, A.T_STRING, 1)
           + P("kxo_write_string", b"k", 1) + P("kxo_write_string", b"vv", 2)
           + P("kxo_write_field_begin", A.T_LIST, 3) + P("kxo_write_list_begin", A.T_STRING, 3)
           + P("kxo_write_string", b"a", 1) + P("kxo_write_string", b"", 0) + P("kxo_write_string", b"bcd", 3)
           + b"\x00")
    data = np.frombuffer(one, dtype=np.uint8).copy()
    rc, out, st, _ = oracle.decode(sch, data, 1)
    assert rc == 0
    ko, keo, kb = out.cols[1]
    vo, veo, vb = out.cols[2]
    lo, leo, lb = out.cols[3]
    assert (ko[1] - ko[0], bytes(kb[keo[0]:keo[1]])) == (1, b"k")
    assert (vo[1] - vo[0], bytes(vb[veo[0]:veo[1]])) == (1, b"vv")
    assert [bytes(lb[leo[k]:leo[k + 1]]) for k in range(lo[0], lo[1])] == [b"a", b"", b"bcd"]
    assert list(st.var_total[:7]) == [2, 1, 1, 1, 2, 3, 4]
    rc, wire, _ = oracle.encode(sch, out)
    assert rc == 0 and bytes(wire) == one


# ---- pkg/remote/codec/thrift/codec_apache_test.go ----------------------------------------------
def gen_test_skip_decoder_bytes(oracle) -> bytes:                              # :115-184
    P = oracle.prim
    structb = P("kxo_write_field_begin", A.T_I64, 10001) + P("kxo_write_i64", 100010) + P("kxo_write_field_stop")
    b = b""
    b += P("kxo_write_field_begin", A.T_BOOL, 1) + P("kxo_write_bool", 1)
    b += P("kxo_write_field_begin", A.T_BYTE, 2) + P("kxo_write_byte", 2)
    b += P("kxo_write_field_begin", A.T_DOUBLE, 3) + P("kxo_write_double", 3.0)
    b += P("kxo_write_field_begin", A.T_I16, 4) + P("kxo_write_i16", 4)
    b += P("kxo_write_field_begin", A.T_I32, 5) + P("kxo_write_i32", 5)
    b += P("kxo_write_field_begin", A.T_I64, 6) + P("kxo_write_i64", 6)
    b += P("kxo_write_field_begin", A.T_STRUCT, 7) + structb
    b += P("kxo_write_field_begin", A.T_LIST, 101) + P("kxo_write_list_begin", A.T_I64, 10)
    b += P("kxo_write_i64", 1011) * 10
    b += P("kxo_write_field_begin", A.T_LIST, 102) + P("kxo_write_list_begin", A.T_STRUCT, 10)
    b += structb * 10
    b += P("kxo_write_field_begin", A.T_MAP, 201) + P("kxo_write_map_begin", A.T_I64, A.T_DOUBLE, 10)
    b += (P("kxo_write_i64", 2011) + P("kxo_write_double", 2012.2)) * 10
    b += P("kxo_write_field_begin", A.T_MAP, 202) + P("kxo_write_map_begin", A.T_STRING, A.T_I64, 10)
    b += (P("kxo_write_string", b"hello-202", 9) + P("kxo_write_i64", 2022)) * 10
    b += P("kxo_write_field_begin", A.T_MAP, 203) + P("kxo_write_map_begin", A.T_I64, A.T_STRUCT, 10)
    b += (P("kxo_write_i64", 2031) + structb) * 10
    return b + P("kxo_write_field_stop")


def test_skip_decoder_fixture(oracle):                                        # :186-200
    b = gen_test_skip_decoder_bytes(oracle)
    assert oracle.skip(b, A.T_STRUCT) == (0, len(b))


def test_skip_truncated(oracle):                                              # :38-54
    P = oracle.prim
    good = P("kxo_write_field_begin", A.T_BOOL, 1) + P("kxo_write_bool", 1) + P("kxo_write_field_stop")
    assert oracle.skip(good, A.T_STRUCT) == (0, len(good))
    rc, _ = oracle.skip(P("kxo_write_field_begin", A.T_BOOL, 1), A.T_STRUCT)
    assert rc == A.ERR_EOF


def test_skip_depth_limit(oracle):
    """skipType checks maxdepth before anything else (codec_apache.go:192-194): 63 nested structs
    holding a scalar skip fine, a string field at depth 64 hits the limit."""
    P = oracle.prim
    inner = P("kxo_write_field_begin", A.T_I64, 1) + P("kxo_write_i64", 7) + P("kxo_write_field_stop")
    b = inner
    for _ in range(63):
        b = P("kxo_write_field_begin", A.T_STRUCT, 1) + b + P("kxo_write_field_stop")
    assert oracle.skip(b, A.T_STRUCT) == (0, len(b))
    deep = P("kxo_write_field_begin", A.T_STRING, 1) + P("kxo_write_string", b"x", 1) + P("kxo_write_field_stop")
    for _ in range(63):
        deep = P("kxo_write_field_begin", A.T_STRUCT, 1) + deep + P("kxo_write_field_stop")
    assert oracle.skip(deep, A.T_STRUCT)[0] == A.ERR_DEPTH_LIMIT


def test_skip_negative_and_unknown(oracle):
    P = oracle.prim
    neg = P("kxo_write_field_begin", A.T_STRING, 1) + bytes.fromhex("ffffffff")
    assert oracle.skip(neg, A.T_STRUCT)[0] == A.ERR_INVALID_DATA               # errDataLength
    unk = bytes([20, 0, 1, 0])
    assert oracle.skip(unk, A.T_STRUCT)[0] == A.ERR_INVALID_DATA               # unknown data type


# ---- pkg/remote/codec/protobuf/protobuf_test.go ------------------------------------------------
def test_pb_fast_codec_fixture(oracle):
    """mockFastCodecReq{num: 7, v: "hello"}: tag varint(7<<3|2), varint len, bytes (:85-140)."""
    body = bytes([7 << 3 | 2, 5]) + b"hello"
    sch = Schema(Struct("Req", [Field(7, A.T_STRING, "v")]))
    data = np.frombuffer(body, dtype=np.uint8).copy()
    rc, out, st, _ = oracle.decode(sch, data, 1, offsets=np.array([0, len(body)], np.uint64), pb=True)
    assert rc == 0
    offs, blob = out.cols[0]
    assert bytes(blob[offs[0]:offs[1]]) == b"hello"


def test_pb_meta(oracle):
    """Kitex-Protobuf meta: u32 magic|type, u32 len + method, u32 seqID (protobuf.go:24-47,77-90)."""
    b = oracle.prim("kxo_pb_write_meta", b"mock", 4, 1, 7)
    assert b.hex() == "90010001" + "00000004" + b"mock".hex() + "00000007"
