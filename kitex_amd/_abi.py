"""ctypes mirror of include/kxcodec.h (the C-ABI boundary).

Kept in one place so that the product binding (kitex_amd._lib) and the test-only oracle binding
(oracle/oracle.py) describe the very same structs. Any change here must match kxcodec.h; the
layout is checked by tests/test_abi.py against the compiled library.
"""
import ctypes as C

KX_ABI_VERSION = 7

# Thrift TType ids (gopkg protocol/thrift; pinned by pkg/protocol/bthrift/binary_test.go)
T_STOP, T_VOID, T_BOOL, T_BYTE, T_DOUBLE = 0, 1, 2, 3, 4
T_I16, T_I32, T_I64, T_STRING, T_STRUCT = 6, 8, 10, 11, 12
T_MAP, T_SET, T_LIST = 13, 14, 15

MSG_CALL, MSG_REPLY, MSG_EXCEPTION, MSG_ONEWAY = 1, 2, 3, 4

OK = 0
ERR_INVALID_DATA = 1
ERR_NEGATIVE_SIZE = 2
ERR_SIZE_LIMIT = 3
ERR_BAD_VERSION = 4
ERR_NOT_IMPLEMENTED = 5
ERR_DEPTH_LIMIT = 6
ERR_EOF = 8
ELEM_MAP_VALUE = 0x80
ELEM_STRUCT_FIELD = 0x40
ELEM_PRESENCE = 0x20     # nested schemas: a column of per-element presence words
ERR_APPLICATION_EXCEPTION = 9
ERR_UNKNOWN_PROTOCOL = 10
ERR_PAYLOAD_VALIDATION = 11
# framing sniff kinds (kx_frame_scan): transport.Protocol | FRAME_PB | FRAME_MESH
TRANS_PURE, TRANS_TTHEADER, TRANS_FRAMED, TRANS_TTHEADER_FRAMED = 0, 2, 4, 6
FRAME_PB, FRAME_MESH = 0x10, 0x20
ERR_INVALID_ARG = 100
ERR_HIP = 101
ERR_NO_DEVICE = 102
ERR_INTERNAL = 103

REQ_DEFAULT, REQ_REQUIRED, REQ_OPTIONAL = 0, 1, 2
FIELD_BINARY = 1  # kx_field_desc.reserved0 flag: protobuf `bytes` (no UTF-8 validation)
FIELD_STRING_DEFAULT = 2  # ... default_bits points at the field's NUL-terminated string default
STRUCT_PROTOBUF = 1  # kx_struct_desc.reserved0 of the root struct: a Kitex-Protobuf schema (ABI v4)
# proto scalar kinds (default_bits of a Kitex-Protobuf field: bits 0..7 field / element / key, 8..15 map value)
PB_NATURAL, PB_SINT, PB_FIXED, PB_UINT, PB_BYTES = 0, 1, 2, 3, 4

COL_FIXED, COL_BYTES, COL_LIST, COL_LIST_BYTES = 1, 2, 3, 4
COL_LIST2, COL_LIST2_BYTES = 5, 6   # nested schemas: two container levels down
STRING_KINDS = (COL_BYTES, COL_LIST_BYTES, COL_LIST2_BYTES)
COLF_VIEW = 1  # kx_column.flags: zero-copy (offset, length) string views
MAX_COLUMNS = 64
MAX_STRUCTS = 16

TYPE_SIZE = {T_BOOL: 1, T_BYTE: 1, T_I16: 2, T_I32: 4, T_I64: 8, T_DOUBLE: 8}


class FieldDesc(C.Structure):
    _fields_ = [
        ("id", C.c_int16),
        ("ttype", C.c_uint8),
        ("req", C.c_uint8),
        ("elem_ttype", C.c_uint8),
        ("reserved0", C.c_uint8),
        ("child", C.c_int16),
        ("default_bits", C.c_int64),
    ]


class StructDesc(C.Structure):
    _fields_ = [("fields", C.POINTER(FieldDesc)), ("nfields", C.c_uint32), ("reserved0", C.c_uint32)]


class ColumnInfo(C.Structure):
    _fields_ = [
        ("kind", C.c_uint32),
        ("width", C.c_uint32),
        ("ttype", C.c_uint8),
        ("elem_ttype", C.c_uint8),
        ("field_id", C.c_int16),
        ("presence_bit", C.c_int32),
        ("depth", C.c_uint32),
        ("path", C.c_int16 * 8),
        ("level", C.c_uint8),
        ("reserved1", C.c_uint8 * 3),
    ]


class Column(C.Structure):
    _fields_ = [("data", C.c_void_p), ("offsets", C.c_void_p), ("capacity", C.c_uint64),
                ("elem_offsets", C.c_void_p), ("elem_capacity", C.c_uint64),
                ("offset_bytes", C.c_uint32), ("flags", C.c_uint32),
                ("sub_offsets", C.c_void_p), ("sub_capacity", C.c_uint64)]


class Columns(C.Structure):
    _fields_ = [
        ("cols", Column * MAX_COLUMNS),
        ("ncols", C.c_uint32),
        ("reserved0", C.c_uint32),
        ("presence", C.c_void_p),
    ]


class Status(C.Structure):
    _fields_ = [
        ("code", C.c_int32),
        ("reserved0", C.c_int32),
        ("record", C.c_uint64),
        ("offset", C.c_uint64),
        ("n_records", C.c_uint64),
        ("consumed", C.c_uint64),
        ("var_total", C.c_uint64 * 16),
        ("diag", C.c_uint64 * 3),
    ]


class TTStreamKeys(C.Structure):
    """kx_ttstream_keys: the gopkg ttheader streaming constants the frame scan uses (include/kxcodec.h)"""
    _fields_ = [("frame_type_key", C.c_uint16), ("to_method_key", C.c_uint16), ("streaming_flag", C.c_uint16),
                ("reserved", C.c_uint16), ("type_names", (C.c_char * 8) * 5)]


TTS_META, TTS_HEADER, TTS_DATA, TTS_TRAILER, TTS_RST = 1, 2, 3, 4, 5

# shard concatenation (kx_concat_plan): the arrays of a column a piece belongs to
PIECE_OFFSETS, PIECE_ELEM_OFFSETS, PIECE_SUB_OFFSETS, PIECE_DATA = 0, 1, 2, 3


class ConcatPiece(C.Structure):
    _fields_ = [("rank", C.c_uint32), ("column", C.c_uint32), ("array", C.c_uint32), ("elem_bytes", C.c_uint32),
                ("src_first", C.c_uint64), ("count", C.c_uint64), ("dst_first", C.c_uint64), ("rebase", C.c_int64)]


class ConcatSizes(C.Structure):
    _fields_ = [("n", C.c_uint64), ("in_len", C.c_uint64), ("units", (C.c_uint64 * 4) * MAX_COLUMNS)]

assert C.sizeof(TTStreamKeys) == 48
assert C.sizeof(FieldDesc) == 16
assert C.sizeof(Status) == 192
assert C.sizeof(Column) == 64
assert C.sizeof(Columns) == MAX_COLUMNS * 64 + 16
assert C.sizeof(ColumnInfo) == 40
assert C.sizeof(ConcatPiece) == 48


def n_arrays(ci) -> int:
    """offsets arrays of a column: one per container level above it, one more for a string's bytes"""
    return ci.level + (1 if ci.kind in STRING_KINDS else 0)

ERROR_NAMES = {
    OK: "ok",
    ERR_INVALID_DATA: "invalid data",
    ERR_NEGATIVE_SIZE: "negative size",
    ERR_SIZE_LIMIT: "size limit",
    ERR_BAD_VERSION: "bad version",
    ERR_NOT_IMPLEMENTED: "not implemented",
    ERR_DEPTH_LIMIT: "depth limit exceeded",
    ERR_EOF: "unexpected EOF",
    ERR_APPLICATION_EXCEPTION: "application exception message",
    ERR_UNKNOWN_PROTOCOL: "unknown protocol (framing sniff)",
    ERR_PAYLOAD_VALIDATION: "payload validation failed (crc32c)",
    ERR_INVALID_ARG: "invalid argument",
    ERR_HIP: "HIP runtime error",
    ERR_NO_DEVICE: "no device",
    ERR_INTERNAL: "internal error",
}
