"""list<struct> parity cases (FieldFastReadList / FieldFastWriteList of a struct, struct_tpl.go:583-625,
1011-1036), shared by the CPU oracle + emulator tests and the GPU suite. Test infrastructure only."""
import struct

import numpy as np

from kitex_amd import _abi as A
from kitex_amd import schema as S
from tests.helpers import random_columns


def be16(v):
    return struct.pack(">h", v)


def be32(v):
    return struct.pack(">i", v)


def fld(t, fid, payload):
    return bytes([t]) + be16(fid) + payload


def point(x=None, y=None, w=None, b=None, extra=b"", order=(1, 2, 3, 4), dup_x=None):
    """one Point element (1: i64 x, 2: required i32 y, 3: double w = 1.5, 4: bool b) with the given
    fields in `order`, optional extra (unknown) fields, a duplicate x after the others"""
    parts = {1: None if x is None else fld(A.T_I64, 1, struct.pack(">q", x)),
             2: None if y is None else fld(A.T_I32, 2, be32(y)),
             3: None if w is None else fld(A.T_DOUBLE, 3, struct.pack(">d", w)),
             4: None if b is None else fld(A.T_BOOL, 4, bytes([b]))}
    out = b"".join(parts[k] for k in order if parts[k] is not None) + extra
    if dup_x is not None:
        out += fld(A.T_I64, 1, struct.pack(">q", dup_x))
    return out + b"\x00"


def record(rid, pts, tags=None):
    """LS1 record body: 1: i64 id, 2: list<Point>, 3: optional set<Tag>"""
    out = fld(A.T_I64, 1, struct.pack(">q", rid))
    out += fld(A.T_LIST, 2, bytes([A.T_STRUCT]) + be32(len(pts)) + b"".join(pts))
    if tags is not None:
        out += fld(A.T_SET, 3, bytes([A.T_STRUCT]) + be32(len(tags)) + b"".join(tags))
    return out + b"\x00"


def tag(k, v):
    return fld(A.T_I16, 7, be16(k)) + fld(A.T_BYTE, 9, bytes([v])) + b"\x00"


def handmade():
    """records exercising the element FastRead: reordered fields, unknown fields (scalar, string,
    struct, list), a mistyped id, duplicates (last wins), defaults, an empty list, a set of Tags"""
    recs = [
        record(1, [point(10, 20, 2.5, 1), point(-1, 7, order=(2, 1))]),
        record(2, [point(5, 6, extra=fld(A.T_STRING, 99, be32(3) + b"abc") + fld(A.T_I32, 3, be32(9)))]),
        record(3, [point(1, 2, dup_x=77), point(y=5)], tags=[tag(1, 2), tag(-3, 255)]),
        record(4, []),
        record(5, [point(9, 9, extra=fld(A.T_STRUCT, 50, fld(A.T_I64, 1, struct.pack(">q", 3)) + b"\x00")
                          + fld(A.T_LIST, 51, bytes([A.T_I32]) + be32(2) + be32(1) + be32(2)))], tags=[]),
    ]
    return recs


def missing_required():
    """an element without its required field y -> INVALID_DATA (RequiredFieldNotSetError)"""
    return record(6, [point(1, 2), point(x=3)])


def wire_of(recs):
    wire = np.frombuffer(b"".join(recs), dtype=np.uint8).copy()
    offs = np.zeros(len(recs) + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(r) for r in recs])
    return wire, offs


def random_batch(oracle, n, seed=5):
    sch = S.schema_ls1()
    rc, infos, npres = oracle.flatten(sch)
    assert rc == 0
    cs = random_columns(infos, npres, n, seed=seed)
    rc, wire, offs = oracle.encode(sch, cs)
    assert rc == 0
    return sch, infos, npres, cs, wire, offs
