"""Schema model: the flattened IDL the codec is driven by.

Kitex drives its FastCodec with per-type generated code (tool/internal_pkg/pluginmode/thriftgo/
struct_tpl.go:41-391); the batch codec is instead driven by a schema table built from the IDL, the
same information pkg/generic/descriptor/descriptor.go:64-80 (StructDescriptor / FieldDescriptor)
carries. `Struct` / `Field` below are that table; `Schema.struct_table()` lowers it to the C-ABI's
kx_struct_desc array (root struct first).

Decoded records are struct-of-arrays columns, one per leaf field, flattened depth-first (nested
struct fields inlined) — see include/kxcodec.h (kx_column_info).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field as dc_field
from typing import List, Optional

from . import _abi as A


@dataclass
class Field:
    id: int
    ttype: int
    name: str = ""
    req: int = A.REQ_DEFAULT
    elem: int = 0                       # LIST/SET element type; MAP key type
    val: int = 0                        # MAP value type
    child: Optional["Struct"] = None    # STRUCT fields
    default: int = 0                    # scalar default (two's complement / IEEE bits)
    binary: bool = False                # protobuf `bytes` (no UTF-8 check); thrift: same wire as string


@dataclass
class Struct:
    name: str
    fields: List[Field] = dc_field(default_factory=list)


class Schema:
    """A root struct and every struct reachable from it, lowered to kx_struct_desc[]."""

    def __init__(self, root: Struct):
        self.root = root
        self.structs: List[Struct] = []
        self._index = {}
        self._collect(root)
        self._field_arrays = []
        self._table = (A.StructDesc * len(self.structs))()
        for i, s in enumerate(self.structs):
            arr = (A.FieldDesc * max(1, len(s.fields)))()
            for j, f in enumerate(s.fields):
                arr[j].id = f.id
                arr[j].ttype = f.ttype
                arr[j].req = f.req
                arr[j].elem_ttype = f.elem | (f.val << 4 if f.ttype == A.T_MAP else 0)
                arr[j].reserved0 = A.FIELD_BINARY if f.binary else 0
                arr[j].child = self._index[id(f.child)] if f.child is not None else -1
                arr[j].default_bits = _signed64(f.default)
            self._field_arrays.append(arr)
            self._table[i].fields = C.cast(arr, C.POINTER(A.FieldDesc))
            self._table[i].nfields = len(s.fields)

    def _collect(self, s: Struct):
        if id(s) in self._index:
            return
        self._index[id(s)] = len(self.structs)
        self.structs.append(s)
        for f in s.fields:
            if f.child is not None:
                self._collect(f.child)

    def struct_table(self):
        return self._table, len(self.structs)


def _signed64(v: int) -> int:
    v &= (1 << 64) - 1
    return v - (1 << 64) if v >= 1 << 63 else v


# ---------------------------------------------------------------------------------------------
# The benchmark / parity schemas.
# ---------------------------------------------------------------------------------------------

def schema_r1() -> Schema:
    """R1 = struct{1..8: i64}; wire body 89 B."""
    return Schema(Struct("R1", [Field(i, A.T_I64, f"a{i}") for i in range(1, 9)]))


def schema_r2() -> Schema:
    """R2 = struct{1..8: i64; 9,10: string}; wire body 167 B at 32-byte strings, Go struct 96 B."""
    fs = [Field(i, A.T_I64, f"a{i}") for i in range(1, 9)]
    fs += [Field(9, A.T_STRING, "s9"), Field(10, A.T_STRING, "s10")]
    return Schema(Struct("R2", fs))


def schema_r3() -> Schema:
    """R3 = struct{1: i64 id; 2: list<i64> vals; 3: Inner inner; 4: i32 kind},
    Inner = struct{1: i64 x; 2: i32 y; 3: string tag}. Encoder order: id, kind, vals, inner."""
    inner = Struct("Inner", [Field(1, A.T_I64, "x"), Field(2, A.T_I32, "y"), Field(3, A.T_STRING, "tag")])
    return Schema(Struct("R3", [
        Field(1, A.T_I64, "id"),
        Field(2, A.T_LIST, "vals", elem=A.T_I64),
        Field(3, A.T_STRUCT, "inner", child=inner),
        Field(4, A.T_I32, "kind"),
    ]))


def schema_pf() -> Schema:
    """PF = proto3 {int64 a1..a8 = 1..8; string s9 = 9; string s10 = 10} (Kitex-Protobuf body)."""
    fs = [Field(i, A.T_I64, f"a{i}") for i in range(1, 9)]
    fs += [Field(9, A.T_STRING, "s9"), Field(10, A.T_STRING, "s10")]
    return Schema(Struct("PF", fs))


def schema_mockreq() -> Schema:
    """MockReq (internal/mocks/thrift/k-mock.go:116-184): 1: string Msg, 2: map<string,string>
    strMap, 3: list<string> strList."""
    return Schema(Struct("MockReq", [Field(1, A.T_STRING, "Msg"),
                                     Field(2, A.T_MAP, "strMap", elem=A.T_STRING, val=A.T_STRING),
                                     Field(3, A.T_LIST, "strList", elem=A.T_STRING)]))


def schema_cx1() -> Schema:
    """Containers beyond list<scalar>, MockReq's shapes next to an i64: id, msg, map<string,string>,
    list<string> (7 var slots: the device handles 8 per schema)."""
    return Schema(Struct("CX1", [Field(1, A.T_I64, "id"), Field(2, A.T_STRING, "msg"),
                                 Field(3, A.T_MAP, "strMap", elem=A.T_STRING, val=A.T_STRING),
                                 Field(4, A.T_LIST, "strList", elem=A.T_STRING)]))


def schema_cx2() -> Schema:
    """set<string>, map<i64,double> and an optional map<i32,string> next to an i64."""
    return Schema(Struct("CX2", [Field(1, A.T_I64, "id"), Field(5, A.T_SET, "tags", elem=A.T_STRING),
                                 Field(6, A.T_MAP, "scores", elem=A.T_I64, val=A.T_DOUBLE),
                                 Field(7, A.T_MAP, "names", elem=A.T_I32, val=A.T_STRING, req=A.REQ_OPTIONAL)]))


def schema_ls1() -> Schema:
    """list<struct>: Point{1: i64 x; 2: required i32 y; 3: double w = 1.5; 4: bool b} in a list and a set
    next to an i64 (internal/mocks style; FieldFastReadList of structs, struct_tpl.go:583-625)."""
    import struct as _st
    pt = Struct("Point", [Field(1, A.T_I64, "x"), Field(2, A.T_I32, "y", req=A.REQ_REQUIRED),
                          Field(3, A.T_DOUBLE, "w", default=_st.unpack("<q", _st.pack("<d", 1.5))[0]),
                          Field(4, A.T_BOOL, "b")])
    tag = Struct("Tag", [Field(7, A.T_I16, "k"), Field(9, A.T_BYTE, "v")])
    return Schema(Struct("LS1", [Field(1, A.T_I64, "id"), Field(2, A.T_LIST, "pts", elem=A.T_STRUCT, child=pt),
                                 Field(3, A.T_SET, "tags", elem=A.T_STRUCT, child=tag, req=A.REQ_OPTIONAL)]))


SCHEMAS = {"r1": schema_r1, "r2": schema_r2, "r3": schema_r3, "pf": schema_pf}
