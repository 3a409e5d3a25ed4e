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
    elem: object = 0                    # LIST/SET element type; MAP key type. A container element: a Field
                                        # describing it (its id is ignored), e.g. list<list<i64>>
    val: object = 0                     # MAP value type (a Field for a container value)
    child: Optional["Struct"] = None    # STRUCT fields; the struct of list<S> / set<S> / map<K, S>
    default: object = 0                 # scalar default (two's complement / IEEE bits) or a string default
    binary: bool = False                # protobuf `bytes` (no UTF-8 check); thrift: same wire as string
    pb: int = 0                         # Kitex-Protobuf schemas: proto kind (A.PB_*) of the field / its
                                        # elements / a map's key
    pbv: int = 0                        # ... of a map's value


@dataclass
class Struct:
    name: str
    fields: List[Field] = dc_field(default_factory=list)


class Schema:
    """A root struct and every struct reachable from it, lowered to kx_struct_desc[]."""

    def __init__(self, root: Struct, protobuf: bool = False):
        self.root = root
        self.protobuf = protobuf   # KX_STRUCT_PROTOBUF: proto3 messages, kinds in default_bits
        self.structs: List[Struct] = []
        self._index = {}
        self._elem_struct = {}     # id(field) -> the one-field struct describing its container element
        self._strings = []         # string defaults kept alive for the C-ABI
        self._collect(root)
        self._field_arrays = []
        self._table = (A.StructDesc * len(self.structs))()
        for i, s in enumerate(self.structs):
            arr = (A.FieldDesc * max(1, len(s.fields)))()
            for j, f in enumerate(s.fields):
                arr[j].id = f.id
                arr[j].ttype = f.ttype
                arr[j].req = f.req
                et = f.elem.ttype if isinstance(f.elem, Field) else f.elem
                vt = f.val.ttype if isinstance(f.val, Field) else f.val
                arr[j].elem_ttype = et | (vt << 4 if f.ttype == A.T_MAP else 0)
                arr[j].reserved0 = A.FIELD_BINARY if f.binary else 0
                if id(f) in self._elem_struct:
                    arr[j].child = self._index[id(self._elem_struct[id(f)])]
                else:
                    arr[j].child = self._index[id(f.child)] if f.child is not None else -1
                if isinstance(f.default, (str, bytes)):
                    b = f.default.encode() if isinstance(f.default, str) else f.default
                    buf = C.create_string_buffer(b)
                    self._strings.append(buf)
                    arr[j].default_bits = C.addressof(buf) if b else 0
                    arr[j].reserved0 |= A.FIELD_STRING_DEFAULT if b else 0
                elif protobuf:   # proto3: no defaults; the proto scalar kinds instead
                    arr[j].default_bits = (f.pb & 0xff) | ((f.pbv & 0xff) << 8)
                else:
                    arr[j].default_bits = _signed64(f.default)
            self._field_arrays.append(arr)
            self._table[i].fields = C.cast(arr, C.POINTER(A.FieldDesc))
            self._table[i].nfields = len(s.fields)
            self._table[i].reserved0 = A.STRUCT_PROTOBUF if protobuf and i == 0 else 0

    def _collect(self, s: Struct):
        if id(s) in self._index:
            return
        self._index[id(s)] = len(self.structs)
        self.structs.append(s)
        for f in s.fields:
            self._collect_field(f)

    def _collect_field(self, f: Field):
        sub = f.val if f.ttype == A.T_MAP else f.elem
        if isinstance(sub, Field):   # a container element / map value that is a container
            es = Struct(f"{f.name or f.id}.elem", [sub])
            self._elem_struct[id(f)] = es
            self._collect(es)
        elif f.child is not None:
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


def schema_simple() -> Struct:
    """baseline.thrift Simple (pkg/generic/json_test/idl/baseline.thrift:3-10)"""
    return Struct("Simple", [Field(1, A.T_BYTE, "ByteField"), Field(2, A.T_I64, "I64Field"),
                             Field(3, A.T_DOUBLE, "DoubleField"), Field(4, A.T_I32, "I32Field"),
                             Field(5, A.T_STRING, "StringField"), Field(6, A.T_STRING, "BinaryField", binary=True)])


def schema_nesting() -> Schema:
    """baseline.thrift Nesting (:12-28): list<Simple>, map<string, Simple>, a Simple field and maps /
    lists of scalars and strings: 42 columns, a nested schema"""
    sim = schema_simple()
    S = A.T_STRING
    return Schema(Struct("Nesting", [
        Field(1, S, "String"), Field(2, A.T_LIST, "ListSimple", elem=A.T_STRUCT, child=sim),
        Field(3, A.T_DOUBLE, "Double"), Field(4, A.T_I32, "I32"), Field(5, A.T_LIST, "ListI32", elem=A.T_I32),
        Field(6, A.T_I64, "I64"), Field(7, A.T_MAP, "MapStringString", elem=S, val=S),
        Field(8, A.T_STRUCT, "SimpleStruct", child=sim), Field(9, A.T_MAP, "MapI32I64", elem=A.T_I32, val=A.T_I64),
        Field(10, A.T_LIST, "ListString", elem=S), Field(11, S, "Binary", binary=True),
        Field(12, A.T_MAP, "MapI64String", elem=A.T_I64, val=S), Field(13, A.T_LIST, "ListI64", elem=A.T_I64),
        Field(14, A.T_BYTE, "Byte"), Field(15, A.T_MAP, "MapStringSimple", elem=S, val=A.T_STRUCT, child=sim),
    ]))


def schema_nx() -> Schema:
    """Shapes beyond baseline.thrift: nested containers one level down (list<list<i64>>, map<string,
    list<string>>, list<set<i32>>), a list of structs with optional fields, a nested struct and a
    list inside, a string default, and a recursive struct kept as bytes."""
    S = A.T_STRING
    leaf = Struct("Leaf", [Field(1, A.T_I32, "k", req=A.REQ_REQUIRED), Field(2, S, "v", default="none")])
    item = Struct("Item", [Field(1, A.T_I64, "id"), Field(2, S, "name", req=A.REQ_OPTIONAL),
                           Field(3, A.T_STRUCT, "leaf", child=leaf, req=A.REQ_OPTIONAL),
                           Field(4, A.T_LIST, "tags", elem=A.T_I32), Field(5, A.T_BOOL, "on", req=A.REQ_OPTIONAL)])
    node = Struct("Node", [Field(1, A.T_I64, "v")])
    node.fields.append(Field(2, A.T_STRUCT, "next", child=node, req=A.REQ_OPTIONAL))
    return Schema(Struct("NX", [
        Field(1, A.T_I64, "id"), Field(2, S, "title", default="untitled"),
        Field(3, A.T_LIST, "grid", elem=Field(0, A.T_LIST, elem=A.T_I64)),
        Field(4, A.T_MAP, "index", elem=S, val=Field(0, A.T_LIST, elem=S)),
        Field(5, A.T_LIST, "items", elem=A.T_STRUCT, child=item),
        Field(6, A.T_SET, "groups", elem=Field(0, A.T_SET, elem=A.T_I32), req=A.REQ_OPTIONAL),
        Field(7, A.T_STRUCT, "node", child=node),
        Field(8, A.T_MAP, "byid", elem=A.T_I32, val=A.T_STRUCT, child=leaf),
    ]))


SCHEMAS = {"r1": schema_r1, "r2": schema_r2, "r3": schema_r3, "pf": schema_pf}
