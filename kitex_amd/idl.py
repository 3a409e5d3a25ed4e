"""Thrift IDL -> descriptors -> codec schema (the descriptor-to-schema compiler).

Kitex's generic path builds a ServiceDescriptor from an IDL (pkg/generic/thrift/parse.go, over the
thriftgo parser) whose model is pkg/generic/descriptor/descriptor.go:40-140 (FieldDescriptor,
TypeDescriptor, StructDescriptor, FunctionDescriptor, ServiceDescriptor). This module restates that
front end for the batch codec:

  parse_idl(path or text)        -> Document (structs, enums, typedefs, services; includes resolved)
  Document.service(name)         -> ServiceDescriptor (functions -> request / response TypeDescriptors;
                                    the request is the method's Args struct, the response its Result
                                    struct: field 0 success + the declared exceptions, as parse.go wraps
                                    them and k-mock.go:422-517 generates them)
  to_schema(struct descriptor)   -> kitex_amd.schema.Schema (the flattened table kx_schema_create takes)

Every shape compiles: what the flat column model cannot hold (maps of structs, lists of structs with
string / nested / optional fields, containers of containers, recursive structs, string defaults) becomes a
nested schema (include/kxcodec.h "Nested schemas"); map keys that are structs or containers, and leaves
more than two container levels down, raise NotImplementedError (KX_ERR_NOT_IMPLEMENTED). Supported grammar: namespace / include / cpp_include, typedef, const (skipped),
enum (-> i32), struct / union / exception, service (extends, oneway, throws), annotations `(k = "v")`,
`//`, `#` and `/* */` comments, `,` / `;` separators.
"""
from __future__ import annotations

import os
import re
import struct as _struct
from dataclasses import dataclass, field as dc_field
from typing import Dict, List, Optional, Tuple, Union

from . import _abi as A
from .schema import Field, Schema, Struct

# descriptor.go Type ids = thrift TType (descriptor/type.go)
BASE_TYPES = {"bool": A.T_BOOL, "byte": A.T_BYTE, "i8": A.T_BYTE, "i16": A.T_I16, "i32": A.T_I32,
              "i64": A.T_I64, "double": A.T_DOUBLE, "string": A.T_STRING, "binary": A.T_STRING,
              "void": A.T_VOID}


@dataclass
class TypeDescriptor:
    """descriptor.go TypeDescriptor"""
    name: str
    type: int
    key: Optional["TypeDescriptor"] = None
    elem: Optional["TypeDescriptor"] = None
    struct: Optional["StructDescriptor"] = None
    binary: bool = False


@dataclass
class FieldDescriptor:
    """descriptor.go FieldDescriptor"""
    name: str
    id: int
    type: TypeDescriptor
    required: bool = False
    optional: bool = False
    default_value: object = None
    is_exception: bool = False


@dataclass
class StructDescriptor:
    """descriptor.go StructDescriptor (fields in IDL order; the maps are views over them)"""
    name: str
    fields: List[FieldDescriptor] = dc_field(default_factory=list)

    @property
    def fields_by_id(self) -> Dict[int, FieldDescriptor]:
        return {f.id: f for f in self.fields}

    @property
    def fields_by_name(self) -> Dict[str, FieldDescriptor]:
        return {f.name: f for f in self.fields}

    @property
    def required_fields(self) -> Dict[int, FieldDescriptor]:
        return {f.id: f for f in self.fields if f.required}

    @property
    def default_fields(self) -> Dict[str, FieldDescriptor]:
        return {f.name: f for f in self.fields if f.default_value is not None}


@dataclass
class FunctionDescriptor:
    """descriptor.go FunctionDescriptor: request = the Args struct, response = the Result struct"""
    name: str
    oneway: bool
    request: TypeDescriptor
    response: TypeDescriptor


@dataclass
class ServiceDescriptor:
    name: str
    functions: Dict[str, FunctionDescriptor]

    def lookup_function_by_method(self, method: str) -> FunctionDescriptor:
        if method not in self.functions:
            raise KeyError(f"missing method: {method} in service: {self.name}")
        return self.functions[method]


# ------------------------------------------------------------------------------------------------
# tokenizer + parser
# ------------------------------------------------------------------------------------------------
_TOKEN = re.compile(r"""
    (?P<ws>\s+) | (?P<c1>//[^\n]*) | (?P<c2>\#[^\n]*) | (?P<c3>/\*.*?\*/) |
    (?P<str>"(?:[^"\\]|\\.)*"|'(?:[^'\\]|\\.)*') |
    (?P<num>[+-]?(?:0x[0-9a-fA-F]+|\d+\.\d*(?:[eE][+-]?\d+)?|\d+(?:[eE][+-]?\d+)?)) |
    (?P<id>[A-Za-z_][A-Za-z0-9_.]*) |
    (?P<sym>[{}()<>\[\]:,;=])
""", re.X | re.S)


def _tokens(text: str) -> List[Tuple[str, str]]:
    out, pos = [], 0
    while pos < len(text):
        m = _TOKEN.match(text, pos)
        if not m:
            raise SyntaxError(f"IDL: unexpected character {text[pos]!r} at offset {pos}")
        pos = m.end()
        kind = m.lastgroup
        if kind in ("ws", "c1", "c2", "c3"):
            continue
        out.append((kind, m.group(kind)))
    return out


@dataclass
class _RawField:
    id: int
    req: str
    type: object
    name: str
    default: object


@dataclass
class _RawStruct:
    kind: str
    name: str
    fields: List[_RawField]


@dataclass
class _RawFunc:
    name: str
    oneway: bool
    ret: object
    args: List[_RawField]
    throws: List[_RawField]


class _Parser:
    def __init__(self, text: str):
        self.t = _tokens(text)
        self.i = 0

    def peek(self, k=0):
        return self.t[self.i + k][1] if self.i + k < len(self.t) else None

    def next(self):
        if self.i >= len(self.t):
            raise SyntaxError("IDL: unexpected end of input")
        v = self.t[self.i][1]
        self.i += 1
        return v

    def expect(self, v):
        got = self.next()
        if got != v:
            raise SyntaxError(f"IDL: expected {v!r}, got {got!r}")

    def sep(self):
        while self.peek() in (",", ";"):
            self.i += 1

    def annotations(self):
        if self.peek() == "(":
            depth = 0
            while True:
                v = self.next()
                depth += v == "("
                depth -= v == ")"
                if depth == 0:
                    return

    def type_(self):
        name = self.next()
        if name in ("list", "set"):
            self.expect("<")
            e = self.type_()
            self.expect(">")
            self.annotations()
            return (name, e)
        if name == "map":
            self.expect("<")
            k = self.type_()
            self.expect(",")
            v = self.type_()
            self.expect(">")
            self.annotations()
            return ("map", k, v)
        self.annotations()
        return name

    def const_value(self):
        v = self.next()
        if v == "[":
            while self.peek() != "]":
                self.const_value()
                self.sep()
            self.next()
            return None
        if v == "{":
            while self.peek() != "}":
                self.const_value()
                self.expect(":")
                self.const_value()
                self.sep()
            self.next()
            return None
        if v[0] in "\"'":
            return bytes(v[1:-1], "utf-8").decode("unicode_escape")
        if re.fullmatch(r"[+-]?(0x[0-9a-fA-F]+|\d+)", v):
            return int(v, 0)
        if re.fullmatch(r"[+-]?[\d.]+([eE][+-]?\d+)?", v):
            return float(v)
        return ("ident", v)  # true / false / an enum or const name

    def field(self):
        fid = int(self.next(), 0)
        self.expect(":")
        req = ""
        if self.peek() in ("required", "optional"):
            req = self.next()
        ty = self.type_()
        name = self.next()
        default = None
        if self.peek() == "=":
            self.next()
            default = self.const_value()
        self.annotations()
        self.sep()
        return _RawField(fid, req, ty, name, default)

    def field_list(self, close):
        out = []
        while self.peek() != close:
            out.append(self.field())
        self.next()
        return out

    def document(self):
        doc = {"includes": [], "structs": {}, "enums": {}, "typedefs": {}, "consts": {}, "services": {}}
        while self.peek() is not None:
            kw = self.next()
            if kw in ("namespace",):
                self.next()
                self.next()
            elif kw in ("include", "cpp_include"):
                p = self.next()[1:-1]
                if kw == "include":
                    doc["includes"].append(p)
            elif kw == "typedef":
                ty = self.type_()
                doc["typedefs"][self.next()] = ty
                self.annotations()
            elif kw == "const":
                self.type_()
                name = self.next()
                self.expect("=")
                doc["consts"][name] = self.const_value()
            elif kw in ("enum", "senum"):
                name = self.next()
                self.expect("{")
                vals, nxt = {}, 0
                while self.peek() != "}":
                    k = self.next()
                    if self.peek() == "=":
                        self.next()
                        nxt = int(self.next(), 0)
                    vals[k] = nxt
                    nxt += 1
                    self.annotations()
                    self.sep()
                self.next()
                self.annotations()
                doc["enums"][name] = vals
            elif kw in ("struct", "union", "exception"):
                name = self.next()
                self.expect("{")
                fs = self.field_list("}")
                self.annotations()
                doc["structs"][name] = _RawStruct(kw, name, fs)
            elif kw == "service":
                name = self.next()
                ext = None
                if self.peek() == "extends":
                    self.next()
                    ext = self.next()
                self.expect("{")
                funcs = []
                while self.peek() != "}":
                    oneway = False
                    if self.peek() == "oneway":
                        self.next()
                        oneway = True
                    ret = self.type_()
                    fname = self.next()
                    self.expect("(")
                    args = self.field_list(")")
                    throws = []
                    if self.peek() == "throws":
                        self.next()
                        self.expect("(")
                        throws = self.field_list(")")
                    self.annotations()
                    self.sep()
                    funcs.append(_RawFunc(fname, oneway, ret, args, throws))
                self.next()
                self.annotations()
                doc["services"][name] = (ext, funcs)
            elif kw in (",", ";"):
                continue
            else:
                raise SyntaxError(f"IDL: unexpected {kw!r}")
        return doc


class Document:
    """A parsed IDL file with its includes (referenced as `<file stem>.<Name>`)."""

    def __init__(self, raw: dict, includes: Dict[str, "Document"], name: str = ""):
        self.raw = raw
        self.includes = includes
        self.name = name
        self._structs: Dict[str, StructDescriptor] = {}

    # -- name resolution --
    def _resolve(self, name: str):
        """(document, local name) of a possibly include-qualified name"""
        if "." in name:
            pre, rest = name.split(".", 1)
            if pre in self.includes:
                return self.includes[pre]._resolve(rest)
        return self, name

    def type_descriptor(self, ty) -> TypeDescriptor:
        if isinstance(ty, tuple):
            if ty[0] in ("list", "set"):
                return TypeDescriptor(ty[0], A.T_LIST if ty[0] == "list" else A.T_SET, elem=self.type_descriptor(ty[1]))
            return TypeDescriptor("map", A.T_MAP, key=self.type_descriptor(ty[1]), elem=self.type_descriptor(ty[2]))
        if ty in BASE_TYPES:
            return TypeDescriptor(ty, BASE_TYPES[ty], binary=ty == "binary")
        doc, local = self._resolve(ty)
        if local in doc.raw["typedefs"]:
            return doc.type_descriptor(doc.raw["typedefs"][local])
        if local in doc.raw["enums"]:
            return TypeDescriptor(local, A.T_I32)
        if local in doc.raw["structs"]:
            return TypeDescriptor(local, A.T_STRUCT, struct=doc.struct(local))
        raise KeyError(f"IDL: unknown type {ty!r}")

    def struct(self, name: str) -> StructDescriptor:
        doc, local = self._resolve(name)
        if doc is not self:
            return doc.struct(local)
        if local in self._structs:
            return self._structs[local]
        rs = self.raw["structs"][local]
        sd = StructDescriptor(local)
        self._structs[local] = sd  # before the fields: recursive structs refer to themselves
        for f in rs.fields:
            sd.fields.append(self._field(f, rs.kind == "exception"))
        return sd

    def _field(self, f: _RawField, exc=False) -> FieldDescriptor:
        d = f.default
        if isinstance(d, tuple) and d[0] == "ident":
            d = {"true": True, "false": False}.get(d[1], self._enum_value(d[1]))
        return FieldDescriptor(f.name, f.id, self.type_descriptor(f.type), required=f.req == "required",
                               optional=f.req == "optional", default_value=d, is_exception=exc)

    def _enum_value(self, name):
        doc, local = self._resolve(name)
        if "." in local:  # Enum.VALUE
            en, v = local.rsplit(".", 1)
            d2, en = doc._resolve(en)
            return d2.raw["enums"].get(en, {}).get(v)
        return doc.raw["consts"].get(local)

    def service(self, name: Optional[str] = None) -> ServiceDescriptor:
        """descriptor of a service (the last one in the file by default, as parse.go picks it), with the
        functions of the services it extends"""
        if name is None:
            name = list(self.raw["services"])[-1]
        doc, local = self._resolve(name)
        ext, funcs = doc.raw["services"][local]
        out: Dict[str, FunctionDescriptor] = {}
        if ext:
            out.update(doc.service(ext).functions)
        for fn in funcs:
            args = StructDescriptor(f"{local}{fn.name[:1].upper()}{fn.name[1:]}Args",
                                    [doc._field(a) for a in fn.args])
            res = StructDescriptor(f"{local}{fn.name[:1].upper()}{fn.name[1:]}Result")
            if fn.ret != "void":
                res.fields.append(FieldDescriptor("success", 0, doc.type_descriptor(fn.ret), optional=True))
            for t in fn.throws:
                fd = doc._field(t, exc=True)
                fd.optional = True
                res.fields.append(fd)
            out[fn.name] = FunctionDescriptor(fn.name, fn.oneway, TypeDescriptor(args.name, A.T_STRUCT, struct=args),
                                              TypeDescriptor(res.name, A.T_STRUCT, struct=res))
        return ServiceDescriptor(local, out)


def parse_idl(src: str, include_dirs=()) -> Document:
    """Parse an IDL file path (includes resolved next to it, then in include_dirs) or IDL text."""
    if os.path.exists(src):
        path = os.path.abspath(src)
        with open(path) as fh:
            text = fh.read()
        base = os.path.dirname(path)
        name = os.path.splitext(os.path.basename(path))[0]
    else:
        text, base, name = src, os.getcwd(), ""
    raw = _Parser(text).document()
    incs = {}
    for inc in raw["includes"]:
        for d in (base, *include_dirs):
            p = os.path.join(d, inc)
            if os.path.exists(p):
                incs[os.path.splitext(os.path.basename(inc))[0]] = parse_idl(p, include_dirs)
                break
        else:
            raise FileNotFoundError(f"IDL include {inc!r} not found")
    return Document(raw, incs, name)


# ------------------------------------------------------------------------------------------------
# descriptor -> schema
# ------------------------------------------------------------------------------------------------
_LEAF = (A.T_BOOL, A.T_BYTE, A.T_I16, A.T_I32, A.T_I64, A.T_DOUBLE, A.T_STRING)


def _default_bits(fd: FieldDescriptor):
    """a scalar default as its bits, a string default as the string (include/kxcodec.h: string defaults
    are nested-schema data)"""
    d = fd.default_value
    if d is None:
        return 0
    t = fd.type.type
    if t == A.T_STRING:
        return d if d != "" else 0
    if t == A.T_DOUBLE:
        return _struct.unpack("<q", _struct.pack("<d", float(d)))[0]
    if t in (A.T_BOOL, A.T_BYTE, A.T_I16, A.T_I32, A.T_I64):
        return int(d)
    raise NotImplementedError(f"field {fd.name}: default value for a container or struct")


def _elem(td: TypeDescriptor, memo):
    """a container's element (or map value) type: (wire type or element-type Field, element struct)"""
    if td.type in _LEAF:
        return td.type, None
    if td.type == A.T_STRUCT:
        return A.T_STRUCT, _struct_of(td.struct, memo)
    if td.type in (A.T_LIST, A.T_SET, A.T_MAP):   # a container of containers: described by a Field
        return _container(Field(0, td.type, td.name, binary=td.binary), td, memo), None
    raise NotImplementedError(f"element type {td.name}")


def _container(f: Field, td: TypeDescriptor, memo) -> Field:
    if td.type == A.T_MAP:
        if td.key.type not in _LEAF:
            raise NotImplementedError(f"map<{td.key.name},{td.elem.name}>: struct / container keys")
        f.elem = td.key.type
        f.val, child = _elem(td.elem, memo)
    else:
        f.elem, child = _elem(td.elem, memo)
    if child is not None:
        f.child = child
    return f


def _field(fd: FieldDescriptor, memo) -> Field:
    td = fd.type
    req = A.REQ_REQUIRED if fd.required else A.REQ_OPTIONAL if fd.optional else A.REQ_DEFAULT
    f = Field(fd.id, td.type, fd.name, req=req, default=_default_bits(fd), binary=td.binary)
    if td.type == A.T_STRUCT:
        f.child = _struct_of(td.struct, memo)
    elif td.type in (A.T_LIST, A.T_SET, A.T_MAP):
        _container(f, td, memo)
    elif td.type not in _LEAF:
        raise NotImplementedError(f"field {fd.name}: type {td.name}")
    return f


def _struct_of(sd: StructDescriptor, memo) -> Struct:
    # one Struct per descriptor: a recursive type refers to itself (the codec keeps such a field's bytes)
    s = memo.get(id(sd))
    if s is None:
        s = memo[id(sd)] = Struct(sd.name, [])
        s.fields.extend(_field(f, memo) for f in sd.fields)
    return s


def to_schema(sd: Union[StructDescriptor, TypeDescriptor]) -> Schema:
    """The codec schema of a struct descriptor (a request's Args struct decodes its record through
    body_field 1; pass `fn.request.struct.fields_by_id[1].type` for the record itself)."""
    if isinstance(sd, TypeDescriptor):
        if sd.struct is None:
            raise ValueError(f"{sd.name} is not a struct")
        sd = sd.struct
    return Schema(_struct_of(sd, {}))


def request_schema(doc: Document, method: str, service: Optional[str] = None) -> Schema:
    """The record of a method's request (its Args field 1), ready for kx_thrift_decode_messages(body_field=1)."""
    fn = doc.service(service).lookup_function_by_method(method)
    arg = fn.request.struct.fields_by_id.get(1)
    if arg is None or arg.type.type != A.T_STRUCT:
        raise NotImplementedError(f"method {method}: the request's field 1 is not a struct")
    return to_schema(arg.type)
