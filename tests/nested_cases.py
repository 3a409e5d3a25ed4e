"""Test infrastructure: nested-schema batches (include/kxcodec.h "Nested schemas").

Values are generated as Python trees (a struct is {field id: value}, a list a Python list, a map a list of
(key, value) pairs, a string bytes, a double its IEEE bits) and written to Thrift binary by a small
writer here, independent of both the oracle (oracle/kx_oracle_nested.c) and the device walker
(kitex_amd/csrc/kx_nested.h). Canonical writes follow FastWriteNocopy (struct_tpl.go:225-264, fixed-length
fields first per patcher.go:503-522, optional fields only when set, a nil struct as STOP); `noise` writes
fields in shuffled order with unknown ids, mistyped known ids and repeated fields (the last one wins)."""
from __future__ import annotations

import struct as _st

import numpy as np

from kitex_amd import _abi as A
from kitex_amd.schema import Field, Struct

SCALAR_FMT = {A.T_BOOL: ">B", A.T_BYTE: ">B", A.T_I16: ">H", A.T_I32: ">I", A.T_I64: ">Q", A.T_DOUBLE: ">Q"}
MASK = {A.T_BOOL: 1, A.T_BYTE: 0xFF, A.T_I16: 0xFFFF, A.T_I32: 0xFFFFFFFF, A.T_I64: (1 << 64) - 1,
        A.T_DOUBLE: (1 << 64) - 1}


def field_type(f: Field):
    """('scalar', t) | ('string',) | ('struct', S) | ('list', t, elem type) | ('map', key type, value type)"""
    return _type(f.ttype, f.elem, f.val, f.child)


def _type(t, elem, val, child):
    if t in A.TYPE_SIZE:
        return ("scalar", t)
    if t == A.T_STRING:
        return ("string",)
    if t == A.T_STRUCT:
        return ("struct", child)
    if t in (A.T_LIST, A.T_SET):
        return ("list", t, _elem(elem, child))
    return ("map", _elem(elem, None), _elem(val, child))


def _elem(e, child):
    if isinstance(e, Field):
        return field_type(e)
    return _type(e, 0, 0, child)


def wire_type(ty) -> int:
    k = ty[0]
    return ty[1] if k == "scalar" else A.T_STRING if k == "string" else A.T_STRUCT if k == "struct" else \
        ty[1] if k == "list" else A.T_MAP


class Gen:
    def __init__(self, seed: int, max_elems: int = 4, max_str: int = 12, rec_depth: int = 2):
        self.rng = np.random.default_rng(seed)
        self.max_elems, self.max_str, self.rec_depth = max_elems, max_str, rec_depth

    def value(self, ty, stack=()):
        r = self.rng
        k = ty[0]
        if k == "scalar":
            t = ty[1]
            return int(r.integers(0, 2)) if t == A.T_BOOL else int(r.integers(0, 1 << 62)) * 3 & MASK[t]
        if k == "string":
            return bytes(r.integers(0, 256, size=int(r.integers(0, self.max_str + 1)), dtype=np.uint8))
        if k == "struct":
            return self.struct(ty[1], stack)
        if k == "list":
            return [self.value(ty[2], stack) for _ in range(int(r.integers(0, self.max_elems + 1)))]
        return [(self.value(ty[1], stack), self.value(ty[2], stack)) for _ in range(int(r.integers(0, self.max_elems + 1)))]

    def struct(self, s: Struct, stack=()):
        out = {}
        depth = sum(1 for x in stack if x is s)
        for f in s.fields:
            ty = field_type(f)
            if ty[0] == "struct" and depth >= self.rec_depth and any(x is ty[1] for x in stack + (s,)):
                continue  # bound the recursion of a recursive type
            if f.req == A.REQ_OPTIONAL and self.rng.random() < 0.4:
                continue
            if f.req == A.REQ_DEFAULT and ty[0] == "struct" and self.rng.random() < 0.2:
                continue  # a nil struct field (written as STOP)
            out[f.id] = self.value(ty, stack + (s,))
        return out


def _default_value(f: Field, ty):
    if ty[0] == "scalar":
        return int(f.default) & MASK[ty[1]] if isinstance(f.default, int) else 0
    if ty[0] == "string":
        d = f.default
        return d.encode() if isinstance(d, str) else d if isinstance(d, bytes) else b""
    if ty[0] == "list" or ty[0] == "map":
        return []
    return None


class Writer:
    """Thrift binary of value trees (canonical FastWriteNocopy, or noisy)."""

    def __init__(self, noise: bool = False, seed: int = 0):
        self.noise = noise
        self.rng = np.random.default_rng(seed)

    def value(self, ty, v) -> bytes:
        k = ty[0]
        if k == "scalar":
            t = ty[1]
            return _st.pack(SCALAR_FMT[t], (1 if v else 0) if t == A.T_BOOL else v & MASK[t])
        if k == "string":
            return _st.pack(">I", len(v)) + v
        if k == "struct":
            return self.struct(ty[1], v)
        if k == "list":
            return bytes([wire_type(ty[2])]) + _st.pack(">I", len(v)) + b"".join(self.value(ty[2], x) for x in v)
        return bytes([wire_type(ty[1]), wire_type(ty[2])]) + _st.pack(">I", len(v)) + \
            b"".join(self.value(ty[1], a) + self.value(ty[2], b) for a, b in v)

    def struct(self, s: Struct, v) -> bytes:
        if v is None:
            return b"\x00"
        parts = []
        for f in s.fields:
            ty = field_type(f)
            if f.id not in v:
                if f.req == A.REQ_OPTIONAL:
                    continue
                if ty[0] == "struct":
                    parts.append((f, bytes([A.T_STRUCT]) + _st.pack(">h", f.id) + b"\x00"))  # nil *T
                    continue
                val = _default_value(f, ty)
            else:
                val = v[f.id]
            parts.append((f, bytes([wire_type(ty)]) + _st.pack(">h", f.id) + self.value(ty, val)))
        if not self.noise:
            order = [p for p in parts if field_type(p[0])[0] == "scalar"] + \
                    [p for p in parts if field_type(p[0])[0] != "scalar"]
            return b"".join(p[1] for p in order) + b"\x00"
        r = self.rng
        groups = []               # shuffled as units: a repeated field's last occurrence stays last
        for f, b in parts:
            g = []
            if r.random() < 0.25:   # an earlier occurrence of the same field with other content: overwritten
                ty = field_type(f)
                other = Gen(int(r.integers(0, 1 << 30))).value(ty)   # written plainly: bounded depth
                g.append(bytes([wire_type(ty)]) + _st.pack(">h", f.id) + Writer().value(ty, other))
            g.append(b)
            groups.append(g)
            if r.random() < 0.2:    # an unknown field id (skipped)
                groups.append([bytes([A.T_LIST, 0x7F, 0x00, A.T_STRING]) + _st.pack(">I", 1) + _st.pack(">I", 2) +
                               b"zz"])
            if r.random() < 0.15:   # a known id with the wrong wire type (skipped)
                wt = A.T_I64 if field_type(f)[0] != "scalar" or f.ttype != A.T_I64 else A.T_STRING
                body = _st.pack(">Q", 7) if wt == A.T_I64 else _st.pack(">I", 1) + b"x"
                groups.append([bytes([wt]) + _st.pack(">h", f.id) + body])
        order = r.permutation(len(groups))
        return b"".join(b"".join(groups[i]) for i in order) + b"\x00"


def batch(schema, n: int, seed: int = 0, noise: bool = False, **gen_kw):
    """n records of `schema`: (value trees, wire uint8 array, offsets uint64[n+1])"""
    g = Gen(seed, **gen_kw)
    w = Writer(noise=noise, seed=seed + 1)
    vals = [g.struct(schema.root) for _ in range(n)]
    recs = [w.struct(schema.root, v) for v in vals]
    offs = np.zeros(n + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(b) for b in recs])
    wire = np.frombuffer(b"".join(recs), dtype=np.uint8).copy() if recs else np.zeros(0, np.uint8)
    return vals, wire, offs
