"""Kitex-Protobuf nested messages (include/kxcodec.h, KX_STRUCT_PROTOBUF): the test schema, a seeded value
generator and an independent proto3 writer, shared by the CPU suite (oracle vs google.protobuf, host walker vs
oracle: tests/test_pbn.py) and the GPU suite (libkxcodec vs oracle: tests/test_gpu_pbn.py).

The writer produces canonical bytes (proto.Marshal: field-number order, zero scalars omitted, packed repeated
scalars, map entries with key and value) and noisy bytes that decode to the same message (fields shuffled,
repeated scalars unpacked or split over several packed runs, a singular field written twice with the last
value winning, a message field split over several occurrences that merge, unknown fields of every wire
type). The semantics are pinned by google.protobuf (upb, in this image) parsing the same bytes: see
tests/test_pbn.py and tests/golden/make_pbn_golden.py."""
from __future__ import annotations

import random
import struct

import numpy as np

from kitex_amd import _abi as A
from kitex_amd.schema import Field, Schema, Struct

T = A

# proto type name -> (ttype, kind)
PT = {
    "int64": (A.T_I64, A.PB_NATURAL), "uint64": (A.T_I64, A.PB_UINT), "sint64": (A.T_I64, A.PB_SINT),
    "fixed64": (A.T_I64, A.PB_FIXED), "sfixed64": (A.T_I64, A.PB_FIXED),
    "int32": (A.T_I32, A.PB_NATURAL), "uint32": (A.T_I32, A.PB_UINT), "sint32": (A.T_I32, A.PB_SINT),
    "fixed32": (A.T_I32, A.PB_FIXED), "sfixed32": (A.T_I32, A.PB_FIXED), "float": (A.T_I32, A.PB_FIXED),
    "double": (A.T_DOUBLE, A.PB_NATURAL), "bool": (A.T_BOOL, A.PB_NATURAL),
    "string": (A.T_STRING, A.PB_NATURAL), "bytes": (A.T_STRING, A.PB_BYTES), "enum": (A.T_I32, A.PB_NATURAL),
}


def _f(num, name, ptype, label="", child=None, key=None, val=None, val_child=None):
    """a proto field as a schema Field: label '' (singular), 'optional', 'repeated', 'map'"""
    req = A.REQ_OPTIONAL if label == "optional" else A.REQ_DEFAULT
    if label == "map":
        kt, kk = PT[key]
        if val == "message":
            return Field(num, A.T_MAP, name, elem=kt, val=A.T_STRUCT, child=val_child, pb=kk)
        vt, vk = PT[val]
        return Field(num, A.T_MAP, name, elem=kt, val=vt, pb=kk, pbv=vk)
    if ptype == "message":
        if label == "repeated":
            return Field(num, A.T_LIST, name, elem=A.T_STRUCT, child=child)
        return Field(num, A.T_STRUCT, name, child=child)
    tt, kind = PT[ptype]
    if label == "repeated":
        return Field(num, A.T_LIST, name, elem=tt, pb=kind)
    return Field(num, tt, name, req=req, pb=kind)


# the proto3 test messages: (name, [(num, name, type, label, extra)])
INNER = [(1, "x", "int64", ""), (2, "tag", "string", ""), (3, "zs", "sint32", "repeated"),
         (4, "o", "uint32", "optional")]
LEAF = [(1, "f", "fixed32", ""), (2, "g", "float", "")]
PN = [(1, "id", "int64", ""), (2, "s64", "sint64", ""), (3, "s32", "sint32", ""), (4, "f64", "fixed64", ""),
      (5, "f32", "fixed32", ""), (6, "fl", "float", ""), (7, "d", "double", ""), (8, "b", "bool", ""),
      (9, "u32", "uint32", ""), (10, "i32", "int32", ""), (11, "name", "string", ""), (12, "blob", "bytes", ""),
      (13, "vals", "int64", "repeated"), (14, "tags", "string", "repeated"), (15, "inner", "Inner", ""),
      (16, "items", "Inner", "repeated"), (17, "counts", "map<string,int64>", "map"),
      (18, "leaves", "map<int32,Leaf>", "map"), (19, "opt", "int64", "optional"),
      (20, "fx", "fixed32", "repeated"), (21, "names", "map<sint64,string>", "map"),
      (22, "flags", "bool", "repeated"), (23, "u64", "uint64", ""), (24, "sf32", "sfixed32", ""),
      (25, "sf64", "sfixed64", "")]
PK = [(1, "a", "sint64", ""), (2, "b", "fixed32", ""), (3, "c", "float", ""), (4, "d", "uint32", ""),
      (5, "e", "sfixed64", ""), (6, "s", "string", "")]
MESSAGES = {"Inner": INNER, "Leaf": LEAF, "PN": PN, "PK": PK}


def _struct(name, structs):
    if name in structs:
        return structs[name]
    s = Struct(name, [])
    structs[name] = s
    for num, fname, ty, label in MESSAGES[name]:
        if label == "map":
            k, v = ty[4:-1].split(",")
            if v in MESSAGES:
                s.fields.append(_f(num, fname, None, "map", key=k, val="message", val_child=_struct(v, structs)))
            else:
                s.fields.append(_f(num, fname, None, "map", key=k, val=v))
        elif ty in MESSAGES:
            s.fields.append(_f(num, fname, "message", label, child=_struct(ty, structs)))
        else:
            s.fields.append(_f(num, fname, ty, label))
    return s


def schema_pn() -> Schema:
    return Schema(_struct("PN", {}), protobuf=True)


def schema_pk() -> Schema:
    """a flat message whose scalars need the nested path (zig-zag / fixed / float / uint kinds)"""
    return Schema(_struct("PK", {}), protobuf=True)


SCHEMAS = {"PN": schema_pn, "PK": schema_pk}


# ---- values -----------------------------------------------------------------------------------------
class Gen:
    def __init__(self, seed, max_rep=4, max_str=12):
        self.r = random.Random(seed)
        self.max_rep, self.max_str = max_rep, max_str

    def scalar(self, ty):
        r = self.r
        if r.random() < 0.15:
            return {"bool": False, "string": "", "bytes": b"", "double": 0.0, "float": 0.0}.get(ty, 0)
        if ty in ("int64", "sint64", "sfixed64"):
            return r.choice([r.randrange(-(1 << 63), 1 << 63), r.randrange(-300, 300)])
        if ty in ("uint64", "fixed64"):
            return r.choice([r.randrange(0, 1 << 64), r.randrange(0, 300)])
        if ty in ("int32", "sint32", "sfixed32", "enum"):
            return r.choice([r.randrange(-(1 << 31), 1 << 31), r.randrange(-300, 300)])
        if ty in ("uint32", "fixed32"):
            return r.choice([r.randrange(0, 1 << 32), r.randrange(0, 300)])
        if ty == "bool":
            return r.random() < 0.5
        if ty == "double":
            return r.choice([r.uniform(-1e6, 1e6), -0.0, 1.5])
        if ty == "float":
            return struct.unpack("<f", struct.pack("<f", r.uniform(-1e4, 1e4)))[0]
        if ty == "string":
            alpha = "abcdefghij éü中文✓"
            return "".join(r.choice(alpha) for _ in range(r.randrange(0, self.max_str)))
        if ty == "bytes":
            return bytes(r.randrange(256) for _ in range(r.randrange(0, self.max_str)))
        raise ValueError(ty)

    def message(self, name, depth=0):
        r = self.r
        v = {}
        for num, fname, ty, label in MESSAGES[name]:
            if label == "map":
                k, vt = ty[4:-1].split(",")
                m = {}
                for _ in range(r.randrange(0, self.max_rep)):
                    key = self.scalar(k)
                    m[key] = self.message(vt, depth + 1) if vt in MESSAGES else self.scalar(vt)
                v[fname] = dict(sorted(m.items()))
            elif label == "repeated":
                cnt = r.randrange(0, self.max_rep)
                v[fname] = [self.message(ty, depth + 1) if ty in MESSAGES else self.scalar(ty) for _ in range(cnt)]
            elif ty in MESSAGES:
                if r.random() < 0.7:
                    v[fname] = self.message(ty, depth + 1)
            elif label == "optional":
                if r.random() < 0.5:
                    v[fname] = self.scalar(ty)
            else:
                v[fname] = self.scalar(ty)
        return v


# ---- proto3 writer ----------------------------------------------------------------------------------
def uvarint(v: int) -> bytes:
    v &= (1 << 64) - 1
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def tag(num, wt):
    return uvarint((num << 3) | wt)


WT = {"double": 1, "fixed64": 1, "sfixed64": 1, "fixed32": 5, "sfixed32": 5, "float": 5,
      "string": 2, "bytes": 2}


def wt_of(ty):
    return 2 if ty in MESSAGES else WT.get(ty, 0)


def scalar_bytes(ty, v) -> bytes:
    """the value bytes (no tag) of a scalar / string"""
    if ty in ("int64", "uint64", "int32", "enum"):
        return uvarint(v)                      # int32 negative: sign-extended to 10 bytes
    if ty == "uint32":
        return uvarint(v & 0xFFFFFFFF)
    if ty == "sint64":
        return uvarint(((v << 1) ^ (v >> 63)) & ((1 << 64) - 1))
    if ty == "sint32":
        return uvarint(((v << 1) ^ (v >> 31)) & 0xFFFFFFFF)
    if ty == "bool":
        return uvarint(1 if v else 0)
    if ty in ("fixed64", "sfixed64"):
        return struct.pack("<Q", v & ((1 << 64) - 1))
    if ty in ("fixed32", "sfixed32"):
        return struct.pack("<I", v & 0xFFFFFFFF)
    if ty == "float":
        return struct.pack("<f", v)
    if ty == "double":
        return struct.pack("<d", v)
    if ty in ("string", "bytes"):
        b = v.encode() if isinstance(v, str) else v
        return uvarint(len(b)) + b
    raise ValueError(ty)


def is_zero(ty, v):
    if ty == "double" or ty == "float":
        return struct.pack("<d", v) == b"\0" * 8
    return not v


class Writer:
    """canonical (noise=False) or noisy proto3 bytes of a value dict"""

    def __init__(self, noise=False, seed=0):
        self.noise = noise
        self.r = random.Random(seed)

    def message(self, name, v) -> bytes:
        groups = []
        for num, fname, ty, label in sorted(MESSAGES[name], key=lambda f: f[0]):
            if fname not in v:
                continue
            groups.append(self.field(num, ty, label, v[fname]))
        groups = [g for g in groups if g]
        if not self.noise:
            return b"".join(b"".join(g) for g in groups)
        pieces = [p for g in groups for p in g]
        self.r.shuffle(pieces)
        # unknown fields of every wire type, anywhere
        for _ in range(self.r.randrange(0, 3)):
            num = self.r.choice([50, 99, 1000, 123456])
            wt = self.r.choice([0, 1, 2, 5])
            body = {0: uvarint(self.r.randrange(1 << 40)), 1: bytes(8), 2: uvarint(3) + b"xyz", 5: bytes(4)}[wt]
            pieces.insert(self.r.randrange(len(pieces) + 1), tag(num, wt) + body)
        return b"".join(pieces)

    def field(self, num, ty, label, v):
        """pieces (each a whole tagged field occurrence) that decode to v"""
        r = self.r
        if label == "map":
            k, vt = ty[4:-1].split(",")
            out = []
            for key, val in v.items():
                kb = tag(1, wt_of(k)) + scalar_bytes(k, key)
                if vt in MESSAGES:
                    vbody = self.message(vt, val)
                    vb = tag(2, 2) + uvarint(len(vbody)) + vbody
                else:
                    vb = tag(2, wt_of(vt)) + scalar_bytes(vt, val)
                ent = kb + vb
                if self.noise and r.random() < 0.3:
                    ent = vb + kb                  # value before key
                out.append(tag(num, 2) + uvarint(len(ent)) + ent)
            return [b"".join(out)] if (out and not self.noise) else out
        if label == "repeated":
            if not v:
                return []
            if ty in MESSAGES or ty in ("string", "bytes"):
                out = []
                for e in v:
                    if ty in MESSAGES:
                        body = self.message(ty, e)
                        out.append(tag(num, 2) + uvarint(len(body)) + body)
                    else:
                        out.append(tag(num, 2) + scalar_bytes(ty, e))
                return [b"".join(out)] if not self.noise else out
            if self.noise and r.random() < 0.5:       # unpacked, or several packed runs (order kept)
                if r.random() < 0.5:
                    return [b"".join(tag(num, wt_of(ty)) + scalar_bytes(ty, e) for e in v)]
                cut = r.randrange(0, len(v) + 1)
                runs = [v[:cut], v[cut:]]
                return [b"".join(tag(num, 2) + uvarint(len(b"".join(scalar_bytes(ty, e) for e in run)))
                                 + b"".join(scalar_bytes(ty, e) for e in run) for run in runs)]
            body = b"".join(scalar_bytes(ty, e) for e in v)
            return [tag(num, 2) + uvarint(len(body)) + body]
        if ty in MESSAGES:
            body = self.message(ty, v)
            if self.noise and r.random() < 0.4 and len(MESSAGES[ty]) > 1:
                # split into two occurrences that merge (scalar fields disjoint, repeated split in order)
                a, b = {}, {}
                for _, fname, fty, flabel in MESSAGES[ty]:
                    if fname not in v:
                        continue
                    if flabel == "repeated":
                        cut = r.randrange(0, len(v[fname]) + 1)
                        a[fname], b[fname] = v[fname][:cut], v[fname][cut:]
                    elif r.random() < 0.5:
                        a[fname] = v[fname]
                    else:
                        b[fname] = v[fname]
                ba, bb = Writer(False).message(ty, a), Writer(False).message(ty, b)
                return [tag(num, 2) + uvarint(len(ba)) + ba + tag(num, 2) + uvarint(len(bb)) + bb]
            return [tag(num, 2) + uvarint(len(body)) + body]
        if label != "optional" and is_zero(ty, v):
            return []
        piece = tag(num, wt_of(ty)) + scalar_bytes(ty, v)
        if self.noise and r.random() < 0.25:          # an earlier occurrence that the last one replaces
            other = Gen(r.randrange(1 << 30)).scalar(ty)
            return [tag(num, wt_of(ty)) + scalar_bytes(ty, other) + piece]
        return [piece]


def batch(n, seed=0, noise=False, name="PN", framed=False, **gen_kw):
    """n records: (values, wire uint8, offsets uint64[n+1]); framed: Batch frames (0x0A, uvarint, body)
    with offsets at the bodies"""
    g = Gen(seed, **gen_kw)
    w = Writer(noise=noise, seed=seed + 1)
    vals = [g.message(name) for _ in range(n)]
    bodies = [w.message(name, v) for v in vals]
    if framed:
        parts, offs, pos = [], np.zeros(n + 1, dtype=np.uint64), 0
        for i, b in enumerate(bodies):
            h = b"\x0a" + uvarint(len(b))
            parts.append(h + b)
            offs[i] = pos + len(h)
            pos += len(h) + len(b)
        offs[n] = pos
        blob = b"".join(parts)
    else:
        offs = np.zeros(n + 1, dtype=np.uint64)
        offs[1:] = np.cumsum([len(b) for b in bodies]) if bodies else []
        blob = b"".join(bodies)
    wire = np.frombuffer(blob, dtype=np.uint8).copy() if blob else np.zeros(0, np.uint8)
    return vals, wire, offs


# ---- google.protobuf (upb) classes of the same messages, for the semantic pin -----------------------
def upb_classes(messages=None, packed=True):
    """{name: message class} built from MESSAGES with google.protobuf's descriptor pool (proto3)"""
    from google.protobuf import descriptor_pb2, descriptor_pool, message_factory
    messages = messages or MESSAGES
    F = descriptor_pb2.FieldDescriptorProto
    tmap = {"int64": F.TYPE_INT64, "uint64": F.TYPE_UINT64, "sint64": F.TYPE_SINT64, "fixed64": F.TYPE_FIXED64,
            "sfixed64": F.TYPE_SFIXED64, "int32": F.TYPE_INT32, "uint32": F.TYPE_UINT32, "sint32": F.TYPE_SINT32,
            "fixed32": F.TYPE_FIXED32, "sfixed32": F.TYPE_SFIXED32, "float": F.TYPE_FLOAT, "double": F.TYPE_DOUBLE,
            "bool": F.TYPE_BOOL, "string": F.TYPE_STRING, "bytes": F.TYPE_BYTES}
    fdp = descriptor_pb2.FileDescriptorProto(name=f"pn_{int(packed)}.proto", package=f"pn{int(packed)}",
                                             syntax="proto3")
    pkg = fdp.package
    for name, fields in messages.items():
        m = fdp.message_type.add(name=name)
        oneof_i = 0
        for num, fname, ty, label in fields:
            if label == "map":
                k, v = ty[4:-1].split(",")
                ent = m.nested_type.add(name=fname.capitalize() + "Entry")
                ent.options.map_entry = True
                ent.field.add(name="key", number=1, type=tmap[k], label=F.LABEL_OPTIONAL)
                vf = ent.field.add(name="value", number=2, label=F.LABEL_OPTIONAL)
                if v in messages:
                    vf.type = F.TYPE_MESSAGE
                    vf.type_name = f".{pkg}.{v}"
                else:
                    vf.type = tmap[v]
                fd = m.field.add(name=fname, number=num, label=F.LABEL_REPEATED, type=F.TYPE_MESSAGE,
                                 type_name=f".{pkg}.{name}.{ent.name}")
                continue
            fd = m.field.add(name=fname, number=num)
            if ty in messages:
                fd.type = F.TYPE_MESSAGE
                fd.type_name = f".{pkg}.{ty}"
            else:
                fd.type = tmap[ty]
            fd.label = F.LABEL_REPEATED if label == "repeated" else F.LABEL_OPTIONAL
            if label == "repeated" and ty not in messages and ty not in ("string", "bytes") and not packed:
                fd.options.packed = False
            if label == "optional":          # proto3 `optional`: a synthetic oneof
                m.oneof_decl.add(name=f"_{fname}")
                fd.oneof_index = oneof_i
                fd.proto3_optional = True
                oneof_i += 1
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fdp)
    return {name: message_factory.GetMessageClass(pool.FindMessageTypeByName(f"{pkg}.{name}"))
            for name in messages}


def fill(cls_map, name, msg, v):
    """set a upb message from a value dict"""
    for num, fname, ty, label in MESSAGES[name]:
        if fname not in v:
            continue
        x = v[fname]
        if label == "map":
            k, vt = ty[4:-1].split(",")
            mf = getattr(msg, fname)
            for key, val in x.items():
                if vt in MESSAGES:
                    fill(cls_map, vt, mf[key], val)
                else:
                    mf[key] = val
        elif label == "repeated":
            rf = getattr(msg, fname)
            for e in x:
                if ty in MESSAGES:
                    fill(cls_map, ty, rf.add(), e)
                else:
                    rf.append(e)
        elif ty in MESSAGES:
            sub = getattr(msg, fname)
            sub.SetInParent()
            fill(cls_map, ty, sub, x)
        else:
            setattr(msg, fname, x)
