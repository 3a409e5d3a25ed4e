"""Synthetic record batches.

Deterministic: value = splitmix64(seed + i*16 + field) with seed = 0x4B495445 ^ config_id, so the
same batch can be produced on the host (numpy, for the CPU oracle and tests) or directly in HBM
(torch on the GPU, for bench.py) and the two are bit-identical (tests/test_synth.py).

A batch is a `ColumnSet`: one entry per flattened schema column —
  FIXED -> array[n] (int64 / int32 / int16 / uint8, host byte order)
  BYTES -> (offsets u32[n+1], data u8[total])
  LIST  -> (offsets u32[n+1], elements[total])
plus `presence` (u64[n]) when the schema tracks presence.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional

import numpy as np

from . import _abi as A

M64 = (1 << 64) - 1
ALPHABET = b"abcdefghijklmnopqrstuvwxyz0123456789"
SEED_BASE = 0x4B495445
CONFIG_ID = {"cx": 7, "r1": 1, "r2": 2, "r3": 3, "pf": 4}


def seed_for(config: str) -> int:
    return SEED_BASE ^ CONFIG_ID[config]


def _s64(v: int) -> int:
    v &= M64
    return v - (1 << 64) if v >= 1 << 63 else v


@dataclass
class ColumnSet:
    cols: list
    presence: Optional[object]
    n: int

    def var_total(self, c):
        off = self.cols[c][0]
        return int(off[-1])


# ------------------------------------------------------------------------------------------------
# backends: numpy uint64 (wrapping) and torch int64 (two's complement, logical shifts by masking)
# ------------------------------------------------------------------------------------------------
class _NP:
    def __init__(self):
        self.u64 = np.uint64

    def arange(self, n):
        return np.arange(n, dtype=np.uint64)

    def const(self, v):
        return np.uint64(v & M64)

    def srl(self, x, s):
        return x >> np.uint64(s)

    def shl(self, x, s):
        return x << np.uint64(s)

    def mod(self, x, m):
        return x % np.uint64(m)

    def to_i64(self, x):
        return x.view(np.int64)

    def low_bytes(self, x, nbytes):  # x: uint64 [n, k] -> uint8 [n, k*8]
        return x.astype("<u8").view(np.uint8).reshape(x.shape[0], -1)[:, :nbytes]


def splitmix64_np(x):
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def _key_np(seed, i, f):
    with np.errstate(over="ignore"):
        return np.uint64(seed) + i * np.uint64(16) + np.uint64(f)


def _sub_np(key, k):
    """sub-stream k (0..254) of a (record, field) key: chunks of strings, list elements"""
    with np.errstate(over="ignore"):
        return splitmix64_np((key << np.uint64(8)) ^ np.uint64(k + 1))


def _string_bytes_np(key, length):
    """[n] keys -> uint8 [n, length] drawn from ALPHABET"""
    n = key.shape[0]
    nchunk = (length + 7) // 8
    alpha = np.frombuffer(ALPHABET, dtype=np.uint8)
    if nchunk == 0:
        return np.zeros((n, 0), dtype=np.uint8)
    hs = np.stack([_sub_np(key, k) for k in range(nchunk)], axis=1)
    raw = hs.astype("<u8").view(np.uint8).reshape(n, nchunk * 8)[:, :length]
    return alpha[raw % len(ALPHABET)]


def _fixed_strings_np(key, length):
    n = key.shape[0]
    data = _string_bytes_np(key, length).reshape(-1)
    offs = (np.arange(n + 1, dtype=np.uint64) * np.uint64(length)).astype(np.uint32)
    return offs, data


def _ragged_strings_np(key, lens, maxlen):
    n = key.shape[0]
    full = _string_bytes_np(key, maxlen)
    mask = np.arange(maxlen)[None, :] < lens[:, None]
    data = full[mask]
    offs = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(lens, out=offs[1:])
    return offs.astype(np.uint32), data


# ------------------------------------------------------------------------------------------------
# host (numpy) generators
# ------------------------------------------------------------------------------------------------
def gen_r1(n: int, start: int = 0) -> ColumnSet:
    seed = seed_for("r1")
    i = np.arange(start, start + n, dtype=np.uint64)
    cols = [splitmix64_np(_key_np(seed, i, f)).view(np.int64) for f in range(1, 9)]
    return ColumnSet(cols, None, n)


def gen_r2(n: int, start: int = 0, strlen: int = 32) -> ColumnSet:
    seed = seed_for("r2")
    i = np.arange(start, start + n, dtype=np.uint64)
    cols: List[object] = [splitmix64_np(_key_np(seed, i, f)).view(np.int64) for f in range(1, 9)]
    for f in (9, 10):
        cols.append(_fixed_strings_np(_key_np(seed, i, f), strlen))
    return ColumnSet(cols, None, n)


def gen_r3(n: int, start: int = 0, maxlist: int = 128, maxtag: int = 16) -> ColumnSet:
    """columns (DFS): id, vals(list), inner.x, inner.y, inner.tag, kind; presence bits: vals=0, inner=1"""
    seed = seed_for("r3")
    i = np.arange(start, start + n, dtype=np.uint64)
    k1, k2, k4 = _key_np(seed, i, 1), _key_np(seed, i, 2), _key_np(seed, i, 4)
    k5, k6, k7 = _key_np(seed, i, 5), _key_np(seed, i, 6), _key_np(seed, i, 7)
    ids = splitmix64_np(k1).view(np.int64)
    lens = (splitmix64_np(k2) % np.uint64(maxlist + 1)).astype(np.int64)
    elems = np.stack([_sub_np(k2, e) for e in range(maxlist)], axis=1).view(np.int64) if maxlist else np.zeros((n, 0), np.int64)
    mask = np.arange(maxlist)[None, :] < lens[:, None]
    vals_data = elems[mask]
    vals_off = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(lens, out=vals_off[1:])
    x = splitmix64_np(k5).view(np.int64)
    y = splitmix64_np(k6).astype(np.uint32).view(np.int32)
    tlen = (splitmix64_np(k7) % np.uint64(maxtag + 1)).astype(np.int64)
    tag = _ragged_strings_np(k7, tlen, maxtag)
    kind = splitmix64_np(k4).astype(np.uint32).view(np.int32)
    cols = [ids, (vals_off.astype(np.uint32), vals_data), x, y, tag, kind]
    presence = np.full(n, 0b11, dtype=np.uint64)  # vals and inner always set
    return ColumnSet(cols, presence, n)


def _pf_int_np(key):
    h = splitmix64_np(key)
    h2 = splitmix64_np(key ^ np.uint64(0xA5A5A5A5A5A5A5A5))
    c = (h2 % np.uint64(10)).astype(np.int64) + 1               # target varint length 1..10
    zero = ((h2 >> np.uint64(8)) & np.uint64(15)) == 0           # 1/16 forced to 0 (omitted)
    out = np.empty(key.shape[0], dtype=np.uint64)
    neg = c == 10
    out[neg] = h[neg] | np.uint64(1 << 63)
    pos = ~neg
    bits = (7 * c[pos]).astype(np.uint64)
    v = h[pos] >> (np.uint64(64) - bits)
    v |= np.uint64(1) << (bits - np.uint64(1))
    out[pos] = v
    out[zero] = 0
    return out.view(np.int64)


def gen_pf(n: int, start: int = 0, strlen: int = 32) -> ColumnSet:
    seed = seed_for("pf")
    i = np.arange(start, start + n, dtype=np.uint64)
    cols: List[object] = [_pf_int_np(_key_np(seed, i, f)) for f in range(1, 9)]
    for f in (9, 10):
        cols.append(_fixed_strings_np(_key_np(seed, i, f), strlen))
    return ColumnSet(cols, None, n)


_ALPHA_NP = np.frombuffer(ALPHABET, dtype=np.uint8)


def _strings(rng, counts, lo, hi):
    """LIST_BYTES column parts for per-record element counts: (record offsets, element byte
    offsets, bytes) with element lengths in [lo, hi] from [a-z0-9]"""
    ne = int(counts.sum())
    lens = rng.integers(lo, hi + 1, size=ne)
    eoff = np.zeros(ne + 1, dtype=np.uint32)
    eoff[1:] = np.cumsum(lens)
    roff = np.zeros(counts.size + 1, dtype=np.uint32)
    roff[1:] = np.cumsum(counts)
    data = _ALPHA_NP[rng.integers(0, len(ALPHABET), size=max(1, int(eoff[-1])))]
    return roff, eoff, data


def gen_cx1(n: int, start: int = 0) -> ColumnSet:
    """records of schema.schema_cx1(): i64 id, string msg, map<string,string> (0..3 entries),
    list<string> (0..4 elements)"""
    rng = np.random.default_rng(seed_for("cx") + start)
    ids = rng.integers(-2**63, 2**63 - 1, size=n, dtype=np.int64)
    msg_len = rng.integers(0, 21, size=n)
    moff = np.zeros(n + 1, dtype=np.uint32)
    moff[1:] = np.cumsum(msg_len)
    msg = _ALPHA_NP[rng.integers(0, len(ALPHABET), size=max(1, int(moff[-1])))]
    c_map = rng.integers(0, 4, size=n)
    km = _strings(rng, c_map, 1, 6)
    vm = _strings(rng, c_map, 0, 8)
    lst = _strings(rng, rng.integers(0, 5, size=n), 0, 10)
    pres = np.full(n, 0b11, dtype=np.uint64)  # strMap 0, strList 1 (always written)
    return ColumnSet([ids, (moff, msg), km, vm, lst], pres, n)


def gen_cx2(n: int, start: int = 0) -> ColumnSet:
    """records of schema.schema_cx2(): i64 id, set<string> (0..3), map<i64,double> (0..3), optional
    map<i32,string> (present in half the records, 0..2 entries)"""
    rng = np.random.default_rng(seed_for("cx") + 1000003 + start)
    ids = rng.integers(-2**63, 2**63 - 1, size=n, dtype=np.int64)
    tags = _strings(rng, rng.integers(0, 4, size=n), 1, 5)
    c_sc = rng.integers(0, 4, size=n)
    soff = np.zeros(n + 1, dtype=np.uint32)
    soff[1:] = np.cumsum(c_sc)
    sk = rng.integers(-2**40, 2**40, size=max(1, int(soff[-1])), dtype=np.int64)
    sv = rng.standard_normal(size=max(1, int(soff[-1]))).view(np.int64)
    has = rng.integers(0, 2, size=n).astype(bool)
    c_nm = np.where(has, rng.integers(0, 3, size=n), 0)
    noff = np.zeros(n + 1, dtype=np.uint32)
    noff[1:] = np.cumsum(c_nm)
    nk = rng.integers(-2**31, 2**31 - 1, size=max(1, int(noff[-1])), dtype=np.int64).astype(np.int32)
    nv = _strings(rng, c_nm, 0, 7)
    pres = (np.uint64(0b11) | (has.astype(np.uint64) << np.uint64(2))).astype(np.uint64)  # tags 0, scores 1, names 2
    return ColumnSet([ids, tags, (soff, sk), (soff.copy(), sv), (noff, nk), nv], pres, n)


GENERATORS = {"r1": gen_r1, "r2": gen_r2, "r3": gen_r3, "pf": gen_pf}


# ------------------------------------------------------------------------------------------------
# device (torch) generators — same values, produced directly in HBM
# ------------------------------------------------------------------------------------------------
def _t_consts():
    import torch
    return {k: torch.tensor(_s64(v), dtype=torch.int64) for k, v in {
        "g": 0x9E3779B97F4A7C15, "m1": 0xBF58476D1CE4E5B9, "m2": 0x94D049BB133111EB}.items()}


def _srl_t(x, s):
    return (x >> s) & ((1 << (64 - s)) - 1)


def splitmix64_t(x):
    z = x + _s64(0x9E3779B97F4A7C15)
    z = (z ^ _srl_t(z, 30)) * _s64(0xBF58476D1CE4E5B9)
    z = (z ^ _srl_t(z, 27)) * _s64(0x94D049BB133111EB)
    return z ^ _srl_t(z, 31)


def _key_t(seed, i, f):
    return i * 16 + _s64(seed + f)


def _sub_t(key, k):
    return splitmix64_t((key << 8) ^ (k + 1))


def _umod_t(x, m):
    """unsigned 64-bit x mod m (m < 2^31) for int64 tensors"""
    hi = _srl_t(x, 32)
    lo = x & 0xFFFFFFFF
    return (((hi % m) * ((1 << 32) % m)) % m + lo % m) % m


def _string_bytes_t(key, length):
    import torch
    n = key.shape[0]
    nchunk = (length + 7) // 8
    alpha = torch.tensor(list(ALPHABET), dtype=torch.uint8, device=key.device)
    hs = torch.stack([_sub_t(key, k) for k in range(nchunk)], dim=1)           # [n, nchunk] int64
    raw = hs.contiguous().view(torch.uint8).reshape(n, nchunk * 8)[:, :length]   # little-endian bytes
    return alpha[(raw.to(torch.int64) % len(ALPHABET))]


def _offsets_t(off):
    """an offset column as the C-ABI takes it: 4-byte (uint32 values in int32) unless the arena
    reaches 2^32 units, then 8-byte"""
    import torch
    return off if int(off[-1].item()) >= (1 << 32) else off.to(torch.int32)


def gen_r2_torch(n: int, device, start: int = 0, strlen: int = 32, chunk: int = 1 << 22) -> ColumnSet:
    import torch
    seed = seed_for("r2")
    cols = [torch.empty(n, dtype=torch.int64, device=device) for _ in range(8)]
    sdata = [torch.empty(n * strlen, dtype=torch.uint8, device=device) for _ in range(2)]
    for c0 in range(0, n, chunk):
        c1 = min(n, c0 + chunk)
        i = torch.arange(start + c0, start + c1, dtype=torch.int64, device=device)
        for f in range(1, 9):
            cols[f - 1][c0:c1] = splitmix64_t(_key_t(seed, i, f))
        for j, f in enumerate((9, 10)):
            sdata[j][c0 * strlen:c1 * strlen] = _string_bytes_t(_key_t(seed, i, f), strlen).reshape(-1)
    offs = _offsets_t(torch.arange(n + 1, dtype=torch.int64, device=device) * strlen)
    out: List[object] = list(cols) + [(offs, sdata[0]), (offs.clone(), sdata[1])]
    return ColumnSet(out, None, n)


def gen_r1_torch(n: int, device, start: int = 0) -> ColumnSet:
    import torch
    seed = seed_for("r1")
    i = torch.arange(start, start + n, dtype=torch.int64, device=device)
    return ColumnSet([splitmix64_t(_key_t(seed, i, f)) for f in range(1, 9)], None, n)


def gen_pf_torch(n: int, device, start: int = 0, strlen: int = 32, chunk: int = 1 << 22) -> ColumnSet:
    import torch
    seed = seed_for("pf")
    cols = [torch.empty(n, dtype=torch.int64, device=device) for _ in range(8)]
    sdata = [torch.empty(n * strlen, dtype=torch.uint8, device=device) for _ in range(2)]
    for c0 in range(0, n, chunk):
        c1 = min(n, c0 + chunk)
        i = torch.arange(start + c0, start + c1, dtype=torch.int64, device=device)
        for f in range(1, 9):
            key = _key_t(seed, i, f)
            h = splitmix64_t(key)
            h2 = splitmix64_t(key ^ _s64(0xA5A5A5A5A5A5A5A5))
            c = _umod_t(h2, 10) + 1
            zero = (_srl_t(h2, 8) & 15) == 0
            bits = 7 * c
            sh = torch.clamp(64 - bits, 0, 63)
            v = _srl_var_t(h, sh) | (torch.ones_like(h) << (bits - 1).clamp(0, 63))
            v = torch.where(c == 10, h | _s64(1 << 63), v)
            v = torch.where(zero, torch.zeros_like(v), v)
            cols[f - 1][c0:c1] = v
        for j, f in enumerate((9, 10)):
            sdata[j][c0 * strlen:c1 * strlen] = _string_bytes_t(_key_t(seed, i, f), strlen).reshape(-1)
    offs = _offsets_t(torch.arange(n + 1, dtype=torch.int64, device=device) * strlen)
    out: List[object] = list(cols) + [(offs, sdata[0]), (offs.clone(), sdata[1])]
    return ColumnSet(out, None, n)


def _srl_var_t(x, s):
    """logical right shift of int64 tensor x by per-element s in [0, 63]"""
    import torch
    mask = torch.where(s == 0, torch.full_like(x, -1), (torch.ones_like(x) << (64 - s)) - 1)
    return (x >> s) & mask


def gen_r3_torch(n: int, device, start: int = 0, maxlist: int = 128, maxtag: int = 16,
                 chunk: int = 1 << 20) -> ColumnSet:
    import torch
    seed = seed_for("r3")
    ids, x, y, kind = [torch.empty(n, dtype=t, device=device) for t in
                       (torch.int64, torch.int64, torch.int32, torch.int32)]
    lens = torch.empty(n, dtype=torch.int64, device=device)
    tlen = torch.empty(n, dtype=torch.int64, device=device)
    for c0 in range(0, n, chunk):
        c1 = min(n, c0 + chunk)
        i = torch.arange(start + c0, start + c1, dtype=torch.int64, device=device)
        ids[c0:c1] = splitmix64_t(_key_t(seed, i, 1))
        lens[c0:c1] = _umod_t(splitmix64_t(_key_t(seed, i, 2)), maxlist + 1)
        x[c0:c1] = splitmix64_t(_key_t(seed, i, 5))
        y[c0:c1] = (splitmix64_t(_key_t(seed, i, 6)) & 0xFFFFFFFF).to(torch.int64).to(torch.int32)
        tlen[c0:c1] = _umod_t(splitmix64_t(_key_t(seed, i, 7)), maxtag + 1)
        kind[c0:c1] = (splitmix64_t(_key_t(seed, i, 4)) & 0xFFFFFFFF).to(torch.int32)
    voff = torch.zeros(n + 1, dtype=torch.int64, device=device)
    voff[1:] = torch.cumsum(lens, 0)
    toff = torch.zeros(n + 1, dtype=torch.int64, device=device)
    toff[1:] = torch.cumsum(tlen, 0)
    vdata = torch.empty(int(voff[-1]), dtype=torch.int64, device=device)
    tdata = torch.empty(int(toff[-1]), dtype=torch.uint8, device=device)
    ar_l = torch.arange(maxlist, device=device)
    ar_t = torch.arange(maxtag, device=device)
    for c0 in range(0, n, chunk):
        c1 = min(n, c0 + chunk)
        i = torch.arange(start + c0, start + c1, dtype=torch.int64, device=device)
        k2 = _key_t(seed, i, 2)
        el = torch.stack([_sub_t(k2, e) for e in range(maxlist)], dim=1)
        m = ar_l[None, :] < lens[c0:c1, None]
        vdata[int(voff[c0]):int(voff[c1])] = el[m]
        tb = _string_bytes_t(_key_t(seed, i, 7), maxtag)
        mt = ar_t[None, :] < tlen[c0:c1, None]
        tdata[int(toff[c0]):int(toff[c1])] = tb[mt]
    pres = torch.full((n,), 3, dtype=torch.int64, device=device)
    cols = [ids, (_offsets_t(voff), vdata), x, y, (_offsets_t(toff), tdata), kind]
    return ColumnSet(cols, pres, n)


TORCH_GENERATORS = {"r1": gen_r1_torch, "r2": gen_r2_torch, "r3": gen_r3_torch, "pf": gen_pf_torch}


# ---------------------------------------------------------------------------------------------
# Any schema: k distinct Thrift-binary records written on the host (the nested-path bench input, tiled
# on the device). Fields in IDL order, every field present; containers of 0..maxn entries, strings of
# 0..maxs bytes. numpy's PCG64 stream seeded with `seed`.
# ---------------------------------------------------------------------------------------------
def _tw_value(out: bytearray, t: int, node, child, rng, maxn: int, maxs: int, depth: int):
    import struct
    if t == A.T_BOOL:
        out.append(int(rng.integers(0, 2)))
    elif t == A.T_BYTE:
        out += struct.pack(">b", int(rng.integers(-128, 128)))
    elif t == A.T_I16:
        out += struct.pack(">h", int(rng.integers(-2**15, 2**15)))
    elif t == A.T_I32:
        out += struct.pack(">i", int(rng.integers(-2**31, 2**31)))
    elif t == A.T_I64:
        out += struct.pack(">q", int(rng.integers(-2**63, 2**63 - 1)))
    elif t == A.T_DOUBLE:
        out += struct.pack(">d", float(rng.standard_normal()))
    elif t == A.T_STRING:
        s = rng.integers(97, 123, size=int(rng.integers(0, maxs + 1)), dtype=np.uint8).tobytes()
        out += struct.pack(">I", len(s)) + s
    elif t == A.T_STRUCT:
        _tw_struct(out, child, rng, maxn, maxs, depth + 1)
    elif t in (A.T_LIST, A.T_SET):
        et, enode, echild = _tw_sub(node.elem, node.child)
        k = int(rng.integers(0, maxn + 1)) if depth < 3 else 0
        out += struct.pack(">bi", et, k)
        for _ in range(k):
            _tw_value(out, et, enode, echild, rng, maxn, maxs, depth)
    elif t == A.T_MAP:
        kt, knode, kchild = _tw_sub(node.elem, None)
        vt, vnode, vchild = _tw_sub(node.val, node.child)
        k = int(rng.integers(0, maxn + 1)) if depth < 3 else 0
        out += struct.pack(">bbi", kt, vt, k)
        for _ in range(k):
            _tw_value(out, kt, knode, kchild, rng, maxn, maxs, depth)
            _tw_value(out, vt, vnode, vchild, rng, maxn, maxs, depth)
    else:
        raise ValueError(f"type {t}")


def _tw_sub(sub, child):
    """(ttype, container node, struct) of a container's element / key / value"""
    from .schema import Field
    if isinstance(sub, Field):
        return sub.ttype, sub, sub.child
    return sub, None, child


def _tw_struct(out: bytearray, st, rng, maxn: int, maxs: int, depth: int):
    import struct
    for f in st.fields:
        out += struct.pack(">bh", f.ttype, f.id)
        _tw_value(out, f.ttype, f, f.child, rng, maxn, maxs, depth)
    out.append(A.T_STOP)


def thrift_records(schema, k: int, seed: int = 1, maxn: int = 4, maxs: int = 24) -> List[bytes]:
    rng = np.random.default_rng(seed)
    recs = []
    for _ in range(k):
        out = bytearray()
        _tw_struct(out, schema.root, rng, maxn, maxs, 0)
        recs.append(bytes(out))
    return recs
