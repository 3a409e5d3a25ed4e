"""TEST INFRASTRUCTURE ONLY: ctypes binding of the CPU restatement (oracle/kx_oracle.c).

Imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, never by the product
(kitex_amd). It is the parity checker: the device codec's outputs are compared with it.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from typing import List, Optional, Sequence, Tuple

import numpy as np

from kitex_amd import _abi as A
from kitex_amd.columns import alloc_host, to_kx_columns
from kitex_amd.schema import Schema
from kitex_amd.synth import ColumnSet

HERE = os.path.dirname(os.path.abspath(__file__))
# KX_ORACLE_SAN=1: the ASan + UBSan build of the same sources (make asan; tests/test_sanitizers.py)
SAN = os.environ.get("KX_ORACLE_SAN") == "1"
LIB_PATH = os.path.join(HERE, "lib", "libkxoracle_asan.so" if SAN else "libkxoracle.so")

_lib = None


def build(quiet: bool = True) -> str:
    subprocess.run(["make", "-C", HERE, "-s"] + (["asan"] if SAN else []), check=True,
                   stdout=subprocess.DEVNULL if quiet else None)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if SAN or not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        u8p, u64p = C.POINTER(C.c_uint8), C.POINTER(C.c_uint64)
        vp, sz = C.c_void_p, C.c_size_t
        sdp = C.POINTER(A.StructDesc)
        for name in ("kxo_write_field_begin",):
            getattr(L, name).argtypes = [vp, C.c_uint8, C.c_int16]
        L.kxo_write_field_stop.argtypes = [vp]
        L.kxo_write_map_begin.argtypes = [vp, C.c_uint8, C.c_uint8, C.c_int32]
        L.kxo_write_list_begin.argtypes = [vp, C.c_uint8, C.c_int32]
        L.kxo_write_set_begin.argtypes = [vp, C.c_uint8, C.c_int32]
        L.kxo_write_bool.argtypes = [vp, C.c_int]
        L.kxo_write_byte.argtypes = [vp, C.c_int8]
        L.kxo_write_i16.argtypes = [vp, C.c_int16]
        L.kxo_write_i32.argtypes = [vp, C.c_int32]
        L.kxo_write_i64.argtypes = [vp, C.c_int64]
        L.kxo_write_double.argtypes = [vp, C.c_double]
        L.kxo_write_string.argtypes = [vp, vp, C.c_uint32]
        L.kxo_write_message_begin.argtypes = [vp, C.c_char_p, C.c_uint32, C.c_int32, C.c_int32]
        L.kxo_message_begin_length.argtypes = [C.c_uint32]
        L.kxo_read_message_begin.argtypes = [vp, sz, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32),
                                             C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.POINTER(sz)]
        for n in ("kxo_write_field_begin", "kxo_write_field_stop", "kxo_write_map_begin",
                  "kxo_write_list_begin", "kxo_write_set_begin", "kxo_write_bool", "kxo_write_byte",
                  "kxo_write_i16", "kxo_write_i32", "kxo_write_i64", "kxo_write_double",
                  "kxo_write_string", "kxo_write_message_begin", "kxo_message_begin_length",
                  "kxo_pb_write_meta", "kxo_put_uvarint"):
            getattr(L, n).restype = sz
        L.kxo_skip.argtypes = [vp, sz, C.c_uint8, C.c_int, C.POINTER(sz)]
        L.kxo_skip_batch.argtypes = [vp, sz, C.c_uint64, vp, C.POINTER(C.c_uint64)]
        L.kxo_frame_scan.argtypes = [vp, C.c_uint64, C.c_uint64, C.c_uint64, vp, vp, vp, vp,
                                     C.POINTER(C.c_uint64)]
        L.kxo_grpc_frame_scan.argtypes = L.kxo_frame_scan.argtypes
        L.kxo_ttstream_frame_scan.argtypes = [vp, C.c_uint64, C.c_uint64, C.POINTER(A.TTStreamKeys), vp, vp, vp, vp,
                                              vp, vp, vp, C.POINTER(C.c_uint64)]
        L.kxo_raw_messages.argtypes = [vp, C.c_uint64, vp, C.c_uint64, vp, vp, vp, vp, vp]
        L.kxo_set_seqids.argtypes = [vp, C.c_uint64, vp, C.c_uint64, vp, vp]
        L.kxo_crc32c.argtypes = [C.c_uint32, vp, C.c_uint64]
        L.kxo_crc32c.restype = C.c_uint32
        L.kxo_crc32c_batch.argtypes = [vp, C.c_uint64, vp, C.c_uint64, vp]
        L.kxo_frame_crc32c_validate.argtypes = [vp, C.c_uint64, vp, C.c_uint64, vp, vp, C.POINTER(C.c_uint64)]
        L.kxo_flatten.argtypes = [sdp, C.c_uint32, C.POINTER(A.ColumnInfo), C.POINTER(C.c_uint32),
                                  C.POINTER(C.c_uint32)]
        dec = [sdp, C.c_uint32, vp, C.c_uint64, vp, C.c_uint64, C.POINTER(A.Columns), vp,
               C.POINTER(A.Status)]
        L.kxo_thrift_decode.argtypes = dec
        L.kxo_pb_decode.argtypes = dec
        decmt = [sdp, C.c_uint32, vp, C.c_uint64, vp, C.c_uint64, C.POINTER(A.Columns),
                 C.POINTER(A.Status), C.c_int]
        L.kxo_thrift_decode_mt.argtypes = decmt
        L.kxo_pb_decode_mt.argtypes = decmt
        L.kxo_thrift_sizes.argtypes = [sdp, C.c_uint32, C.POINTER(A.Columns), C.c_uint64, vp]
        L.kxo_thrift_encode.argtypes = [sdp, C.c_uint32, C.POINTER(A.Columns), C.c_uint64, vp,
                                        C.c_uint64, vp, C.POINTER(C.c_uint64)]
        L.kxo_thrift_encode_mt.argtypes = L.kxo_thrift_encode.argtypes + [C.c_int]
        L.kxo_pb_encode.argtypes = L.kxo_thrift_encode.argtypes
        L.kxo_pb_write_meta.argtypes = [vp, C.c_char_p, C.c_uint32, C.c_int32, C.c_int32]
        L.kxo_pb_read_meta.argtypes = L.kxo_read_message_begin.argtypes
        L.kxo_put_uvarint.argtypes = [vp, C.c_uint64]
        L.kxo_get_uvarint.argtypes = [vp, sz, C.POINTER(C.c_uint64), C.POINTER(sz)]
        L.kxo_is_nested.argtypes = [sdp, C.c_uint32]
        L.kxo_is_nested.restype = C.c_int
        L.kxo_splitmix64.argtypes = [C.c_uint64]
        L.kxo_splitmix64.restype = C.c_uint64
        _lib = L
    return _lib


def _buf(n: int = 256):
    return (C.c_uint8 * n)()


def prim(fn: str, *args) -> bytes:
    """Call a kxo_write_* primitive and return the bytes it wrote."""
    extra = sum(len(a) for a in args if isinstance(a, (bytes, bytearray)))
    b = _buf(1024 + extra)
    n = getattr(lib(), fn)(b, *args)
    return bytes(b[:n])


def read_message_begin(data: bytes):
    arr = np.frombuffer(data, dtype=np.uint8).copy()
    no, nl, t, s, u = C.c_uint32(), C.c_uint32(), C.c_int32(), C.c_int32(), C.c_size_t()
    rc = lib().kxo_read_message_begin(arr.ctypes.data, len(data), C.byref(no), C.byref(nl),
                                      C.byref(t), C.byref(s), C.byref(u))
    if rc:
        return rc, None
    return 0, (data[no.value:no.value + nl.value].decode(), t.value, s.value, u.value)


def skip(data: bytes, ttype: int, maxdepth: int = 64) -> Tuple[int, int]:
    arr = np.frombuffer(data, dtype=np.uint8).copy() if data else np.zeros(1, np.uint8)
    u = C.c_size_t()
    rc = lib().kxo_skip(arr.ctypes.data, len(data), ttype, maxdepth, C.byref(u))
    return rc, u.value


def skip_batch(data: np.ndarray, n: int):
    offs = np.zeros(n + 1, dtype=np.uint64)
    done = C.c_uint64()
    rc = lib().kxo_skip_batch(data.ctypes.data, data.size, n, offs.ctypes.data, C.byref(done))
    return rc, offs, done.value


def frame_scan(data: np.ndarray, n: int, max_payload: int = 0):
    """framing sniff over n messages (kxo_frame_scan): rc, frame offsets[n+1], payload starts[n],
    payload ends[n], kinds[n], frames done"""
    fo = np.zeros(n + 1, dtype=np.uint64)
    ps = np.zeros(max(1, n), dtype=np.uint64)
    pe = np.zeros(max(1, n), dtype=np.uint64)
    kd = np.zeros(max(1, n), dtype=np.uint8)
    done = C.c_uint64()
    rc = lib().kxo_frame_scan(data.ctypes.data, data.size, n, max_payload, fo.ctypes.data, ps.ctypes.data,
                              pe.ctypes.data, kd.ctypes.data, C.byref(done))
    return rc, fo, ps[:n], pe[:n], kd[:n], done.value


def raw_messages(data: np.ndarray, offsets: np.ndarray):
    """binary generic ingress (kxo_raw_messages): rc, names (list of bytes), msg types, seqids, codes"""
    n = offsets.size - 1
    npos = np.zeros(max(1, n), dtype=np.uint64)
    nlen = np.zeros(max(1, n), dtype=np.uint64)
    ty = np.zeros(max(1, n), dtype=np.int32)
    sq = np.zeros(max(1, n), dtype=np.int32)
    rs = np.zeros(max(1, n), dtype=np.uint8)
    offs = np.ascontiguousarray(offsets, dtype=np.uint64)
    rc = lib().kxo_raw_messages(data.ctypes.data if data.size else None, data.size, offs.ctypes.data, n,
                                npos.ctypes.data, nlen.ctypes.data, ty.ctypes.data, sq.ctypes.data, rs.ctypes.data)
    names = [data[int(npos[i]):int(npos[i]) + int(nlen[i])].tobytes() for i in range(n)]
    return rc, names, ty[:n], sq[:n], rs[:n]


def set_seqids(data: np.ndarray, offsets: np.ndarray, seqids: np.ndarray):
    """SetSeqID over n raw messages, in place on a copy: rc, new bytes, codes"""
    out = data.copy()
    n = offsets.size - 1
    rs = np.zeros(max(1, n), dtype=np.uint8)
    offs = np.ascontiguousarray(offsets, dtype=np.uint64)
    sq = np.ascontiguousarray(seqids, dtype=np.int32)
    rc = lib().kxo_set_seqids(out.ctypes.data if out.size else None, out.size, offs.ctypes.data, n, sq.ctypes.data,
                              rs.ctypes.data)
    return rc, out, rs[:n]


def grpc_frame_scan(data: np.ndarray, n: int, max_payload: int = 0):
    """gRPC length-prefixed messages (kxo_grpc_frame_scan): rc, frame offsets[n+1], payload starts[n],
    payload ends[n], flags[n], messages done"""
    fo = np.zeros(n + 1, dtype=np.uint64)
    ps = np.zeros(max(1, n), dtype=np.uint64)
    pe = np.zeros(max(1, n), dtype=np.uint64)
    fl = np.zeros(max(1, n), dtype=np.uint8)
    done = C.c_uint64()
    rc = lib().kxo_grpc_frame_scan(data.ctypes.data if data.size else None, data.size, n, max_payload,
                                   fo.ctypes.data, ps.ctypes.data, pe.ctypes.data, fl.ctypes.data, C.byref(done))
    return rc, fo, ps[:n], pe[:n], fl[:n], done.value


def ttstream_frame_scan(data: np.ndarray, n: int, keys):
    """ttstream DecodeFrame over n frames (kxo_ttstream_frame_scan): rc, frame offsets[n+1], payload
    starts[n], payload ends[n], frame types[n], stream ids[n], method positions[n], method lengths[n],
    frames done"""
    fo = np.zeros(n + 1, dtype=np.uint64)
    ps = np.zeros(max(1, n), dtype=np.uint64)
    pe = np.zeros(max(1, n), dtype=np.uint64)
    ft = np.zeros(max(1, n), dtype=np.uint8)
    sd = np.zeros(max(1, n), dtype=np.int32)
    mp = np.zeros(max(1, n), dtype=np.uint64)
    ml = np.zeros(max(1, n), dtype=np.uint32)
    done = C.c_uint64()
    rc = lib().kxo_ttstream_frame_scan(data.ctypes.data if data.size else None, data.size, n, C.byref(keys),
                                       fo.ctypes.data, ps.ctypes.data, pe.ctypes.data, ft.ctypes.data, sd.ctypes.data,
                                       mp.ctypes.data, ml.ctypes.data, C.byref(done))
    return rc, fo, ps[:n], pe[:n], ft[:n], sd[:n], mp[:n], ml[:n], done.value


def crc32c(data: bytes, crc: int = 0) -> int:
    """crc32.Update(crc, Castagnoli, data) (validate.go:208-217 getCRC32C with crc = 0)"""
    buf = np.frombuffer(bytes(data), dtype=np.uint8)
    return lib().kxo_crc32c(crc, buf.ctypes.data if buf.size else None, buf.size)


def crc32c_batch(data: np.ndarray, offsets: np.ndarray):
    """rc, CRC-32C of each range [offsets[i], offsets[i+1])"""
    n = offsets.size - 1
    out = np.zeros(max(1, n), dtype=np.uint32)
    offs = np.ascontiguousarray(offsets, dtype=np.uint64)
    rc = lib().kxo_crc32c_batch(data.ctypes.data if data.size else None, data.size, offs.ctypes.data, n,
                                out.ctypes.data)
    return rc, out[:n]


def frame_crc32c_validate(data: np.ndarray, frame_offsets: np.ndarray, n: int):
    """rc, per-frame CRC-32C of the TTHeader payload, per-frame codes, first failing frame (n: none)"""
    crc = np.zeros(max(1, n), dtype=np.uint32)
    rs = np.zeros(max(1, n), dtype=np.uint8)
    first = C.c_uint64()
    fo = np.ascontiguousarray(frame_offsets, dtype=np.uint64)
    rc = lib().kxo_frame_crc32c_validate(data.ctypes.data if data.size else None, data.size, fo.ctypes.data, n,
                                         crc.ctypes.data, rs.ctypes.data, C.byref(first))
    return rc, crc[:n], rs[:n], first.value


def flatten(schema: Schema) -> Tuple[int, List[A.ColumnInfo], int]:
    tab, ns = schema.struct_table()
    cols = (A.ColumnInfo * A.MAX_COLUMNS)()
    nc, npres = C.c_uint32(), C.c_uint32()
    rc = lib().kxo_flatten(tab, ns, cols, C.byref(nc), C.byref(npres))
    return rc, [cols[i] for i in range(nc.value)] if rc == 0 else [], npres.value


def _infos(schema: Schema):
    rc, infos, npres = flatten(schema)
    if rc:
        raise ValueError(f"oracle flatten failed: {rc}")
    return infos, npres


def decode(schema: Schema, data: np.ndarray, n: int, offsets: Optional[np.ndarray] = None,
           var_caps: Optional[Sequence[int]] = None, pb: bool = False, threads: int = 0, views: bool = False,
           wide: bool = False):
    """Decode n records with the restated FastRead (or proto3 body when pb=True). views: string
    columns as zero-copy (offset, length) pairs (KX_COLF_VIEW)."""
    infos, npres = _infos(schema)
    if var_caps is None:
        var_caps = [0 if ci.kind == A.COL_FIXED else max(1, data.size) for ci in infos]
    out = alloc_host(infos, n, var_caps, npres, views=views, wide=wide)
    kc = to_kx_columns(out, infos, var_caps)
    st = A.Status()
    rs = np.zeros(max(1, n), dtype=np.uint8)
    tab, ns = schema.struct_table()
    dptr = data.ctypes.data if data.size else None
    optr = offsets.ctypes.data if offsets is not None else None
    L = lib()
    if threads:
        fn = L.kxo_pb_decode_mt if pb else L.kxo_thrift_decode_mt
        rc = fn(tab, ns, dptr, data.size, optr, n, C.byref(kc), C.byref(st), threads)
    else:
        fn = L.kxo_pb_decode if pb else L.kxo_thrift_decode
        rc = fn(tab, ns, dptr, data.size, optr, n, C.byref(kc), rs.ctypes.data, C.byref(st))
    return rc, out, st, rs[:n]


def encode(schema: Schema, cs: ColumnSet, pb: bool = False, threads: int = 1):
    infos, _ = _infos(schema)
    kc = to_kx_columns(cs, infos)
    tab, ns = schema.struct_table()
    L = lib()
    total = C.c_uint64()
    offs = np.zeros(cs.n + 1, dtype=np.uint64)
    if pb:
        cap = 64
        while True:
            out = np.zeros(cap, dtype=np.uint8)
            rc = L.kxo_pb_encode(tab, ns, C.byref(kc), cs.n, out.ctypes.data, cap, offs.ctypes.data,
                                 C.byref(total))
            if rc != A.ERR_SIZE_LIMIT:
                break
            cap *= 4
        return rc, out[:total.value], offs
    sizes = np.zeros(max(1, cs.n), dtype=np.uint64)
    rc = L.kxo_thrift_sizes(tab, ns, C.byref(kc), cs.n, sizes.ctypes.data)
    if rc:
        return rc, None, None
    cap = int(sizes[:cs.n].sum())
    out = np.zeros(max(1, cap), dtype=np.uint8)
    rc = L.kxo_thrift_encode_mt(tab, ns, C.byref(kc), cs.n, out.ctypes.data, cap, offs.ctypes.data,
                                C.byref(total), threads)
    return rc, out[:total.value], offs


def splitmix64(x: int) -> int:
    return lib().kxo_splitmix64(x)


def hexs(b: bytes) -> str:
    return b.hex()
