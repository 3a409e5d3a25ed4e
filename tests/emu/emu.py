"""Test infrastructure only: ctypes binding of the CPU SIMT emulation of the decode kernel."""
import ctypes as C
import os
import subprocess

import numpy as np

from kitex_amd import _abi as A
from kitex_amd.columns import alloc_host, to_kx_columns

HERE = os.path.dirname(os.path.abspath(__file__))
# KX_EMU_SAN=1: a host AddressSanitizer + UndefinedBehaviorSanitizer build (tests/test_sanitizers.py runs the
# emulator suites in a child process with the ASan runtime preloaded)
SAN = os.environ.get("KX_EMU_SAN") == "1"
SAN_FLAGS = "-fsanitize=address,undefined -fno-sanitize-recover=undefined -fno-omit-frame-pointer -shared-libasan"
OUT = "_build_san" if SAN else "_build"
LIB = os.path.join(HERE, OUT, "libkxemu.so")
_lib = None


def build():
    env = dict(os.environ, EMU_OUT=OUT)
    if SAN:
        env["EMU_EXTRA"] = SAN_FLAGS
    subprocess.run([os.path.join(HERE, "build_emu.sh")], check=True, stdout=subprocess.DEVNULL, env=env)


def lib():
    global _lib
    if _lib is None:
        csrc = os.path.join(HERE, "..", "..", "kitex_amd", "csrc")
        srcs = [os.path.join(csrc, f) for f in ("kx_decode.hip", "kx_crc.hip", "kx_nested.h", "kx_nested_schema.cpp",
                                                "kx_schema.cpp", "kx_internal.h", "kx_knobs.cpp",
                                                "kx_knobs.h")] + \
            [os.path.join(HERE, f) for f in ("emu_driver.cpp", "emu_rt.cpp", "nested_host.cpp",
                                             os.path.join("hip", "hip_runtime.h"))]
        import fcntl
        os.makedirs(os.path.join(HERE, OUT), exist_ok=True)
        # one build at a time (pytest -n workers share the build directory); the check is repeated under the lock
        with open(os.path.join(HERE, OUT, ".lock"), "w") as lk:
            fcntl.flock(lk, fcntl.LOCK_EX)
            if not os.path.exists(LIB) or os.path.getmtime(LIB) < max(os.path.getmtime(f) for f in srcs):
                build()
        _lib = C.CDLL(LIB)
        _lib.emu_decode.restype = C.c_int
        _lib.emu_decode.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64,
                                    C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]
        _lib.emu_nested_decode.restype = C.c_int
        _lib.emu_nested_decode.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64,
                                           C.c_void_p, C.c_void_p, C.c_void_p]
        _lib.emu_nested_encode.restype = C.c_int
        _lib.emu_nested_encode.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64,
                                           C.c_void_p, C.c_void_p]
        _lib.emu_split.restype = C.c_int
        _lib.emu_split.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint64, C.c_uint64, C.c_uint32,
                                   C.c_void_p, C.c_void_p, C.c_int]
        _lib.emu_crc.restype = C.c_int
        _lib.emu_crc.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64, C.c_int, C.c_void_p, C.c_void_p,
                                 C.c_void_p]
        _lib.emu_pb_frames.restype = C.c_int
        _lib.emu_pb_frames.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64] + [C.c_void_p] * 4
        _lib.emu_frames.restype = C.c_int
        _lib.emu_frames.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.c_uint64] + [C.c_void_p] * 5 + [C.c_int,
                                                                                                  C.c_void_p]
        _lib.emu_tts_frames.restype = C.c_int
        _lib.emu_tts_frames.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.POINTER(A.TTStreamKeys)] + \
            [C.c_void_p] * 8
    return _lib


def tts_frames(data: np.ndarray, n: int, keys, threads: int = 8):
    """the ttstream frame scan of the kernel source: rc, fo, ps, pe, frame types, stream ids, method pos, len, st"""
    os.environ["KX_EMU_THREADS"] = str(threads)
    fo = np.zeros(n + 1, dtype=np.uint64)
    ps = np.zeros(max(1, n), dtype=np.uint64)
    pe = np.zeros(max(1, n), dtype=np.uint64)
    ft = np.zeros(max(1, n), dtype=np.uint8)
    sd = np.zeros(max(1, n), dtype=np.int32)
    mp = np.zeros(max(1, n), dtype=np.uint64)
    ml = np.zeros(max(1, n), dtype=np.uint32)
    st = A.Status()
    rc = lib().emu_tts_frames(data.ctypes.data, data.size, n, C.byref(keys), fo.ctypes.data, ps.ctypes.data,
                              pe.ctypes.data, ft.ctypes.data, sd.ctypes.data, mp.ctypes.data, ml.ctypes.data,
                              C.addressof(st))
    return rc, fo, ps[:n], pe[:n], ft[:n], sd[:n], mp[:n], ml[:n], st


def decode(schema, infos, npres, data: np.ndarray, n: int, offsets=None, var_caps=None, threads: int = 8,
           pb: bool = False, views: bool = False, wide: bool = False):
    os.environ["KX_EMU_THREADS"] = str(threads)
    if var_caps is None:
        var_caps = [0 if ci.kind == A.COL_FIXED else max(1, data.size) for ci in infos]
    out = alloc_host(infos, n, var_caps, npres, views=views, wide=wide)
    kc = to_kx_columns(out, infos, var_caps)
    st = A.Status()
    rs = np.zeros(max(1, n), dtype=np.uint8)
    tab, ns = schema.struct_table()
    rc = lib().emu_decode(C.cast(tab, C.c_void_p), ns, data.ctypes.data, data.size,
                          offsets.ctypes.data if offsets is not None else None, n, C.addressof(kc),
                          rs.ctypes.data, C.addressof(st), 2 if pb else 0, None)
    return rc, out, st, rs[:n]


def skip(data: np.ndarray, n: int, threads: int = 8):
    os.environ["KX_EMU_THREADS"] = str(threads)
    offs = np.zeros(n + 1, dtype=np.uint64)
    st = A.Status()
    rc = lib().emu_decode(None, 0, data.ctypes.data, data.size, None, n, None, None, C.addressof(st), 1,
                          offs.ctypes.data)
    return rc, offs, st


def split_points(schema, data: np.ndarray, n: int, parts: int, threads: int = 8):
    """kx_launch_split under the emulator: rc, points (parts + 1), status; schema None: the skip walker"""
    os.environ["KX_EMU_THREADS"] = str(threads)
    pts = np.full(parts + 1, 0xDEAD, dtype=np.uint64)
    st = A.Status()
    tab, ns = schema.struct_table() if schema is not None else (None, 0)
    rc = lib().emu_split(C.cast(tab, C.c_void_p) if tab is not None else None, ns, data.ctypes.data, data.size, n,
                         parts, pts.ctypes.data, C.addressof(st), 1 if schema is None else 0)
    return rc, pts, st


def pb_frames(data: np.ndarray, n: int, threads: int = 8):
    """the Kitex-PB Batch frame pass of the kernel source: rc, frame offsets (n + 1), body starts, body ends,
    status"""
    os.environ["KX_EMU_THREADS"] = str(threads)
    fo = np.zeros(n + 1, dtype=np.uint64)
    bs = np.zeros(max(1, n), dtype=np.uint64)
    be = np.zeros(max(1, n), dtype=np.uint64)
    st = A.Status()
    rc = lib().emu_pb_frames(data.ctypes.data, data.size, n, fo.ctypes.data, bs.ctypes.data, be.ctypes.data,
                             C.addressof(st))
    return rc, fo, bs[:n], be[:n], st


def frames(data: np.ndarray, n: int, max_payload: int = 0, threads: int = 8, grpc: bool = False, crc: bool = False):
    """the frame scan of the kernel source; crc=True also returns the fused CRC32Check codes per frame"""
    os.environ["KX_EMU_THREADS"] = str(threads)
    fo = np.zeros(n + 1, dtype=np.uint64)
    ps = np.zeros(max(1, n), dtype=np.uint64)
    pe = np.zeros(max(1, n), dtype=np.uint64)
    kd = np.zeros(max(1, n), dtype=np.uint8)
    cc = np.full(max(1, n), 0xEE, dtype=np.uint8)
    st = A.Status()
    rc = lib().emu_frames(data.ctypes.data, data.size, n, max_payload, fo.ctypes.data, ps.ctypes.data,
                          pe.ctypes.data, kd.ctypes.data, C.addressof(st), 1 if grpc else 0,
                          cc.ctypes.data if crc else None)
    if crc:
        return rc, fo, ps[:n], pe[:n], kd[:n], st, cc[:n]
    return rc, fo, ps[:n], pe[:n], kd[:n], st


def crc32c(data: np.ndarray, offs: np.ndarray, n: int, val: bool, threads: int = 8):
    """the CRC32C kernel source: crc per range (val=False) or per TTHeader frame (val=True), codes, status"""
    os.environ["KX_EMU_THREADS"] = str(threads)
    crc = np.zeros(max(1, n), dtype=np.uint32)
    rs = np.zeros(max(1, n), dtype=np.uint8)
    st = A.Status()
    o = np.ascontiguousarray(offs, dtype=np.uint64)
    rc = lib().emu_crc(data.ctypes.data if data.size else None, data.size, o.ctypes.data, n, 1 if val else 0,
                       crc.ctypes.data, rs.ctypes.data, C.addressof(st))
    assert rc == 0, rc
    return crc[:n], rs[:n], st


def nested_decode(schema, infos, npres, data: np.ndarray, n: int, offsets=None, var_caps=None, elem_caps=None,
                  sub_caps=None, wide: bool = False):
    """the nested walker of the kernel source on the host: rc, columns, status, record codes"""
    if var_caps is None:
        var_caps = [0 if ci.kind == A.COL_FIXED else max(1, data.size) for ci in infos]
    out = alloc_host(infos, n, var_caps, npres, wide=wide, elem_caps=elem_caps, sub_caps=sub_caps)
    kc = to_kx_columns(out, infos, var_caps)
    st = A.Status()
    rs = np.zeros(max(1, n), dtype=np.uint8)
    tab, ns = schema.struct_table()
    offs = None if offsets is None else np.ascontiguousarray(offsets, dtype=np.uint64)
    rc = lib().emu_nested_decode(C.cast(tab, C.c_void_p), ns, data.ctypes.data if data.size else None, data.size,
                                 None if offs is None else offs.ctypes.data, n, C.addressof(kc), rs.ctypes.data,
                                 C.addressof(st))
    return rc, out, st, rs[:n]


def nested_encode(schema, infos, cs):
    """rc, wire bytes, record offsets of the kernel source's nested encoder on the host"""
    kc = to_kx_columns(cs, infos)
    tab, ns = schema.struct_table()
    total = C.c_uint64()
    offs = np.zeros(cs.n + 1, dtype=np.uint64)
    rc = lib().emu_nested_encode(C.cast(tab, C.c_void_p), ns, C.addressof(kc), cs.n, None, 0, None, C.byref(total))
    if rc and rc != A.ERR_SIZE_LIMIT:
        return rc, None, None
    out = np.zeros(max(1, total.value), dtype=np.uint8)
    rc = lib().emu_nested_encode(C.cast(tab, C.c_void_p), ns, C.addressof(kc), cs.n, out.ctypes.data, total.value,
                                 offs.ctypes.data, C.byref(total))
    return rc, out[:total.value], offs
