"""ttstream (TTHeader streaming) frames for the oracle / emulator / GPU tests (test infrastructure).

A frame = TTHeader (gopkg protocol/ttheader layout, as restated in oracle/kx_oracle.c) with protocol id
ThriftStruct (0x10), the streaming flag, IntInfo {FrameType, ToMethod} (+ extra keys), optional string
KV info (META / HEADER / TRAILER frames carry headers, ttstream frame.go:108-114), padding to 4 bytes,
then the payload (a bare FastMarshal struct for DATA frames, frame.go:192-205)."""
import struct

import numpy as np

from kitex_amd import _abi as A


def default_keys():
    from kitex_amd.codec import default_ttstream_keys
    return default_ttstream_keys()


def type_name(keys, t):
    return bytes(keys.type_names[t - 1].value)


def frame(keys, sid, ftype, method=b"", payload=b"", strinfo=None, flags=None, proto=0x10, extra_int=None,
          type_value=None, ntrans=0, acl=None):
    ints = {}
    if extra_int:
        ints.update(extra_int)
    ints[keys.frame_type_key] = type_value if type_value is not None else type_name(keys, ftype)
    if method is not None:
        ints[keys.to_method_key] = method
    h = bytes([proto, ntrans]) + bytes(range(1, ntrans + 1))
    h += b"\x10" + struct.pack(">H", len(ints)) + b"".join(struct.pack(">HH", k, len(v)) + v for k, v in ints.items())
    if strinfo:
        h += b"\x01" + struct.pack(">H", len(strinfo)) + b"".join(
            struct.pack(">H", len(k)) + k + struct.pack(">H", len(v)) + v for k, v in strinfo.items())
    if acl is not None:
        h += b"\x11" + struct.pack(">H", len(acl)) + acl
    h += b"\x00" * (-len(h) % 4)
    fl = keys.streaming_flag if flags is None else flags
    body = struct.pack(">HHIH", 0x1000, fl, sid & 0xFFFFFFFF, len(h) // 4) + h + payload
    return struct.pack(">I", len(body)) + body


def stream_batch(oracle, sch, cs, keys, streams=3, seed=0):
    """n records sent as DATA frames over `streams` interleaved streams, each stream opened by META +
    HEADER frames and closed by a TRAILER frame. Returns (wire uint8, frames: list of (type, sid, method,
    payload start, payload end), record order of the DATA frames)."""
    rng = np.random.default_rng(seed)
    rc, wire, offs = oracle.encode(sch, cs)
    assert rc == 0
    recs = [bytes(wire[int(offs[i]):int(offs[i + 1])]) for i in range(cs.n)]
    out, info, pos = [], [], 0

    def put(fb, t, sid, m, plen):
        nonlocal pos
        out.append(fb)
        ps = pos + len(fb) - plen
        info.append((t, sid, m, ps, pos + len(fb)))
        pos += len(fb)
    for s in range(streams):
        m = b"Method%d" % s
        put(frame(keys, 100 + s, A.TTS_META, m, strinfo={b"k": b"v%d" % s}), A.TTS_META, 100 + s, m, 0)
        put(frame(keys, 100 + s, A.TTS_HEADER, m, strinfo={b"h": b"x"}, extra_int={1: b"val1"}), A.TTS_HEADER,
            100 + s, m, 0)
    for i, r in enumerate(recs):
        s = int(rng.integers(0, streams))
        m = b"Method%d" % s
        put(frame(keys, 100 + s, A.TTS_DATA, m, payload=r), A.TTS_DATA, 100 + s, m, len(r))
    for s in range(streams):
        m = b"Method%d" % s
        put(frame(keys, 100 + s, A.TTS_TRAILER, m, strinfo={b"biz-status": b"0"}), A.TTS_TRAILER, 100 + s, m, 0)
    return np.frombuffer(b"".join(out), dtype=np.uint8).copy(), info


ERROR_CASES = ["no_stream_flag", "bad_type", "bad_magic", "truncated", "bad_info"]


def error_batch(oracle, keys, case, n_good=50):
    """n_good valid DATA frames, then one bad frame, then more; (wire, index of the bad frame, code)"""
    from kitex_amd import schema as S, synth
    sch = S.schema_r1()
    rc, wire, offs = oracle.encode(sch, synth.gen_r1(n_good * 2))
    recs = [bytes(wire[int(offs[i]):int(offs[i + 1])]) for i in range(n_good * 2)]
    good = [frame(keys, 7, A.TTS_DATA, b"m", payload=r) for r in recs]
    if case == "no_stream_flag":
        bad, code = frame(keys, 7, A.TTS_DATA, b"m", payload=recs[0], flags=0), A.ERR_INVALID_DATA
    elif case == "bad_type":
        bad, code = frame(keys, 7, A.TTS_DATA, b"m", payload=recs[0], type_value=b"zz"), A.ERR_INVALID_DATA
    elif case == "bad_magic":
        b = bytearray(frame(keys, 7, A.TTS_DATA, b"m", payload=recs[0]))
        b[4] = 0x20
        bad, code = bytes(b), A.ERR_UNKNOWN_PROTOCOL
    elif case == "bad_info":
        b = bytearray(frame(keys, 7, A.TTS_DATA, b"m", payload=recs[0]))
        b[16] = 0x7F  # the first info id (after protocol id, transform count)
        bad, code = bytes(b), A.ERR_UNKNOWN_PROTOCOL
    else:  # truncated: the last frame of the buffer is cut short
        fb = frame(keys, 7, A.TTS_DATA, b"m", payload=recs[0])
        w = b"".join(good[:n_good]) + fb[:-3]
        return np.frombuffer(w, dtype=np.uint8).copy(), n_good, A.ERR_EOF, n_good + 1
    w = b"".join(good[:n_good]) + bad + b"".join(good[n_good:])
    return np.frombuffer(w, dtype=np.uint8).copy(), n_good, code, 2 * n_good + 1
