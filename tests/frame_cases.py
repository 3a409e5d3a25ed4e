"""Framing-sniff parity cases (kx_frame_scan / kx_*_decode_frames), shared by the CPU oracle tests,
the SIMT-emulator tests and the GPU suite. Frames are built here byte by byte from the layouts the
reference reads (default_codec.go:328-427; Mesh header header_codec.go:172-212; TTHeader meta /
info blocks of gopkg protocol/ttheader): test infrastructure only."""
import struct

import numpy as np

from kitex_amd import _abi as A
from kitex_amd import schema as S
from kitex_amd import synth


def be16(v):
    return struct.pack(">H", v)


def be32(v):
    return struct.pack(">I", v & 0xFFFFFFFF)


def thrift_message(name: bytes, seqid: int, record: bytes, mtype: int = 1, field: int = 1) -> bytes:
    """MessageBegin (strict) + Args{field: record} + STOP"""
    return (be32(0x80010000 | mtype) + be32(len(name)) + name + be32(seqid)
            + bytes([A.T_STRUCT]) + be16(field) + record + b"\x00")


def pb_message(name: bytes, seqid: int, body: bytes, mtype: int = 1) -> bytes:
    """Kitex-PB meta header (protobuf.go:77-90) + body"""
    return be32(0x90010000 | mtype) + be32(len(name)) + name + be32(seqid) + body


def framed(payload: bytes) -> bytes:
    return be32(len(payload)) + payload


def _kv_strings(kv):
    out = be16(len(kv))
    for k, v in kv:
        out += be16(len(k)) + k + be16(len(v)) + v
    return out


def ttheader(payload: bytes, seqid: int = 7, flags: int = 0, proto: int = 0, transforms=(), int_kv=(),
             str_kv=(), acl: bytes = None, pad_extra: int = 0) -> bytes:
    """LENGTH | 0x1000 | FLAGS | SEQID | HEADER SIZE/4 | proto, #transforms, ids, info blocks, padding"""
    info = bytes([proto, len(transforms)]) + bytes(transforms)
    if int_kv:
        info += b"\x10" + be16(len(int_kv)) + b"".join(be16(k) + be16(len(v)) + v for k, v in int_kv)
    if str_kv:
        info += b"\x01" + _kv_strings(str_kv)
    if acl is not None:
        info += b"\x11" + be16(len(acl)) + acl
    info += b"\x00" * ((-len(info)) % 4 + 4 * pad_extra)
    meta = be16(0x1000) + be16(flags) + be32(seqid) + be16(len(info) // 4)
    return be32(len(meta) + len(info) + len(payload)) + meta + info + payload


def mesh(payload: bytes, kv=()) -> bytes:
    hdr = _kv_strings(kv)
    return be16(0xFFAF) + be16(len(hdr)) + hdr + payload


def records(n, start=0):
    """n R2 record bodies (oracle-encoded)"""
    from oracle import oracle as o
    sch = S.schema_r2()
    rc, wire, offs = o.encode(sch, synth.gen_r2(n, start=start))
    assert rc == 0
    return sch, [bytes(wire[int(offs[i]):int(offs[i + 1])]) for i in range(n)]


KINDS = ["framed", "ttheader", "ttheader_framed", "pure", "mesh", "mesh_framed", "pb_framed", "ttheader_pb"]


def make_frame(kind, i, rec):
    name = b"Method%d" % (i % 7)
    if kind in ("pb_framed", "ttheader_pb"):
        m = pb_message(name, i, rec)
        return framed(m) if kind == "pb_framed" else ttheader(framed(m), seqid=i, proto=4)
    m = thrift_message(name, i, rec)
    if kind == "framed":
        return framed(m)
    if kind == "pure":
        return m
    if kind == "ttheader":
        kv = [(b"k%d" % j, b"v" * (i % 5)) for j in range(i % 3)]
        return ttheader(m, seqid=i, int_kv=[(1, b"svc"), (2, b"x" * (i % 4))], str_kv=kv,
                        acl=b"tok" if i % 2 else None, transforms=[1] if i % 3 == 0 else ())
    if kind == "ttheader_framed":
        return ttheader(framed(m), seqid=i, flags=1)
    if kind == "mesh":
        return mesh(m, kv=[(b"from", b"svc%d" % i)])
    if kind == "mesh_framed":
        return mesh(framed(m))
    raise ValueError(kind)


def expected_kind(kind):
    return {"framed": 4, "ttheader": 2, "ttheader_framed": 6, "pure": 0, "mesh": 0x20, "mesh_framed": 0x24,
            "pb_framed": 0x14, "ttheader_pb": 0x16}[kind]


def batch(kinds, n, start=0, pb_body=None):
    """n frames cycling over `kinds`, R2 records as the Args payload (Thrift) or a PF body (PB)"""
    sch, recs = records(n, start)
    frames = [make_frame(kinds[i % len(kinds)], i, recs[i]) for i in range(n)]
    wire = np.frombuffer(b"".join(frames), dtype=np.uint8).copy()
    fo = np.zeros(n + 1, dtype=np.uint64)
    fo[1:] = np.cumsum([len(f) for f in frames])
    return sch, recs, frames, wire, fo


def check_scan(scan, oracle, wire, n, max_payload=0):
    """scan(wire, n, max_payload) -> (fo, ps, pe, kinds, status) compared with the oracle"""
    rc, efo, eps, epe, ekd, done = oracle.frame_scan(wire, n, max_payload)
    fo, ps, pe, kd, st = scan(wire, n, max_payload)
    assert st.code == rc, (st.code, rc)
    assert st.n_records == done, (st.n_records, done)
    k = done
    assert np.array_equal(np.asarray(fo[:k + (0 if rc else 1)], dtype=np.uint64), efo[:k + (0 if rc else 1)])
    assert np.array_equal(np.asarray(ps[:k], dtype=np.uint64), eps[:k])
    assert np.array_equal(np.asarray(pe[:k], dtype=np.uint64), epe[:k])
    assert np.array_equal(np.asarray(kd[:k], dtype=np.uint8), ekd[:k])
    if rc:
        assert st.record == done and st.offset == int(efo[done]), (st.record, st.offset, int(efo[done]))
    return rc, done


SCAN_CASES = ["each_kind", "mixed", "many", "large_frames", "bad_magic", "truncated", "bad_tth_info",
              "max_payload", "short_count"]


def case_scan(scan, oracle, case, n=2000):
    if case == "each_kind":
        for kd in KINDS:
            sch, recs, frames, wire, fo = batch([kd], n)
            rc, done = check_scan(scan, oracle, wire, n)
            assert rc == 0 and done == n
            _, _, _, _, kinds, _ = oracle.frame_scan(wire, n)
            assert (kinds == expected_kind(kd)).all(), kd
        return
    if case in ("mixed", "many"):   # many: 25 000 frames, several groups of tiles
        n = 25000 if case == "many" else n
        sch, recs, frames, wire, fo = batch(KINDS if case == "mixed" else ["ttheader", "pure", "framed"], n)
        rc, done = check_scan(scan, oracle, wire, n)
        assert rc == 0
        return
    if case == "large_frames":   # frames longer than a tile, TTHeader padding words
        big = [ttheader(thrift_message(b"Big", i, _big_struct(i)), pad_extra=i % 9)
               for i in range(40)]
        wire = np.frombuffer(b"".join(big), dtype=np.uint8).copy()
        check_scan(scan, oracle, wire, 40)
        return
    sch, recs, frames, wire, fo = batch(["ttheader", "framed"], n)
    k = n // 2 + 3
    if case == "bad_magic":
        wire[int(fo[k]) + 4:int(fo[k]) + 6] = (0x70, 0x01)
        rc, done = check_scan(scan, oracle, wire, n)
        assert rc == A.ERR_UNKNOWN_PROTOCOL and done == k
    elif case == "truncated":
        rc, done = check_scan(scan, oracle, wire[:int(fo[k]) + 9].copy(), n)
        assert rc == A.ERR_EOF and done == k
    elif case == "bad_tth_info":
        j = k if k % 2 == 0 else k + 1      # a TTHeader frame: its first info byte -> invalid id 0x7f
        wire[int(fo[j]) + 14 + 2] = 0x7F
        rc, done = check_scan(scan, oracle, wire, n)
        assert rc == A.ERR_UNKNOWN_PROTOCOL and done == j
    elif case == "max_payload":   # frame k carries a 20 KiB payload, the limit is 1000 bytes
        frames = list(frames)
        frames[k] = framed(thrift_message(b"Big", k, _big_struct(k)))
        wire = np.frombuffer(b"".join(frames), dtype=np.uint8).copy()
        rc, done = check_scan(scan, oracle, wire, n, max_payload=1000)
        assert rc == A.ERR_INVALID_DATA and done == k
    elif case == "short_count":      # fewer frames than asked for
        rc, done = check_scan(scan, oracle, wire, n + 2)
        assert rc == A.ERR_EOF and done == n


def _big_struct(i):
    """an R2-shaped record with one 20 KiB string (field 9)"""
    s = bytes([97 + (i % 26)]) * 20000
    out = b""
    for f in range(1, 9):
        out += bytes([A.T_I64]) + be16(f) + struct.pack(">q", i * 1000 + f)
    out += bytes([A.T_STRING]) + be16(9) + be32(len(s)) + s + bytes([A.T_STRING]) + be16(10) + be32(3) + b"abc"
    return out + b"\x00"


def sniff_matrix_frames():
    """The reference's framing-sniff matrix (default_codec_test.go:58-199), restated as whole frames:
    each case's first 8 payload bytes and its length 10, decoded with size limits 10 and 9
    (PayloadLen 10 passes a 10-byte limit and fails a 9-byte one, :123-126, :141-144, :191-194)."""
    ten = bytes(range(10))
    tv1 = be32(0x80010000)
    pb1 = be32(0x90010000)
    return {
        # 1. TTHeader + unframed thrift (:73-91); the payload is a complete message so it delimits
        "ttheader": (ttheader(thrift_message(b"m", 1, b"\x00")), 2),
        # 2. TTHeader + framed thrift (:93-111)
        "ttheader_framed": (ttheader(be32(10) + tv1 + ten[:6]), 6),
        # 3. thrift Framed, payload length 10 (:113-129)
        "framed": (be32(10) + tv1 + ten[:6], 4),
        # 4. thrift PurePayload (:131-147)
        "pure": (thrift_message(b"m", 1, b"\x00"), 0),
        # protobuf 1. TTHeader framed (:162-178), 2. Framed (:182-196)
        "pb_ttheader_framed": (ttheader(be32(10) + pb1 + ten[:6], proto=4), 0x16),
        "pb_framed": (be32(10) + pb1 + ten[:6], 0x14),
    }


# ---- gRPC length-prefixed messages (decodeGRPCFrame, grpc_compress.go:37-60) ----
def grpc_message(payload: bytes, flag: int = 0) -> bytes:
    return bytes([flag]) + be32(len(payload)) + payload


def grpc_batch(n, pb=False, start=0, compressed=(), sizes=None):
    """n gRPC messages whose payloads are R2 record bodies (Thrift) or PF bodies (pb); message indices in
    `compressed` carry flag 1; sizes (optional) replaces record i by a string-heavy record of that size"""
    if pb:
        from oracle import oracle as o
        from tests import pb_cases as PC
        sch = S.schema_pf()
        rc, w, _ = o.encode(sch, synth.gen_pf(n, start=start), pb=True)
        assert rc == 0
        recs = [bytes(b) for b in PC.split_frames(w)]
    else:
        sch, recs = records(n, start)
    msgs = [grpc_message(recs[i], 1 if i in compressed else (2 if i % 97 == 5 else 0)) for i in range(n)]
    wire = np.frombuffer(b"".join(msgs), dtype=np.uint8).copy()
    fo = np.zeros(n + 1, dtype=np.uint64)
    fo[1:] = np.cumsum([len(m) for m in msgs])
    return sch, recs, msgs, wire, fo
