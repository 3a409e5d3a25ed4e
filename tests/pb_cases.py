"""Kitex-Protobuf decode parity cases, shared by the GPU suite
(tests/test_gpu_pb.py, libkxcodec through the C-ABI) and the CPU emulation suite
(tests/test_emu_decode.py, the same kernel source under the SIMT emulator).

Concatenated mode = the Batch framing the oracle restates (`0x0A`, uvarint(len), body per record);
offsets mode = bare proto3 bodies with known [offsets[r], offsets[r+1]) extents, i.e. the
`proto.Unmarshal(payload)` each message gets in protobuf.go:135-170. Every case is compared with the
oracle bit-exact: columns, error code, failing record and byte offset.
"""
import numpy as np

from kitex_amd import _abi as A
from kitex_amd import schema as S
from kitex_amd import synth
from tests.helpers import assert_columns_equal, to_np


def uvarint(v: int) -> bytes:
    v &= (1 << 64) - 1
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def tag(num: int, wt: int) -> bytes:
    return uvarint((num << 3) | wt)


def f_varint(num, v):
    return tag(num, 0) + uvarint(v)


def f_bytes(num, b: bytes):
    return tag(num, 2) + uvarint(len(b)) + b


def f_fixed64(num, v):
    return tag(num, 1) + int(v & ((1 << 64) - 1)).to_bytes(8, "little")


def f_fixed32(num, v):
    return tag(num, 5) + int(v & 0xFFFFFFFF).to_bytes(4, "little")


def frame(body: bytes) -> bytes:
    return b"\x0a" + uvarint(len(body)) + body


def split_frames(wire: np.ndarray):
    """framed batch -> list of bodies"""
    b = wire.tobytes()
    pos, out = 0, []
    while pos < len(b):
        assert b[pos] == 0x0A
        pos += 1
        ln, sh = 0, 0
        while True:
            c = b[pos]
            pos += 1
            ln |= (c & 0x7F) << sh
            sh += 7
            if c < 0x80:
                break
        out.append(b[pos:pos + ln])
        pos += ln
    return out


def join(parts, framed):
    recs = [frame(p) for p in parts] if framed else list(parts)
    wire = np.frombuffer(b"".join(recs), dtype=np.uint8).copy()
    offs = np.zeros(len(recs) + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(r) for r in recs])
    return wire, offs


def check_pb(dec, oracle, sch, wire, n, offsets=None):
    rc, exp, est, ers = oracle.decode(sch, wire, n, offsets=offsets, pb=True)
    cols, st, rs = dec.decode(sch, wire, n, offsets, pb=True)
    assert st.code == est.code, (st.code, est.code)
    if est.code:
        assert (st.record, st.offset) == (est.record, est.offset), ((st.record, st.offset), (est.record, est.offset))
    assert st.n_records == est.n_records
    if offsets is None:
        assert st.consumed == est.consumed
    else:
        assert np.array_equal(to_np(rs)[:n], ers[:n])
    _, infos, _ = oracle.flatten(sch)
    ok_rows = est.n_records if offsets is None else n
    assert_columns_equal(cols, exp, infos, ok_rows)
    for k in range(min(8, sum(ci.kind != A.COL_FIXED for ci in infos))):
        assert st.var_total[k] == est.var_total[k]
    return cols, st


def case_pb_concat(dec, oracle, n):
    sch = S.schema_pf()
    cs = synth.gen_pf(n)
    rc, wire, _ = oracle.encode(sch, cs, pb=True)
    assert rc == 0
    cols, st = check_pb(dec, oracle, sch, wire, n)
    assert st.code == 0 and st.consumed == wire.size


def case_pb_offsets(dec, oracle, n):
    sch = S.schema_pf()
    cs = synth.gen_pf(n, start=999)
    rc, wire, _ = oracle.encode(sch, cs, pb=True)
    bodies = split_frames(wire)
    w2, offs = join(bodies, framed=False)
    check_pb(dec, oracle, sch, w2, n, offsets=offs)


def _pf_body(rng, order=None, extra=(), dup=False, strs=(b"hello", b"world")):
    fs = []
    for f in range(1, 9):
        v = int(rng.integers(-2**63, 2**63 - 1))
        if f % 3 == 0:
            v = int(rng.integers(0, 300))
        if v:
            fs.append(f_varint(f, v))
    fs.append(f_bytes(9, strs[0]))
    fs.append(f_bytes(10, strs[1]))
    if order is not None:
        fs = [fs[k] for k in order if k < len(fs)]
    fs = fs[:2] + list(extra) + fs[2:]
    if dup:
        fs.append(f_varint(2, 77))
        fs.append(f_bytes(9, b"last"))
    return b"".join(fs)


def mixed_bodies(count=3000, seed=5):
    """unknown fields of every wire type, known ids with the wrong wire type (skipped), repeated
    fields (last wins), overlong varints, zero-valued fields present, multi-byte UTF-8, empty bodies"""
    rng = np.random.default_rng(seed)
    unknown = [f_varint(100, 5), f_fixed64(101, -1), f_fixed32(102, 7), f_bytes(103, b"\xff\x00raw"),
               tag(3, 2) + uvarint(2) + b"ab",          # field 3 (int64) sent as bytes: skipped
               f_fixed64(4, 123)]                         # field 4 sent as fixed64: skipped
    out = []
    for i in range(count):
        k = i % 9
        if k == 1:
            out.append(_pf_body(rng, order=list(rng.permutation(10))))
        elif k == 2:
            out.append(_pf_body(rng, extra=unknown))
        elif k == 3:
            out.append(_pf_body(rng, dup=True))
        elif k == 4:
            out.append(f_varint(1, 0) + b"\x88\x80\x80\x00" + b"\x01" + f_bytes(9, "héllo wörld €𝄞".encode()))
        elif k == 5:
            out.append(b"")
        elif k == 6:
            s = bytes(rng.integers(97, 123, size=int(rng.integers(0, 300)), dtype=np.uint8))
            out.append(_pf_body(rng, strs=(s, b"")))
        else:
            out.append(_pf_body(rng))
    return out


def case_pb_noncanonical(dec, oracle, mode):
    sch = S.schema_pf()
    bodies = mixed_bodies()
    framed = mode == "concat"
    wire, offs = join(bodies, framed)
    check_pb(dec, oracle, sch, wire, len(bodies), offsets=None if framed else offs)


PB_ERRORS = ["truncated_varint", "varint_10th", "group_wt", "field_zero", "len_overflow", "bad_utf8",
             "bad_frame", "truncated_input", "short_input"]


def case_pb_error(dec, oracle, case, mode):
    sch = S.schema_pf()
    rng = np.random.default_rng(6)
    bodies = [_pf_body(rng) for _ in range(900)]
    n = len(bodies)
    framed = mode == "concat"
    bad = {
        "truncated_varint": f_varint(1, 5) + tag(2, 0) + b"\xff\xff",
        "varint_10th": f_varint(1, 5) + tag(2, 0) + b"\xff" * 9 + b"\x02",
        "group_wt": f_varint(1, 5) + tag(50, 3),
        "field_zero": f_varint(1, 5) + b"\x00\x01",
        "len_overflow": f_varint(1, 5) + tag(9, 2) + uvarint(1000) + b"abc",
        "bad_utf8": f_bytes(10, b"ok\xc3\x28"),
    }
    if case in bad:
        bodies[401] = bad[case]
        wire, offs = join(bodies, framed)
    elif case == "bad_frame":
        if not framed:
            return
        wire, offs = join(bodies, framed)
        wire[int(offs[300])] = 0x12                  # record 300's frame is not field 1 / LEN
    elif case == "truncated_input":
        wire, offs = join(bodies, framed)
        wire = wire[:-9]
        offs[-1] = wire.size
    else:
        if not framed:
            return
        wire, offs = join(bodies, framed)
        n += 3
    check_pb(dec, oracle, sch, wire, n, offsets=None if framed else offs)
