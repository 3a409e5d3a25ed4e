"""Binary generic ingress cases (binaryThriftCodec, pkg/generic/binarythrift_codec.go), shared by the CPU
oracle tests and the GPU suite. Test infrastructure only."""
import numpy as np

from tests import frame_cases as FC


def _empty_mockreq_body() -> bytes:
    """kt.NewMockReq() FastWrite: Msg "" (field 1), strMap {} (field 2), strList [] (field 3), STOP"""
    return (b"\x0b\x00\x01" + FC.be32(0) + b"\x0d\x00\x02\x0b\x0b" + FC.be32(0)
            + b"\x0f\x00\x03\x0b" + FC.be32(0) + b"\x00")


# TestBinaryThriftCodec (binarythrift_codec_test.go:36-105): MarshalFastMsg("mock", CALL, 100,
# MockTestArgs{Req: NewMockReq()}) -> GetSeqID == 100; SetSeqID(1) -> 1; method "mock"
REF_SEQID = [(FC.thrift_message(b"mock", 100, _empty_mockreq_body()), 100)]

# (kind, raw code, set code) cycled over the batch
_KINDS = [("ok", 0, 0), ("exception", 9, 0), ("zero_name", 1, 0), ("long_name", 1, 1), ("short3", 8, 1),
          ("short6", 1, 1), ("bad_version", 0, 4), ("positive_first", 0, 1), ("no_seqid", 0, 1), ("oneway", 0, 0)]


def _message(kind, i):
    name = b"Method%d" % (i % 13)
    body = _empty_mockreq_body()
    if kind == "ok":
        return FC.thrift_message(name, i * 7, body), name
    if kind == "oneway":
        return FC.thrift_message(name, i * 7, body, mtype=4), name
    if kind == "exception":
        return FC.thrift_message(name, i * 7, body, mtype=3), name
    if kind == "zero_name":
        return FC.be32(0x80010001) + FC.be32(0) + FC.be32(i * 7) + b"\x00", b""
    if kind == "long_name":
        return FC.be32(0x80010001) + FC.be32(50) + b"abc", b""
    if kind == "short3":
        return b"\x80\x01\x00", b""
    if kind == "short6":
        return b"\x80\x01\x00\x01\x00\x00", b""
    if kind == "bad_version":  # readBinaryMethod does not look at the version; GetSeqID does
        return FC.be32(0x80020001) + FC.be32(len(name)) + name + FC.be32(i * 7) + body, name
    if kind == "positive_first":
        return FC.be32(0x00000001) + FC.be32(len(name)) + name + FC.be32(i * 7), name
    if kind == "no_seqid":
        return FC.be32(0x80010001) + FC.be32(len(name)) + name, name
    raise ValueError(kind)


def raw_batch(n):
    msgs, names, codes = [], [], []
    for i in range(n):
        kind, rc, _ = _KINDS[i % len(_KINDS)]
        m, nm = _message(kind, i)
        msgs.append(m)
        names.append(nm if rc == 0 else b"")
        codes.append(rc)
    wire = np.frombuffer(b"".join(msgs), dtype=np.uint8).copy()
    offs = np.zeros(n + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(m) for m in msgs])
    return wire, offs, names, codes


def set_codes(n):
    return [_KINDS[i % len(_KINDS)][2] for i in range(n)]


def raw_seqids(n):
    """expected seqids from Unmarshal (0 where the message fails or has none)"""
    out = []
    for i in range(n):
        kind, rc, _ = _KINDS[i % len(_KINDS)]
        out.append(0 if rc or kind in ("no_seqid",) else i * 7)
    return out
