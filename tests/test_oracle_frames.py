"""The oracle's framing sniff (kxo_frame_scan) against the reference's sniff matrix
(default_codec_test.go:58-199) and hand-built TTHeader / Mesh / Framed / PurePayload frames."""
import numpy as np
import pytest

from kitex_amd import _abi as A
from tests import frame_cases as FC


@pytest.mark.parametrize("name", list(FC.sniff_matrix_frames()))
def test_sniff_matrix(oracle, name):
    frame, kind = FC.sniff_matrix_frames()[name]
    w = np.frombuffer(frame, dtype=np.uint8).copy()
    rc, fo, ps, pe, kd, done = oracle.frame_scan(w, 1)
    assert rc == 0 and done == 1 and int(fo[1]) == len(frame)
    assert kd[0] == kind
    framed = kind & (A.TRANS_FRAMED)
    if framed:   # PayloadLen 10: passes a 10-byte limit, fails a 9-byte one (checkPayloadSize)
        assert int(pe[0] - ps[0]) == 10
        assert oracle.frame_scan(w, 1, 10)[0] == 0
        assert oracle.frame_scan(w, 1, 9)[0] == A.ERR_INVALID_DATA
    elif kind == A.TRANS_PURE:   # PurePayload: the length is unknown when the limit is checked
        assert oracle.frame_scan(w, 1, 1)[0] == 0
    # the payload the payload codec sees starts with the MessageBegin / Kitex-PB magic
    assert w[int(ps[0])] in (0x80, 0x90)


def test_not_a_frame(oracle):
    """checkPayload's last branch (default_codec.go:411-416): the telnet interrupt 0xfff4fffd"""
    w = np.frombuffer(FC.be32(0xFFF4FFFD) + FC.be32(0) + bytes(8), dtype=np.uint8).copy()
    assert oracle.frame_scan(w, 1)[0] == A.ERR_UNKNOWN_PROTOCOL
    assert oracle.frame_scan(w[:7].copy(), 1)[0] == A.ERR_EOF   # Peek(8) fails


def test_ttheader_header_checks(oracle):
    good = FC.ttheader(FC.thrift_message(b"m", 1, b"\x00"))
    for mut, code in [((12, 0), A.ERR_UNKNOWN_PROTOCOL),     # header size 0 words
                      ((14, 9), A.ERR_UNKNOWN_PROTOCOL)]:    # protocol id 9 (checkProtocolID)
        b = bytearray(good)
        b[mut[0]], b[mut[0] + 1] = (0, 0) if mut[0] == 12 else (mut[1], b[mut[0] + 1])
        rc = oracle.frame_scan(np.frombuffer(bytes(b), dtype=np.uint8).copy(), 1)[0]
        assert rc == code
    # LENGTH shorter than the header: negative payload length
    b = bytearray(good)
    b[0:4] = FC.be32(8)
    assert oracle.frame_scan(np.frombuffer(bytes(b), dtype=np.uint8).copy(), 1)[0] == A.ERR_UNKNOWN_PROTOCOL


@pytest.mark.parametrize("case", FC.SCAN_CASES)
def test_oracle_scan_cases(oracle, case):
    """the shared cases with the oracle as both sides: exercises the builders and expectations"""
    def scan(wire, n, mx):
        rc, fo, ps, pe, kd, done = oracle.frame_scan(wire, n, mx)
        st = A.Status()
        st.code, st.n_records = rc, done
        if rc:
            st.record, st.offset = done, int(fo[done])
        return fo, ps, pe, kd, st
    FC.case_scan(scan, oracle, case, n=300)
