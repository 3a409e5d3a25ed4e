"""CPU: the oracle's CRC32C payload validator (kxo_crc32c*, restating validate.go:168-217) pinned by the
published CRC-32C check values and by the reference's own validator tests (validate_test.go:147-178,
default_codec_test.go:269-316)."""
import numpy as np
import pytest

from tests import crc_cases as CC


@pytest.mark.parametrize("data,want", CC.KNOWN)
def test_known_answers(oracle, data, want):
    assert oracle.crc32c(data) == want
    assert CC.py_crc32c(data) == want


def test_update_continues(oracle):
    """crc32.Update(crc, tab, p) continues a running CRC: Update(Update(0, a), b) == Update(0, a + b)"""
    a, b = b"hello, ", b"kitex payload"
    assert oracle.crc32c(b, oracle.crc32c(a)) == oracle.crc32c(a + b)


def test_batch_matches_independent_restatement(oracle):
    data, offs = CC.ragged_ranges(1, 300, big=False)
    rc, crc = oracle.crc32c_batch(data, offs)
    assert rc == 0
    for i in range(300):
        assert crc[i] == CC.py_crc32c(data[int(offs[i]):int(offs[i + 1])].tobytes()), i


def test_batch_range_outside_input(oracle):
    data = np.arange(10, dtype=np.uint8)
    rc, crc = oracle.crc32c_batch(data, np.array([0, 4, 20], dtype=np.uint64))
    assert rc == 100 and crc[1] == 0 and crc[0] == CC.py_crc32c(bytes(range(4)))


def test_reference_validator_cases(oracle):
    """TestCRCPayloadValidator: Generate, Validate(value) passes, value + "0" fails, "" passes"""
    from tests import frame_cases as FC
    p = CC.ref_payload()
    val = CC.crc_hex(oracle.crc32c(p))
    for hv, code in ((val, 0), (val + b"0", 11), (b"", 0)):
        fr = FC.ttheader(p, str_kv=[(b"crc32c", hv)])
        wire = np.frombuffer(fr, dtype=np.uint8).copy()
        rc, crc, rs, first = oracle.frame_crc32c_validate(wire, np.array([0, len(fr)], dtype=np.uint64), 1)
        assert rc == code and rs[0] == code and crc[0] == oracle.crc32c(p)


def test_reference_codec_tamper_case(oracle):
    """TestDefaultCodecWithCRC32_Encode_Decode: a 32 KiB TTHeaderFramed payload validates; overwriting
    its last 9 bytes with 123 fails validation"""
    from tests import frame_cases as FC
    body = FC.framed(bytes((i * 7) & 0xFF for i in range(32 * 1024)))
    fr = bytearray(FC.ttheader(body, flags=1, str_kv=[(b"crc32c", CC.crc_hex(CC.py_crc32c(body)))]))
    fo = np.array([0, len(fr)], dtype=np.uint64)
    rc, _, _, _ = oracle.frame_crc32c_validate(np.frombuffer(bytes(fr), dtype=np.uint8).copy(), fo, 1)
    assert rc == 0
    for i in range(len(fr) - 1, len(fr) - 10, -1):
        fr[i] = 123
    rc, _, _, first = oracle.frame_crc32c_validate(np.frombuffer(bytes(fr), dtype=np.uint8).copy(), fo, 1)
    assert rc == 11 and first == 0


def test_frame_modes(oracle):
    sch, recs, frames, wire, fo, exp = CC.crc_batch(64, CC.MODES_PASS + CC.MODES_FAIL)
    rc, crc, rs, first = oracle.frame_crc32c_validate(wire, fo, 64)
    assert (rs == exp).all()
    assert first == int(np.nonzero(exp)[0][0]) and rc == 11
    # the frames are still well-formed for the framing sniff
    src, *_ = oracle.frame_scan(wire, 64)
    assert src == 0


# ---- the CRC32C kernel source under the SIMT emulator (tests/emu), oracle-checked ----
@pytest.mark.parametrize("seed,n,big,maxlen", [(1, 1, False, 600), (2, 300, False, 600), (5, 700, True, 600),
                                                (6, 700, False, 180), (7, 1000, True, 120)])
def test_emu_generate(oracle, seed, n, big, maxlen):
    from tests.emu import emu
    data, offs = CC.ragged_ranges(seed, n, big, maxlen)
    rc, exp = oracle.crc32c_batch(data, offs)
    crc, _, st = emu.crc32c(data, offs, n, False)
    assert rc == 0 and st.code == 0 and st.n_records == n and st.consumed == offs[n]
    assert np.array_equal(crc, exp)


def test_emu_validate_frames(oracle):
    from tests.emu import emu
    n = 200
    sch, recs, frames, wire, fo, exp = CC.crc_batch(n, CC.MODES_PASS + CC.MODES_FAIL)
    rc, ecrc, ers, first = oracle.frame_crc32c_validate(wire, fo, n)
    crc, rs, st = emu.crc32c(wire, fo, n, True)
    assert np.array_equal(rs, ers) and np.array_equal(crc, ecrc)
    assert st.code == rc == 11 and st.record == first


@pytest.mark.parametrize("n", [1, 200, 3000])
def test_emu_fused_frame_check(oracle, n):
    """CRC32Check fused into the frame scan's emit pass (kx_decode.hip frame_crc_check): the per-frame codes
    equal the oracle's validator and the checksum kernel's"""
    from tests.emu import emu
    sch, recs, frames, wire, fo, exp = CC.crc_batch(n, CC.MODES_PASS + CC.MODES_FAIL)
    rc, ecrc, ers, first = oracle.frame_crc32c_validate(wire, fo, n)
    src, sfo, ps, pe, kd, st, codes = emu.frames(wire, n, crc=True)
    assert src == 0 and st.code == 0 and np.array_equal(sfo[:n + 1], fo[:n + 1])
    assert np.array_equal(codes, ers)
