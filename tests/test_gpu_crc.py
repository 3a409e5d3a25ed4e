"""GPU parity of the CRC32C payload validator (kx_crc32c_batch, kx_frame_crc32c_validate, CRC32Check in
kx_thrift_decode_frames) against the oracle's bitwise restatement of crcPayloadValidator
(validate.go:168-217), through the C-ABI."""
import numpy as np
import pytest

from tests import crc_cases as CC
from tests import frame_cases as FC
from tests.helpers import assert_rows_equal, to_np

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as t
    if not t.cuda.is_available():
        pytest.skip("no GPU")
    return t


def _u32(t):
    return to_np(t).astype(np.uint64).astype(np.uint32)


@pytest.mark.parametrize("seed,n,big,maxlen", [(1, 1, False, 600), (2, 257, False, 600), (3, 3000, True, 600),
                                                (4, 40000, False, 600), (5, 40000, False, 180), (6, 9000, True, 120)])
def test_generate_matches_oracle(torch, oracle, seed, n, big, maxlen):
    from kitex_amd.codec import CRC32PayloadValidator
    data, offs = CC.ragged_ranges(seed, n, big, maxlen)
    rc, exp = oracle.crc32c_batch(data, offs)
    assert rc == 0
    v = CRC32PayloadValidator()
    got = v.Generate(torch.from_numpy(data).to("cuda:0"), torch.from_numpy(offs.astype(np.int64)).to("cuda:0"))
    assert np.array_equal(_u32(got), exp)


def test_generate_known_answers(torch):
    from kitex_amd.codec import CRC32PayloadValidator
    blobs = [d for d, _ in CC.KNOWN]
    data = np.frombuffer(b"".join(blobs), dtype=np.uint8).copy()
    offs = np.zeros(len(blobs) + 1, dtype=np.int64)
    offs[1:] = np.cumsum([len(b) for b in blobs])
    got = CRC32PayloadValidator().Generate(torch.from_numpy(data).to("cuda:0"), torch.from_numpy(offs).to("cuda:0"))
    assert list(_u32(got)) == [w for _, w in CC.KNOWN]


def test_generate_one_large_range(torch, oracle):
    """one 24 MiB payload at an unaligned start: the wave-cooperative path with many 256 KiB stretches"""
    from kitex_amd.codec import CRC32PayloadValidator
    rng = np.random.default_rng(9)
    data = rng.integers(0, 256, size=24 * 1024 * 1024 + 77, dtype=np.uint8)
    offs = np.array([5, 5, 24 * 1024 * 1024 + 70, 24 * 1024 * 1024 + 77], dtype=np.int64)
    _, exp = oracle.crc32c_batch(data, offs.astype(np.uint64))
    got = CRC32PayloadValidator().Generate(torch.from_numpy(data).to("cuda:0"), torch.from_numpy(offs).to("cuda:0"))
    assert np.array_equal(_u32(got), exp)


def test_generate_range_outside_input(torch):
    from kitex_amd._lib import KxError
    from kitex_amd.codec import CRC32PayloadValidator
    data = torch.zeros(10, dtype=torch.uint8, device="cuda:0")
    with pytest.raises(KxError) as e:
        CRC32PayloadValidator().Generate(data, torch.tensor([0, 4, 20], dtype=torch.int64, device="cuda:0"))
    assert e.value.code == 100 and e.value.record == 1


@pytest.mark.parametrize("n", [1, 8, 5000])
def test_validate_frames_matches_oracle(torch, oracle, n):
    from kitex_amd.codec import CRC32PayloadValidator
    sch, recs, frames, wire, fo, exp = CC.crc_batch(n, CC.MODES_PASS + CC.MODES_FAIL)
    rc, ecrc, ers, first = oracle.frame_crc32c_validate(wire, fo, n)
    rs, crc, st = CRC32PayloadValidator().ValidateFrames(torch.from_numpy(wire).to("cuda:0"),
                                                          torch.from_numpy(fo.astype(np.int64)).to("cuda:0"), n)
    assert np.array_equal(to_np(rs), ers) and np.array_equal(ers, exp[:n])
    assert np.array_equal(_u32(crc), ecrc)
    assert st.code == rc and (rc == 0 or st.record == first)


def test_validate_reference_tamper_case(torch, oracle):
    """default_codec_test.go:269-316: a 32 KiB TTHeaderFramed payload passes; its last 9 bytes
    overwritten fail (KX_ERR_PAYLOAD_VALIDATION), exactly as the oracle says"""
    from kitex_amd.codec import CRC32PayloadValidator
    body = FC.framed(bytes((i * 7) & 0xFF for i in range(32 * 1024)))
    good = FC.ttheader(body, flags=1, str_kv=[(b"crc32c", CC.crc_hex(CC.py_crc32c(body)))])
    bad = bytearray(good)
    bad[-9:] = b"\x7b" * 9
    wire = np.frombuffer(good + bytes(bad), dtype=np.uint8).copy()
    fo = np.array([0, len(good), 2 * len(good)], dtype=np.int64)
    rs, crc, st = CRC32PayloadValidator().ValidateFrames(torch.from_numpy(wire).to("cuda:0"),
                                                          torch.from_numpy(fo).to("cuda:0"), 2)
    assert list(to_np(rs)) == [0, 11] and st.code == 11 and st.record == 1
    _, ecrc, _, _ = oracle.frame_crc32c_validate(wire, fo.astype(np.uint64), 2)
    assert np.array_equal(_u32(crc), ecrc)


@pytest.mark.parametrize("form", ["fused", "separate_no_fo"])
def test_decode_frames_with_crc32_check(torch, oracle, form, monkeypatch):
    """UnmarshalFrames(crc32_check=True): failing frames carry ERR_PAYLOAD_VALIDATION, every other
    message decodes exactly as the oracle decodes its record; without the check all decode.
    separate_no_fo: the separate checksum kernel (KX_CRC_FUSED=0) with frame_offsets NULL, so the frame
    offsets live in the library's scratch next to the CRC status (the status used to overlap
    them); the first failing frame is frame 5"""
    from kitex_amd.codec import ThriftCodec
    n = 6000
    sch, recs, frames, wire, fo, exp = CC.crc_batch(n, CC.MODES_PASS + CC.MODES_FAIL)
    assert int(np.nonzero(exp)[0][0]) < 8
    from kitex_amd._lib import lib
    from tests.helpers import knob
    cdc = ThriftCodec(sch)
    buf = torch.from_numpy(wire).to("cuda:0")
    with knob(lib(), "KX_CRC_FUSED", 0 if form == "separate_no_fo" else 1, 1):
        res = cdc.UnmarshalFrames(buf, n, raise_on_error=False, crc32_check=True,
                                  frame_offsets=form == "fused")
    st = res.read_status()
    rs = to_np(res.record_status)[:n]
    assert np.array_equal(rs, exp)
    first = int(np.nonzero(exp)[0][0])
    assert st.code == 11 and st.record == first and st.offset == fo[first]
    ok = np.nonzero(exp == 0)[0]
    wire_ok = np.frombuffer(b"".join(recs[i] for i in ok), dtype=np.uint8).copy()
    offs = np.zeros(len(ok) + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(recs[i]) for i in ok])
    rc, eout, est, _ = oracle.decode(sch, wire_ok, len(ok), offsets=offs)
    _, infos, _ = oracle.flatten(sch)
    assert_rows_equal(res.columns, eout, infos, ok)
    res2 = cdc.UnmarshalFrames(buf, n, raise_on_error=False, crc32_check=False)
    assert res2.read_status().code == 0 and (to_np(res2.record_status)[:n] == 0).all()
