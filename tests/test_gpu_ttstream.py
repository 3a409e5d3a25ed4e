"""GPU parity of the ttstream caller: a connection buffer of TTHeader streaming frames
(META / HEADER / DATA / TRAILER of several interleaved streams, ttstream frame.go:92-185) located and
classified on the device (kx_ttstream_frame_scan) and the DATA payloads decoded as bare FastRead bodies
(kx_*_decode_extents, DecodePayload frame.go:223-233), against the oracle."""
import numpy as np
import pytest

from kitex_amd import _abi as A
from kitex_amd import schema as S
from kitex_amd import synth
from tests import tts_cases as T
from tests.helpers import assert_columns_equal, to_np

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as t
    if not t.cuda.is_available():
        pytest.skip("no GPU")
    return t


@pytest.mark.parametrize("name,n", [("r2", 20000), ("r3", 3000), ("r1", 1)])
def test_ttstream_decode_matches_oracle(torch, oracle, name, n):
    from kitex_amd.codec import ThriftCodec
    keys = T.default_keys()
    sch = S.SCHEMAS[name]()
    cs = synth.GENERATORS[name](n, start=3)
    wire, info = T.stream_batch(oracle, sch, cs, keys, streams=5, seed=n)
    nf = len(info)
    dev = torch.device("cuda", 0)
    d = torch.from_numpy(wire).to(dev)
    res = ThriftCodec(sch).UnmarshalStream(d, nf, keys)
    exp = oracle.ttstream_frame_scan(wire, nf, keys)
    assert exp[0] == 0 and res.scan_status.code == 0 and res.scan_status.n_records == nf
    for got, want in zip((res.frame_offsets, res.payload_start, res.payload_end, res.frame_types, res.stream_ids,
                          res.method_pos, res.method_len), exp[1:8]):
        assert np.array_equal(to_np(got).astype(np.int64), want.astype(np.int64))
    assert res.method(nf - 1) == info[-1][2].decode()
    st = res.read_status()
    assert st.code == 0 and st.n_records == n
    assert to_np(res.data_frames).tolist() == [i for i, f in enumerate(info) if f[0] == A.TTS_DATA]
    rc, ew, eo = oracle.encode(sch, cs)
    _, infos, _ = oracle.flatten(sch)
    rc, exp_cols, est, _ = oracle.decode(sch, ew, n, offsets=eo)
    assert_columns_equal(res.columns, exp_cols, infos, n)


def test_ttstream_protobuf_struct_frames(torch, oracle):
    """ProtobufStruct payloads (protocol id 0x11): DATA payloads are bare proto bodies"""
    from kitex_amd.codec import ProtobufCodec
    from tests.test_gpu_messages import _records
    keys = T.default_keys()
    sch = S.schema_pf()
    n = 5000
    cs = synth.gen_pf(n, start=9)
    recs = _records(oracle, sch, cs, pb=True)
    frames = [T.frame(keys, 1, A.TTS_META, b"pb")]
    frames += [T.frame(keys, 1, A.TTS_DATA, b"pb", payload=r, proto=0x11) for r in recs]
    frames += [T.frame(keys, 1, A.TTS_TRAILER, b"pb")]
    wire = np.frombuffer(b"".join(frames), dtype=np.uint8).copy()
    res = ProtobufCodec(sch).UnmarshalStream(torch.from_numpy(wire).cuda(), len(frames), keys)
    assert res.read_status().code == 0
    _, infos, _ = oracle.flatten(sch)
    body = np.frombuffer(b"".join(recs), dtype=np.uint8).copy()
    offs = np.zeros(n + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(r) for r in recs])
    rc, exp, est, _ = oracle.decode(sch, body, n, offsets=offs, pb=True)
    assert_columns_equal(res.columns, exp, infos, n)


@pytest.mark.parametrize("case", T.ERROR_CASES)
def test_ttstream_scan_errors_match_oracle(torch, oracle, case):
    from kitex_amd.codec import read_status, ttstream_frame_scan
    keys = T.default_keys()
    wire, bad, code, n = T.error_batch(oracle, keys, case)
    fo, ps, pe, ft, sid, mp, ml, st = ttstream_frame_scan(torch.from_numpy(wire).cuda(), n, keys)
    s = read_status(st)
    assert s.code == code and s.record == bad, (s.code, s.record)
    e = oracle.ttstream_frame_scan(wire, n, keys)
    assert np.array_equal(to_np(fo)[:bad].astype(np.uint64), e[1][:bad])
    assert np.array_equal(to_np(ft)[:bad], e[4][:bad])


def test_decode_extents_with_gaps_and_errors(torch, oracle):
    """records at explicit extents with junk between them; a truncated extent fails alone"""
    from kitex_amd.codec import ThriftCodec
    sch = S.schema_r2()
    n = 7000
    cs = synth.gen_r2(n, start=1)
    rc, w, o = oracle.encode(sch, cs)
    recs = [bytes(w[int(o[i]):int(o[i + 1])]) for i in range(n)]
    rng = np.random.default_rng(3)
    parts, starts, ends, pos = [], [], [], 0
    for i, r in enumerate(recs):
        gap = bytes(rng.integers(0, 256, size=int(rng.integers(0, 40)), dtype=np.uint8))
        parts.append(gap)
        pos += len(gap)
        starts.append(pos)
        cut = 5 if i == 4321 else 0
        ends.append(pos + len(r) - cut)
        parts.append(r)
        pos += len(r)
    wire = np.frombuffer(b"".join(parts), dtype=np.uint8).copy()
    dev = torch.device("cuda", 0)
    res = ThriftCodec(sch).UnmarshalExtents(torch.from_numpy(wire).to(dev), torch.tensor(starts, device=dev),
                                            torch.tensor(ends, device=dev), raise_on_error=False)
    st = res.read_status()
    assert st.code == A.ERR_EOF and st.record == 4321 and st.offset == starts[4321]
    rs = to_np(res.record_status)[:n]
    assert rs[4321] == A.ERR_EOF and int((rs != 0).sum()) == 1
    _, infos, _ = oracle.flatten(sch)
    keep = [i for i in range(n) if i != 4321]
    for c in range(8):
        assert np.array_equal(to_np(res.columns.cols[c])[keep], cs.cols[c][keep])
