"""GPU parity of the framing sniff (kx_frame_scan) and of socket-buffer decode (kx_*_decode_frames):
frame boundaries, payload extents and kinds identical to the oracle's kxo_frame_scan; the records
inside identical to the oracle's decode of the same record bytes; method names / seqids as written."""
import numpy as np
import pytest

from kitex_amd import _abi as A
from tests import frame_cases as FC
from tests.helpers import assert_columns_equal, to_np

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as t
    if not t.cuda.is_available():
        pytest.skip("no GPU")
    return t


def _gpu_scan(torch):
    from kitex_amd.codec import frame_scan, read_status

    def scan(wire, n, mx):
        buf = torch.from_numpy(wire).to("cuda:0")
        fo, ps, pe, kd, st = frame_scan(buf, n, mx)
        return to_np(fo).astype(np.uint64), to_np(ps).astype(np.uint64), to_np(pe).astype(np.uint64), \
            to_np(kd), read_status(st)
    return scan


@pytest.mark.parametrize("case", FC.SCAN_CASES)
def test_frame_scan_matches_oracle(torch, oracle, case):
    FC.case_scan(_gpu_scan(torch), oracle, case)


def _oracle_records(oracle, sch, recs):
    wire = np.frombuffer(b"".join(recs), dtype=np.uint8).copy()
    offs = np.zeros(len(recs) + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(r) for r in recs])
    return oracle.decode(sch, wire, len(recs), offsets=offs)


@pytest.mark.parametrize("kinds", [["ttheader"], ["framed", "ttheader_framed", "pure", "mesh", "mesh_framed"]])
def test_thrift_frames_end_to_end(torch, oracle, kinds):
    from kitex_amd.codec import ThriftCodec
    n = 20000
    sch, recs, frames, wire, fo = FC.batch(kinds, n)
    cdc = ThriftCodec(sch)
    res = cdc.UnmarshalFrames(torch.from_numpy(wire).to("cuda:0"), n, raise_on_error=False)
    st = res.read_status()
    assert st.code == 0 and st.n_records == n and st.consumed == wire.size
    assert np.array_equal(to_np(res.frame_offsets).astype(np.uint64), fo)
    assert (to_np(res.kinds) == [FC.expected_kind(kinds[i % len(kinds)]) for i in range(n)]).all()
    rc, exp, est, _ = _oracle_records(oracle, sch, recs)
    _, infos, _ = oracle.flatten(sch)
    assert_columns_equal(res.columns, exp, infos, n)
    assert (to_np(res.seqid) == np.arange(n)).all()
    assert [res.name(i) for i in (0, 1, 6, 7, n - 1)] == ["Method%d" % (i % 7) for i in (0, 1, 6, 7, n - 1)]


def test_pb_frames_end_to_end(torch, oracle):
    from kitex_amd import schema as S
    from kitex_amd import synth
    from kitex_amd.codec import ProtobufCodec
    from tests.pb_cases import split_frames
    n = 5000
    sch = S.schema_pf()
    rc, w, _ = oracle.encode(sch, synth.gen_pf(n, start=3), pb=True)
    bodies = split_frames(w)
    frames = [FC.make_frame(["pb_framed", "ttheader_pb"][i % 2], i, bodies[i]) for i in range(n)]
    wire = np.frombuffer(b"".join(frames), dtype=np.uint8).copy()
    res = ProtobufCodec(sch).UnmarshalFrames(torch.from_numpy(wire).to("cuda:0"), n, raise_on_error=False)
    st = res.read_status()
    assert st.code == 0 and st.n_records == n
    bw = np.frombuffer(b"".join(bodies), dtype=np.uint8).copy()
    bo = np.zeros(n + 1, dtype=np.uint64)
    bo[1:] = np.cumsum([len(b) for b in bodies])
    rc, exp, est, _ = oracle.decode(sch, bw, n, offsets=bo, pb=True)
    _, infos, _ = oracle.flatten(sch)
    assert_columns_equal(res.columns, exp, infos, n)
    assert (to_np(res.seqid) == np.arange(n)).all()


def test_frames_error_ends_batch(torch, oracle):
    """a frame that cannot be delimited: earlier messages decode, it and later ones carry its code"""
    from kitex_amd.codec import ThriftCodec
    n = 6000
    sch, recs, frames, wire, fo = FC.batch(["ttheader", "framed"], n)
    k = 4321
    wire[int(fo[k]) + 4:int(fo[k]) + 6] = (0x70, 0x01)
    res = ThriftCodec(sch).UnmarshalFrames(torch.from_numpy(wire).to("cuda:0"), n, raise_on_error=False)
    st = res.read_status()
    assert (st.code, st.record, st.offset) == (A.ERR_UNKNOWN_PROTOCOL, k, int(fo[k]))
    rs = to_np(res.record_status)[:n]
    assert (rs[:k] == 0).all() and (rs[k:] == A.ERR_UNKNOWN_PROTOCOL).all()
    rc, exp, est, _ = _oracle_records(oracle, sch, recs[:k])
    _, infos, _ = oracle.flatten(sch)
    assert_columns_equal(res.columns, exp, infos, k)
