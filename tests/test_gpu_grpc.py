"""GPU parity of gRPC message delimiting (kx_grpc_frame_scan) and gRPC payload decode
(kx_thrift_decode_grpc / kx_pb_decode_grpc) against the oracle: decodeGRPCFrame
(grpc_compress.go:37-60) + grpcCodec.Decode (grpc.go:202-270), through the C-ABI."""
import numpy as np
import pytest

from tests import frame_cases as FC
from tests.helpers import assert_rows_equal, to_np

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as t
    if not t.cuda.is_available():
        pytest.skip("no GPU")
    return t


def _scan(torch, wire, n, mx=0):
    from kitex_amd.codec import grpc_frame_scan, read_status
    fo, ps, pe, fl, st = grpc_frame_scan(torch.from_numpy(wire).to("cuda:0"), n, mx)
    u = lambda t: to_np(t).astype(np.uint64)
    return u(fo), u(ps), u(pe), to_np(fl), read_status(st)


@pytest.mark.parametrize("n,pb", [(1, False), (777, False), (30000, False), (30000, True)])
def test_grpc_scan_matches_oracle(torch, oracle, n, pb):
    sch, recs, msgs, wire, fo = FC.grpc_batch(n, pb=pb, compressed={0, n // 3})
    rc, efo, eps, epe, efl, done = oracle.grpc_frame_scan(wire, n)
    gfo, gps, gpe, gfl, st = _scan(torch, wire, n)
    assert st.code == rc == 0 and st.n_records == n and st.consumed == wire.size
    assert np.array_equal(gfo, efo) and np.array_equal(gps, eps) and np.array_equal(gpe, epe)
    assert np.array_equal(gfl, efl)


@pytest.mark.parametrize("case", ["truncated_payload", "truncated_header", "max_payload"])
def test_grpc_scan_errors(torch, oracle, case):
    n = 20000
    sch, recs, msgs, wire, fo = FC.grpc_batch(n)
    mx = 0
    if case == "truncated_payload":
        wire = wire[:int(fo[15000]) + 40]
    elif case == "truncated_header":
        wire = wire[:int(fo[15000]) + 3]
    else:
        mx = len(recs[0]) - 1
    rc, efo, eps, epe, efl, done = oracle.grpc_frame_scan(wire, n, mx)
    gfo, gps, gpe, gfl, st = _scan(torch, wire, n, mx)
    assert rc != 0 and st.code == rc and st.record == done and st.n_records == done
    assert np.array_equal(gfo[:done + 1], efo[:done + 1])


@pytest.mark.parametrize("pb", [False, True])
def test_grpc_decode_matches_oracle(torch, oracle, pb):
    from kitex_amd.codec import ProtobufCodec, ThriftCodec
    n = 20000
    comp = {7, 8, 12345}
    sch, recs, msgs, wire, fo = FC.grpc_batch(n, pb=pb, compressed=comp)
    cdc = ProtobufCodec(sch) if pb else ThriftCodec(sch)
    res = cdc.UnmarshalGRPC(torch.from_numpy(wire).to("cuda:0"), n, raise_on_error=False)
    st = res.read_status()
    rs = to_np(res.record_status)[:n]
    exp = np.zeros(n, dtype=np.uint8)
    exp[sorted(comp)] = 5
    assert np.array_equal(rs, exp)
    assert st.code == 5 and st.record == 7 and st.offset == fo[7]
    assert np.array_equal(to_np(res.frame_offsets).astype(np.uint64), fo)
    ok = np.nonzero(exp == 0)[0]
    body = np.frombuffer(b"".join(recs[i] for i in ok), dtype=np.uint8).copy()
    offs = np.zeros(ok.size + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(recs[i]) for i in ok])
    rc, eout, est, _ = oracle.decode(sch, body, ok.size, offsets=offs, pb=pb)
    assert rc == 0
    _, infos, _ = oracle.flatten(sch)
    assert_rows_equal(res.columns, eout, infos, ok)


def test_grpc_decode_empty_and_short_payloads(torch, oracle):
    """an empty Thrift payload is EOF (fastUnmarshal of 0 bytes); an empty proto payload is a message of
    defaults (proto.Unmarshal of nil)"""
    from kitex_amd.codec import ProtobufCodec, ThriftCodec
    from kitex_amd import schema as S
    wire = np.frombuffer(FC.grpc_message(b"") * 3, dtype=np.uint8).copy()
    r = ThriftCodec(S.schema_r2()).UnmarshalGRPC(torch.from_numpy(wire).to("cuda:0"), 3, raise_on_error=False)
    assert list(to_np(r.record_status)[:3]) == [8, 8, 8]
    r = ProtobufCodec(S.schema_pf()).UnmarshalGRPC(torch.from_numpy(wire).to("cuda:0"), 3, raise_on_error=False)
    assert list(to_np(r.record_status)[:3]) == [0, 0, 0] and r.read_status().code == 0
