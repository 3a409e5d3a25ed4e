"""CPU: the oracle's gRPC message delimiting (kxo_grpc_frame_scan, restating decodeGRPCFrame,
pkg/remote/codec/grpc/grpc_compress.go:37-60) and the SIMT-emulated device scan against it."""
import numpy as np
import pytest

from tests import frame_cases as FC


def test_grpc_scan_layout(oracle):
    sch, recs, msgs, wire, fo = FC.grpc_batch(50, compressed={3})
    rc, efo, ps, pe, fl, done = oracle.grpc_frame_scan(wire, 50)
    assert rc == 0 and done == 50 and np.array_equal(efo, fo)
    for i in range(50):
        assert wire[int(ps[i]):int(pe[i])].tobytes() == recs[i]
    assert fl[3] == 1 and fl[5] == 2 and fl[0] == 0


def test_grpc_scan_errors(oracle):
    sch, recs, msgs, wire, fo = FC.grpc_batch(20)
    rc, *_, done = oracle.grpc_frame_scan(wire[:-1], 20)            # last payload cut short
    assert rc == 8 and done == 19
    rc, *_, done = oracle.grpc_frame_scan(wire[:int(fo[7]) + 3], 20)  # header cut short
    assert rc == 8 and done == 7
    rc, *_, done = oracle.grpc_frame_scan(wire, 20, max_payload=len(recs[0]) - 1)
    assert rc == 1 and done == 0
    rc, *_, done = oracle.grpc_frame_scan(np.zeros(0, dtype=np.uint8), 0)
    assert rc == 0 and done == 0


@pytest.mark.parametrize("n,pb", [(1, False), (3000, False), (3000, True)])
def test_emu_grpc_scan(oracle, n, pb):
    from tests.emu import emu
    sch, recs, msgs, wire, fo = FC.grpc_batch(n, pb=pb, compressed={1, n // 2})
    rc, efo, eps, epe, efl, done = oracle.grpc_frame_scan(wire, n)
    grc, gfo, gps, gpe, gfl, st = emu.frames(wire, n, grpc=True)
    assert st.code == rc == 0 and st.n_records == n
    assert np.array_equal(gfo, efo) and np.array_equal(gps, eps) and np.array_equal(gpe, epe)
    assert np.array_equal(gfl, efl)


def test_emu_grpc_scan_truncated(oracle):
    from tests.emu import emu
    n = 2000
    sch, recs, msgs, wire, fo = FC.grpc_batch(n)
    cut = wire[:int(fo[1500]) + 40]
    rc, efo, *_, done = oracle.grpc_frame_scan(cut, n)
    grc, gfo, gps, gpe, gfl, st = emu.frames(cut, n, grpc=True)
    assert st.code == rc == 8 and st.n_records == done == 1500 and st.record == 1500
    assert np.array_equal(gfo[:1501], efo[:1501])
