"""GPU parity for the Kitex-Protobuf path (kx_pb_decode_batch, HIP, gfx950) vs the CPU oracle,
through the C-ABI: columns field-for-field, error code / failing record / byte offset identical."""
import numpy as np
import pytest

from kitex_amd import schema as S
from kitex_amd import synth
from tests import pb_cases as PC
from tests.helpers import assert_columns_equal

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as t
    if not t.cuda.is_available():
        pytest.skip("no GPU")
    return t


class PbGpuDecoder:
    """decode through libkxcodec (HIP) with host inputs copied to HBM"""

    def __init__(self, torch):
        self.torch = torch
        self.dev = torch.device("cuda", 0)

    def decode(self, sch, wire, n, offsets=None, pb=True):
        from kitex_amd.codec import ProtobufCodec
        torch, dev = self.torch, self.dev
        cdc = ProtobufCodec(sch)
        buf = torch.from_numpy(wire.copy()).to(dev) if wire.size else torch.empty(0, dtype=torch.uint8, device=dev)
        offs = torch.from_numpy(offsets.astype(np.int64)).to(dev) if offsets is not None else None
        res = cdc.Unmarshal(buf, n, offsets=offs, record_status=offsets is not None, raise_on_error=False)
        return res.columns, res.read_status(), res.record_status


@pytest.fixture(scope="module")
def pdec(torch):
    return PbGpuDecoder(torch)


@pytest.mark.parametrize("n", [1, 7, 1000, 25000])
def test_pb_decode_concat_matches_oracle(pdec, oracle, n):
    PC.case_pb_concat(pdec, oracle, n)


@pytest.mark.parametrize("n", [1, 300, 5000])
def test_pb_decode_offsets_matches_oracle(pdec, oracle, n):
    PC.case_pb_offsets(pdec, oracle, n)


@pytest.mark.parametrize("mode", ["concat", "offsets"])
def test_pb_noncanonical(pdec, oracle, mode):
    PC.case_pb_noncanonical(pdec, oracle, mode)


@pytest.mark.parametrize("mode", ["concat", "offsets"])
@pytest.mark.parametrize("case", PC.PB_ERRORS)
def test_pb_errors(pdec, oracle, case, mode):
    PC.case_pb_error(pdec, oracle, case, mode)


def test_pb_large_batch_roundtrip(pdec, oracle):
    """2M records (varints of every length, zero fields omitted): decode(encode(x)) == x"""
    sch = S.schema_pf()
    n = 1 << 21
    cs = synth.gen_pf(n)
    rc, wire, _ = oracle.encode(sch, cs, pb=True)
    assert rc == 0
    cols, st, _ = pdec.decode(sch, wire, n)
    assert st.code == 0 and st.n_records == n and st.consumed == wire.size
    _, infos, _ = oracle.flatten(sch)
    assert_columns_equal(cols, cs, infos, n)


@pytest.mark.parametrize("n", [1, 1000, 30000])
def test_pb_encode_bit_exact(torch, oracle, n):
    """kx_pb_encode_batch bytes == the oracle's proto3 Marshal (pinned against google.protobuf by
    tests/golden), frame starts == the framed record boundaries, sizes == BLength"""
    from kitex_amd.codec import ProtobufCodec
    from tests.test_gpu_thrift import cs_to_device
    sch = S.schema_pf()
    cs = synth.gen_pf(n, start=31)
    rc, exp, _ = oracle.encode(sch, cs, pb=True)
    assert rc == 0
    cdc = ProtobufCodec(sch)
    dev = torch.device("cuda", 0)
    dcs = cs_to_device(torch, dev, cs)
    wire, offs = cdc.Marshal(dcs)
    got = wire.cpu().numpy()
    assert got.size == exp.size and np.array_equal(got, exp)
    _, ref_offs = PC.join(PC.split_frames(exp), framed=True)
    assert np.array_equal(offs.cpu().numpy().astype(np.uint64), ref_offs)
    sizes = cdc.BLength(dcs).cpu().numpy()
    assert np.array_equal(sizes.astype(np.uint64), np.diff(ref_offs))


def test_pb_marshal_unmarshal_roundtrip_device(torch):
    """GPU encode -> GPU decode of 1M records generated in HBM equals the source columns"""
    from kitex_amd.codec import ProtobufCodec
    n = 1 << 20
    dev = torch.device("cuda", 0)
    cdc = ProtobufCodec(S.schema_pf())
    src = synth.gen_pf_torch(n, dev)
    wire, offs = cdc.Marshal(src)
    res = cdc.Unmarshal(wire, n)
    st = res.read_status()
    assert st.code == 0 and st.n_records == n and st.consumed == wire.numel()
    for c, col in enumerate(src.cols):
        got = res.columns.cols[c]
        if isinstance(col, tuple):
            assert torch.equal(got[0][:n + 1], col[0][:n + 1]) and torch.equal(got[1][:col[1].numel()], col[1])
        else:
            assert torch.equal(got[:n], col)


def test_pb_golden_fixture_on_gpu(torch, oracle):
    """tests/golden/pf_batch_64.bin (google.protobuf serialization, pinned by the oracle) decoded by
    kx_pb_decode_batch: the generator's 64 records field-for-field"""
    import os

    from kitex_amd.codec import ProtobufCodec
    golden = np.fromfile(os.path.join(os.path.dirname(__file__), "golden", "pf_batch_64.bin"), dtype=np.uint8)
    sch = S.schema_pf()
    cdc = ProtobufCodec(sch)
    dev = torch.device("cuda", 0)
    res = cdc.Unmarshal(torch.from_numpy(golden).to(dev), 64)
    st = res.read_status()
    assert st.code == 0 and st.n_records == 64 and st.consumed == golden.size
    _, infos, _ = oracle.flatten(sch)
    assert_columns_equal(res.columns, synth.gen_pf(64), infos, 64)


def test_pb_split_points_refused(torch):
    """SplitPoints on a flat Kitex-Protobuf codec: NOT_IMPLEMENTED, never a Thrift walk over protobuf Batch
    bytes (a nested proto3 schema is refused by kx_thrift_split_points itself)"""
    from kitex_amd.codec import ProtobufCodec
    sch = S.schema_pf()
    cdc = ProtobufCodec(sch)
    assert not cdc.dschema.nested
    buf = torch.zeros(64, dtype=torch.uint8, device="cuda:0")
    from kitex_amd import _abi as A
    from kitex_amd._lib import KxError
    with pytest.raises(KxError) as ei:
        cdc.SplitPoints(buf, 4, 2)
    assert ei.value.code == A.ERR_NOT_IMPLEMENTED
