"""GPU parity of the binary generic ingress (kx_thrift_raw_messages / kx_thrift_set_seqids) against the
oracle's restatement of binaryThriftCodec (pkg/generic/binarythrift_codec.go:83-199), and of a decode
driven by an IDL-compiled schema (kitex_amd.idl over the reference's IDL fixtures)."""
import os

import numpy as np
import pytest

from tests import generic_cases as GC
from tests.helpers import assert_columns_equal, random_columns, to_np

pytestmark = pytest.mark.gpu
IDL = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "idl")


@pytest.fixture(scope="module")
def torch():
    import torch as t
    if not t.cuda.is_available():
        pytest.skip("no GPU")
    return t


@pytest.mark.parametrize("n", [1, 10, 30000])
def test_raw_messages_match_oracle(torch, oracle, n):
    from kitex_amd.generic import BinaryThriftCodec
    wire, offs, names, codes = GC.raw_batch(n)
    rc, enames, ety, esq, ers = oracle.raw_messages(wire, offs)
    buf = torch.from_numpy(wire).to("cuda:0")
    toffs = torch.from_numpy(offs.astype(np.int64)).to("cuda:0")
    res = BinaryThriftCodec().Unmarshal(buf, n, toffs, raise_on_error=False)
    assert np.array_equal(to_np(res.record_status), ers)
    assert np.array_equal(to_np(res.msg_type), ety) and np.array_equal(to_np(res.seqid), esq)
    pick = [i for i in range(n) if i < 50 or i == n - 1]
    assert [res.name(i).encode() for i in pick] == [enames[i] for i in pick]
    st = res.status.cpu().numpy()
    first = next((i for i in range(n) if ers[i]), None)
    from kitex_amd.codec import read_status
    s = read_status(res.status)
    assert (s.code == 0) if first is None else (s.code == ers[first] and s.record == first)


@pytest.mark.parametrize("n", [1, 30000])
def test_set_seqids_matches_oracle(torch, oracle, n):
    from kitex_amd.generic import BinaryThriftCodec
    wire, offs, names, codes = GC.raw_batch(n)
    seq = (np.arange(n, dtype=np.int64) * 31 - 5).astype(np.int32)
    rc, eout, ers = oracle.set_seqids(wire, offs, seq)
    buf = torch.from_numpy(wire).to("cuda:0")
    rs = BinaryThriftCodec().SetSeqID(buf, torch.from_numpy(offs.astype(np.int64)).to("cuda:0"),
                                      torch.from_numpy(seq).to("cuda:0"), raise_on_error=False)
    assert np.array_equal(to_np(rs), ers)
    assert np.array_equal(to_np(buf), eout)


def test_reference_binary_codec_case(torch):
    """TestBinaryThriftCodec: GetSeqID 100, SetSeqID(1) -> 1, method "mock" """
    from kitex_amd.generic import BinaryThriftCodec
    buf_b, seq = GC.REF_SEQID[0]
    buf = torch.from_numpy(np.frombuffer(buf_b, dtype=np.uint8).copy()).to("cuda:0")
    offs = torch.tensor([0, len(buf_b)], dtype=torch.int64, device="cuda:0")
    c = BinaryThriftCodec()
    r = c.Unmarshal(buf, 1, offs)
    assert int(r.seqid[0]) == 100 and r.name(0) == "mock"
    c.SetSeqID(buf, offs, torch.tensor([1], dtype=torch.int32, device="cuda:0"))
    r = c.Unmarshal(buf, 1, offs)
    assert int(r.seqid[0]) == 1 and r.name(0) == "mock"


@pytest.mark.parametrize("idl_file,struct", [("example.thrift", "base.BaseResp"), ("baseline.thrift", "Simple"),
                                             ("mock.thrift", "MockReq")])
def test_idl_schema_decode_matches_oracle(torch, oracle, idl_file, struct):
    """a schema compiled from the reference's IDL fixtures drives the device decode (known offsets and
    concatenated), identical to the oracle"""
    from kitex_amd import idl
    from kitex_amd.codec import ThriftCodec
    sch = idl.to_schema(idl.parse_idl(os.path.join(IDL, idl_file)).struct(struct))
    rc, infos, npres = oracle.flatten(sch)
    n = 5000
    cs = random_columns(infos, npres, n, seed=11)
    rc, wire, offs = oracle.encode(sch, cs)
    assert rc == 0
    rc, exp, est, _ = oracle.decode(sch, wire, n, offsets=offs)
    assert rc == 0 and est.code == 0
    cdc = ThriftCodec(sch)
    buf = torch.from_numpy(wire).to("cuda:0")
    for o in (torch.from_numpy(offs.astype(np.int64)).to("cuda:0"), None):
        res = cdc.Unmarshal(buf, n, offsets=o)
        assert_columns_equal(res.columns, exp, infos, n)


@pytest.mark.parametrize("f", ["testservice.thrift", "http_binary_echo.thrift", "http_annotation.thrift",
                               "http_baseline.thrift", "grpcjson_api.thrift"])
def test_reference_fixture_methods_decode_encode_on_gpu(torch, oracle, f):
    """every method's Args / Result of the reference's other IDL fixtures: concatenated decode on the GPU
    equals the oracle's, and the GPU's encode of those columns equals the oracle's bytes"""
    from kitex_amd import synth
    from kitex_amd.codec import ThriftCodec
    from tests.helpers import assert_columns_equal, to_np
    from tests.test_idl import fixture_schemas
    for name, sch in fixture_schemas(f):
        n = 3000
        wire = np.frombuffer(b"".join(synth.thrift_records(sch, n, seed=13)), dtype=np.uint8).copy()
        rc, exp, est, _ = oracle.decode(sch, wire, n)
        _, infos, _ = oracle.flatten(sch)
        cdc = ThriftCodec(sch)
        res = cdc.Unmarshal(torch.from_numpy(wire).to("cuda:0"), n)
        assert_columns_equal(res.columns, exp, infos, n)
        rc, ow, _ = oracle.encode(sch, exp)
        got, _ = cdc.Marshal(res.columns)
        assert np.array_equal(to_np(got), ow), name
