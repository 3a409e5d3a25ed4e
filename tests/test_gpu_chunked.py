"""GPU parity of the chunked decode pipeline (kx_ctx_set_pipeline): the index + group passes of
chunk k run on the ctx's second stream while chain + emit of chunk k - ahead run on the caller's
stream. Small chunks (512 KiB = one group of tiles) so every batch spans several chunks; results
must be identical to the oracle (and therefore to the one-chunk path) for every `ahead`."""
import numpy as np
import pytest

from tests import decode_cases as DC

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as t
    if not t.cuda.is_available():
        pytest.skip("no GPU")
    return t


class ChunkedGpuDecoder:
    def __init__(self, torch, ahead):
        self.torch, self.ahead = torch, ahead
        self.dev = torch.device("cuda", 0)
        self._codecs = {}

    def decode(self, sch, wire, n, offsets=None, pb=False):
        from kitex_amd.codec import ProtobufCodec, ThriftCodec
        torch, dev = self.torch, self.dev
        key = (id(sch), pb)
        if key not in self._codecs:
            cdc = (ProtobufCodec if pb else ThriftCodec)(sch)
            cdc.set_pipeline(512 * 1024, self.ahead)
            self._codecs[key] = (sch, cdc)
        cdc = self._codecs[key][1]
        buf = torch.from_numpy(wire.copy()).to(dev) if wire.size else torch.empty(0, dtype=torch.uint8, device=dev)
        offs = torch.from_numpy(offsets.astype(np.int64)).to(dev) if offsets is not None else None
        res = cdc.Unmarshal(buf, n, offsets=offs, record_status=offsets is not None, raise_on_error=False)
        return res.columns, res.read_status(), res.record_status


@pytest.mark.parametrize("ahead", [0, 1, 3])
@pytest.mark.parametrize("case", DC.CHUNK_CASES)
def test_chunked_matches_oracle(torch, oracle, case, ahead):
    DC.case_chunked(ChunkedGpuDecoder(torch, ahead), oracle, case)


def test_chunked_large_batch_equals_source(torch):
    """4 M R2 records (700 MB) in default-size chunks and in one chunk: identical columns"""
    from kitex_amd import schema as S
    from kitex_amd import synth
    from kitex_amd.codec import ThriftCodec
    dev = torch.device("cuda", 0)
    n = 4 << 20
    src = synth.gen_r2_torch(n, dev)
    one = ThriftCodec(S.schema_r2())
    one.set_pipeline(0)
    wire, _ = one.Marshal(src)
    outs = []
    for chunk in (0, 64 << 20, 16 << 20):
        cdc = ThriftCodec(S.schema_r2())
        cdc.set_pipeline(chunk, 1)
        res = cdc.Unmarshal(wire, n, raise_on_error=False)
        st = res.read_status()
        assert st.code == 0 and st.n_records == n and st.consumed == wire.numel(), (chunk, st.code)
        outs.append(res.columns)
    for c in range(10):
        for o in outs:
            if isinstance(src.cols[c], tuple):
                assert torch.equal(o.cols[c][0].to(torch.int64), src.cols[c][0].to(torch.int64)), c
                assert torch.equal(o.cols[c][1][:32 * n], src.cols[c][1][:32 * n]), c
            else:
                assert torch.equal(o.cols[c], src.cols[c]), c
