"""GPU parity of list<struct> fields (kxcodec.h: list/set of a struct of fixed-width scalars): device
decode (known offsets and concatenated) and encode / BLength bit-exact against the oracle."""
import numpy as np
import pytest

from kitex_amd import schema as S
from tests import list_struct_cases as LC
from tests.helpers import assert_columns_equal, to_np

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as t
    if not t.cuda.is_available():
        pytest.skip("no GPU")
    return t


@pytest.mark.parametrize("n", [1, 700, 40000])
@pytest.mark.parametrize("mode", ["offsets", "concat"])
def test_decode_matches_oracle(torch, oracle, n, mode):
    from kitex_amd.codec import ThriftCodec
    sch, infos, npres, cs, wire, offs = LC.random_batch(oracle, n, seed=n)
    rc, exp, est, _ = oracle.decode(sch, wire, n, offsets=offs if mode == "offsets" else None)
    assert rc == 0 and est.code == 0
    cdc = ThriftCodec(sch)
    o = torch.from_numpy(offs.astype(np.int64)).to("cuda:0") if mode == "offsets" else None
    res = cdc.Unmarshal(torch.from_numpy(wire).to("cuda:0"), n, offsets=o)
    assert_columns_equal(res.columns, exp, infos, n)


def test_handmade_and_required(torch, oracle):
    from kitex_amd.codec import ThriftCodec
    sch = S.schema_ls1()
    recs = LC.handmade() + [LC.missing_required()]
    wire, offs = LC.wire_of(recs)
    n = len(recs)
    rc, exp, est, ers = oracle.decode(sch, wire, n, offsets=offs)
    res = ThriftCodec(sch).Unmarshal(torch.from_numpy(wire).to("cuda:0"), n,
                                     offsets=torch.from_numpy(offs.astype(np.int64)).to("cuda:0"),
                                     record_status=True, raise_on_error=False)
    st = res.read_status()
    assert st.code == est.code == 1 and st.record == est.record == n - 1
    assert np.array_equal(to_np(res.record_status)[:n], ers)
    _, infos, _ = oracle.flatten(sch)
    assert_columns_equal(res.columns, exp, infos, n - 1)


def test_encode_bit_exact(torch, oracle):
    from kitex_amd.codec import ThriftCodec
    from kitex_amd.columns import to_kx_columns  # noqa: F401
    sch, infos, npres, cs, wire, offs = LC.random_batch(oracle, 30000, seed=2)
    cdc = ThriftCodec(sch)
    dev = [c if not isinstance(c, tuple) else tuple(torch.from_numpy(x.astype(np.int64) if x.dtype == np.uint32
                                                                     else x).to("cuda:0") for x in c)
           for c in cs.cols]
    dev = [torch.from_numpy(c).to("cuda:0") if isinstance(c, np.ndarray) else c for c in dev]
    from kitex_amd.synth import ColumnSet
    dcs = ColumnSet(dev, torch.from_numpy(cs.presence.view(np.int64)).to("cuda:0"), cs.n)
    sizes = cdc.BLength(dcs)
    assert np.array_equal(to_np(sizes), np.diff(offs.astype(np.int64)))
    out, o2 = cdc.Marshal(dcs)
    assert np.array_equal(to_np(out), wire)
