"""Config 5 in miniature on one GPU (BASELINE.json configs[4]): record-range shards of an
R2 batch, an R3 batch and a container batch (map<string,string>, list<string>) are decoded by
libkxcodec on two contexts and two streams, concatenated with the same plan and device rebase the RCCL
path uses (kitex_amd.shard), and compared field for field with the oracle's decode of the whole batch."""
import numpy as np
import pytest

from kitex_amd import schema as S
from kitex_amd import synth
from kitex_amd.shard import shard_range
from tests.helpers import assert_columns_equal

pytestmark = pytest.mark.gpu

_GEN = {"r2": (S.schema_r2, synth.gen_r2), "r3": (S.schema_r3, synth.gen_r3),
        "cx1": (S.schema_cx1, synth.gen_cx1), "cx2": (S.schema_cx2, synth.gen_cx2)}


@pytest.fixture(scope="module")
def torch():
    import torch as t
    if not t.cuda.is_available():
        pytest.skip("no GPU")
    return t


@pytest.mark.parametrize("name,n,parts,views", [("r2", 60001, 4, False), ("r3", 9001, 3, False),
                                                 ("cx1", 5003, 3, False), ("cx2", 4001, 2, False),
                                                 ("r2", 30001, 3, True)])
def test_c5_shards_concat_matches_whole(torch, oracle, name, n, parts, views):
    from kitex_amd.codec import ThriftCodec
    from kitex_amd.shard import concat_local
    mk, gen = _GEN[name]
    sch = mk()
    _, infos, _ = oracle.flatten(sch)
    dev = torch.device("cuda", 0)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    codecs = [ThriftCodec(sch), ThriftCodec(sch)]          # two contexts (workspaces)
    shards, wires, keep = [], [], []
    for r in range(parts):
        s0, cnt = shard_range(n, parts, r)
        rc, w, _ = oracle.encode(sch, gen(cnt, start=s0))
        assert rc == 0
        wires.append(w)
        st = streams[r % 2]
        with torch.cuda.stream(st):
            d = torch.from_numpy(w).to(dev, non_blocking=False)
            keep.append(d)
            res = codecs[r % 2].Unmarshal(d, cnt, stream=st, views=views, raise_on_error=False)
        shards.append((res, cnt, w.size))
    for st in streams:
        st.synchronize()
    for res, cnt, _ in shards:
        s = res.read_status()
        assert s.code == 0 and s.n_records == cnt, (s.code, s.n_records, cnt)
    out = concat_local([(res.columns, cnt, ln) for res, cnt, ln in shards], infos)
    torch.cuda.synchronize()
    rc, exp, est, _ = oracle.decode(sch, np.concatenate(wires), n, views=views)
    assert rc == 0 and est.code == 0
    assert out.n == n
    assert_columns_equal(out, exp, infos, n)
