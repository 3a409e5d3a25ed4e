"""GPU parity: libkxcodec (HIP, gfx950) vs the CPU oracle on the same inputs, through the C-ABI.

Bit-exact for everything (integer/byte work): decoded columns field-for-field, encoded bytes
byte-for-byte, error codes / failing record / byte offset identical.
"""
import numpy as np
import pytest

from kitex_amd import _abi as A
from kitex_amd import schema as S
from kitex_amd import synth
from tests import decode_cases as DC
from tests.helpers import assert_columns_equal, to_np

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as t
    if not t.cuda.is_available():
        pytest.skip("no GPU")
    return t


@pytest.fixture(scope="module")
def dev(torch):
    return torch.device("cuda", 0)


_codecs = {}


def codec(sch_name_or_schema):
    from kitex_amd.codec import ThriftCodec
    key = sch_name_or_schema if isinstance(sch_name_or_schema, str) else id(sch_name_or_schema)
    if key not in _codecs:
        sch = S.SCHEMAS[key]() if isinstance(key, str) else sch_name_or_schema
        _codecs[key] = (sch, ThriftCodec(sch))
    return _codecs[key]


class GpuDecoder:
    """decode through libkxcodec (HIP) with host inputs copied to HBM"""

    def __init__(self, torch, dev):
        self.torch, self.dev = torch, dev

    def decode(self, sch, wire: np.ndarray, n, offsets=None, caps=None):
        torch, dev = self.torch, self.dev
        cdc = codec(sch)[1]
        buf = torch.from_numpy(wire.copy()).to(dev) if wire.size else torch.empty(0, dtype=torch.uint8, device=dev)
        offs = torch.from_numpy(offsets.astype(np.int64)).to(dev) if offsets is not None else None
        res = cdc.Unmarshal(buf, n, offsets=offs, var_caps=caps, record_status=offsets is not None,
                            raise_on_error=False)
        return res.columns, res.read_status(), res.record_status

    def decode_views(self, sch, wire, n, offsets=None, pb=False, wide=False):
        from kitex_amd.codec import ProtobufCodec, ThriftCodec
        from kitex_amd.columns import alloc_device
        torch, dev = self.torch, self.dev
        cdc = ProtobufCodec(sch) if pb else codec(sch)[1]
        buf = torch.from_numpy(wire.copy()).to(dev)
        offs = torch.from_numpy(offsets.astype(np.int64)).to(dev) if offsets is not None else None
        ds = cdc.dschema
        caps = [0 if ci.kind == A.COL_FIXED else max(1, wire.size) for ci in ds.infos]
        out = alloc_device(ds.infos, n, caps, ds.npresence, dev, views=True, wide=wide)
        res = cdc.Unmarshal(buf, n, offsets=offs, out=out, var_caps=caps, record_status=offsets is not None,
                            raise_on_error=False)
        return res.columns, res.read_status()


@pytest.fixture(scope="module")
def gdec(torch, dev):
    return GpuDecoder(torch, dev)


@pytest.mark.parametrize("name", ["r1", "r2", "r3"])
@pytest.mark.parametrize("n", [1, 7, 1000, 25000])
def test_decode_concat_matches_oracle(gdec, oracle, name, n):
    DC.case_concat(gdec, oracle, name, n)


@pytest.mark.parametrize("name", ["r1", "r2", "r3"])
@pytest.mark.parametrize("n", [1, 300, 5000])
def test_decode_offsets_matches_oracle(gdec, oracle, name, n):
    DC.case_offsets(gdec, oracle, name, n)


def test_decode_roundtrip_equals_source_columns(gdec, oracle):
    DC.case_roundtrip(gdec, oracle)


@pytest.mark.parametrize("mode", ["concat", "offsets"])
def test_noncanonical_records(gdec, oracle, mode):
    DC.case_noncanonical(gdec, oracle, mode)


@pytest.mark.parametrize("mode", ["concat", "offsets"])
def test_ragged_and_huge_strings(gdec, oracle, mode):
    DC.case_ragged(gdec, oracle, mode)


def test_empty_records_and_defaults(gdec, oracle):
    DC.case_empty(gdec, oracle)


def test_slot_overflow(gdec, oracle):
    """a run of 1-byte records after large ones: tiles with more records than the mean-size slot estimate"""
    DC.case_slot_overflow(gdec, oracle)


@pytest.mark.parametrize("seed", [3, 4])
def test_long_strings(gdec, oracle, seed):
    """strings at and past the wave-copy threshold, inside and outside the tile window"""
    DC.case_long_strings(gdec, oracle, n=3000, seed=seed)


@pytest.mark.parametrize("name", ["r2", "r3", "cx1"])
def test_slotcap_64(gdec, oracle, name):
    """64 record-start slots per tile (KX_SLOTCAP): records past them are emitted from the chain"""
    from kitex_amd._lib import lib
    from tests.helpers import knob
    with knob(lib(), "KX_SLOTCAP", 64, 0):
        if name == "cx1":
            DC.case_containers(gdec, oracle, "cx1", 3000, "concat")
        else:
            DC.case_concat(gdec, oracle, name, 20000)


def test_nested_struct_repeated_and_required(gdec, oracle):
    DC.case_nested(gdec, oracle)


@pytest.mark.parametrize("case", DC.ERROR_CASES)
def test_error_cases(gdec, oracle, case):
    DC.case_error(gdec, oracle, case)


# ---------------------------------------------------------------------------------------------
# encode
# ---------------------------------------------------------------------------------------------
def cs_to_device(torch, dev, cs):
    cols = []
    for c in cs.cols:
        if isinstance(c, tuple):
            parts = [torch.from_numpy(x.view(np.int32).copy() if x.dtype == np.uint32 else x.copy()).to(dev)
                     for x in c[:-1]]
            cols.append(tuple(parts) + (torch.from_numpy(c[-1].copy()).to(dev),))
        else:
            cols.append(torch.from_numpy(c.copy()).to(dev))
    pres = torch.from_numpy(cs.presence.view(np.int64).copy()).to(dev) if cs.presence is not None else None
    return synth.ColumnSet(cols, pres, cs.n)


@pytest.mark.parametrize("name", ["r1", "r2", "r3"])
@pytest.mark.parametrize("n", [1, 1000, 20000])
def test_encode_bit_exact(torch, dev, oracle, name, n):
    sch, cdc = codec(name)
    cs = synth.GENERATORS[name](n, start=31)
    rc, wire, offs = oracle.encode(sch, cs)
    dcs = cs_to_device(torch, dev, cs)
    sizes = cdc.BLength(dcs)
    assert np.array_equal(to_np(sizes), np.diff(offs).astype(np.int64))
    got, goffs = cdc.Marshal(dcs)
    assert np.array_equal(to_np(got), wire)
    assert np.array_equal(to_np(goffs).astype(np.uint64), offs)


def test_encode_optional_and_nil(torch, dev, oracle):
    inner = S.Struct("In", [S.Field(1, A.T_I64), S.Field(2, A.T_STRING, req=A.REQ_OPTIONAL)])
    sch = S.Schema(S.Struct("Out", [S.Field(1, A.T_STRING), S.Field(2, A.T_STRUCT, child=inner),
                                    S.Field(3, A.T_BOOL, req=A.REQ_OPTIONAL), S.Field(4, A.T_LIST, elem=A.T_BOOL),
                                    S.Field(5, A.T_I16)]))
    from kitex_amd.codec import ThriftCodec
    cdc = ThriftCodec(sch)
    n = 3000
    rng = np.random.default_rng(5)
    lens = rng.integers(0, 9, size=n)
    s_off = np.zeros(n + 1, np.uint32); s_off[1:] = np.cumsum(lens)
    s_dat = rng.integers(0, 256, size=int(s_off[-1]), dtype=np.uint8)
    llen = rng.integers(0, 5, size=n)
    l_off = np.zeros(n + 1, np.uint32); l_off[1:] = np.cumsum(llen)
    l_dat = rng.integers(0, 2, size=int(l_off[-1]), dtype=np.uint8)
    t_off = np.zeros(n + 1, np.uint32); t_off[1:] = np.cumsum(lens[::-1])
    t_dat = rng.integers(0, 256, size=int(t_off[-1]), dtype=np.uint8)
    cols = [(s_off, s_dat), rng.integers(-9, 9, size=n).astype(np.int64), (t_off, t_dat),
            rng.integers(0, 2, size=n).astype(np.uint8), (l_off, l_dat), rng.integers(-99, 99, size=n).astype(np.int16)]
    # presence bits in DFS order: inner=0, inner.tag=1, flag=2, list=3
    pres = rng.integers(0, 16, size=n).astype(np.uint64)
    cs = synth.ColumnSet(cols, pres, n)
    rc, wire, offs = oracle.encode(sch, cs)
    assert rc == 0
    got, goffs = cdc.Marshal(cs_to_device(torch, dev, cs))
    assert np.array_equal(to_np(got), wire)
    DC.check_decode(GpuDecoder(torch, dev), oracle, sch, wire, n)


def test_skip_batch_matches_oracle(torch, dev, oracle):
    sch, cdc = codec("r3")
    DC.case_skip(lambda wire, n: cdc.Skip(torch.from_numpy(wire).to(dev), n), oracle)


@pytest.mark.parametrize("mode", ["concat", "offsets"])
def test_r2_base_flat_path(torch, dev, oracle, mode):
    """R2 + base.Base (base.thrift:10-17): 11 var slots stay on the flat tile pipeline (kx_schema_is_nested
    == 0) and decode like the oracle"""
    from kitex_amd.codec import DeviceSchema
    assert not DeviceSchema(DC.schema_r2_base()).nested
    DC.case_r2_base(GpuDecoder(torch, dev), oracle, mode, n=20000)


@pytest.mark.parametrize("mode", ["concat", "offsets"])
def test_r2_base_repeated_struct(torch, dev, oracle, mode):
    """a repeated 255:Base whose second copy omits Extra: the struct is replaced wholesale, so the
    first copy's Extra (var slots past 8) is dropped, as the oracle does"""
    DC.case_r2_base(GpuDecoder(torch, dev), oracle, mode, n=20000, repeat=True)


def _gpu_split(torch, dev):
    from kitex_amd.codec import ThriftCodec, read_status, status_tensor
    from kitex_amd._lib import lib
    from kitex_amd.codec import _ptr

    def split(sch, wire, n, parts):
        cdc = ThriftCodec(sch)
        buf = torch.from_numpy(wire.copy()).to(dev) if wire.size else torch.empty(0, dtype=torch.uint8, device=dev)
        pts = torch.full((parts + 1,), 0xDEAD, dtype=torch.int64, device=dev)
        st = status_tensor(dev)
        ss = torch.cuda.current_stream(dev)
        rc = lib().kx_thrift_split_points(cdc._ctx(ss).handle, cdc.dschema.handle, _ptr(buf), buf.numel(), n, parts,
                                          _ptr(pts), _ptr(st), int(ss.cuda_stream))
        assert rc == 0
        return pts, read_status(st, ss)
    return split


@pytest.mark.parametrize("case", DC.SPLIT_CASES)
def test_split_points_match_oracle(torch, dev, oracle, case):
    """kx_thrift_split_points: record floor(k n / G)'s start for every k (the oracle's record offsets)"""
    DC.case_split(_gpu_split(torch, dev), oracle, case)


def test_split_points_errors(torch, dev, oracle):
    DC.case_split_errors(_gpu_split(torch, dev), oracle)


def test_split_points_codec_method_shards_decode(torch, dev, oracle):
    """ThriftCodec.SplitPoints cuts one concatenated batch into shards that decode on their own to the
    whole batch's columns (the c5 bench's sharding)"""
    from kitex_amd.codec import ThriftCodec
    sch = S.schema_r2()
    n = 50000
    cs = synth.gen_r2(n)
    rc, wire, offs = oracle.encode(sch, cs)
    buf = torch.from_numpy(wire).to(dev)
    cdc = ThriftCodec(sch)
    pts = to_np(cdc.SplitPoints(buf, n, 4))
    assert np.array_equal(pts.astype(np.uint64), DC.expected_points(offs, n, 4))
    _, infos, _ = oracle.flatten(sch)
    for k in range(4):
        r0, r1 = (k * n) // 4, ((k + 1) * n) // 4
        res = cdc.Unmarshal(buf[int(pts[k]):int(pts[k + 1])], r1 - r0)
        rc, exp, est, _ = oracle.decode(sch, wire[int(offs[r0]):int(offs[r1])], r1 - r0)
        assert_columns_equal(res.columns, exp, infos, r1 - r0)


def test_decode_beyond_2gib(torch, dev):
    """positions past 2^31 and 2^32 bytes: 26M R2 records (4.3 GB) generated and encoded in HBM,
    decoded in both modes and compared with the source columns on the device"""
    from kitex_amd.columns import alloc_device
    from kitex_amd.codec import status_tensor, read_status
    sch, cdc = codec("r2")
    n = 26_000_000
    src = synth.gen_r2_torch(n, dev)
    wire, offs = cdc.Marshal(src)
    assert wire.numel() > (1 << 32)
    infos = cdc.dschema.infos
    caps = [0 if ci.kind == A.COL_FIXED else int(src.cols[c][0][-1].item()) for c, ci in enumerate(infos)]
    for o in (None, offs):
        out = alloc_device(infos, n, caps, cdc.dschema.npresence, dev)
        st = status_tensor(dev)
        cdc.Unmarshal(wire, n, offsets=o, out=out, var_caps=caps, raise_on_error=False, status=st)
        s = read_status(st)
        assert s.code == 0 and s.n_records == n
        for c, ci in enumerate(infos):
            if ci.kind == A.COL_FIXED:
                assert torch.equal(out.cols[c], src.cols[c])
            else:
                assert torch.equal(out.cols[c][0], src.cols[c][0])
                assert torch.equal(out.cols[c][1][:caps[c]], src.cols[c][1][:caps[c]])
        del out
    del wire, src
    torch.cuda.empty_cache()


def test_decode_arena_beyond_4gib(torch, dev):
    """one string arena past 2^32 bytes: 2M records with a 2100-byte string (4.4 GB arena), encoded
    on the GPU from 8-byte-offset columns and decoded in both modes. 8-byte offsets give the source
    columns back; 4-byte offsets fail with SIZE_LIMIT instead of wrapping."""
    from kitex_amd.codec import ThriftCodec, read_status, status_tensor
    from kitex_amd.columns import alloc_device
    sch = S.Schema(S.Struct("Big", [S.Field(1, A.T_I64), S.Field(2, A.T_STRING), S.Field(3, A.T_STRING)]))
    cdc = ThriftCodec(sch)
    n, L = 1 << 21, 2100
    ids = torch.arange(n, dtype=torch.int64, device=dev) * 7 - 5
    big_off = torch.arange(n + 1, dtype=torch.int64, device=dev) * L
    big = (torch.arange(n * L, dtype=torch.int64, device=dev) % 251).to(torch.uint8)
    sm_len = (torch.arange(n, device=dev) % 5).to(torch.int64)
    sm_off = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    sm_off[1:] = torch.cumsum(sm_len, 0)
    small = (torch.arange(int(sm_off[-1]), device=dev) % 26 + 97).to(torch.uint8)
    src = synth.ColumnSet([ids, (big_off, big), (sm_off, small)], None, n)
    wire, offs = cdc.Marshal(src)
    assert big.numel() > (1 << 32) and wire.numel() > (1 << 32)
    infos = cdc.dschema.infos
    caps = [0, n * L, int(sm_off[-1])]
    for o in (None, offs):
        out = alloc_device(infos, n, caps, 0, dev, wide=True)
        st = status_tensor(dev)
        cdc.Unmarshal(wire, n, offsets=o, out=out, var_caps=caps, raise_on_error=False, status=st)
        s = read_status(st)
        assert s.code == 0 and s.n_records == n and s.var_total[0] == n * L
        assert torch.equal(out.cols[0], ids)
        assert torch.equal(out.cols[1][0], big_off) and torch.equal(out.cols[2][0], sm_off)
        assert torch.equal(out.cols[1][1], big) and torch.equal(out.cols[2][1][:small.numel()], small)
        del out
        narrow = alloc_device(infos, n, caps, 0, dev)
        st = status_tensor(dev)
        cdc.Unmarshal(wire, n, offsets=o, out=narrow, var_caps=caps, raise_on_error=False, status=st)
        assert read_status(st).code == A.ERR_SIZE_LIMIT
        del narrow
    del wire, offs, src, big
    torch.cuda.empty_cache()


# ---------------------------------------------------------------------------------------------
# host-memory entry point (kx_host_decode_batch: H2D -> decode -> D2H)
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("mode", ["concat", "offsets"])
@pytest.mark.parametrize("name", ["r2", "r3"])
def test_host_decode_matches_oracle(torch, oracle, name, mode):
    sch, cdc = codec(name)
    cs = synth.GENERATORS[name](20000, start=5)
    rc, wire, offs = oracle.encode(sch, cs)
    o = offs if mode == "offsets" else None
    out, st = cdc.UnmarshalHost(wire, cs.n, offsets=o)
    rc2, exp, est, _ = oracle.decode(sch, wire, cs.n, offsets=o)
    assert st.code == est.code == 0 and st.n_records == cs.n
    _, infos, _ = oracle.flatten(sch)
    from tests.helpers import assert_columns_equal
    assert_columns_equal(out, exp, infos, cs.n)


def test_host_decode_error_status(torch, oracle):
    sch, cdc = codec("r2")
    cs = synth.gen_r2(3000)
    rc, wire, offs = oracle.encode(sch, cs)
    wire = wire[:-5]
    out, st = cdc.UnmarshalHost(wire, cs.n, raise_on_error=False)
    _, _, est, _ = oracle.decode(sch, wire, cs.n)
    assert (st.code, st.record, st.offset) == (est.code, est.record, est.offset) and st.code == A.ERR_EOF


# ---------------------------------------------------------------------------------------------
# streams: a call on a side stream reports its own status; two streams never share a workspace
# ---------------------------------------------------------------------------------------------
def test_side_streams_status_and_workspaces(torch, dev, oracle):
    from kitex_amd.codec import ProtocolError, ThriftCodec
    sch = S.schema_r2()
    cdc = ThriftCodec(sch)
    batches = []
    for k in range(2):
        cs = synth.gen_r2(60000, start=1000 * k)
        rc, wire, _ = oracle.encode(sch, cs)
        if k == 1:
            wire = wire[:-9]                      # the second batch ends in a truncated record
        batches.append((cs, torch.from_numpy(wire).to(dev), oracle.decode(sch, wire, cs.n)))
    torch.cuda.synchronize()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    res = []
    for _ in range(3):                            # repeated, interleaved calls on both streams
        res = [cdc.Unmarshal(b[1], b[0].n, stream=s, raise_on_error=False) for b, s in zip(batches, (s1, s2))]
    assert len(cdc._ctxs) >= 3                    # the default stream's ctx + one per side stream
    _, infos, _ = oracle.flatten(sch)
    from tests.helpers import assert_columns_equal
    for (cs, _, (rc, exp, est, _)), r in zip(batches, res):
        st = r.read_status()
        assert (st.code, st.record, st.offset, st.n_records) == (est.code, est.record, est.offset, est.n_records)
        assert_columns_equal(r.columns, exp, infos, est.n_records)
    with pytest.raises(ProtocolError):
        cdc.Unmarshal(batches[1][1], batches[1][0].n, stream=s2)


# ---------------------------------------------------------------------------------------------
# the reference's own skip-decoder vectors through kx_thrift_skip_batch (codec_apache_test.go)
# ---------------------------------------------------------------------------------------------
def test_skip_batch_reference_fixture(torch, dev, oracle):
    """genTestSkipDecoderBytes (codec_apache_test.go:115-184: map<i64,double>, map<string,i64>,
    map<i64,struct>, list<struct>, nested struct) repeated 3000x, skipped on the GPU"""
    from kitex_amd.codec import ThriftCodec
    from tests.test_oracle_kat import gen_test_skip_decoder_bytes
    one = gen_test_skip_decoder_bytes(oracle)
    assert oracle.skip(one, A.T_STRUCT) == (0, len(one))
    n = 3000
    wire = np.frombuffer(one * n, dtype=np.uint8).copy()
    cdc = ThriftCodec(S.schema_r1())
    offs = to_np(cdc.Skip(torch.from_numpy(wire).to(dev), n))
    assert np.array_equal(offs, np.arange(n + 1, dtype=np.int64) * len(one))


def test_skip_batch_truncated_vector(torch, dev, oracle):
    """codec_apache_test.go:38-54: a struct cut after its first field header fails with EOF, at the
    same record and offset as the oracle"""
    from kitex_amd.codec import ProtocolError, ThriftCodec
    P = oracle.prim
    good = P("kxo_write_field_begin", A.T_BOOL, 1) + P("kxo_write_bool", 1) + P("kxo_write_field_stop")
    cut = P("kxo_write_field_begin", A.T_BOOL, 1)
    n = 5000
    wire = np.frombuffer(good * (n - 1) + cut, dtype=np.uint8).copy()
    exp_rc, exp_offs, done = oracle.skip_batch(wire, n)
    assert exp_rc == A.ERR_EOF and done == n - 1
    cdc = ThriftCodec(S.schema_r1())
    with pytest.raises(ProtocolError) as e:
        cdc.Skip(torch.from_numpy(wire).to(dev), n)
    assert (e.value.code, e.value.record, e.value.offset) == (A.ERR_EOF, n - 1, len(good) * (n - 1))


@pytest.mark.parametrize("name", ["r2", "r3", "pf"])
def test_host_decode_chunked_pipeline(torch, oracle, name):
    """kx_host_decode_batch / kx_host_pb_decode_batch with offsets and >= 65536 records: the 8-chunk
    pipeline (arena continued across chunks), field-for-field against the oracle; a failing record
    in the 5th chunk reports its global index"""
    from kitex_amd.codec import ProtobufCodec, ThriftCodec
    sch = S.SCHEMAS[name]()
    pb = name == "pf"
    cdc = ProtobufCodec(sch) if pb else ThriftCodec(sch)
    n = 100_000
    cs = synth.GENERATORS[name](n, start=17)
    rc, wire, offs = oracle.encode(sch, cs, pb=pb)
    if pb:  # bare bodies with known extents
        from tests.test_gpu_messages import _frame, _records
        bodies = _records(oracle, sch, cs, pb=True)
        wire, offs = _frame(bodies)
        offs = offs.astype(np.uint64)
    out, st = cdc.UnmarshalHost(wire, n, offsets=offs)
    rc2, exp, est, _ = oracle.decode(sch, wire, n, offsets=offs, pb=pb)
    assert st.code == est.code == 0 and st.n_records == n
    _, infos, _ = oracle.flatten(sch)
    from tests.helpers import assert_columns_equal
    assert_columns_equal(out, exp, infos, n)
    if not pb:
        bad = wire.copy()
        k = 63_000
        bad[int(offs[k])] = 99                    # an unknown field type in record k
        out, st = cdc.UnmarshalHost(bad, n, offsets=offs, raise_on_error=False)
        _, _, est, _ = oracle.decode(sch, bad, n, offsets=offs)
        assert (st.code, st.record, st.offset) == (est.code, est.record, est.offset) and st.record == k


@pytest.mark.parametrize("n", [20_000, 100_000])
@pytest.mark.parametrize("name", ["r2", "r3", "pf", "cx1", "cx2"])
def test_host_encode_bit_exact(torch, oracle, name, n):
    """kx_host_encode_batch / kx_host_pb_encode_batch (fastMarshal from host columns to host wire, the
    16-chunk pipeline at 100 000 records with each chunk's output placed by the previous chunk's device
    status): bytes and record offsets identical to the oracle's encoder"""
    from kitex_amd.codec import ProtobufCodec, ThriftCodec
    if name in DC.CONTAINER_SCHEMAS:   # list<string>, set<string>, maps: LIST_BYTES columns
        mk, gen = DC.CONTAINER_SCHEMAS[name]
        sch, cs = mk(), gen(n, start=23)
    else:
        sch, cs = S.SCHEMAS[name](), synth.GENERATORS[name](n, start=23)
    pb = name == "pf"
    cdc = ProtobufCodec(sch) if pb else ThriftCodec(sch)
    rc, exp, eoffs = oracle.encode(sch, cs, pb=pb)
    assert rc == 0
    wire, offs, st = cdc.MarshalHost(cs)
    assert st.code == 0 and st.consumed == exp.size
    assert np.array_equal(wire, exp)
    if pb:   # kx_pb_encode_batch's offsets are the Batch frame starts (the oracle's: the bodies)
        from tests import pb_cases as PC
        _, eoffs = PC.join(PC.split_frames(exp), framed=True)
    assert np.array_equal(offs.astype(np.uint64), eoffs.astype(np.uint64))
    # too small an output: SIZE_LIMIT, reported, never a partial overrun
    small = np.zeros(exp.size // 2, dtype=np.uint8)
    _, _, st2 = cdc.MarshalHost(cs, out=small, raise_on_error=False)
    # consumed = the size the whole batch needs (a caller sizes its retry from it)
    assert st2.code == A.ERR_SIZE_LIMIT and st2.consumed == exp.size and st2.n_records == n


@pytest.mark.parametrize("name", ["cx1", "cx2"])
@pytest.mark.parametrize("mode", ["concat", "offsets"])
@pytest.mark.parametrize("n", [1, 20000])
def test_decode_containers_match_oracle(gdec, oracle, name, mode, n):
    DC.case_containers(gdec, oracle, name, n, mode)


@pytest.mark.parametrize("et,w", DC.COOP_TYPES)
@pytest.mark.parametrize("mode", ["concat", "offsets"])
def test_coop_list_edges(gdec, oracle, et, w, mode):
    """the wave-cooperative list copy: i16 .. double elements, a 1500-element list, mostly empty lists"""
    DC.case_coop_lists(gdec, oracle, et, w, mode, n=5000)


@pytest.mark.parametrize("mode", ["concat", "offsets"])
def test_coop_list_arena_too_small(gdec, oracle, mode):
    """a list arena one element short: SIZE_LIMIT, as the oracle reports"""
    sch = DC.coop_schema(A.T_I64)
    cs = DC.coop_columns(A.T_I64, 8, 3000, seed=9)
    rc, wire, offs = oracle.encode(sch, cs)
    need = int(cs.cols[1][0][-1])
    caps = [0, need - 1, int(cs.cols[2][0][-1])]
    _, st, _ = gdec.decode(sch, wire, 3000, offsets=offs if mode == "offsets" else None, caps=caps)
    rc, _, est, _ = oracle.decode(sch, wire, 3000, offsets=offs if mode == "offsets" else None, var_caps=caps)
    assert st.code == est.code == A.ERR_SIZE_LIMIT


def test_mock_req_fault_vector_on_gpu(gdec, oracle):
    DC.case_mock_req_fault(gdec, oracle)


@pytest.mark.parametrize("name", ["cx1", "cx2"])
def test_encode_containers_bit_exact(torch, dev, oracle, name):
    """list<string> / set<string> / map columns written by the GPU encoder == the oracle's
    FastWriteNocopy bytes (maps in column order), and decode back to the source columns"""
    from kitex_amd.codec import ThriftCodec
    mk, gen = DC.CONTAINER_SCHEMAS[name]
    sch = mk()
    cdc = ThriftCodec(sch)
    cs = gen(20000, start=3)
    rc, wire, offs = oracle.encode(sch, cs)
    got, goffs = cdc.Marshal(cs_to_device(torch, dev, cs))
    assert np.array_equal(to_np(got), wire)
    assert np.array_equal(to_np(goffs), offs.astype(np.int64))
    DC.check_decode(GpuDecoder(torch, dev), oracle, sch, wire, cs.n)


@pytest.mark.parametrize("case", DC.VIEW_CASES)
def test_decode_views_match_oracle(gdec, oracle, case):
    DC.case_views(gdec, oracle, case)


def _r2_with_big_strings(n, big, seed=0):
    """R2 columns where a few records carry a huge string (the encoder's direct path and its
    wave-cooperative payload copies), the rest 0..40-byte strings at arbitrary alignments"""
    rng = np.random.default_rng(seed)
    cs = synth.gen_r2(n, start=seed)
    cols = list(cs.cols)
    for c in (8, 9):
        lens = rng.integers(0, 41, size=n)
        for i, L in big.items():
            if c == 8:
                lens[i] = L
        off = np.zeros(n + 1, np.uint32)
        off[1:] = np.cumsum(lens)
        cols[c] = (off, rng.integers(0, 256, size=max(1, int(off[-1])), dtype=np.uint8))
    return synth.ColumnSet(cols, None, n)


@pytest.mark.parametrize("big", [{5: 1 << 20}, {0: 8 << 20, 777: 1 << 20, 4999: 3000}])
def test_encode_huge_strings_bit_exact(torch, dev, oracle, big):
    """1 MiB and 8 MiB strings mixed into an R2 batch: bit-exact with the oracle, and decoded back"""
    sch, cdc = codec("r2")
    n = 5000
    cs = _r2_with_big_strings(n, big, seed=len(big))
    rc, wire, offs = oracle.encode(sch, cs)
    assert rc == 0
    got, goffs = cdc.Marshal(cs_to_device(torch, dev, cs))
    assert np.array_equal(to_np(got), wire)
    assert np.array_equal(to_np(goffs).astype(np.uint64), offs)


@pytest.mark.parametrize("et,w", [(A.T_I64, 8), (A.T_I32, 4), (A.T_I16, 2), (A.T_DOUBLE, 8), (A.T_BYTE, 1)])
def test_encode_long_lists_bit_exact(torch, dev, oracle, et, w):
    """list<scalar> of 0..3000 elements (R3-like large records: direct path, lists copied by the wave
    with every destination alignment), strings of 0..200 bytes between them"""
    from kitex_amd.codec import ThriftCodec
    sch = S.Schema(S.Struct("L", [S.Field(1, A.T_I32, "a"), S.Field(2, A.T_LIST, "v", elem=et),
                                  S.Field(3, A.T_STRING, "s"), S.Field(4, A.T_LIST, "u", elem=A.T_I64)]))
    cdc = ThriftCodec(sch)
    n = 3000
    rng = np.random.default_rng(w)
    dt = {1: np.uint8, 2: np.int16, 4: np.int32, 8: np.int64}[w]
    l1 = rng.integers(0, 3001, size=n)
    l1[::7] = 0
    o1 = np.zeros(n + 1, np.uint32); o1[1:] = np.cumsum(l1)
    v1 = rng.integers(-(1 << 62), 1 << 62, size=max(1, int(o1[-1]))).astype(dt)
    ls = rng.integers(0, 201, size=n)
    os_ = np.zeros(n + 1, np.uint32); os_[1:] = np.cumsum(ls)
    sd = rng.integers(0, 256, size=max(1, int(os_[-1])), dtype=np.uint8)
    l2 = rng.integers(0, 9, size=n)
    o2 = np.zeros(n + 1, np.uint32); o2[1:] = np.cumsum(l2)
    v2 = rng.integers(-(1 << 62), 1 << 62, size=max(1, int(o2[-1]))).astype(np.int64)
    cs = synth.ColumnSet([rng.integers(-9, 9, size=n).astype(np.int32), (o1, v1), (os_, sd), (o2, v2)],
                          np.zeros(n, np.uint64), n)   # containers: the schema has a presence word
    rc, wire, offs = oracle.encode(sch, cs)
    assert rc == 0
    got, goffs = cdc.Marshal(cs_to_device(torch, dev, cs))
    assert np.array_equal(to_np(got), wire)
    assert np.array_equal(to_np(goffs).astype(np.uint64), offs)
