"""GPU parity of the host-memory entry points (kx_host_decode_batch / kx_host_pb_decode_batch /
kx_host_encode_batch / kx_host_pb_encode_batch, ABI 7) on the reference's own request shapes, through the
C-ABI, field-for-field / byte-for-byte against the oracle:

  mockreq  MockReq{Msg, map<string,string>, list<string>} (internal/mocks/thrift/mock.thrift:3-6, generated
           reader k-mock.go:39-114): flat LIST_BYTES columns;
  r2base   the R2 record carrying base.Base with Extra map<string,string> set (base.thrift:10-17);
  nesting  baseline.thrift NestingMethod's request (the nested record walker, 34 columns);
  pn       a nested Kitex-Protobuf message (every proto3 shape; the walker in proto mode).

100 000 records (the 16-chunk pipeline with offsets; one chunk when concatenated), a record failing inside
chunk 5 that reports only its own code (fastUnmarshal fails each message alone, codec_fast.go:60-71), and
the reply path bit-exact with a too-small output reporting the size the batch needs."""
import numpy as np
import pytest

from kitex_amd import _abi as A
from kitex_amd import schema as S
from tests import decode_cases as DC
from tests import nested_cases as NC
from tests import pbn_cases as P
from tests.helpers import assert_columns_equal, offsets_u64

pytestmark = pytest.mark.gpu

N = 100_000
DISTINCT = 2048
BAD = 33_333            # inside chunk 5 of 16 (records 31 250 .. 37 499)


@pytest.fixture(scope="module")
def torch():
    import torch as t
    if not t.cuda.is_available():
        pytest.skip("no GPU")
    return t


def _schema(name):
    if name == "mockreq":
        return S.schema_mockreq()
    if name == "r2base":
        return DC.schema_r2_base()
    if name == "nesting":
        from tests.test_nested import SCHEMAS
        return SCHEMAS["idl_nesting"]
    return P.schema_pn()


def _bodies(oracle, name, sch):
    """DISTINCT record bodies of the case (bytes)"""
    if name == "r2base":
        rng = np.random.default_rng(8)
        return [DC.r2_base_record(oracle, rng, i) for i in range(DISTINCT)]
    if name == "pn":
        _, w, o = P.batch(DISTINCT, seed=5)
    else:
        _, w, o = NC.batch(sch, DISTINCT, seed=5, noise=True)
    return [w[int(o[i]):int(o[i + 1])].tobytes() for i in range(DISTINCT)]


def _join(bodies, framed=False):
    if framed:   # Kitex-PB concatenated: the body of `message Batch { repeated Rec recs = 1; }`
        bodies = [b"\x0a" + P.uvarint(len(b)) + b for b in bodies]
    offs = np.zeros(len(bodies) + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(b) for b in bodies])
    return np.frombuffer(b"".join(bodies), dtype=np.uint8).copy(), offs


_cache = {}


def _case(oracle, name):
    if name not in _cache:
        sch = _schema(name)
        one = _bodies(oracle, name, sch)
        _cache[name] = (sch, [one[i % DISTINCT] for i in range(N)])
    return _cache[name]


def _codec(name, sch):
    from kitex_amd.codec import ProtobufCodec, ThriftCodec
    return ProtobufCodec(sch) if name == "pn" else ThriftCodec(sch)


def _caps(exp, infos, n):
    """the exact units of every column's arrays, from the oracle's decode (var, elem, sub capacities)"""
    var, elem, sub = [], [], []
    for c, ci in enumerate(infos):
        if ci.kind == A.COL_FIXED:
            var.append(0), elem.append(0), sub.append(0)
            continue
        hi, levels = n, []
        for arr in exp.cols[c][:-1]:
            hi = int(offsets_u64(arr)[hi])
            levels.append(hi)
        var.append(max(1, levels[-1]))
        elem.append(levels[0] if len(levels) >= 2 else 0)
        sub.append(levels[1] if len(levels) >= 3 else 0)
    return var, elem, sub


@pytest.mark.parametrize("mode", ["offsets", "concat"])
@pytest.mark.parametrize("name", ["mockreq", "r2base", "nesting", "pn"])
def test_host_decode_reference_shapes(torch, oracle, name, mode):
    sch, bodies = _case(oracle, name)
    pb = name == "pn"
    wire, offs = _join(bodies, framed=pb and mode == "concat")
    o = offs if mode == "offsets" else None
    rc, exp, est, _ = oracle.decode(sch, wire, N, offsets=o, pb=pb)
    assert est.code == 0
    _, infos, _ = oracle.flatten(sch)
    var, elem, sub = _caps(exp, infos, N)
    cdc = _codec(name, sch)
    out, st, rs = cdc.UnmarshalHost(wire, N, offsets=o, var_caps=var, elem_caps=elem, sub_caps=sub,
                                    record_status=True)
    assert st.code == 0 and st.n_records == N and st.consumed == wire.size
    assert not rs.any()
    assert_columns_equal(out, exp, infos, N)


@pytest.mark.parametrize("name", ["mockreq", "r2base", "nesting", "pn"])
def test_host_decode_failing_record_reports_alone(torch, oracle, name):
    """record BAD (chunk 5 of 16) is malformed: only it carries a code; every other record decodes"""
    sch, bodies = _case(oracle, name)
    pb = name == "pn"
    bodies = list(bodies)
    # Thrift: an unknown field type in the first header; proto: field 1 as a start-group tag (groups are
    # refused, protowire) followed by the rest of the record
    b = bodies[BAD]
    bodies[BAD] = (b"\x0b" + b) if pb else (b"\x63" + b[1:])
    wire, offs = _join(bodies)
    rc, exp, est, ers = oracle.decode(sch, wire, N, offsets=offs, pb=pb)
    assert est.code != 0 and est.record == BAD
    assert np.count_nonzero(ers) == 1
    _, infos, _ = oracle.flatten(sch)
    var, elem, sub = _caps(exp, infos, N)
    cdc = _codec(name, sch)
    out, st, rs = cdc.UnmarshalHost(wire, N, offsets=offs, var_caps=var, elem_caps=elem, sub_caps=sub,
                                    record_status=True, raise_on_error=False)
    assert (st.code, st.record, st.offset) == (est.code, est.record, est.offset)
    assert np.array_equal(rs, ers[:N])
    assert np.nonzero(rs)[0].tolist() == [BAD]
    assert_columns_equal(out, exp, infos, N)


@pytest.mark.parametrize("name", ["mockreq", "nesting"])
def test_host_decode_arena_too_small(torch, oracle, name):
    """one column's arena a unit short: SIZE_LIMIT, from the chunk that overflows on, and nothing past
    the arenas the caller gave"""
    sch, bodies = _case(oracle, name)
    wire, offs = _join(bodies)
    rc, exp, est, _ = oracle.decode(sch, wire, N, offsets=offs)
    _, infos, _ = oracle.flatten(sch)
    var, elem, sub = _caps(exp, infos, N)
    c = next(k for k, ci in enumerate(infos) if ci.kind != A.COL_FIXED and var[k] > 1)
    var[c] -= 1
    cdc = _codec(name, sch)
    out, st, rs = cdc.UnmarshalHost(wire, N, offsets=offs, var_caps=var, elem_caps=elem, sub_caps=sub,
                                    record_status=True, raise_on_error=False)
    assert st.code == A.ERR_SIZE_LIMIT
    assert rs[-1] == A.ERR_SIZE_LIMIT and rs.max() == A.ERR_SIZE_LIMIT


@pytest.mark.parametrize("name", ["mockreq", "r2base", "nesting", "pn"])
def test_host_encode_reference_shapes(torch, oracle, name):
    """the reply path: host columns -> host wire, bit-exact with the oracle's encoder at 100 000 records
    (16 chunks); too small an output is SIZE_LIMIT with consumed = the size the batch needs, and the
    records of the chunks that fitted are in `out`"""
    sch, bodies = _case(oracle, name)
    pb = name == "pn"
    wire, offs = _join(bodies)
    rc, cols, est, _ = oracle.decode(sch, wire, N, offsets=offs, pb=pb)
    assert est.code == 0
    rc, exp, eoffs = oracle.encode(sch, cols, pb=pb)
    assert rc == 0
    cdc = _codec(name, sch)
    got, goffs, st, rs = cdc.MarshalHost(cols, record_status=True)
    assert st.code == 0 and st.consumed == exp.size and not rs.any()
    assert np.array_equal(got, exp)
    if not pb:   # (a Kitex-PB batch's offsets are its frame starts)
        assert np.array_equal(goffs, eoffs.astype(np.uint64))
    small = np.zeros(exp.size // 2, dtype=np.uint8)
    w2, _, st2, rs2 = cdc.MarshalHost(cols, out=small, record_status=True, raise_on_error=False)
    assert st2.code == A.ERR_SIZE_LIMIT and st2.consumed == exp.size and st2.n_records == N
    ok = int(np.count_nonzero(rs2 == 0))
    assert rs2[ok:].min() == A.ERR_SIZE_LIMIT and ok == st2.record
    if ok and not pb:   # the chunks that fitted are complete records
        assert np.array_equal(small[:int(eoffs[ok])], exp[:int(eoffs[ok])])
