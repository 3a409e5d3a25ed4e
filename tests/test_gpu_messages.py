"""GPU parity of the message level (kx_thrift_decode_messages / kx_pb_decode_messages): N framed
RPC messages = MessageBegin (or the Kitex-PB meta header) + the method's Args struct holding one
record, decoded on the device and compared with the oracle (records) and with what was written
(method name, message type, seqid), including the MessageBegin KATs of binary_test.go:387-457."""
import numpy as np
import pytest

from kitex_amd import _abi as A
from kitex_amd import schema as S
from kitex_amd import synth
from tests.helpers import assert_columns_equal, to_np

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as t
    if not t.cuda.is_available():
        pytest.skip("no GPU")
    return t


def _records(oracle, sch, cs, pb=False):
    rc, wire, offs = oracle.encode(sch, cs, pb=pb)
    assert rc == 0
    if not pb:
        return [bytes(wire[int(offs[i]):int(offs[i + 1])]) for i in range(cs.n)]
    recs, pos, raw = [], 0, bytes(wire)   # Batch frames (0x0A, uvarint length, body): bare bodies
    for _ in range(cs.n):
        assert raw[pos] == 0x0A
        pos += 1
        ln = sh = 0
        while True:
            b = raw[pos]
            pos += 1
            ln |= (b & 0x7F) << sh
            sh += 7
            if b < 0x80:
                break
        recs.append(raw[pos:pos + ln])
        pos += ln
    return recs


def _frame(msgs):
    wire = np.frombuffer(b"".join(msgs), dtype=np.uint8).copy()
    offs = np.zeros(len(msgs) + 1, dtype=np.int64)
    offs[1:] = np.cumsum([len(m) for m in msgs])
    return wire, offs


def _decode(torch, cdc, wire, offs, n, **kw):
    dev = torch.device("cuda", 0)
    return cdc.UnmarshalMessages(torch.from_numpy(wire).to(dev), n, torch.from_numpy(offs).to(dev),
                                 raise_on_error=False, **kw)


def _expect(oracle, sch, recs):
    data, roffs = _frame(recs)
    rc, exp, est, ers = oracle.decode(sch, data, len(recs), offsets=roffs.astype(np.uint64))
    return exp, est, ers


@pytest.mark.parametrize("name", ["r2", "r3"])
def test_thrift_messages_match_oracle(torch, oracle, name):
    from kitex_amd.codec import ThriftCodec, write_message_begin
    sch = S.SCHEMAS[name]()
    cdc = ThriftCodec(sch)
    n = 5000
    recs = _records(oracle, sch, synth.GENERATORS[name](n, start=3))
    P = oracle.prim
    msgs, body = [], []
    for i, r in enumerate(recs):
        mb = write_message_begin(f"method{i % 7}", A.MSG_CALL if i % 5 else A.MSG_ONEWAY, i * 3 - 100)
        k = i % 10
        if k == 3:    # an unknown field before the record field (skipped: list<string>, map<i64,struct>)
            extra = (P("kxo_write_field_begin", A.T_LIST, 9) + P("kxo_write_list_begin", A.T_STRING, 2)
                     + P("kxo_write_string", b"ab", 2) + P("kxo_write_string", b"", 0)
                     + P("kxo_write_field_begin", A.T_MAP, 4) + P("kxo_write_map_begin", A.T_I64, A.T_STRUCT, 1)
                     + P("kxo_write_i64", 5) + P("kxo_write_field_begin", A.T_I32, 1) + P("kxo_write_i32", 1)
                     + b"\x00")
            args = extra + P("kxo_write_field_begin", A.T_STRUCT, 1) + r + b"\x00"
        elif k == 6:  # the record field, then an unknown one
            args = (P("kxo_write_field_begin", A.T_STRUCT, 1) + r + P("kxo_write_field_begin", A.T_STRING, 2)
                    + P("kxo_write_string", b"trailer", 7) + b"\x00")
        elif k == 8:  # no record field at all: an empty Args -> the record decodes as an empty struct
            args = b"\x00"
            r = b"\x00"
        else:
            args = P("kxo_write_field_begin", A.T_STRUCT, 1) + r + b"\x00"
        msgs.append(mb + args)
        body.append(r)
    wire, offs = _frame(msgs)
    res = _decode(torch, cdc, wire, offs, n)
    st = res.read_status()
    exp, est, ers = _expect(oracle, sch, body)
    assert st.code == est.code and st.n_records == n
    assert np.array_equal(to_np(res.record_status)[:n], ers[:n])
    _, infos, _ = oracle.flatten(sch)
    assert_columns_equal(res.columns, exp, infos, n)
    assert to_np(res.msg_type).tolist() == [A.MSG_CALL if i % 5 else A.MSG_ONEWAY for i in range(n)]
    assert to_np(res.seqid).tolist() == [i * 3 - 100 for i in range(n)]
    no = to_np(res.names[0])
    arena = bytes(to_np(res.names[1])[:int(no[n])])
    assert [arena[no[i]:no[i + 1]].decode() for i in range(n)] == [f"method{i % 7}" for i in range(n)]


@pytest.mark.parametrize("mtype", [A.MSG_CALL, A.MSG_REPLY, A.MSG_ONEWAY])
def test_message_begin_kat_through_device(torch, oracle, mtype):
    """binary_test.go:387-457: MessageBegin("messageBegin", type, 1) bytes, decoded on the GPU"""
    from kitex_amd.codec import ThriftCodec
    sch = S.schema_r1()
    cdc = ThriftCodec(sch)
    mb = bytes.fromhex(f"8001000{mtype}0000000c6d657373616765426567696e00000001")
    rec = _records(oracle, sch, synth.gen_r1(1))[0]
    wire, offs = _frame([mb + oracle.prim("kxo_write_field_begin", A.T_STRUCT, 1) + rec + b"\x00"])
    res = _decode(torch, cdc, wire, offs, 1)
    assert res.read_status().code == 0
    assert res.name(0) == "messageBegin" and int(res.msg_type[0]) == mtype and int(res.seqid[0]) == 1
    exp, _, _ = _expect(oracle, sch, [rec])
    _, infos, _ = oracle.flatten(sch)
    assert_columns_equal(res.columns, exp, infos, 1)


def test_message_errors(torch, oracle):
    """per-message codes: bad version, negative name length, truncated header, an EXCEPTION message,
    a truncated record, an unknown field type inside Args; the first failing message is the status"""
    from kitex_amd.codec import ThriftCodec, write_message_begin
    sch = S.schema_r2()
    cdc = ThriftCodec(sch)
    n = 600
    recs = _records(oracle, sch, synth.gen_r2(n, start=11))
    P = oracle.prim
    good = lambda i: write_message_begin("m", A.MSG_CALL, i) + P("kxo_write_field_begin", A.T_STRUCT, 1) + recs[i] + b"\x00"
    msgs = [good(i) for i in range(n)]
    want = {}
    msgs[100] = bytes.fromhex("00000005") + msgs[100][4:]; want[100] = A.ERR_BAD_VERSION
    msgs[150] = msgs[150][:4] + bytes.fromhex("fffffff0") + msgs[150][8:]; want[150] = A.ERR_NEGATIVE_SIZE
    msgs[200] = msgs[200][:6]; want[200] = A.ERR_EOF
    msgs[250] = write_message_begin("m", A.MSG_EXCEPTION, 1) + b"\x00"; want[250] = A.ERR_APPLICATION_EXCEPTION
    msgs[300] = msgs[300][:-20]; want[300] = A.ERR_EOF
    msgs[350] = write_message_begin("m", A.MSG_CALL, 1) + bytes([99, 0, 5]) + b"\x00"; want[350] = A.ERR_INVALID_DATA
    wire, offs = _frame(msgs)
    res = _decode(torch, cdc, wire, offs, n)
    st = res.read_status()
    rs = to_np(res.record_status)[:n]
    assert {i: int(rs[i]) for i in np.nonzero(rs)[0]} == want
    assert (st.code, st.record, st.offset) == (A.ERR_BAD_VERSION, 100, int(offs[100]))
    good_rows = [i for i in range(n) if i not in want]
    exp, _, _ = _expect(oracle, sch, [recs[i] for i in good_rows])
    _, infos, _ = oracle.flatten(sch)
    got = res.columns
    for j, c in enumerate(infos):
        if c.kind == A.COL_FIXED:
            assert np.array_equal(to_np(got.cols[j])[good_rows], to_np(exp.cols[j])[:len(good_rows)])


def test_pb_messages_match_oracle(torch, oracle):
    from kitex_amd.codec import ProtobufCodec, write_pb_meta
    sch = S.schema_pf()
    cdc = ProtobufCodec(sch)
    n = 4000
    recs = _records(oracle, sch, synth.gen_pf(n, start=9), pb=True)
    msgs = [write_pb_meta(f"pb{i % 3}", A.MSG_CALL, i) + r for i, r in enumerate(recs)]
    msgs[77] = bytes.fromhex("80010001") + msgs[77][4:]          # a thrift magic: bad version
    wire, offs = _frame(msgs)
    res = _decode(torch, cdc, wire, offs, n)
    st = res.read_status()
    assert (st.code, st.record) == (A.ERR_BAD_VERSION, 77)
    rs = to_np(res.record_status)[:n]
    assert np.nonzero(rs)[0].tolist() == [77]
    data, roffs = _frame(recs)
    rc, exp, est, ers = oracle.decode(sch, data, n, offsets=roffs.astype(np.uint64), pb=True)
    _, infos, _ = oracle.flatten(sch)
    rows = [i for i in range(n) if i != 77]
    for j, c in enumerate(infos):
        if c.kind == A.COL_FIXED:
            assert np.array_equal(to_np(res.columns.cols[j])[rows], to_np(exp.cols[j])[rows])
    assert to_np(res.seqid)[rows].tolist() == rows
    assert res.name(5) == "pb2"


@pytest.mark.parametrize("name,body_field,mtype", [("r2", 1, 1), ("r3", 0, 2)])
def test_marshal_messages_matches_oracle_and_round_trips(torch, oracle, name, body_field, mtype):
    """fastMarshal on the device (kx_thrift_encode_messages): every message equals the oracle's
    WriteMessageBegin + Args/Result wrapper + the oracle-encoded record + STOP, and decodes back"""
    import numpy as np
    from kitex_amd import schema as S, synth
    from kitex_amd.codec import ThriftCodec, write_message_begin
    from kitex_amd.columns import alloc_device  # noqa: F401
    from tests.helpers import assert_columns_equal
    n = 3000
    sch = S.SCHEMAS[name]()
    cs = synth.GENERATORS[name](n, start=11)
    rc, wire, offs = oracle.encode(sch, cs)
    assert rc == 0
    dev = torch.device("cuda:0")
    dcs = synth.ColumnSet([torch.from_numpy(c).to(dev) if not isinstance(c, tuple) else
                           tuple(torch.from_numpy(x.view(np.int32) if x.dtype == np.uint32 else x).to(dev) for x in c)
                           for c in cs.cols],
                          torch.from_numpy(cs.presence.view(np.int64)).to(dev) if cs.presence is not None else None, n)
    seq = torch.arange(n, dtype=torch.int32, device=dev) * 3 - 7
    cdc = ThriftCodec(sch)
    msgs, moffs = cdc.MarshalMessages(dcs, "Method_%s" % name, seq, msg_type=mtype, body_field=body_field)
    exp = b"".join(write_message_begin("Method_%s" % name, mtype, i * 3 - 7) + bytes([12, 0, body_field])
                   + bytes(wire[int(offs[i]):int(offs[i + 1])]) + b"\x00" for i in range(n))
    assert bytes(msgs.cpu().numpy()) == exp
    res = cdc.UnmarshalMessages(msgs, n, moffs, body_field=body_field)
    _, infos, _ = oracle.flatten(sch)
    rc, eout, est, _ = oracle.decode(sch, wire, n, offsets=offs)
    assert_columns_equal(res.columns, eout, infos, n)
    assert np.array_equal(res.seqid.cpu().numpy(), np.arange(n) * 3 - 7)
    assert (res.msg_type.cpu().numpy() == mtype).all()


def test_marshal_messages_short_scratch_is_size_limit(torch, oracle):
    """kx_thrift_encode_messages with a record scratch too small for the bodies and a large `out`: the
    call reports SIZE_LIMIT and the message pass never reads the (unwritten) record offsets"""
    import ctypes as C
    from kitex_amd import schema as S, synth
    from kitex_amd._lib import lib
    from kitex_amd.codec import ThriftCodec, read_status, status_tensor
    from kitex_amd.columns import to_kx_columns
    n = 4000
    dev = torch.device("cuda:0")
    sch = S.schema_r2()
    cdc = ThriftCodec(sch)
    src = synth.TORCH_GENERATORS["r2"](n, dev)
    body = int(cdc.BLength(src).sum().item())
    seq = torch.arange(n, dtype=torch.int32, device=dev)
    # run a bigger call first so the context's offset buffer holds stale entries past this call's n + 1
    big = synth.TORCH_GENERATORS["r2"](2 * n, dev)
    cdc.MarshalMessages(big, "m", torch.arange(2 * n, dtype=torch.int32, device=dev))
    nb = b"Method"
    for scratch_len in (1, body // 2, body - 1):
        scratch = torch.empty(scratch_len, dtype=torch.uint8, device=dev)
        out = torch.full((body * 4 + n * 64,), 0xAB, dtype=torch.uint8, device=dev)
        offs = torch.empty(n + 1, dtype=torch.int64, device=dev)
        st = status_tensor(dev)
        kc = to_kx_columns(src, cdc.dschema.infos)
        s = torch.cuda.current_stream()
        rc = lib().kx_thrift_encode_messages(cdc.ctx.handle, cdc.dschema.handle, C.byref(kc), n, nb, len(nb), 1,
                                             seq.data_ptr(), 1, scratch.data_ptr(), scratch.numel(), out.data_ptr(),
                                             out.numel(), offs.data_ptr(), st.data_ptr(), int(s.cuda_stream))
        assert rc == 0
        stt = read_status(st, s)
        assert stt.code == A.ERR_SIZE_LIMIT, (scratch_len, stt.code)
        assert bool((out == 0xAB).all()), "no message may be written from unwritten offsets"


def test_marshal_messages_checks_seqids(torch):
    from kitex_amd import schema as S, synth
    from kitex_amd._lib import KxError
    from kitex_amd.codec import ThriftCodec
    dev = torch.device("cuda:0")
    cdc = ThriftCodec(S.schema_r2())
    src = synth.TORCH_GENERATORS["r2"](100, dev)
    with pytest.raises(KxError):
        cdc.MarshalMessages(src, "m", torch.arange(50, dtype=torch.int32, device=dev))      # too short
    with pytest.raises(KxError):
        cdc.MarshalMessages(src, "m", torch.zeros(100, dtype=torch.float32, device=dev))   # not integers
    # int64 host tensor: converted (values fit) and moved to the device
    msgs, offs = cdc.MarshalMessages(src, "m", torch.arange(100, dtype=torch.int64))
    res = cdc.UnmarshalMessages(msgs, 100, offs)
    assert res.seqid.cpu().tolist() == list(range(100))
