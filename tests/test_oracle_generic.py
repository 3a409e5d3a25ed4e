"""CPU: the oracle's binary generic ingress (kxo_raw_messages / kxo_set_seqids, restating
binaryThriftCodec.Unmarshal / readBinaryMethod / SetSeqID, pkg/generic/binarythrift_codec.go:83-199),
pinned by the reference's GetSeqID / SetSeqID test bytes (binarythrift_codec_test.go)."""
import numpy as np

from tests import generic_cases as GC


def test_reference_seqid_vectors(oracle):
    for buf, seq in GC.REF_SEQID:
        wire = np.frombuffer(buf, dtype=np.uint8).copy()
        offs = np.array([0, len(buf)], dtype=np.uint64)
        rc, names, ty, sq, rs = oracle.raw_messages(wire, offs)
        assert rc == 0 and sq[0] == seq
        rc, out, rs = oracle.set_seqids(wire, offs, np.array([seq + 1], dtype=np.int32))
        rc2, _, _, sq2, _ = oracle.raw_messages(out, offs)
        assert rc == 0 and sq2[0] == seq + 1


def test_raw_batch_cases(oracle):
    wire, offs, exp_names, exp_codes = GC.raw_batch(200)
    rc, names, ty, sq, rs = oracle.raw_messages(wire, offs)
    assert list(rs) == exp_codes
    assert names == exp_names and list(sq) == GC.raw_seqids(200)
    rc, out, rs = oracle.set_seqids(wire, offs, np.arange(200, dtype=np.int32) + 1000)
    assert list(rs) == GC.set_codes(200)


def test_idl_request_schema_decodes_reference_message(oracle):
    """the MockReq schema compiled from the reference's mock.thrift decodes the reference's
    TestBinaryThriftCodec request body"""
    import os
    from kitex_amd.generic import schema_from_idl
    sch = schema_from_idl(os.path.join(os.path.dirname(__file__), "golden", "idl", "mock.thrift"), "Test")
    body = np.frombuffer(GC._empty_mockreq_body(), dtype=np.uint8).copy()
    rc, out, st, rs = oracle.decode(sch, body, 1, offsets=np.array([0, body.size], dtype=np.uint64))
    assert rc == 0 and st.code == 0 and rs[0] == 0
