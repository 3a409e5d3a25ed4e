"""CPU: the Thrift codec-selection mirror (unmarshalThriftData / marshalThriftData, thrift_data.go:56-127;
IsDataLenDeterministic thrift.go:102-105; fastUnmarshal's skip-then-read, codec_fast.go:60-82)."""
import pytest

from kitex_amd.codec import CodecType as T, TypeCodec, KxError, select_marshal, select_unmarshal, \
    is_data_len_deterministic


@pytest.mark.parametrize("ct,dlen,tc,want", [
    (T.FastReadWrite, 100, TypeCodec(), "fast"),
    (T.FastReadWrite, 0, TypeCodec(), "fast"),                         # fallback: skip-then-read
    (T.FastRead | T.EnableSkipDecoder, 0, TypeCodec(), "fast"),
    (T.Basic, 100, TypeCodec(Apache=True), "apache"),
    (T.FastRead, 100, TypeCodec(FastCodec=False, Apache=True), "apache"),
    (T.FrugalRead, 100, TypeCodec(FastCodec=True, Frugal=True), "frugal"),
    (T.FrugalRead, 0, TypeCodec(FastCodec=True, Frugal=True, Apache=True), "apache"),  # dataLen unknown
    (T.FrugalRead | T.EnableSkipDecoder, 0, TypeCodec(FastCodec=False, Frugal=True), "frugal"),
    (T.Basic, 0, TypeCodec(FastCodec=False, Frugal=True), "frugal"),
])
def test_unmarshal_selection(ct, dlen, tc, want):
    assert select_unmarshal(ct, dlen, tc) == want


def test_mismatch_and_marshal():
    with pytest.raises(KxError):
        select_unmarshal(T.FastReadWrite, 10, TypeCodec(FastCodec=False))
    assert select_marshal(T.FastWrite) == "fast"
    assert select_marshal(T.FrugalWrite, TypeCodec(Frugal=True)) == "frugal"
    assert select_marshal(T.Basic, TypeCodec(Apache=True)) == "apache"
    assert not is_data_len_deterministic(T.FastRead, 0) and is_data_len_deterministic(T.EnableSkipDecoder, 0)
