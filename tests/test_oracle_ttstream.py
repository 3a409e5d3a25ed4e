"""Oracle restatement of ttstream DecodeFrame (pkg/remote/trans/ttstream/frame.go:137-185) against
frames built by tests/tts_cases.py (the gopkg ttheader constants are the library's defaults:
kx_ttstream_default_keys, parity unpinned)."""
import numpy as np
import pytest

from kitex_amd import _abi as A
from kitex_amd import schema as S
from kitex_amd import synth
from tests import tts_cases as T


def test_oracle_ttstream_stream(oracle):
    keys = T.default_keys()
    sch = S.schema_r2()
    wire, info = T.stream_batch(oracle, sch, synth.gen_r2(500), keys)
    n = len(info)
    rc, fo, ps, pe, ft, sd, mp, ml, done = oracle.ttstream_frame_scan(wire, n, keys)
    assert rc == 0 and done == n and int(fo[n]) == wire.size
    for i, (t, sid, m, a, b) in enumerate(info):
        assert ft[i] == t and sd[i] == sid and (int(ps[i]), int(pe[i])) == (a, b)
        assert bytes(wire[int(mp[i]):int(mp[i]) + int(ml[i])]) == m
    # the DATA payloads are the records, decoded by FastRead at their extents
    data = [i for i in range(n) if ft[i] == A.TTS_DATA]
    assert len(data) == 500
    rc0, wire0, offs0 = oracle.encode(sch, synth.gen_r2(500))
    for j, i in enumerate(data[:50]):
        assert bytes(wire[int(ps[i]):int(pe[i])]) == bytes(wire0[int(offs0[j]):int(offs0[j + 1])])


def test_oracle_ttstream_keys_follow_caller(oracle):
    """another set of gopkg constants (key ids, type values, flag) is honoured"""
    keys = T.default_keys()
    keys.frame_type_key, keys.to_method_key, keys.streaming_flag = 30, 12, 0x40
    for k, nm in enumerate([b"meta", b"header", b"data", b"trailer", b"rst"]):
        keys.type_names[k].value = nm
    fb = T.frame(keys, 9, A.TTS_TRAILER, b"Foo", strinfo={b"a": b"b"}, acl=b"tok", ntrans=2)
    w = np.frombuffer(fb, dtype=np.uint8).copy()
    rc, fo, ps, pe, ft, sd, mp, ml, done = oracle.ttstream_frame_scan(w, 1, keys)
    assert rc == 0 and ft[0] == A.TTS_TRAILER and sd[0] == 9 and int(pe[0]) == w.size
    assert bytes(w[int(mp[0]):int(mp[0]) + int(ml[0])]) == b"Foo"
    rc, *_ = oracle.ttstream_frame_scan(w, 1, T.default_keys())  # default keys: no frame type -> error
    assert rc == A.ERR_INVALID_DATA


@pytest.mark.parametrize("case", T.ERROR_CASES)
def test_oracle_ttstream_errors(oracle, case):
    keys = T.default_keys()
    wire, bad, code, n = T.error_batch(oracle, keys, case)
    rc, fo, ps, pe, ft, sd, mp, ml, done = oracle.ttstream_frame_scan(wire, n, keys)
    assert rc == code and done == bad


# ---- the device frame walker's source under the SIMT emulator, against the oracle ----
@pytest.fixture(scope="module")
def emu_lib():
    from tests.emu import emu
    emu.lib()
    return emu


@pytest.mark.parametrize("n", [1, 200, 3000])
def test_emu_ttstream_matches_oracle(oracle, emu_lib, n):
    keys = T.default_keys()
    wire, info = T.stream_batch(oracle, S.schema_r2(), synth.gen_r2(n), keys, streams=4, seed=n)
    nf = len(info)
    exp = oracle.ttstream_frame_scan(wire, nf, keys)
    rc, fo, ps, pe, ft, sd, mp, ml, st = emu_lib.tts_frames(wire, nf, keys)
    assert rc == 0 and st.code == 0 and st.n_records == nf
    for got, want in zip((fo, ps, pe, ft, sd, mp, ml), exp[1:8]):
        assert np.array_equal(got, want)


@pytest.mark.parametrize("case", T.ERROR_CASES)
def test_emu_ttstream_errors(oracle, emu_lib, case):
    keys = T.default_keys()
    wire, bad, code, n = T.error_batch(oracle, keys, case)
    rc, fo, ps, pe, ft, sd, mp, ml, st = emu_lib.tts_frames(wire, n, keys)
    assert rc == 0 and st.code == code and st.record == bad, (st.code, st.record)
    e = oracle.ttstream_frame_scan(wire, n, keys)
    assert np.array_equal(fo[:bad], e[1][:bad]) and np.array_equal(ft[:bad], e[4][:bad])
