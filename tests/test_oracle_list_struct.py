"""CPU: list<struct> in the oracle (restating FieldFastReadList / StructLikeFastRead / FieldFastWriteList,
struct_tpl.go:41-149, 583-625, 1011-1036), the schema compiler's columns, and the decode kernel source
under the SIMT emulator against the oracle."""
import struct

import numpy as np
import pytest

from kitex_amd import _abi as A
from kitex_amd import schema as S
from tests import list_struct_cases as LC
from tests.helpers import assert_columns_equal, offsets_u64


def test_columns_match_device_schema(oracle):
    from kitex_amd.codec import DeviceSchema
    sch = S.schema_ls1()
    ds = DeviceSchema(sch)
    rc, infos, npres = oracle.flatten(sch)
    assert rc == 0 and ds.ncols == len(infos) == 7 and ds.npresence == npres
    for a, b in zip(ds.infos, infos):
        assert bytes(a) == bytes(b)
    assert [ci.elem_ttype for ci in infos[1:5]] == [A.T_I64 | 0x40, A.T_I32 | 0x40, A.T_DOUBLE | 0x40, A.T_BOOL | 0x40]


def test_other_element_structs_are_nested(oracle):
    """element structs with strings or optional fields: the nested model (include/kxcodec.h), in both the
    library and the oracle; the optional field's bit lives in the elements' presence column"""
    from kitex_amd.codec import DeviceSchema
    wide = [S.Struct("E", [S.Field(1, A.T_STRING, "s")]),
            S.Struct("E", [S.Field(1, A.T_I64, "x", req=A.REQ_OPTIONAL)])]
    for k, es in enumerate(wide):
        sch = S.Schema(S.Struct("R", [S.Field(1, A.T_LIST, "l", elem=A.T_STRUCT, child=es)]))
        rc, infos, _ = oracle.flatten(sch)
        assert rc == 0 and DeviceSchema(sch).nested
        assert infos[0].kind == (A.COL_LIST_BYTES if k == 0 else A.COL_LIST)
        if k == 1:
            assert infos[-1].elem_ttype == A.ELEM_PRESENCE and infos[0].presence_bit == 0


def test_handmade_semantics(oracle):
    sch = S.schema_ls1()
    recs = LC.handmade()
    wire, offs = LC.wire_of(recs)
    rc, out, st, rs = oracle.decode(sch, wire, len(recs), offsets=offs)
    assert rc == 0 and list(rs) == [0] * len(recs)
    cnt = np.diff(offsets_u64(out.cols[1][0])[:6])
    assert list(cnt) == [2, 1, 2, 0, 1]
    xs = out.cols[1][1][:6].view(np.int64)
    ys = out.cols[2][1][:6].view(np.int32)
    ws = out.cols[3][1][:6].view(np.float64)
    bs = out.cols[4][1][:6]
    assert list(xs) == [10, -1, 5, 77, 0, 9]          # dup x: last wins; missing x: default 0
    assert list(ys) == [20, 7, 6, 2, 5, 9]
    assert list(ws) == [2.5, 1.5, 1.5, 1.5, 1.5, 1.5]  # mistyped id 3 (i32) skipped: default 1.5
    assert list(bs) == [1, 0, 0, 0, 0, 0]
    assert list(np.diff(offsets_u64(out.cols[5][0])[:6])) == [0, 0, 2, 0, 0]
    assert list(out.cols[5][1][:2].view(np.int16)) == [1, -3] and list(out.cols[6][1][:2]) == [2, 255]


def test_missing_required_element_field(oracle):
    sch = S.schema_ls1()
    wire, offs = LC.wire_of([LC.missing_required()])
    rc, out, st, rs = oracle.decode(sch, wire, 1, offsets=offs)
    assert st.code == A.ERR_INVALID_DATA and rs[0] == A.ERR_INVALID_DATA


def test_round_trip(oracle):
    sch, infos, npres, cs, wire, offs = LC.random_batch(oracle, 400)
    for o in (offs, None):
        rc, out, st, rs = oracle.decode(sch, wire, 400, offsets=o)
        assert rc == 0 and st.code == 0
        assert_columns_equal(out, cs, infos, 400, check_presence=False)
    rc2, wire2, _ = oracle.encode(sch, out)
    assert rc2 == 0 and np.array_equal(wire2, wire)


@pytest.mark.parametrize("mode", ["offsets", "concat"])
def test_emu_matches_oracle(oracle, mode):
    from tests.emu import emu
    sch, infos, npres, cs, wire, offs = LC.random_batch(oracle, 3000)
    hm, hoffs = LC.wire_of(LC.handmade() + [LC.missing_required()] if mode == "offsets" else LC.handmade())
    for w, o, n in ((wire, offs, 3000), (hm, hoffs, int(hoffs.size - 1))):
        oo = o if mode == "offsets" else None
        rc, exp, est, ers = oracle.decode(sch, w, n, offsets=oo)
        rc2, got, gst, grs = emu.decode(sch, infos, npres, w, n, offsets=oo)
        assert rc2 == 0 and gst.code == est.code and gst.record == est.record
        if mode == "offsets":
            assert np.array_equal(grs, ers)
        ok = n if est.code == 0 else int(est.record)
        assert_columns_equal(got, exp, infos, ok)
