"""The per-type Go glue generator (kitex_amd/gogen.py): shape of the generated FillFromRow / VarBytes /
WriteToRow for the reference's flat request types, column indices against the library's own column table,
and the fall-through (NotImplementedError) for the shapes it leaves to the stock codec. The Go text is not
compiled (no Go toolchain in this image)."""
import os
import re

import pytest

from kitex_amd import gogen, idl
from kitex_amd import schema as S
from kitex_amd.codec import DeviceSchema

IDL = os.path.join(os.path.dirname(__file__), "golden", "idl")


def _balanced(src: str) -> bool:
    depth = 0
    for ch in re.sub(r'"[^"\n]*"', '""', src):
        depth += ch == "{"
        depth -= ch == "}"
        if depth < 0:
            return False
    return depth == 0


def _mockreq():
    return idl.to_schema(idl.parse_idl(os.path.join(IDL, "mock.thrift")).struct("MockReq"))


def _base():   # base.Base (base.thrift:10-17): strings, an optional struct, a map<string,string>
    return idl.to_schema(idl.parse_idl(os.path.join(IDL, "base.thrift")).struct("Base"))


@pytest.mark.parametrize("make", [_mockreq, _base, S.schema_r1, S.schema_r2, S.schema_r3, S.schema_cx1, S.schema_cx2])
def test_glue_shape(make):
    sch = make()
    src = gogen.go_glue(sch, "kxglue")
    t = gogen.go_name(sch.root.name)
    for sig in (f"func (p *{t}) FillFromRow(cols *C.kx_columns, row int) error {{",
                f"func (p *{t}) VarBytes() []uint64 {{",
                f"func (p *{t}) WriteToRow(cols *C.kx_columns, row int) error {{"):
        assert sig in src
    assert _balanced(src)
    ncols = len(DeviceSchema(sch).infos)
    used = {int(m) for m in re.findall(r"cols\.cols\[(\d+)\]", src)}
    assert used == set(range(ncols))   # every column, each index valid
    # every root field is read and written
    for f in sch.root.fields:
        name = gogen.go_name(f.name or f"field{f.id}")
        assert f"p.{name} =" in src.split("VarBytes")[0]
        assert f"p.{name}" in src.split("func (p *%s) WriteToRow" % t)[1]
    # one (units, elements) pair per var column
    nvar = sum(1 for ci in DeviceSchema(sch).infos if ci.kind != 1)
    body = src.split("func (p *%s) VarBytes" % t)[1].split("return u")[0]
    # (an absent struct's var columns append zeros in an else branch)
    present = re.sub(r"\} else \{[^}]*\}", "}", body)
    assert present.count("u = append(u,") == nvar


def test_mockreq_text():
    src = gogen.go_glue(_mockreq(), "mock", preamble=False)
    assert "p.StrMap = make(map[string]string, b-a)" in src
    assert "p.StrList = append(p.StrList, string(kxBytes(c, kxOff(c, c.elem_offsets, int(e))" in src
    assert "kxSetPresent(cols, row, 0, p.StrMap != nil)" in src
    # no name declared twice in one map entry's write
    assert "kb := kxOff(k, k.elem_offsets" in src and "vb := kxOff(v, v.elem_offsets" in src


def test_names():
    assert gogen.go_name("str_map") == "StrMap"
    assert gogen.go_name("Msg") == "Msg"
    assert gogen.go_name("log_id") == "LogId"


def test_fallthrough():
    doc = idl.parse_idl(os.path.join(IDL, "baseline.thrift"))
    with pytest.raises(NotImplementedError, match="ListSimple"):
        gogen.go_glue(idl.to_schema(doc.struct("Nesting")))
    with pytest.raises(NotImplementedError):
        gogen.go_glue(S.schema_pf_proto() if hasattr(S, "schema_pf_proto") else S.Schema(S.schema_pf().root,
                                                                                           protobuf=True))
