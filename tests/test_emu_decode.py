"""CPU runs of the decode KERNEL SOURCE (kitex_amd/csrc/kx_decode.hip) under the SIMT emulator
(tests/emu): same parity cases as the GPU suite, oracle-checked. This covers the kernel's
cross-tile logic (speculative entries, repair rounds, decoupled look-back, error paths) on every
CPU test run; the emulator is test infrastructure and is never linked into the product."""
import numpy as np
import pytest

from kitex_amd import schema as S
from kitex_amd import synth
from kitex_amd import _abi as A
from tests import decode_cases as DC
from tests import frame_cases as FC
from tests import pb_cases as PC
from tests.emu import emu


class EmuDecoder:
    def __init__(self, oracle, threads=8):
        self.oracle = oracle
        self.threads = threads

    def decode(self, sch, wire, n, offsets=None, pb=False):
        _, infos, npres = self.oracle.flatten(sch)
        rc, out, st, rs = emu.decode(sch, infos, npres, wire, n, offsets=offsets, threads=self.threads, pb=pb)
        assert rc == 0, rc
        return out, st, rs

    def decode_views(self, sch, wire, n, offsets=None, pb=False, wide=False):
        _, infos, npres = self.oracle.flatten(sch)
        rc, out, st, rs = emu.decode(sch, infos, npres, wire, n, offsets=offsets, threads=self.threads, pb=pb,
                                     views=True, wide=wide)
        assert rc == 0, rc
        return out, st


@pytest.fixture(scope="module")
def edec(oracle):
    emu.lib()
    return EmuDecoder(oracle)


@pytest.mark.parametrize("name", ["r1", "r2", "r3"])
@pytest.mark.parametrize("n", [1, 7, 1000, 25000])
def test_emu_concat(edec, oracle, name, n):
    DC.case_concat(edec, oracle, name, n)


@pytest.mark.parametrize("name", ["r1", "r2", "r3"])
@pytest.mark.parametrize("n", [1, 300, 5000])
def test_emu_offsets(edec, oracle, name, n):
    DC.case_offsets(edec, oracle, name, n)


def test_emu_roundtrip(edec, oracle):
    DC.case_roundtrip(edec, oracle)


@pytest.mark.parametrize("mode", ["concat", "offsets"])
def test_emu_noncanonical(edec, oracle, mode):
    DC.case_noncanonical(edec, oracle, mode)


@pytest.mark.parametrize("mode", ["concat", "offsets"])
def test_emu_ragged(edec, oracle, mode):
    DC.case_ragged(edec, oracle, mode)


def test_emu_empty_records(edec, oracle):
    DC.case_empty(edec, oracle)


def test_emu_slot_overflow(edec, oracle):
    DC.case_slot_overflow(edec, oracle)


@pytest.mark.parametrize("case", ["r1", "r2", "r3", "pb", "containers", "noncanonical", "empty", "ragged", "skip"])
def test_emu_slotcap_64(edec, oracle, case):
    """64 record-start slots per tile (KX_SLOTCAP): every record past a tile's first 64 is emitted one per
    round from the previous record's end"""
    from tests.helpers import knob
    with knob(emu.lib(), "KX_SLOTCAP", 64, 0):
        _slotcap_case(edec, oracle, case)


def _slotcap_case(edec, oracle, case):
    if case in ("r1", "r2", "r3"):
        DC.case_concat(edec, oracle, case, 3000)
    elif case == "pb":
        PC.case_pb_concat(edec, oracle, 3000)
    elif case == "containers":
        DC.case_containers(edec, oracle, "cx1", 3000, "concat")
    elif case == "noncanonical":
        DC.case_noncanonical(edec, oracle, "concat")
    elif case == "empty":
        DC.case_empty(edec, oracle)
    elif case == "ragged":
        DC.case_ragged(edec, oracle, "concat")
    else:
        DC.case_skip(lambda wire, n: emu.skip(wire, n)[1], oracle)


def test_emu_nested(edec, oracle):
    DC.case_nested(edec, oracle)


@pytest.mark.parametrize("case", DC.ERROR_CASES)
def test_emu_errors(edec, oracle, case):
    DC.case_error(edec, oracle, case)


def test_emu_skip(edec, oracle):
    DC.case_skip(lambda wire, n: emu.skip(wire, n)[1], oracle)


@pytest.mark.parametrize("mode", ["concat", "offsets"])
def test_emu_r2_base_flat(edec, oracle, mode):
    """R2 + base.Base: 11 var slots on the flat pipeline (the 16-slot instantiation)"""
    from kitex_amd.codec import DeviceSchema
    assert not DeviceSchema(DC.schema_r2_base()).nested
    DC.case_r2_base(edec, oracle, mode, n=1500)


@pytest.mark.parametrize("mode", ["concat", "offsets"])
def test_emu_r2_base_repeated_struct(edec, oracle, mode):
    """a second 255:Base without Extra replaces the first wholesale: var slots 8..15 are reset too
    (vslot_mask is 16 bits)"""
    DC.case_r2_base(edec, oracle, mode, n=600, repeat=True)


def _emu_split(sch, wire, n, parts, skip=False):
    rc, pts, st = emu.split_points(None if skip else sch, wire, n, parts)
    assert rc == 0
    return pts, st


@pytest.mark.parametrize("case", DC.SPLIT_CASES)
def test_emu_split_points(edec, oracle, case):
    DC.case_split(_emu_split, oracle, case)


@pytest.mark.parametrize("case", ["r3", "noncanonical", "slot_overflow"])
def test_emu_split_points_skip_walker(edec, oracle, case):
    """the schema-free walker (nested schemas' split points)"""
    DC.case_split(lambda sch, w, n, p: _emu_split(sch, w, n, p, skip=True), oracle, case, parts_list=(3, 8))


def test_emu_split_points_errors(edec, oracle):
    DC.case_split_errors(_emu_split, oracle)


@pytest.mark.parametrize("name,n", [("r2", 75000), ("r3", 20000), ("r1", 60000)])
def test_emu_deep_lookback(oracle, name, n):
    """64 co-resident workgroups, one super-tile each: look-back windows that reach past their
    first 16 predecessors before finding an inclusive prefix"""
    DC.case_concat(EmuDecoder(oracle, threads=64), oracle, name, n)


def test_emu_deep_lookback_pb(oracle):
    PC.case_pb_concat(EmuDecoder(oracle, threads=64), oracle, 25000)


@pytest.mark.parametrize("name,n", [("r2", 120000), ("r3", 30000)])
def test_emu_persistent_loop(oracle, name, n):
    """3 workgroups, each looping over many super-tiles (the persistent grid of the GPU)"""
    DC.case_concat(EmuDecoder(oracle, threads=3), oracle, name, n)
    DC.case_offsets(EmuDecoder(oracle, threads=3), oracle, name, n // 4)


# ---- Kitex-Protobuf (same kernels, M_PB walker) ----
@pytest.mark.parametrize("n", [1, 7, 1000, 20000])
def test_emu_pb_concat(edec, oracle, n):
    PC.case_pb_concat(edec, oracle, n)


@pytest.mark.parametrize("n", [1, 300, 5000])
def test_emu_pb_offsets(edec, oracle, n):
    PC.case_pb_offsets(edec, oracle, n)


@pytest.mark.parametrize("mode", ["concat", "offsets"])
def test_emu_pb_noncanonical(edec, oracle, mode):
    PC.case_pb_noncanonical(edec, oracle, mode)


@pytest.mark.parametrize("mode", ["concat", "offsets"])
@pytest.mark.parametrize("case", PC.PB_ERRORS)
def test_emu_pb_errors(edec, oracle, case, mode):
    PC.case_pb_error(edec, oracle, case, mode)


@pytest.mark.parametrize("name", ["cx1", "cx2"])
@pytest.mark.parametrize("mode", ["concat", "offsets"])
def test_emu_containers(edec, oracle, name, mode):
    DC.case_containers(edec, oracle, name, 3000, mode)


@pytest.mark.parametrize("et,w", DC.COOP_TYPES)
@pytest.mark.parametrize("mode", ["concat", "offsets"])
def test_emu_coop_list_edges(edec, oracle, et, w, mode):
    DC.case_coop_lists(edec, oracle, et, w, mode, n=300)


def test_emu_mock_req_fault(edec, oracle):
    DC.case_mock_req_fault(edec, oracle)


@pytest.mark.parametrize("ahead", [0, 1, 3])
@pytest.mark.parametrize("case", DC.CHUNK_CASES)
def test_emu_chunked(edec, oracle, case, ahead, monkeypatch):
    """the chunked two-stream pipeline (64-tile chunks, index pass 0/1/3 chunks ahead of emit)"""
    monkeypatch.setenv("KX_EMU_CHUNK", "64")
    monkeypatch.setenv("KX_EMU_AHEAD", str(ahead))
    DC.case_chunked(edec, oracle, case)


# ---- framing sniff (M_FRAME walker, kx_launch_frames) ----
def _emu_scan(threads=8):
    def scan(wire, n, mx):
        rc, fo, ps, pe, kd, st = emu.frames(wire, n, mx, threads=threads)
        assert rc == 0, rc
        return fo, ps, pe, kd, st
    return scan


@pytest.mark.parametrize("case", FC.SCAN_CASES)
def test_emu_frames(edec, oracle, case):
    FC.case_scan(_emu_scan(), oracle, case)


@pytest.mark.parametrize("case", DC.VIEW_CASES)
def test_emu_views(edec, oracle, case):
    DC.case_views(edec, oracle, case)


@pytest.mark.parametrize("name,n", [("r1", 20000), ("r2", 15000), ("r3", 4000)])
def test_emu_fast_index_path_taken(edec, oracle, name, n):
    """canonical batches: every tile but the last few takes the fast index path (status diag[2] counts
    the tiles that fell back to walk_tile), and the decode equals the oracle's"""
    from tests.helpers import assert_columns_equal
    sch = S.SCHEMAS[name]()
    _, infos, npres = oracle.flatten(sch)
    rc, wire, _ = oracle.encode(sch, synth.GENERATORS[name](n, start=5))
    erc, cols, st, _ = emu.decode(sch, infos, npres, wire, n, threads=8)
    assert erc == 0 and st.code == 0 and st.n_records == n
    tiles = (wire.size + 8191) // 8192
    assert st.diag[2] <= 2, (st.diag[2], tiles)
    rc, exp, est, _ = oracle.decode(sch, wire, n)
    assert_columns_equal(cols, exp, infos, n)


def test_emu_long_strings(edec, oracle):
    """strings past the wave-copy threshold, inside and outside the tile window"""
    DC.case_long_strings(edec, oracle)


def test_emu_bimodal_no_chain_repair(edec, oracle):
    """1 % of the records at 64 KiB (tests/test_gpu_adversarial.py's batch, 20 000 records): decoded as the
    oracle does, and no group needs the chain pass's repair (a tile holding the start of a record longer
    than its window leaves the fast index path instead of reading as a tile with no record start)"""
    from tests.test_gpu_adversarial import _bimodal_batch
    sch = S.Schema(S.Struct("Bi", [S.Field(1, A.T_I64, "id"), S.Field(2, A.T_STRING, "s")]))
    _, _, _, wire = _bimodal_batch(20000)
    _, st = DC.check_decode(edec, oracle, sch, wire, 20000)
    assert st.code == 0 and (st.diag[0], st.diag[1]) == (0, 0), list(st.diag)


def test_emu_skip_encoder_order_nesting(oracle):
    """baseline.thrift Nesting records as Kitex's encoder writes them (fixed-length fields first: double,
    i32, i64, byte — the way its Simple elements start too): the skip decoder delimits them as the oracle
    does with no tile re-walk and no group re-scan (data_sig2)"""
    import os
    from kitex_amd import idl
    doc = idl.parse_idl(os.path.join(os.path.dirname(__file__), "golden", "idl", "baseline.thrift"))
    sch = idl.to_schema(doc.struct("Nesting"))
    recs = synth.thrift_records(sch, 1500, seed=7)
    wire = np.frombuffer(b"".join(recs), dtype=np.uint8).copy()
    _, infos, npres = oracle.flatten(sch)
    rc, out, st, _ = emu.nested_decode(sch, infos, npres, wire, 1500)
    assert rc == 0 and st.code == 0
    rc, w2, offs = emu.nested_encode(sch, infos, out)
    assert rc == 0 and w2[0] == A.T_DOUBLE          # encoder order: the double first
    rc, got, st = emu.skip(w2, 1500)
    assert rc == 0 and st.code == 0 and st.n_records == 1500
    assert np.array_equal(got, offs)
    assert (st.diag[0], st.diag[1]) == (0, 0), list(st.diag)


def test_emu_pb_frames_nested_no_repair():
    """Kitex-PB Batch frames of nested PN records (tests/pbn_cases.py: maps with string keys and repeated
    messages put 0x0A bytes inside every record): delimited exactly, and no group needs the chain pass's
    re-scan (a candidate frame must be followed by another; a lane tries its segment's later 0x0A bytes)"""
    from tests import pbn_cases as PB
    k = 4000
    _, bodies, boffs = PB.batch(k, seed=7, name="PN")
    lens = np.diff(boffs).astype(np.int64)
    recs = [b"\x0a" + PB.uvarint(int(lens[i])) + bodies[int(boffs[i]):int(boffs[i + 1])].tobytes() for i in range(k)]
    wire = np.frombuffer(b"".join(recs), dtype=np.uint8).copy()
    rc, fo, bs, be, st = emu.pb_frames(wire, k)
    exp = np.zeros(k + 1, dtype=np.uint64)
    exp[1:] = np.cumsum([len(r) for r in recs])
    assert rc == 0 and st.code == 0 and st.n_records == k
    assert np.array_equal(fo, exp)
    assert np.array_equal(be - bs, lens.astype(np.uint64))
    assert (st.diag[0], st.diag[1]) == (0, 0), list(st.diag)
