"""Shared test helpers: column-set comparison (host numpy or device torch)."""
import numpy as np

from kitex_amd import _abi as A


def knob(L, name: str, value: int, default: int):
    """set one of the library's tuning switches (kx_knobs.h, read from the environment once per process) for
    the duration of a `with` block, through the test-only kx_debug_set_knob of library L (libkxcodec or
    the emulator)"""
    import contextlib
    import ctypes as C

    @contextlib.contextmanager
    def cm():
        L.kx_debug_set_knob.argtypes = [C.c_char_p, C.c_int]
        L.kx_debug_set_knob.restype = C.c_int
        assert L.kx_debug_set_knob(name.encode(), value) == 0, name
        try:
            yield
        finally:
            L.kx_debug_set_knob(name.encode(), default)
    return cm()


def to_np(x):
    if isinstance(x, np.ndarray):
        return x
    return x.detach().cpu().numpy()


def offsets_u64(x):
    """record offsets as int64 values: 4-byte columns hold uint32, 8-byte columns int64/uint64"""
    a = to_np(x)
    return a.view(np.uint64).astype(np.int64) if a.itemsize == 8 else a.view(np.uint32).astype(np.int64)


def _assert_list_bytes(got, exp, n, c, ci):
    """LIST_BYTES: per-record element counts, per-element lengths, element bytes"""
    go, ge, gd = (to_np(v) for v in got)
    eo, ee, ed = (to_np(v) for v in exp)
    go, eo = offsets_u64(go)[:n + 1], offsets_u64(eo)[:n + 1]
    assert np.array_equal(np.diff(go), np.diff(eo)), f"list column {c} (field {ci.field_id}) counts differ"
    ge = offsets_u64(ge)[int(go[0]):int(go[-1]) + 1]
    ee = offsets_u64(ee)[int(eo[0]):int(eo[-1]) + 1]
    assert np.array_equal(np.diff(ge), np.diff(ee)), f"list column {c} (field {ci.field_id}) element lengths differ"
    gb = gd.view(np.uint8)[int(ge[0]):int(ge[-1])]
    eb = ed.view(np.uint8)[int(ee[0]):int(ee[-1])]
    assert np.array_equal(gb, eb), f"list column {c} (field {ci.field_id}) bytes differ"


def _assert_levels(got, exp, n, c, ci):
    """any var column: each offsets array level by level (counts per parent), then the data they reach"""
    g = [to_np(v) for v in got]
    e = [to_np(v) for v in exp]
    glo, ghi, elo, ehi = 0, n, 0, n
    for k in range(len(g) - 1):
        ga = offsets_u64(g[k])[glo:ghi + 1]
        ea = offsets_u64(e[k])[elo:ehi + 1]
        bad = np.nonzero(np.diff(ga) != np.diff(ea))[0]
        assert bad.size == 0, f"column {c} (field {ci.field_id}) array {k} counts differ at {bad[:8]}"
        glo, ghi, elo, ehi = int(ga[0]), int(ga[-1]), int(ea[0]), int(ea[-1])
    gd, ed = g[-1], e[-1]
    w = gd.itemsize
    gb = gd.view(np.uint8)[glo * w:ghi * w]
    eb = ed.view(np.uint8)[elo * w:ehi * w]
    assert np.array_equal(gb, eb), f"column {c} (field {ci.field_id}) data differ"


def assert_columns_equal(got, exp, infos, n, check_presence=True):
    """Field-for-field equality of the first n records (fixed values, var bytes/elements, offsets)."""
    from kitex_amd.columns import Views
    for c, ci in enumerate(infos):
        if isinstance(got.cols[c], Views) or isinstance(exp.cols[c], Views):
            assert isinstance(got.cols[c], Views) and isinstance(exp.cols[c], Views), f"column {c}: view vs copy"
            g = to_np(got.cols[c].pairs)[:n].astype(np.uint64)
            e = to_np(exp.cols[c].pairs)[:n].astype(np.uint64)
            bad = np.nonzero((g != e).any(axis=1))[0]
            assert bad.size == 0, f"view column {c} (field {ci.field_id}) differs at records {bad[:8]}"
            continue
        if ci.kind == A.COL_FIXED:
            g = to_np(got.cols[c])[:n].view(np.uint8).reshape(n, -1) if n else None
            e = to_np(exp.cols[c])[:n].view(np.uint8).reshape(n, -1) if n else None
            if n:
                bad = np.nonzero((g != e).any(axis=1))[0]
                assert bad.size == 0, f"column {c} (field {ci.field_id}) differs at records {bad[:8]}"
        elif ci.kind in (A.COL_LIST_BYTES, A.COL_LIST2, A.COL_LIST2_BYTES) or ci.level > 0:
            _assert_levels(got.cols[c], exp.cols[c], n, c, ci)
        else:
            go, gd = (to_np(v) for v in got.cols[c])
            eo, ed = (to_np(v) for v in exp.cols[c])
            go = offsets_u64(go)[:n + 1]
            eo = offsets_u64(eo)[:n + 1]
            g0, e0 = int(go[0]), int(eo[0])
            go, eo = go - g0, eo - e0
            lg, le = np.diff(go), np.diff(eo)
            bad = np.nonzero(lg != le)[0]
            assert bad.size == 0, f"var column {c} (field {ci.field_id}) lengths differ at {bad[:8]}"
            tot = int(eo[-1])
            gb = gd.view(np.uint8)[g0 * gd.itemsize:(g0 + tot) * gd.itemsize]
            eb = ed.view(np.uint8)[e0 * ed.itemsize:(e0 + tot) * ed.itemsize]
            assert np.array_equal(gb, eb), f"var column {c} (field {ci.field_id}) payload differs"
    if check_presence and exp.presence is not None:
        assert got.presence is not None
        assert np.array_equal(to_np(got.presence)[:n].view(np.uint64), to_np(exp.presence)[:n].view(np.uint64))


def assert_rows_equal(got, exp, infos, rows):
    """got's records `rows` equal exp's records 0..len(rows)-1 (FIXED and BYTES columns)."""
    rows = np.asarray(rows, dtype=np.int64)
    m = rows.size
    for c, ci in enumerate(infos):
        if ci.kind == A.COL_FIXED:
            g = to_np(got.cols[c]).view(np.uint8).reshape(len(to_np(got.cols[c])), -1)[rows]
            e = to_np(exp.cols[c])[:m].view(np.uint8).reshape(m, -1)
            bad = np.nonzero((g != e).any(axis=1))[0]
            assert bad.size == 0, f"column {c} (field {ci.field_id}) differs at rows {rows[bad[:8]]}"
        elif ci.kind == A.COL_BYTES:
            go, gd = (to_np(v) for v in got.cols[c])
            eo, ed = (to_np(v) for v in exp.cols[c])
            go, eo = offsets_u64(go), offsets_u64(eo)
            gd, ed = gd.view(np.uint8), ed.view(np.uint8)
            for k, r in enumerate(rows):
                a = gd[int(go[r]):int(go[r + 1])]
                b = ed[int(eo[k]):int(eo[k + 1])]
                assert np.array_equal(a, b), f"var column {c} (field {ci.field_id}) differs at row {r}"
        else:
            raise NotImplementedError(ci.kind)


def random_columns(infos, npres, n, seed=0):
    """Random host columns for any flattened schema (test infrastructure): fixed values (bools 0/1),
    strings 0..40 bytes, lists of 0..5 elements, string lists of 0..4 strings of 0..12 bytes; a map's
    value column shares its key column's entry counts; every presence bit set."""
    from kitex_amd.synth import ColumnSet
    rng = np.random.default_rng(seed)
    fixed = {1: np.uint8, 2: np.int16, 4: np.int32, 8: np.int64}
    cols, counts = [], None
    for c, ci in enumerate(infos):
        is_val = bool(ci.elem_ttype & 0x80)
        # a list<struct> element field after the first of its list shares that list's counts
        if ci.elem_ttype & 0x40 and c > 0 and infos[c - 1].elem_ttype & 0x40 and \
                list(infos[c - 1].path[:ci.depth]) == list(ci.path[:ci.depth]):
            is_val = True
        et = ci.elem_ttype & 0x3F
        if ci.kind == A.COL_FIXED:
            v = rng.integers(0, 2, size=n) if ci.ttype == A.T_BOOL else rng.integers(-(1 << 62), 1 << 62, size=n)
            cols.append(v.astype(fixed[ci.width]))
            continue
        cnt = counts if is_val else rng.integers(0, 6 if ci.kind == A.COL_LIST else 5 if ci.kind == A.COL_LIST_BYTES
                                                 else 41, size=n)
        if (ci.ttype == A.T_MAP or ci.elem_ttype & 0x40) and not is_val:
            counts = cnt
        offs = np.zeros(n + 1, dtype=np.uint32)
        offs[1:] = np.cumsum(cnt)
        tot = int(offs[-1])
        if ci.kind == A.COL_BYTES:
            cols.append((offs, rng.integers(0, 256, size=max(1, tot), dtype=np.uint8)))
        elif ci.kind == A.COL_LIST:
            v = rng.integers(0, 2, size=max(1, tot)) if et == A.T_BOOL else rng.integers(-(1 << 62), 1 << 62,
                                                                                         size=max(1, tot))
            cols.append((offs, v.astype(fixed[ci.width])))
        else:
            el = rng.integers(0, 13, size=max(1, tot))[:tot]
            eo = np.zeros(tot + 1, dtype=np.uint32)
            eo[1:] = np.cumsum(el)
            cols.append((offs, eo, rng.integers(0, 256, size=max(1, int(eo[-1])), dtype=np.uint8)))
    pres = np.full(n, (1 << 64) - 1, dtype=np.uint64) if npres else None
    return ColumnSet(cols, pres, n)
