"""Column buffers <-> the C-ABI's kx_columns struct (host numpy or device torch)."""
from __future__ import annotations

import ctypes as C
from typing import List, Sequence

import numpy as np

from . import _abi as A
from .synth import ColumnSet

_NP_FIXED = {1: np.uint8, 2: np.int16, 4: np.int32, 8: np.int64}


class Views:
    """A BYTES column in zero-copy view mode (KX_COLF_VIEW): pairs[n, 2] = (offset into the decode
    call's input, length), 4- or 8-byte integers; no arena."""

    def __init__(self, pairs):
        self.pairs = pairs

    def __repr__(self):
        return f"Views({tuple(self.pairs.shape)})"


def _ptr(x) -> int:
    if x is None:
        return 0
    if isinstance(x, np.ndarray):
        if x.size == 0:
            return 0 if x.ctypes.data is None else x.ctypes.data
        assert x.flags["C_CONTIGUOUS"]
        return x.ctypes.data
    # torch tensor
    assert x.is_contiguous()
    return x.data_ptr()


def _numel(x) -> int:
    return x.numel() if hasattr(x, "numel") else x.size


def _itemsize(x) -> int:
    return x.element_size() if hasattr(x, "element_size") else x.itemsize


def to_kx_columns(cs: ColumnSet, infos: Sequence[A.ColumnInfo], caps: Sequence[int] = None) -> A.Columns:
    """Describe a ColumnSet to the C-ABI. `caps[c]` lowers a var column's arena capacity (never
    above the arena actually allocated). Offsets may be 4- or 8-byte integers (kx_column.offset_bytes)."""
    out = A.Columns()
    out.ncols = len(infos)
    for c, ci in enumerate(infos):
        if ci.kind == A.COL_FIXED:
            out.cols[c].data = _ptr(cs.cols[c])
            out.cols[c].offsets = 0
            out.cols[c].capacity = 0
            continue
        parts = cs.cols[c]
        if isinstance(parts, Views):
            out.cols[c].offsets = _ptr(parts.pairs)
            out.cols[c].offset_bytes = _itemsize(parts.pairs)
            out.cols[c].flags = A.COLF_VIEW
            continue
        offs, data = parts[0], parts[-1]
        out.cols[c].data = _ptr(data)
        out.cols[c].offsets = _ptr(offs)
        out.cols[c].offset_bytes = _itemsize(offs)
        have = _numel(data)
        cap = caps[c] if caps is not None and caps[c] is not None else have
        out.cols[c].capacity = int(min(int(cap), have))
        if ci.kind in (A.COL_LIST_BYTES, A.COL_LIST2, A.COL_LIST2_BYTES):  # (record offsets, element offsets, ..)
            eoffs = parts[1]
            assert _itemsize(eoffs) == _itemsize(offs)
            out.cols[c].elem_offsets = _ptr(eoffs)
            out.cols[c].elem_capacity = max(0, _numel(eoffs) - 1)
        if ci.kind == A.COL_LIST2_BYTES:  # (.., inner element byte offsets, bytes)
            soffs = parts[2]
            assert _itemsize(soffs) == _itemsize(offs)
            out.cols[c].sub_offsets = _ptr(soffs)
            out.cols[c].sub_capacity = max(0, _numel(soffs) - 1)
    out.presence = _ptr(cs.presence)
    return out


def alloc_host(infos: Sequence[A.ColumnInfo], n: int, var_caps: Sequence[int], npresence: int,
               wide: bool = False, elem_caps: Sequence[int] = None, views: bool = False,
               sub_caps: Sequence[int] = None) -> ColumnSet:
    """Host columns. wide: 8-byte offsets. elem_caps[c]: element capacity of LIST_BYTES / LIST2 /
    LIST2_BYTES columns, sub_caps[c]: inner element capacity of LIST2_BYTES columns.
    views: BYTES columns as zero-copy (offset, length) views."""
    odt = np.uint64 if wide else np.uint32
    cols: List[object] = []
    for c, ci in enumerate(infos):
        ec = (elem_caps[c] if elem_caps is not None else max(1, var_caps[c])) if ci.kind != A.COL_FIXED else 0
        if views and ci.kind == A.COL_BYTES:
            cols.append(Views(np.zeros((max(1, n), 2), dtype=odt)))
        elif ci.kind == A.COL_FIXED:
            cols.append(np.zeros(n, dtype=_NP_FIXED[ci.width]))
        elif ci.kind == A.COL_LIST2:
            cols.append((np.zeros(n + 1, dtype=odt), np.zeros(ec + 1, dtype=odt),
                         np.zeros(max(1, var_caps[c]), dtype=_NP_FIXED[ci.width])))
        elif ci.kind == A.COL_LIST2_BYTES:
            sc = sub_caps[c] if sub_caps is not None else max(1, var_caps[c])
            cols.append((np.zeros(n + 1, dtype=odt), np.zeros(ec + 1, dtype=odt), np.zeros(sc + 1, dtype=odt),
                         np.zeros(max(1, var_caps[c]), dtype=np.uint8)))
        elif ci.kind == A.COL_LIST_BYTES:
            cols.append((np.zeros(n + 1, dtype=odt), np.zeros(ec + 1, dtype=odt),
                         np.zeros(max(1, var_caps[c]), dtype=np.uint8)))
        else:
            dt = np.uint8 if ci.kind == A.COL_BYTES else _NP_FIXED[ci.width]
            cols.append((np.zeros(n + 1, dtype=odt), np.zeros(max(1, var_caps[c]), dtype=dt)))
    pres = np.zeros(n, dtype=np.uint64) if npresence else None
    return ColumnSet(cols, pres, n)


def alloc_device(infos: Sequence[A.ColumnInfo], n: int, var_caps: Sequence[int], npresence: int,
                 device, fill: int = None, wide: bool = False, elem_caps: Sequence[int] = None,
                 views: bool = False, sub_caps: Sequence[int] = None) -> ColumnSet:
    """Device columns (torch). wide: 8-byte offsets (int64) instead of 4-byte (int32 storage of
    the unsigned offsets). views: BYTES columns as zero-copy (offset, length) views."""
    import torch
    tdt = {1: torch.uint8, 2: torch.int16, 4: torch.int32, 8: torch.int64}
    odt = torch.int64 if wide else torch.int32
    mk = torch.empty if fill is None else (lambda *a, **k: torch.full(*a[:1], fill, **k))
    cols: List[object] = []
    for c, ci in enumerate(infos):
        ec = (elem_caps[c] if elem_caps is not None else max(1, var_caps[c])) if ci.kind != A.COL_FIXED else 0
        if views and ci.kind == A.COL_BYTES:
            cols.append(Views(mk((max(1, n), 2), dtype=odt, device=device)))
        elif ci.kind == A.COL_FIXED:
            cols.append(mk((n,), dtype=tdt[ci.width], device=device))
        elif ci.kind == A.COL_LIST2:
            cols.append((mk((n + 1,), dtype=odt, device=device), mk((ec + 1,), dtype=odt, device=device),
                         mk((max(1, var_caps[c]),), dtype=tdt[ci.width], device=device)))
        elif ci.kind == A.COL_LIST2_BYTES:
            sc = sub_caps[c] if sub_caps is not None else max(1, var_caps[c])
            cols.append((mk((n + 1,), dtype=odt, device=device), mk((ec + 1,), dtype=odt, device=device),
                         mk((sc + 1,), dtype=odt, device=device),
                         mk((max(1, var_caps[c]),), dtype=torch.uint8, device=device)))
        elif ci.kind == A.COL_LIST_BYTES:
            cols.append((mk((n + 1,), dtype=odt, device=device), mk((ec + 1,), dtype=odt, device=device),
                         mk((max(1, var_caps[c]),), dtype=torch.uint8, device=device)))
        else:
            dt = torch.uint8 if ci.kind == A.COL_BYTES else tdt[ci.width]
            cols.append((mk((n + 1,), dtype=odt, device=device),
                         mk((max(1, var_caps[c]),), dtype=dt, device=device)))
    pres = mk((n,), dtype=torch.int64, device=device) if npresence else None
    return ColumnSet(cols, pres, n)


def var_caps_of(cs: ColumnSet, infos: Sequence[A.ColumnInfo]) -> List[int]:
    caps = []
    for c, ci in enumerate(infos):
        if ci.kind == A.COL_FIXED or isinstance(cs.cols[c], Views):
            caps.append(0)
        else:  # the last entry of the array that indexes the data (bytes / elements)
            offs = cs.cols[c][-2]
            caps.append(int(offs[-1]) & (0xFFFFFFFF if _itemsize(offs) == 4 else (1 << 64) - 1))
    return caps
