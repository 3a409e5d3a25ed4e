"""Column buffers <-> the C-ABI's kx_columns struct (host numpy or device torch)."""
from __future__ import annotations

import ctypes as C
from typing import List, Sequence

import numpy as np

from . import _abi as A
from .synth import ColumnSet

_NP_FIXED = {1: np.uint8, 2: np.int16, 4: np.int32, 8: np.int64}


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


def to_kx_columns(cs: ColumnSet, infos: Sequence[A.ColumnInfo], caps: Sequence[int] = None) -> A.Columns:
    """Describe a ColumnSet to the C-ABI. `caps[c]` overrides a var column's arena capacity."""
    out = A.Columns()
    out.ncols = len(infos)
    for c, ci in enumerate(infos):
        if ci.kind == A.COL_FIXED:
            out.cols[c].data = _ptr(cs.cols[c])
            out.cols[c].offsets = 0
            out.cols[c].capacity = 0
        else:
            offs, data = cs.cols[c]
            out.cols[c].data = _ptr(data)
            out.cols[c].offsets = _ptr(offs)
            cap = caps[c] if caps is not None and caps[c] is not None else (
                data.numel() if hasattr(data, "numel") else data.size)
            out.cols[c].capacity = int(cap)
    out.presence = _ptr(cs.presence)
    return out


def alloc_host(infos: Sequence[A.ColumnInfo], n: int, var_caps: Sequence[int], npresence: int) -> ColumnSet:
    cols: List[object] = []
    for c, ci in enumerate(infos):
        if ci.kind == A.COL_FIXED:
            cols.append(np.zeros(n, dtype=_NP_FIXED[ci.width]))
        else:
            dt = np.uint8 if ci.kind == A.COL_BYTES else _NP_FIXED[ci.width]
            cols.append((np.zeros(n + 1, dtype=np.uint32), np.zeros(max(1, var_caps[c]), dtype=dt)))
    pres = np.zeros(n, dtype=np.uint64) if npresence else None
    return ColumnSet(cols, pres, n)


def alloc_device(infos: Sequence[A.ColumnInfo], n: int, var_caps: Sequence[int], npresence: int,
                 device, fill: int = None) -> ColumnSet:
    import torch
    tdt = {1: torch.uint8, 2: torch.int16, 4: torch.int32, 8: torch.int64}
    mk = torch.empty if fill is None else (lambda *a, **k: torch.full(*a[:1], fill, **k))
    cols: List[object] = []
    for c, ci in enumerate(infos):
        if ci.kind == A.COL_FIXED:
            cols.append(mk((n,), dtype=tdt[ci.width], device=device))
        else:
            dt = torch.uint8 if ci.kind == A.COL_BYTES else tdt[ci.width]
            cols.append((mk((n + 1,), dtype=torch.int32, device=device),
                         mk((max(1, var_caps[c]),), dtype=dt, device=device)))
    pres = mk((n,), dtype=torch.int64, device=device) if npresence else None
    return ColumnSet(cols, pres, n)


def var_caps_of(cs: ColumnSet, infos: Sequence[A.ColumnInfo]) -> List[int]:
    caps = []
    for c, ci in enumerate(infos):
        if ci.kind == A.COL_FIXED:
            caps.append(0)
        else:
            offs = cs.cols[c][0]
            caps.append(int(offs[-1]) & 0xFFFFFFFF)
    return caps
