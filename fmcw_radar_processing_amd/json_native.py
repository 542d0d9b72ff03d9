"""Output files through libfmcw's native jsonencode writer (include/fmcw.h
fmcw_json_write; radar_processing.m:313-321, :362-369, :390-398, :424-431,
:590-593).  ``write(path, obj)`` takes the same struct-like dict as the Python
mirror ``matlab_json.encode`` and produces the same bytes; arrays are passed by
pointer and strides (a transposed numpy view is written without a copy)."""
from __future__ import annotations

import ctypes as ct

import numpy as np

from . import _lib

_KIND = {np.dtype(np.float32): _lib.FMCW_JSON_F32, np.dtype(np.float64): _lib.FMCW_JSON_F64,
         np.dtype(np.int32): _lib.FMCW_JSON_I32, np.dtype(np.uint8): _lib.FMCW_JSON_BOOL}


def _field(name: str, v, keep: list) -> _lib.JsonField:
    f = _lib.JsonField()
    f.name = name.encode()
    keep.append(f.name)
    if isinstance(v, str):
        b = v.encode()
        keep.append(b)
        f.kind, f.data = _lib.FMCW_JSON_STRING, ct.cast(ct.c_char_p(b), ct.c_void_p)
        return f
    a = np.asarray(v)
    if a.dtype == np.bool_:                  # MATLAB logical: true / false
        a = a.astype(np.uint8)
    elif np.issubdtype(a.dtype, np.integer):
        a = a.astype(np.int32) if a.size == 0 or (np.abs(a).max() < 2 ** 31) else a.astype(np.float64)
    elif a.dtype not in _KIND:
        a = a.astype(np.float64)
    if a.ndim == 0:
        a = a.reshape(1, 1)
    elif a.ndim == 1:
        a = a.reshape(1, -1)               # MATLAB row vector
    elif a.ndim != 2:
        raise ValueError(f"field {name}: only scalars, vectors and matrices are encoded")
    keep.append(a)
    isz = a.itemsize
    if any(st % isz for st in a.strides):
        a = np.ascontiguousarray(a)
        keep.append(a)
    f.kind = _KIND[a.dtype]
    f.data = a.ctypes.data if a.size else None
    f.rows, f.cols = a.shape
    f.row_stride, f.col_stride = a.strides[0] // isz, a.strides[1] // isz
    return f


def write(path: str, obj: dict, pretty: bool = True, threads: int = 0) -> int:
    """jsonencode(obj, 'PrettyPrint', pretty) to `path`; returns the bytes written."""
    keep = []
    fields = [_field(k, v, keep) for k, v in obj.items()]
    arr = (_lib.JsonField * max(1, len(fields)))(*fields)
    n = ct.c_int64()
    _lib.check(_lib.load().fmcw_json_write(str(path).encode(), arr, len(fields), int(pretty), int(threads),
                                           ct.byref(n)))
    return n.value
