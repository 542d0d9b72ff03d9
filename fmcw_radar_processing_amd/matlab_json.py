"""MATLAB ``jsonencode(..., 'PrettyPrint', true)`` semantics for the host mirror.

radar_processing.m writes every output through jsonencode (:315, :364, :392,
:425, :590).  The rules that matter for its payloads:
  * struct -> JSON object, fields in assignment order
  * numeric 1x1 -> number; 1xN or Nx1 -> flat array; MxN (M, N > 1) -> array
    of M rows (row-major); 0x0 -> []
  * NaN, Inf, -Inf -> null
  * char row -> string; logical -> true / false (also inside arrays)
  * doubles are printed with up to 15 significant digits
Consumers compare parsed numbers, not bytes.
"""
from __future__ import annotations

import math

import numpy as np


def _num(v) -> str:
    if isinstance(v, (bool, np.bool_)):     # an element of a logical array
        return "true" if v else "false"
    v = float(v)
    if math.isnan(v) or math.isinf(v):
        return "null"
    if v == int(v) and abs(v) < 1e15:
        return str(int(v))
    return "%.15g" % v


def _array(a: np.ndarray, ind: str, pretty: bool) -> str:
    a = np.asarray(a)
    if a.size == 0:
        return "[]"
    if a.ndim == 0 or a.size == 1 and a.ndim <= 2:
        return _num(a.reshape(-1)[0])
    if a.ndim == 1 or (a.ndim == 2 and (a.shape[0] == 1 or a.shape[1] == 1)):
        flat = a.reshape(-1)
        if pretty:
            inner = ind + "  "
            return "[\n" + ",\n".join(inner + _num(x) for x in flat) + "\n" + ind + "]"
        return "[" + ",".join(_num(x) for x in flat) + "]"
    if a.ndim == 2:
        if pretty:
            inner = ind + "  "
            rows = [inner + _array(r, inner, pretty) for r in a]
            return "[\n" + ",\n".join(rows) + "\n" + ind + "]"
        return "[" + ",".join(_array(r, "", False) for r in a) + "]"
    raise ValueError("only scalars, vectors and matrices are encoded")


def encode(obj, pretty: bool = True, ind: str = "") -> str:
    if isinstance(obj, dict):
        if not obj:
            return "{}"
        inner = ind + "  "
        if pretty:
            items = [f'{inner}"{k}": {encode(v, pretty, inner)}' for k, v in obj.items()]
            return "{\n" + ",\n".join(items) + "\n" + ind + "}"
        return "{" + ",".join(f'"{k}":{encode(v, False)}' for k, v in obj.items()) + "}"
    if isinstance(obj, str):
        return '"' + obj.replace("\\", "\\\\").replace('"', '\\"') + '"'
    if isinstance(obj, (bool, np.bool_)):
        return "true" if obj else "false"
    if isinstance(obj, (int, float, np.integer, np.floating)):
        return _num(obj)
    a = np.asarray(obj)
    return _array(a if a.dtype == np.bool_ else a.astype(np.float64), ind, pretty)


def matlab_squeeze_2d(a: np.ndarray) -> np.ndarray:
    """MATLAB squeeze on the Nr x 1 x F result of max(cube,[],2) (:265): an
    Nr x F matrix, or an Nr x 1 column when F == 1."""
    a = np.asarray(a)
    return a.reshape(a.shape[0], -1)
