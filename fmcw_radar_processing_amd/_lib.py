"""ctypes binding of libfmcw.so (include/fmcw.h).

The library is built in-tree (``fmcw_radar_processing_amd/libfmcw.so``, see
``csrc/Makefile`` / ``__graft_entry__.build``).  There is no CPU fallback:
if the shared object is missing, or no gfx950 device is present, the calls
raise ``FmcwError`` instead of silently computing elsewhere.
"""
from __future__ import annotations

import ctypes as ct
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FMCW_LIB", os.path.join(_HERE, "libfmcw.so"))

FMCW_OK = 0
FMCW_E_ARG, FMCW_E_HIP, FMCW_E_OOM, FMCW_E_STATE, FMCW_E_DATA = -1, -2, -3, -4, -5
FMCW_C64, FMCW_C32H = 0, 1
FMCW_PIPE_AUTO, FMCW_PIPE_STREAMS, FMCW_PIPE_ONEPASS, FMCW_PIPE_XCD = 0, 1, 3, 4
ABI_VERSION = 4
STATUS_NAMES = {0: "OK", -1: "E_ARG", -2: "E_HIP", -3: "E_OOM", -4: "E_STATE", -5: "E_DATA"}
STAGES = ("range", "doppler", "detect", "compact", "stft_power", "stft_db", "range_only", "range_doppler", "onepass",
          "render")


class FmcwError(RuntimeError):
    def __init__(self, status: int, msg: str):
        super().__init__(f"fmcw:{STATUS_NAMES.get(status, status)}: {msg}")
        self.status = status


class Params(ct.Structure):
    """fmcw_params (include/fmcw.h)."""
    _fields_ = [
        ("nts", ct.c_int32), ("pn", ct.c_int32), ("nr", ct.c_int32), ("nd", ct.c_int32),
        ("max_targets", ct.c_int32), ("doppler_fallback_idx", ct.c_int32),
        ("if_scale", ct.c_float), ("range_thr", ct.c_float), ("doppler_thr", ct.c_float),
        ("min_d", ct.c_float), ("max_d", ct.c_float), ("dist_per_bin", ct.c_float),
    ]


class JsonField(ct.Structure):
    """fmcw_json_field (include/fmcw.h)."""
    _fields_ = [("name", ct.c_char_p), ("kind", ct.c_int32), ("data", ct.c_void_p),
                ("rows", ct.c_int64), ("cols", ct.c_int64), ("row_stride", ct.c_int64), ("col_stride", ct.c_int64)]


FMCW_JSON_STRING, FMCW_JSON_F32, FMCW_JSON_F64, FMCW_JSON_I32, FMCW_JSON_BOOL = 0, 1, 2, 3, 4

_P = ct.c_void_p
_I32, _I64, _F, _D = ct.c_int32, ct.c_int64, ct.c_float, ct.c_double
_PP = ct.POINTER(Params)

# name -> (restype, argtypes); every symbol declared in include/fmcw.h
SIGNATURES = {
    "fmcw_abi_version": (_I32, []),
    "fmcw_last_error": (ct.c_char_p, []),
    "fmcw_device_count": (ct.c_int, [ct.POINTER(_I32)]),
    "fmcw_default_devices": (ct.c_int, [_I32, ct.POINTER(_I32), ct.POINTER(_I32)]),
    "fmcw_ctx_create": (ct.c_int, [_I32, ct.POINTER(_I32), ct.POINTER(_P)]),
    "fmcw_ctx_destroy": (ct.c_int, [_P]),
    "fmcw_ctx_devices": (ct.c_int, [_P, ct.POINTER(_I32), ct.POINTER(_I32), ct.POINTER(_I32)]),
    "fmcw_set_taps": (ct.c_int, [_P, _PP, _P, _P, _P]),
    "fmcw_process": (ct.c_int, [_P, _PP, _P, _I32, _I64, _P, _P, _P, _P, _P, _P, _P, _P, _I64, _P]),
    "fmcw_range_fft": (ct.c_int, [_P, _PP, _P, _I32, _I64, _P, _P]),
    "fmcw_stft_sizes": (ct.c_int, [_I64, _I32, _I32, _I32, _I32, ct.POINTER(_I64), ct.POINTER(_I32),
                                   ct.POINTER(_I32)]),
    "fmcw_stft": (ct.c_int, [_P, _P, _I64, _P, _I32, _I32, _I32, _D, _I32, _P, _P, _P]),
    "fmcw_process_device": (ct.c_int, [_P, _PP, _P, _I32, _I64, _P, _P, _P, _P, _P, _P, _P, _P, _I32, _I64,
                                       _P, _P]),
    "fmcw_range_fft_device": (ct.c_int, [_P, _PP, _P, _I32, _I64, _P, _I32, _P, _P]),
    "fmcw_process_slow_device": (ct.c_int, [_P, _PP, _P, _I32, _I64, _P, _P, _P, _P, _P, _P, _P, _I32, _P, _P, _P,
                                            _P]),
    "fmcw_compact_device": (ct.c_int, [_P, _P, _I64, _I32, _P, _P, _P]),
    "fmcw_stft_power_device": (ct.c_int, [_P, _P, _P, _P, _I32, _P, _I32, _P, _P, _I32, _I32, _I32, _D, _I64,
                                          _P, _P, _P, _P]),
    "fmcw_stft_db_device": (ct.c_int, [_P, _P, _P, _I64, _I32, _D, _P, _I32, _P, _P]),
    "fmcw_stft_db_direct_device": (ct.c_int, [_P, _P, _P, _P, _I32, _P, _I32, _P, _P, _I32, _I32, _I32, _D, _I64,
                                              _P, _P, _P]),
    "fmcw_synth_device": (ct.c_int, [_P, _PP, _I64, _I64, _P, _I32, _P]),
    "fmcw_timing_enable": (ct.c_int, [_P, _I32]),
    "fmcw_timing_read": (ct.c_int, [_P, _I32, ct.POINTER(_D), ct.POINTER(_I64)]),
    "fmcw_timing_reset": (ct.c_int, [_P]),
    "fmcw_set_chunk_frames": (ct.c_int, [_P, _I64]),
    "fmcw_set_pipeline": (ct.c_int, [_P, _I32]),
    "fmcw_synchronize": (ct.c_int, [_P]),
    "fmcw_rdx_clock": (ct.c_int, [_P, ct.POINTER(_D), ct.POINTER(_D)]),
    "fmcw_copy_device": (ct.c_int, [_P, _P, _P, _I64, _P]),
    "fmcw_json_write": (ct.c_int, [ct.c_char_p, ct.POINTER(JsonField), _I32, _I32, _I32, ct.POINTER(_I64)]),
    "fmcw_stft_png": (ct.c_int, [_P, _P, _I64, _P, _I32, _I32, _I32, _D, _I32, _P, _P, _P, ct.c_char_p, _I32, _I32,
                                 ct.POINTER(_I64)]),
    "fmcw_render_spectrogram_device": (ct.c_int, [_P, _P, _I32, _P, _P, _I32, _D, _D, _D, _I32, _I32, _P, _P]),
}

_lib = None


def load() -> ct.CDLL:
    """Load libfmcw.so once; raise loudly (no fallback) if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    # torch bundles its own libamdhip64.so.7 (same SONAME as /opt/rocm's): when
    # both are used in one process, torch's copy must be the one loaded first
    # so that libfmcw binds to the same HIP runtime instead of a second one.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(LIB_PATH):
        raise FmcwError(FMCW_E_HIP, f"{LIB_PATH} not found: build it with "
                        "`python -c 'import __graft_entry__ as g; g.build()'` (no CPU fallback exists)")
    lib = ct.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.fmcw_abi_version() != ABI_VERSION:
        raise FmcwError(FMCW_E_STATE, "libfmcw ABI version mismatch")
    _lib = lib
    return lib


def check(status: int) -> None:
    if status != FMCW_OK:
        msg = load().fmcw_last_error()
        raise FmcwError(status, msg.decode() if msg else "")
