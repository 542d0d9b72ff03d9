"""ctypes wrapper of oracle/build/liboracle.so (the C restatement) -- TEST INFRASTRUCTURE ONLY.

Same inputs/outputs as oracle.process_frames / oracle.spectrogram_pipeline,
float64 throughout, OpenMP over frames (used as the multi-core CPU baseline).
"""
from __future__ import annotations

import ctypes as ct
import os

import numpy as np

_LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "build", "liboracle.so")
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            raise RuntimeError(f"{_LIB} missing: run `make -C oracle`")
        _lib = ct.CDLL(_LIB)
        P = ct.c_void_p
        _lib.oracle_process.argtypes = [ct.c_int] * 6 + [ct.c_double] * 6 + [P] * 4 + [ct.c_int64] + [P] * 8 + [ct.c_int]
        _lib.oracle_process.restype = ct.c_int
        _lib.oracle_process2.argtypes = [ct.c_int] * 6 + [ct.c_double] * 6 + [P] * 4 + [ct.c_int64] + [P] * 9 + [ct.c_int]
        _lib.oracle_process2.restype = ct.c_int
        _lib.oracle_err2.argtypes = [P, P, ct.c_double, ct.c_int64, ct.c_int64, P, P, ct.c_int]
        _lib.oracle_err2.restype = None
        _lib.oracle_stft.argtypes = [P, ct.c_int64, P, ct.c_int, ct.c_int, ct.c_int, ct.c_double, ct.c_int, P, P, P,
                                     ct.c_int]
        _lib.oracle_stft.restype = ct.c_int64
        _lib.oracle_num_threads.restype = ct.c_int
    return _lib


def _p(a):
    return ct.c_void_p(0) if a is None else ct.c_void_p(a.ctypes.data)


def process_frames(iq, cal, p, wr, wd, want_cube=False, want_rd=False, nthreads=0, rd_out=None, cube_out=None,
                   want_pre=False):
    """rd_out / cube_out: preallocated complex128 [F][nr][nd] / [F][C][nr] that
    receive every row's Doppler spectrum / the range cube (no allocation per call;
    used by bench.py's CPU baseline and full-size check).  want_pre: also return
    'pre' [F], the energy entering the Doppler FFT (relaxed RD normalisation)."""
    iq = np.ascontiguousarray(iq, np.complex64)
    F, C, S = iq.shape
    nr, nd, M = p["nr"], p["nd"], p["max_targets"]
    out = dict(profile=np.zeros((F, nr)), tgt_count=np.zeros(F, np.int32), tgt_range_idx=np.zeros((F, M), np.int32),
               tgt_range_mag=np.zeros((F, M)), tgt_doppler_idx=np.zeros((F, M), np.int32), slow_mag=np.zeros((F, C)))
    cube = np.zeros((F, C, nr), np.complex128) if want_cube else None
    rd = np.zeros((F, nr, nd), np.complex128) if want_rd else None
    if rd_out is not None:
        assert rd_out.dtype == np.complex128 and rd_out.shape == (F, nr, nd) and rd_out.flags.c_contiguous
        rd = rd_out
    if cube_out is not None:
        assert cube_out.dtype == np.complex128 and cube_out.shape == (F, C, nr) and cube_out.flags.c_contiguous
        cube = cube_out
    pre = np.zeros(F) if want_pre else None
    c = np.ascontiguousarray(np.asarray(cal, np.complex128))
    wr = np.ascontiguousarray(wr, np.float64)
    wd = np.ascontiguousarray(wd, np.float64)
    st = lib().oracle_process2(S, C, nr, nd, M, int(p["doppler_fallback_idx"]), p["if_scale"], p["range_thr"],
                               p["doppler_thr"], p["min_d"], p["max_d"], p["dist_per_bin"], _p(wr), _p(wd), _p(c),
                               _p(iq), F, _p(out["profile"]), _p(out["tgt_count"]), _p(out["tgt_range_idx"]),
                               _p(out["tgt_range_mag"]), _p(out["tgt_doppler_idx"]), _p(out["slow_mag"]), _p(cube),
                               _p(rd), _p(pre), int(nthreads))
    if st != 0:
        raise RuntimeError("oracle_process failed")
    if want_cube or cube_out is not None:
        out["cube"] = cube
    if want_rd or rd_out is not None:
        out["rd"] = rd
    if want_pre:
        out["pre"] = pre
    return out


def err2(ref, got, unscale=1.0, nthreads=0):
    """Per-frame (sum |got*unscale - ref|^2, sum |ref|^2): ref complex128 [F][...],
    got complex64 (or float32 [..][2]) of the same shape."""
    ref = np.ascontiguousarray(ref, np.complex128)
    got = np.ascontiguousarray(got)
    if got.dtype == np.complex64:
        got = got.view(np.float32)
    assert got.dtype == np.float32 and got.size == 2 * ref.size
    F = ref.shape[0]
    n = ref.size // max(F, 1)
    num, den = np.zeros(F), np.zeros(F)
    lib().oracle_err2(_p(ref), _p(got), float(unscale), F, n, _p(num), _p(den), int(nthreads))
    return num, den


def spectrogram(x, prt, win, noverlap, nfft, nbins=1024, nthreads=0):
    x = np.ascontiguousarray(x, np.float64)
    w = np.ascontiguousarray(win, np.float64)
    hop = len(w) - noverlap
    nseg = (len(x) - noverlap) // hop
    nb = nfft // 2 + 1
    T = np.zeros(max(nseg, 0))
    Fq = np.zeros(nbins if nbins else nb)
    inten = np.zeros((max(nseg, 0), nbins if nbins else nb))
    got = lib().oracle_stft(_p(x), len(x), _p(w), len(w), noverlap, nfft, 1.0 / prt, nbins, _p(T), _p(Fq), _p(inten),
                            int(nthreads))
    if got < 1:
        raise ValueError("spectrogram: bad size")
    return dict(time=T, frequency=Fq, intensity=inten, nfft=nfft)


def max_threads() -> int:
    return lib().oracle_num_threads()
