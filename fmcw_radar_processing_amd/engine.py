"""Python handle on one libfmcw context (one HIP device, one stream).

Two call styles, both straight through the C-ABI of include/fmcw.h:

* host arrays (numpy) -- the same sequence a MEX gateway performs for MATLAB
  (``process``, ``range_fft``, ``stft``);
* device buffers (torch tensors used purely as HBM allocations, plus the
  torch stream) -- ``process_device`` and friends, for benches and the
  multi-GPU driver.
"""
from __future__ import annotations

import contextlib
import ctypes as ct

import numpy as np

from . import _lib
from ._lib import FMCW_C32H, FMCW_C64, STAGES, FmcwError, check
from .params import FmcwConfig


def _ptr(a) -> ct.c_void_p:
    if a is None:
        return ct.c_void_p(0)
    if isinstance(a, np.ndarray):
        return ct.c_void_p(a.ctypes.data)
    return ct.c_void_p(int(a.data_ptr()))      # torch tensor (device pointer)


def _host_iq(iq: np.ndarray):
    """complex64 [F][C][S]  or  float16 [F][C][S][2] -> (array, dtype code)."""
    if iq.dtype == np.complex64:
        return np.ascontiguousarray(iq), FMCW_C64
    if iq.dtype == np.float16 and iq.shape[-1] == 2:
        return np.ascontiguousarray(iq), FMCW_C32H
    if np.iscomplexobj(iq):
        return np.ascontiguousarray(iq.astype(np.complex64)), FMCW_C64
    raise TypeError("iq must be complex64 [F][C][S] or float16 [F][C][S][2]")


class Engine:
    """fmcw_ctx on HIP device ``device`` -- an int, or a list of device ids for
    one context over several GPUs (the host-array calls then shard their work
    over them; include/fmcw.h fmcw_ctx_create).  No CPU fallback: raises if a
    device is absent."""

    def __init__(self, device: int | list | tuple | None = 0):
        self.lib = _lib.load()
        if device is None:                       # FMCW_DEVICES, else every visible device
            device = default_devices()
        ids = [int(device)] if isinstance(device, int) else [int(d) for d in device]
        arr = (ct.c_int32 * len(ids))(*ids)
        h = ct.c_void_p()
        check(self.lib.fmcw_ctx_create(len(ids), arr, ct.byref(h)))
        self.h = h
        self.device = ids[0]
        self.devices = ids
        self.cfg: FmcwConfig | None = None
        self.p = None

    def device_info(self) -> dict:
        """{'devices': [...], 'rccl': bool} of this context."""
        n, rc = ct.c_int32(), ct.c_int32()
        ids = (ct.c_int32 * 64)()
        check(self.lib.fmcw_ctx_devices(self.h, ct.byref(n), ids, ct.byref(rc)))
        return {"devices": list(ids[: n.value]), "rccl": bool(rc.value)}

    def close(self):
        if getattr(self, "h", None):
            self.lib.fmcw_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- setup ---------------------------------------------------------------
    def set_taps(self, cfg: FmcwConfig, cal: np.ndarray, range_win: np.ndarray | None = None,
                 doppler_win: np.ndarray | None = None) -> None:
        """radar_processing.m:138-139 windows and :174 calib_rx1 to the device."""
        wr = np.ascontiguousarray(cfg.range_window() if range_win is None else range_win, np.float32)
        wd = np.ascontiguousarray(cfg.doppler_window() if doppler_win is None else doppler_win, np.float32)
        c = np.ascontiguousarray(np.asarray(cal, np.complex128).astype(np.complex64))
        if wr.shape != (cfg.nts,) or wd.shape != (cfg.pn,) or c.shape != (cfg.nts,):
            raise ValueError("taps have the wrong length")
        self.cfg, self.p = cfg, cfg.abi()
        check(self.lib.fmcw_set_taps(self.h, ct.byref(self.p), _ptr(wr), _ptr(wd), _ptr(c)))

    def set_chunk_frames(self, n: int) -> None:
        check(self.lib.fmcw_set_chunk_frames(self.h, int(n)))

    def set_pipeline(self, mode: int) -> None:
        """FMCW_PIPE_AUTO / _STREAMS / _ONEPASS (include/fmcw.h)."""
        check(self.lib.fmcw_set_pipeline(self.h, int(mode)))

    # ---- host-array API --------------------------------------------------------
    def process(self, iq: np.ndarray, want_cube: bool = False, want_rd: bool = False,
                probe_column: int = 0) -> dict:
        """Per-frame stages (:197-261, :265) over iq[F][C][S]."""
        cfg = self._need()
        iq, dt = _host_iq(iq)
        F = iq.shape[0]
        if iq.shape[1:3] != (cfg.pn, cfg.nts):
            raise ValueError(f"iq must be [F][{cfg.pn}][{cfg.nts}]")
        M = cfg.max_targets
        out = dict(profile=np.empty((F, cfg.nr), np.float32), tgt_count=np.empty(F, np.int32),
                   tgt_range_idx=np.empty((F, M), np.int32), tgt_range_mag=np.empty((F, M), np.float32),
                   tgt_doppler_idx=np.empty((F, M), np.int32), slow_mag=np.empty((F, cfg.pn), np.float32))
        cube = np.empty((F, cfg.pn, cfg.nr), np.complex64) if want_cube else None
        rd = np.empty((F, cfg.nr, cfg.nd), np.complex64) if want_rd else None
        probe = np.empty(cfg.nr, np.float32) if probe_column else None
        check(self.lib.fmcw_process(self.h, ct.byref(self.p), _ptr(iq), dt, F, _ptr(out["profile"]),
                                    _ptr(out["tgt_count"]), _ptr(out["tgt_range_idx"]), _ptr(out["tgt_range_mag"]),
                                    _ptr(out["tgt_doppler_idx"]), _ptr(out["slow_mag"]), _ptr(cube), _ptr(rd),
                                    int(probe_column), _ptr(probe)))
        if want_cube:
            out["cube"] = cube
        if want_rd:
            out["rd"] = rd
        if probe is not None:
            out["probe_mag"] = probe
        return out

    def range_fft(self, iq: np.ndarray):
        """Config-2 range stage: (cube [F][C][Nr] complex64, profile [F][Nr])."""
        cfg = self._need()
        iq, dt = _host_iq(iq)
        F = iq.shape[0]
        cube = np.empty((F, cfg.pn, cfg.nr), np.complex64)
        prof = np.empty((F, cfg.nr), np.float32)
        check(self.lib.fmcw_range_fft(self.h, ct.byref(self.p), _ptr(iq), dt, F, _ptr(cube), _ptr(prof)))
        return cube, prof

    def stft_sizes(self, L: int, wlen: int, noverlap: int, nfft: int = 0, n_log_bins: int = 1024):
        ns, nf, nb = ct.c_int64(), ct.c_int32(), ct.c_int32()
        check(self.lib.fmcw_stft_sizes(int(L), int(wlen), int(noverlap), int(nfft), int(n_log_bins),
                                       ct.byref(ns), ct.byref(nf), ct.byref(nb)))
        return ns.value, nf.value, nb.value

    def stft(self, x: np.ndarray, win: np.ndarray, noverlap: int, fs: float, nfft: int = 0,
             n_log_bins: int = 1024) -> dict:
        """:270-299 on the device; returns time [nseg], frequency, intensity [nseg][nbins]."""
        x = np.ascontiguousarray(x, np.float32).reshape(-1)
        w = np.ascontiguousarray(win, np.float32)
        nseg, nf, nb = self.stft_sizes(len(x), len(w), noverlap, nfft, n_log_bins)
        T = np.empty(nseg, np.float32)
        Fq = np.empty(nb, np.float32)
        inten = np.empty((nseg, nb), np.float32)
        check(self.lib.fmcw_stft(self.h, _ptr(x), len(x), _ptr(w), len(w), int(noverlap), int(nfft), float(fs),
                                 int(n_log_bins), _ptr(T), _ptr(Fq), _ptr(inten)))
        return dict(time=T, frequency=Fq, intensity=inten, nfft=nf)

    def stft_png(self, x: np.ndarray, win: np.ndarray, noverlap: int, fs: float, png_path: str, nfft: int = 0,
                 n_log_bins: int = 1024, width: int = 0, height: int = 0) -> dict:
        """:270-299 as ``stft`` plus spectrogram.png (:331-348) rendered on the device."""
        x = np.ascontiguousarray(x, np.float32).reshape(-1)
        w = np.ascontiguousarray(win, np.float32)
        nseg, nf, nb = self.stft_sizes(len(x), len(w), noverlap, nfft, n_log_bins)
        T = np.empty(nseg, np.float32)
        Fq = np.empty(nb, np.float32)
        inten = np.empty((nseg, nb), np.float32)
        nbytes = ct.c_int64()
        check(self.lib.fmcw_stft_png(self.h, _ptr(x), len(x), _ptr(w), len(w), int(noverlap), int(nfft), float(fs),
                                     int(n_log_bins), _ptr(T), _ptr(Fq), _ptr(inten), str(png_path).encode(),
                                     int(width), int(height), ct.byref(nbytes)))
        return dict(time=T, frequency=Fq, intensity=inten, nfft=nf, png_bytes=nbytes.value)

    def render_spectrogram_device(self, d_Q, nq: int, d_nseg, d_pmax, nfft: int, fs: float, t0: float, dt: float,
                                  width: int, height: int, d_img, stream=None) -> None:
        with _sided(stream) as hs:
            check(self.lib.fmcw_render_spectrogram_device(self.h, _ptr(d_Q), int(nq), _ptr(d_nseg), _ptr(d_pmax),
                                                          int(nfft), float(fs), float(t0), float(dt), int(width),
                                                          int(height), _ptr(d_img), hs))

    # ---- device API (torch tensors as HBM buffers) -------------------------------
    def process_device(self, d_iq, F: int, in_dtype: int, outs: dict, d_cube=None, d_rd=None,
                       out_dtype: int = FMCW_C64, probe_column: int = 0, stream=None) -> None:
        self._need()
        with _sided(stream) as hs:
            check(self.lib.fmcw_process_device(
                self.h, ct.byref(self.p), _ptr(d_iq), in_dtype, int(F), _ptr(outs["profile"]),
                _ptr(outs["tgt_count"]), _ptr(outs["tgt_range_idx"]), _ptr(outs["tgt_range_mag"]),
                _ptr(outs["tgt_doppler_idx"]), _ptr(outs["slow_mag"]), _ptr(d_cube), _ptr(d_rd), out_dtype,
                int(probe_column), _ptr(outs.get("probe_mag")), hs))

    def process_slow_device(self, d_iq, F: int, in_dtype: int, outs: dict, d_list, d_len, d_pmax=None, d_rd=None,
                            out_dtype: int = FMCW_C64, stream=None) -> None:
        """process_device + compact_device (+ d_pmax = 0) in one call (fmcw_process_slow_device): on
        the single-pass schedule the compaction runs in the detection kernel's last workgroup."""
        self._need()
        with _sided(stream) as hs:
            check(self.lib.fmcw_process_slow_device(
                self.h, ct.byref(self.p), _ptr(d_iq), in_dtype, int(F), _ptr(outs["profile"]),
                _ptr(outs["tgt_count"]), _ptr(outs["tgt_range_idx"]), _ptr(outs["tgt_range_mag"]),
                _ptr(outs["tgt_doppler_idx"]), _ptr(outs["slow_mag"]), _ptr(d_rd), out_dtype, _ptr(d_list),
                _ptr(d_len), _ptr(d_pmax), hs))

    def range_fft_device(self, d_iq, F: int, in_dtype: int, d_cube, d_prof, out_dtype: int = FMCW_C64,
                         stream=None) -> None:
        self._need()
        with _sided(stream) as hs:
            check(self.lib.fmcw_range_fft_device(self.h, ct.byref(self.p), _ptr(d_iq), in_dtype, int(F), _ptr(d_cube),
                                                 out_dtype, _ptr(d_prof), hs))

    def compact_device(self, d_count, F: int, d_list, d_len, stream=None) -> None:
        cfg = self._need()
        with _sided(stream) as hs:
            check(self.lib.fmcw_compact_device(self.h, _ptr(d_count), int(F), cfg.pn, _ptr(d_list), _ptr(d_len),
                                               hs))

    def stft_power_device(self, d_slow, d_list, d_len, pn: int, d_win, wlen: int, noverlap: int, nfft: int,
                          fs: float, max_seg: int, d_P, d_pmax, d_nseg, d_halo=None, n_halo: int = 0,
                          d_halo_len=None, stream=None) -> None:
        with _sided(stream) as hs:
            check(self.lib.fmcw_stft_power_device(self.h, _ptr(d_slow), _ptr(d_list), _ptr(d_len), int(pn),
                                                  _ptr(d_halo), int(n_halo), _ptr(d_halo_len), _ptr(d_win),
                                                  int(wlen), int(noverlap),
                                                  int(nfft), float(fs), int(max_seg), _ptr(d_P), _ptr(d_pmax),
                                                  _ptr(d_nseg), hs))

    def stft_db_direct_device(self, d_slow, d_list, d_len, pn: int, d_win, wlen: int, noverlap: int, nfft: int,
                              fs: float, max_seg: int, d_pmax, d_out, d_halo=None, n_halo: int = 0, d_halo_len=None,
                              stream=None) -> None:
        with _sided(stream) as hs:
            check(self.lib.fmcw_stft_db_direct_device(self.h, _ptr(d_slow), _ptr(d_list), _ptr(d_len), int(pn),
                                                      _ptr(d_halo), int(n_halo), _ptr(d_halo_len), _ptr(d_win),
                                                      int(wlen), int(noverlap), int(nfft), float(fs), int(max_seg),
                                                      _ptr(d_pmax), _ptr(d_out), hs))

    def stft_db_device(self, d_P, d_nseg, max_seg: int, nfft: int, fs: float, d_pmax, n_log_bins: int, d_out,
                       stream=None) -> None:
        with _sided(stream) as hs:
            check(self.lib.fmcw_stft_db_device(self.h, _ptr(d_P), _ptr(d_nseg), int(max_seg), int(nfft), float(fs),
                                               _ptr(d_pmax), int(n_log_bins), _ptr(d_out), hs))

    def synth_device(self, d_iq, frame0: int, F: int, dtype: int = FMCW_C64, stream=None) -> None:
        self._need()
        with _sided(stream) as hs:
            check(self.lib.fmcw_synth_device(self.h, ct.byref(self.p), int(frame0), int(F), _ptr(d_iq), dtype,
                                             hs))

    # ---- timing -----------------------------------------------------------------
    def timing(self, level: int) -> None:
        """0 off, 1 per range+Doppler chunk + STFT launches, 2 per kernel launch, 3 the dominant
        kernel's launches only (k_rdx / range-only K1)."""
        check(self.lib.fmcw_timing_enable(self.h, int(level)))

    def timing_reset(self) -> None:
        check(self.lib.fmcw_timing_reset(self.h))

    def timing_read(self) -> dict:
        out = {}
        for i, name in enumerate(STAGES):
            ms, n = ct.c_double(), ct.c_int64()
            check(self.lib.fmcw_timing_read(self.h, i, ct.byref(ms), ct.byref(n)))
            out[name] = (ms.value, n.value)
        return out

    def synchronize(self) -> None:
        check(self.lib.fmcw_synchronize(self.h))

    def rdx_clock(self) -> tuple:
        """(MHz, us) of the last k_rdx launch: its effective shader clock and stamped span."""
        mhz, us = ct.c_double(), ct.c_double()
        check(self.lib.fmcw_rdx_clock(self.h, ct.byref(mhz), ct.byref(us)))
        return mhz.value, us.value

    def copy_device(self, d_src, d_dst, nbytes: int, stream=None) -> None:
        """16-byte nontemporal device copy (the bench's HBM copy ceiling)."""
        with _sided(stream) as hs:
            check(self.lib.fmcw_copy_device(self.h, _ptr(d_src), _ptr(d_dst), int(nbytes), hs))

    def _need(self) -> FmcwConfig:
        if self.cfg is None:
            raise FmcwError(_lib.FMCW_E_STATE, "set_taps() first")
        return self.cfg


def _stream(stream) -> ct.c_void_p:
    """The hipStream_t of a call: None = the context's own stream (include/fmcw.h: NULL), an int
    = a raw handle, a torch.cuda.Stream = its handle (see _sided for torch's default stream)."""
    if stream is None:
        return ct.c_void_p(0)
    if isinstance(stream, int):
        return ct.c_void_p(stream)
    return ct.c_void_p(int(stream.cuda_stream))   # torch.cuda.Stream


_SIDE = {}


@contextlib.contextmanager
def _sided(stream):
    """The stream handle for a device call on `stream`.  torch's default stream has handle 0,
    which the C-ABI reads as the context's own (non-blocking) stream -- one that does not wait
    for the torch work queued before the call (a flip, a mul_, an RCCL collective) nor the torch
    work after it for the call.  So a call on torch's default stream runs on a side stream that
    waits for it first and that it waits for afterwards: ordered like any torch kernel."""
    if stream is None or isinstance(stream, int) or int(stream.cuda_stream) != 0:
        yield _stream(stream)
        return
    import torch
    side = _SIDE.get(stream.device)
    if side is None:
        side = _SIDE[stream.device] = torch.cuda.Stream(device=stream.device)
    side.wait_stream(stream)
    try:
        yield ct.c_void_p(int(side.cuda_stream))
    finally:
        stream.wait_stream(side)


def device_count() -> int:
    lib = _lib.load()
    n = ct.c_int32()
    st = lib.fmcw_device_count(ct.byref(n))
    return n.value if st == 0 else 0


def default_devices() -> list:
    """include/fmcw.h fmcw_default_devices: FMCW_DEVICES ("0,1,...") or every visible device."""
    lib = _lib.load()
    ids = (ct.c_int32 * 64)()
    n = ct.c_int32()
    check(lib.fmcw_default_devices(64, ids, ct.byref(n)))
    return list(ids[: n.value])
