"""Host mirror of ``radar_processing(process_animal_activity)``
(radar-etl-pipeline/radar_processing.m:56), with the loop and the STFT on the GPU.

The MATLAB host keeps the same structure (see matlab/radar_processing.m and
INTEGRATION.md); this module is the same sequence in Python so the path can be
driven, tested and benchmarked without MATLAB:

  :86       [frame, frame_count, calib_data, sXML] = f_parse_data2(...)  -> arguments
            (f_parse_data2 is absent from the reference; the caller supplies the
            parsed frames, calibration vector and device fields)
  :89-174   params, windows, calibration                    -> params.py (host)
  :197-261  per-frame loop                                   -> Engine.process (libfmcw)
  :242-252  measurement update, incl. its (fr_idx, j) growth  -> measurement_update_no
  :257-260  slow-time concatenation                          -> slow_time_signal
  :265-299  max-abs profile, STFT, dB, log-frequency resample -> Engine.stft (libfmcw)
  :302-436  four JSON files + uploads                        -> write_outputs_no
  :440-607  'yes' branch: per-100-frame spectrogram JSONs     -> _run_yes

The blob uploads are a caller-supplied hook (``upload``, default: none).
"""
from __future__ import annotations

import os
import threading
from typing import Callable

import numpy as np

from . import params as P
from . import json_native
from .matlab_json import matlab_squeeze_2d


# ---------------------------------------------------------------------------
# pure host logic (testable without a GPU)
# ---------------------------------------------------------------------------
def measurement_update_no(per: dict, cfg: P.FmcwConfig, frame_count: int) -> dict:
    """:157-159 + :242-252.  target_measurements.<x>(fr_idx, j) written into a
    max_num_targets x frame_count zeros matrix grows it (MATLAB auto-expands on
    out-of-range assignment) to max(rows) x max(cols)."""
    M = cfg.max_targets
    rows, cols = M, frame_count
    entries = []
    for f in range(frame_count):
        n = int(per["tgt_count"][f])
        for j in range(n):
            entries.append((f, j, float(per["tgt_range_mag"][f, j]),
                            float(cfg.range_m(per["tgt_range_idx"][f, j])),
                            float(cfg.speed(per["tgt_doppler_idx"][f, j]))))
            rows, cols = max(rows, f + 1), max(cols, j + 1)
    out = {k: np.zeros((rows, cols)) for k in ("strength", "range", "speed")}
    for f, j, a, r, s in entries:
        out["strength"][f, j] = a
        out["range"][f, j] = r
        out["speed"][f, j] = s
    return out


def measurement_update_yes(per: dict, cfg: P.FmcwConfig, frames) -> dict:
    """:499-529: (j, fr_idx) orientation, NaN where no target."""
    M = cfg.max_targets
    F = len(per["tgt_count"])
    out = {k: np.zeros((M, F)) for k in ("strength", "range", "speed")}
    for f in frames:
        n = int(per["tgt_count"][f])
        for j in range(M):
            if j < n:
                out["strength"][j, f] = per["tgt_range_mag"][f, j]
                out["range"][j, f] = cfg.range_m(per["tgt_range_idx"][f, j])
                out["speed"][j, f] = cfg.speed(per["tgt_doppler_idx"][f, j])
            else:
                for k in out:
                    out[k][j, f] = np.nan
    return out


def slow_time_signal(per: dict, frames=None) -> np.ndarray:
    """:257-260 (and :515): |X(ridx(1), :, fr)| of the frames with a target, in order."""
    cnt = per["tgt_count"]
    idx = np.arange(len(cnt)) if frames is None else np.asarray(list(frames))
    keep = idx[cnt[idx] > 0]
    return per["slow_mag"][keep].reshape(-1).astype(np.float64)


def write_json(path: str, obj: dict) -> str:
    """jsonencode(obj, 'PrettyPrint', true) + fprintf (:313-321 and friends) through
    libfmcw's native writer (json_native; same bytes as matlab_json.encode)."""
    json_native.write(path, obj, pretty=True)
    return path


def write_outputs_no(out_dir: str, filename: str, cfg: P.FmcwConfig, per: dict, spec: dict,
                     meas: dict, frame_count: int, probe_frame_index: int, probe_mag,
                     upload: Callable[[str], None] | None = None, png: str | None = None) -> list:
    """:302-436: the four JSON files of the 'no' branch, each uploaded right after
    it is written.  ``probe_mag`` None: the cube has fewer than ``probe_frame_index``
    columns, and -- as the reference at :411 -- the fourth file fails after the
    first three were written and uploaded."""
    paths = []

    def emit(path, obj):                                        # write, then upload (:315-328 and friends)
        write_json(path, obj)
        if upload:
            upload(path)
        return path

    # :306-328 spectrogram_data.json
    paths.append(emit(os.path.join(out_dir, "spectrogram_data.json"), {
        "time": spec["time"], "frequency": spec["frequency"],
        "intensity": spec["intensity"],                          # 1024 x nseg (bins down the rows)
        "title": "All Frames - Log-Scaled Spectrogram", "xLabel": "Time (s)", "yLabel": "Frequency (Hz)"}))
    # :331-348 spectrogram.png (rendered by Engine.stft_png), then its upload (:347)
    if png:
        if upload:
            upload(png)
        paths.append(png)
    # :355-377 <filename>_range_fft_data.json
    time_axis = np.arange(frame_count) * 0.15
    paths.append(emit(os.path.join(out_dir, f"{filename}_range_fft_data.json"), {
        "time_axis": time_axis, "array_bin_range": cfg.array_bin_range,
        "range_tx1rx1_max_abs": matlab_squeeze_2d(per["profile"].T),   # Nr x F
        "filename": filename}))
    # :379-407 <filename>_range_speed_data.json
    paths.append(emit(os.path.join(out_dir, f"{filename}_range_speed_data.json"), {
        "time_axis": time_axis, "range": meas["range"], "speed": meas["speed"], "filename": filename}))
    # :409-436 <filename>_fft_data.json (linear column 100 of the Nr x PN x F cube)
    if probe_mag is None:                                       # :411 range_tx1rx1_complete(:,100)
        raise IndexError(f"Index in position 2 exceeds array bounds (must not exceed {cfg.pn * frame_count}).")
    paths.append(emit(os.path.join(out_dir, f"{filename}_fft_data.json"), {
        "range_bins": np.arange(cfg.nr), "magnitude": np.asarray(probe_mag, np.float64),
        "frame_index": probe_frame_index, "filename": filename}))
    return paths


# ---------------------------------------------------------------------------
# the entry point (GPU)
# ---------------------------------------------------------------------------
_DEFAULT_ENGINE = None
_DEFAULT_DEVICES_ENV = None
# The default context is not reentrant: libfmcw's context shares pinned staging, scratch and STFT
# tables between calls, and ctypes releases the GIL inside the library.  Calls that pass no engine
# therefore hold this lock for the whole call (threads that want concurrency pass engines of their
# own, one per thread, as the MEX gateway keeps one context per MATLAB worker process).
_DEFAULT_LOCK = threading.RLock()


def _default_engine():
    """The per-process context of calls that pass no engine, created once (as the MEX gateway's
    static context: mexLock on create, mexAtExit destroy).  Devices: FMCW_DEVICES when it is set
    (fmcw_default_devices, the rule the MEX gateway uses), else GPU 0 only -- a deployed 115-frame
    file does not pay for a context and an RCCL communicator on every GPU of the node, and takes no
    GPU it was not given.  A change of FMCW_DEVICES between calls re-creates the context.
    Call with _DEFAULT_LOCK held."""
    global _DEFAULT_ENGINE, _DEFAULT_DEVICES_ENV
    env = os.environ.get("FMCW_DEVICES")
    if _DEFAULT_ENGINE is not None and env != _DEFAULT_DEVICES_ENV:
        _drop_default_engine()
    if _DEFAULT_ENGINE is None:
        import atexit
        from .engine import Engine
        _DEFAULT_ENGINE = Engine(None if env else 0)
        _DEFAULT_DEVICES_ENV = env
        atexit.register(_drop_default_engine)
    return _DEFAULT_ENGINE


def _drop_default_engine():
    global _DEFAULT_ENGINE
    with _DEFAULT_LOCK:
        eng, _DEFAULT_ENGINE = _DEFAULT_ENGINE, None
        if eng is not None:
            eng.close()


def radar_processing(process_animal_activity: str, *, frames: np.ndarray, calib_data: np.ndarray,
                     device: dict, fdata: str = "radar_data", out_dir: str = ".", engine=None,
                     upload: Callable[[str], None] | None = None, nr: int = 256, nd: int = 16,
                     mode: str = P.PARITY) -> dict:
    """radar_processing(process_animal_activity) with the DSP on the MI355X.

    frames      [F][PN][NTS] complex: frame(fr).Chirp(:,:,1) stacked (:199-202)
    calib_data  the calibration vector of f_parse_data2 (:86, :166-174)
    device      sXML fields (see params.derive_params)
    Returns the paths written and the intermediate arrays.  Raises where
    MATLAB raises (e.g. spectrogram of fewer than 20 slow-time samples).
    """
    filename = os.path.splitext(os.path.basename(fdata))[0]            # :68
    cfg = P.derive_params(device, nr=nr, nd=nd, mode=mode)             # :89-154
    cal = P.calibration(calib_data, cfg.n_rx, cfg.nts)                 # :166-174
    frames = np.asarray(frames)
    if engine is None:                                                 # the shared default context:
        with _DEFAULT_LOCK:                                            # one call at a time
            return _radar_processing(process_animal_activity, frames, cfg, cal, filename, out_dir,
                                     _default_engine(), upload)        # FMCW_DEVICES, else GPU 0
    return _radar_processing(process_animal_activity, frames, cfg, cal, filename, out_dir, engine, upload)


def _radar_processing(process_animal_activity, frames, cfg, cal, filename, out_dir, eng, upload):
    F = frames.shape[0]
    eng.set_taps(cfg, cal)                                             # :138-139 windows
    flag = str(process_animal_activity).lower()
    if flag == "no":
        res = _run_no(eng, cfg, frames, F, filename, out_dir, upload)
    elif flag == "yes":
        res = _run_yes(eng, cfg, frames, F, filename, out_dir, upload)
    else:
        res = {"paths": []}                                            # :195/:440: neither branch
    res["devices"] = list(eng.devices)                                 # the GPUs this call drove
    return res


def _run_no(eng, cfg, frames, F, filename, out_dir, upload):
    probe_col = 100                                                     # :410 fr_idx = 100
    have_probe = probe_col <= F * cfg.pn                                # else :411 fails after three files
    per = eng.process(frames, probe_column=probe_col if have_probe else 0)   # :197-261, :265
    meas = measurement_update_no(per, cfg, F)                           # :242-252
    slow = slow_time_signal(per)                                        # :257-260, :270
    fs = 1.0 / cfg.prt
    png = os.path.join(out_dir, "spectrogram.png")
    spec = eng.stft_png(slow, cfg.stft_window(), cfg.overlap, fs, png, nfft=0, n_log_bins=1024)   # :273-299, :331-344
    spec = {"time": spec["time"].astype(np.float64), "frequency": spec["frequency"].astype(np.float64),
            "intensity": spec["intensity"].T.astype(np.float64), "nfft": spec["nfft"]}
    paths = write_outputs_no(out_dir, filename, cfg, per, spec, meas, F, probe_col,
                             per["probe_mag"] if have_probe else None, upload, png=png)
    return {"paths": paths, "per_frame": per, "target_measurements": meas, "spectrogram": spec,
            "slow_time": slow}


def _run_yes(eng, cfg, frames, F, filename, out_dir, upload):
    per = eng.process(frames)                                           # :457-498 per-frame math
    batch = cfg.batch_size                                              # :189
    nb = -(-F // batch)                                                 # :190 ceil
    fs = 1.0 / cfg.prt
    paths, plot_counter, processed = [], 0, []
    for b in range(1, nb + 1):                                          # :444
        f0, f1 = (b - 1) * batch, min(b * batch, F)
        processed.extend(range(f0, f1))
        slow = slow_time_signal(per, range(f0, f1))                     # :515
        if len(slow) == 0 or len(slow) < cfg.window_length:            # :534
            continue
        plot_counter += 1
        if plot_counter > 4:                                            # :537, :598-599 break
            break
        spec = eng.stft(slow, cfg.stft_window(), cfg.overlap, fs, nfft=0, n_log_bins=1024)   # :538-566
        obj = {"time": spec["time"].astype(np.float64), "frequency": spec["frequency"].astype(np.float64),
               "intensity": spec["intensity"].T.astype(np.float64), "title": f"Spectrogram - Batch {b}",
               "xLabel": "Time (s) (relative to detected activity)", "yLabel": "Frequency (Hz)",
               "start_frame": f0 + 1, "end_frame": f1, "filename_base": filename}
        p_ = write_json(os.path.join(out_dir, f"{filename}_spectrogram_batch_{b}.json"), obj)   # :587-593
        if upload:
            upload(p_)
        paths.append(p_)
    meas = measurement_update_yes(per, cfg, processed)
    return {"paths": paths, "per_frame": per, "target_measurements": meas}
