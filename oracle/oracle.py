"""fp64 CPU restatement of the FMCW hot path -- TEST INFRASTRUCTURE ONLY.

This module is the *checker* for the HIP path in ``fmcw_radar_processing_amd``.
Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import it; the product path never does (it fails loudly instead).

It restates, step by step, ``radar-etl-pipeline/radar_processing.m`` of
alepnabil/fmcw_radar_processing (the reference), in float64 like MATLAB:

  * :89-154  device params + algorithm constants        -> ``derive_params``
  * :166-174 ADC calibration extraction                 -> ``calibration``
  * :138-139, :276 window taps                          -> ``windows`` (scipy,
    an implementation independent of the product's own window code)
  * :199-205 fast-time conditioning + range FFT          -> ``fast_time``
  * :210     range integration (max over chirps)         -> ``range_profile``
  * :211     f_search_peak (ABSENT from the reference)   -> ``search_peak``
  * :216-219 Doppler mean removal, window, FFT, fftshift -> ``doppler_rows``
  * :227-239 Doppler index with threshold + fallback     -> ``doppler_index``
  * :242-252 measurement update (with its (fr_idx,j) growth quirk)
  * :257-260 slow-time concatenation
  * :265     range_tx1rx1_max_abs
  * :270-299 |slow|, nextpow2, spectrogram, fftshift, 20log10, logspace+interp1
  * :457-530, :532-566 the 'yes' branch per-frame NaN semantics + batch guards

PARITY STATUS: **parity unpinned** against MATLAB.  The reference is MATLAB
code with no tests, no fixtures and no golden outputs, and no MATLAB/Octave
runtime exists here.  ``f_search_peak`` and
``f_parse_data2`` are not in the reference repo; the peak rule below is the
documented assumption of SURVEY.md section 8a row a9.  What *is* pinned:
known-answer tests (integer-bin range and Doppler tones, static-target
fallback, Parseval, window taps vs. the documented formulas) in
``tests/test_oracle.py``, and the MATLAB built-in semantics this file relies
on are spelled out next to each call.
"""
from __future__ import annotations

import math

import numpy as np
from scipy.signal import windows as sw

C0 = 3e8  # radar_processing.m:67


# --------------------------------------------------------------------------
# a1: parameters (radar_processing.m:89-154)
# --------------------------------------------------------------------------
def derive_params(device: dict, nr: int = 256, nd: int = 16, parity: bool = True) -> dict:
    """Device params (:94-115) + algorithm constants (:117-129) + derived (:131-154).

    ``device`` carries the sXML fields: chirpDuration_ns, upperFrequency_kHz,
    lowerFrequency_kHz, numAntennasTx, numAntennasRx, numSamplesPerChirp,
    numChirpsPerFrame, samplerateHz.
    """
    up = float(device["chirpDuration_ns"]) * 1e-9                  # :94
    prt = up + 200e-6 + 300e-6                                     # :95-97
    bw = (float(device["upperFrequency_kHz"]) - float(device["lowerFrequency_kHz"])) * 1e3  # :100
    fc = (float(device["upperFrequency_kHz"]) + float(device["lowerFrequency_kHz"])) / 2 * 1e3  # :106
    nts = int(device["numSamplesPerChirp"])                        # :109
    pn = int(device["numChirpsPerFrame"])                          # :112
    if_scale = 16 * 3.3 * nr / nts                                 # :121, :136
    lam = C0 / fc                                                  # :133
    r_max = nts * C0 / (2 * bw)                                    # :142
    dist_per_bin = r_max / nr                                      # :147
    fd_max = 1 / (2 * prt)                                         # :152
    fd_per_bin = fd_max / nd                                       # :153
    return dict(
        frame_time=0.15, prt=prt, bw=bw, fc=fc, nts=nts, pn=pn, nr=nr, nd=nd,
        n_rx=int(device.get("numAntennasRx", 1)), n_tx=int(device.get("numAntennasTx", 1)),
        fs=float(device.get("samplerateHz", 0.0)),
        if_scale=if_scale, range_thr=200.0, doppler_thr=50.0,       # :123-124
        min_d=0.9, max_d=25.0, max_targets=1,                       # :126-129
        lam=lam, hz_to_mps=lam / 2, r_max=r_max, dist_per_bin=dist_per_bin,
        fd_max=fd_max, fd_per_bin=fd_per_bin,
        array_bin_range=np.arange(nr) * dist_per_bin,               # :149
        array_bin_fd=(np.arange(1, nd + 1) - nd / 2 - 1) * -fd_per_bin * (lam / 2),  # :154
        # parity mode keeps the literal 9 of :234; throughput uses the zero bin
        doppler_fallback_idx=9 if parity else nd // 2 + 1,
        window_length=20, overlap=19,                               # :178-179
    )


# --------------------------------------------------------------------------
# a2: calibration (radar_processing.m:166-174)
# --------------------------------------------------------------------------
def calibration(calib_data: np.ndarray, n_rx: int, nts: int) -> np.ndarray:
    n_cal = len(calib_data) // (2 * n_rx)          # :167
    dec = n_cal // nts                             # :169
    i1 = calib_data[0:n_cal:dec]                   # :171  MATLAB 1:dec:N_cal
    q1 = calib_data[n_cal:2 * n_cal:dec]           # :172
    return (i1 + 1j * q1).astype(np.complex128)    # :174 (.' = non-conjugate)


# --------------------------------------------------------------------------
# a3: windows (scipy = independent implementation of MATLAB's formulas)
# --------------------------------------------------------------------------
def windows(nts: int, pn: int):
    wr = 2 * sw.blackman(nts, sym=True)            # :138 2*blackman(NTS)
    wd = 2 * sw.chebwin(pn, at=100)                # :139 2*chebwin(PN) (default 100 dB)
    return wr, wd


def stft_window(kind: str, n: int = 20) -> np.ndarray:
    if kind == "kaiser":
        return sw.kaiser(n, 3)                     # :276 kaiser(window_length, 3)
    if kind == "hann":
        return sw.hann(n, sym=True)                # config 4 (BASELINE.json) Hann
    raise ValueError(kind)


# --------------------------------------------------------------------------
# a5-a11: per-frame math
# --------------------------------------------------------------------------
def _fft_n(x: np.ndarray, n: int, axis: int) -> np.ndarray:
    """MATLAB fft(x, n, dim): zero-pad OR truncate to n along dim."""
    return np.fft.fft(x, n=n, axis=axis)


def fast_time(chirps_sc: np.ndarray, cal: np.ndarray, if_scale: float, wr: np.ndarray,
              nr: int) -> np.ndarray:
    """:202-205. ``chirps_sc`` is S x C (samples down the column, as MATLAB)."""
    m = (chirps_sc - cal[:, None]) * if_scale      # :203 repmat(calib_rx1,1,PN)
    m = m - m.mean(axis=0, keepdims=True)          # :204 bsxfun(@minus, m, mean(m))
    return _fft_n(m * wr[:, None], nr, axis=0)     # :205 fft(m.*repmat(w,1,PN), Nr, 1)


def range_profile(x_rc: np.ndarray) -> np.ndarray:
    """:210 abs(max(X,[],2)); MATLAB max of complex compares |.|, so = max|.|."""
    return np.abs(x_rc).max(axis=1)


def search_peak(prof: np.ndarray, n: int, thr: float, max_targets: int, min_d: float,
                max_d: float, dist_per_bin: float):
    """Restatement of the ABSENT helper f_search_peak (:211) -- SURVEY 8a row a9.

    Candidate i (1-based) must satisfy (i-1)*dist_per_bin in [min_d, max_d],
    prof(i) > thr, prof(i) >= prof(i-1) and prof(i) > prof(i+1) (2 <= i <= n-1).
    The ``max_targets`` largest candidates are returned, descending by
    magnitude, ties broken towards the lower index.  Returns (idx[], mag[]),
    idx 1-based.  PARITY UNPINNED: the Infineon helper is not vendored.
    """
    cands = []
    for i in range(2, n):                          # 1-based 2..n-1
        rng = (i - 1) * dist_per_bin
        if rng < min_d or rng > max_d:
            continue
        v = prof[i - 1]
        if v > thr and v >= prof[i - 2] and v > prof[i]:
            cands.append((-v, i))
    cands.sort()
    sel = cands[:max_targets]
    return [i for _, i in sel], [-nv for nv, _ in sel]


def doppler_rows(x_rc: np.ndarray, ridx, wd: np.ndarray, nd: int) -> np.ndarray:
    """:216-219 for the rows in ``ridx`` (1-based). Returns Nr x Nd (zeros elsewhere)."""
    nr = x_rc.shape[0]
    rd = np.zeros((nr, nd), dtype=np.complex128)   # :216
    if len(ridx) == 0:
        return rd
    rows = np.asarray(ridx) - 1
    sel = x_rc[rows, :]
    sel = sel - sel.mean(axis=1, keepdims=True)    # :217-218 mean over ALL PN chirps
    # :219 fftshift(fft(sel.*repmat(w.',n,1), Nd, 2), 2); fft truncates when Nd < PN
    rd[rows, :] = np.fft.fftshift(_fft_n(sel * wd[None, :], nd, axis=1), axes=1)
    return rd


def doppler_all_rows(x_rc: np.ndarray, wd: np.ndarray, nd: int) -> np.ndarray:
    """The same row operation as :217-219 applied to every range row (the full
    range-Doppler map of configs 3-5; each row is bit-for-bit the reference row op)."""
    sel = x_rc - x_rc.mean(axis=1, keepdims=True)
    return np.fft.fftshift(_fft_n(sel * wd[None, :], nd, axis=1), axes=1)


def doppler_index(rd: np.ndarray, ridx, thr: float, fallback: int):
    """:227-239 [val, idx] = max(abs(row)) (first max) ; keep idx unless val<thr or idx==9."""
    out = []
    for r in ridx:
        mag = np.abs(rd[r - 1, :])
        di = int(np.argmax(mag)) + 1               # MATLAB max: first index of the max
        val = mag[di - 1]
        out.append(di if (val >= thr and di != fallback) else fallback)
    return out


# --------------------------------------------------------------------------
# batch driver for the per-frame stages (a4-a13)
# --------------------------------------------------------------------------
def process_frames(iq_fcs: np.ndarray, cal: np.ndarray, p: dict, wr: np.ndarray,
                   wd: np.ndarray, want_cube: bool = False, want_rd: bool = False,
                   rd_all_rows: bool = False, frame_offset: int = 0) -> dict:
    """Run :197-261 over a stacked cube ``iq_fcs[F][C][S]`` (S fastest, i.e.
    MATLAB cat(3, frame.Chirp(:,:,1)) read as a C array).

    Returns per-frame arrays:
      profile [F][Nr]     = range_tx1rx1_max_abs (:265) transposed to C order
      tgt_range_idx [F][M], tgt_range_mag [F][M], tgt_doppler_idx [F][M] (0 = none)
      tgt_count [F]
      slow_mag [F][C]     = |range_tx1rx1_complete(ridx(1), :, fr)| (:259, :270)
      cube [F][C][Nr]     (optional, = range_tx1rx1_complete in C order)
      rd [F][Nr][Nd]      (optional; target rows only unless rd_all_rows)
    """
    F, C, S = iq_fcs.shape
    nr, nd, M = p["nr"], p["nd"], p["max_targets"]
    out = dict(
        profile=np.zeros((F, nr)), tgt_range_idx=np.zeros((F, M), np.int32),
        tgt_range_mag=np.zeros((F, M)), tgt_doppler_idx=np.zeros((F, M), np.int32),
        tgt_count=np.zeros(F, np.int32), slow_mag=np.zeros((F, C)),
    )
    if want_cube:
        out["cube"] = np.zeros((F, C, nr), np.complex128)
    if want_rd:
        out["rd"] = np.zeros((F, nr, nd), np.complex128)
    for f in range(F):
        x = iq_fcs[f].astype(np.complex128).T                         # S x C  (:199-202)
        X = fast_time(x, cal, p["if_scale"], wr, nr)                  # :203-205
        prof = range_profile(X)                                       # :210
        ridx, rmag = search_peak(prof, nr, p["range_thr"], M, p["min_d"], p["max_d"],
                                 p["dist_per_bin"])                   # :211
        rd = doppler_all_rows(X, wd, nd) if rd_all_rows else doppler_rows(X, ridx, wd, nd)
        didx = doppler_index(rd, ridx, p["doppler_thr"], p["doppler_fallback_idx"])
        n = len(ridx)
        out["profile"][f] = prof
        out["tgt_count"][f] = n
        out["tgt_range_idx"][f, :n] = ridx
        out["tgt_range_mag"][f, :n] = rmag
        out["tgt_doppler_idx"][f, :n] = didx
        if n > 0:                                                      # :257-260
            out["slow_mag"][f] = np.abs(X[ridx[0] - 1, :])
        if want_cube:
            out["cube"][f] = X.T
        if want_rd:
            out["rd"][f] = rd
    return out


def measurement_update_no(per_frame: dict, p: dict, frame_count: int):
    """:157-159 + :242-252 ('no' branch).  Assigning (fr_idx, j) into a
    max_num_targets x frame_count zeros matrix grows it to last_fr x F."""
    M = p["max_targets"]
    shape = [M, frame_count]
    vals = []
    for f in range(frame_count):
        n = int(per_frame["tgt_count"][f])
        for j in range(n):
            r = (per_frame["tgt_range_idx"][f, j] - 1) * p["dist_per_bin"]
            s = (per_frame["tgt_doppler_idx"][f, j] - p["nd"] / 2 - 1) * -p["fd_per_bin"] * p["hz_to_mps"]
            vals.append((f, j, per_frame["tgt_range_mag"][f, j], r, s))
            shape[0] = max(shape[0], f + 1)
            shape[1] = max(shape[1], j + 1)
    strength = np.zeros(shape); rng = np.zeros(shape); spd = np.zeros(shape)
    for f, j, a, r, s in vals:
        strength[f, j] = a; rng[f, j] = r; spd[f, j] = s
    return dict(strength=strength, range=rng, speed=spd)


def measurement_update_yes(per_frame: dict, p: dict, frame_count: int):
    """:499-529 ('yes' branch): (j, fr_idx) orientation, NaN where no target."""
    M = p["max_targets"]
    strength = np.zeros((M, frame_count)); rng = np.zeros((M, frame_count)); spd = np.zeros((M, frame_count))
    for f in range(frame_count):
        n = int(per_frame["tgt_count"][f])
        for j in range(M):
            if j < n:
                strength[j, f] = per_frame["tgt_range_mag"][f, j]
                rng[j, f] = (per_frame["tgt_range_idx"][f, j] - 1) * p["dist_per_bin"]
                spd[j, f] = (per_frame["tgt_doppler_idx"][f, j] - p["nd"] / 2 - 1) * -p["fd_per_bin"] * p["hz_to_mps"]
            else:
                strength[j, f] = rng[j, f] = spd[j, f] = np.nan
    return dict(strength=strength, range=rng, speed=spd)


def slow_time_signal(per_frame: dict) -> np.ndarray:
    """:257-260 + :270: concatenation of |X[ridx(1), :]| over frames with a target."""
    keep = per_frame["tgt_count"] > 0
    return per_frame["slow_mag"][keep].reshape(-1)


# --------------------------------------------------------------------------
# a14-a17: STFT, dB, log-frequency resampling (:270-299)
# --------------------------------------------------------------------------
def nextpow2(n: int) -> int:
    """MATLAB nextpow2: smallest p with 2^p >= |n|."""
    return 0 if n <= 1 else int(math.ceil(math.log2(n)))


def spectrogram(x: np.ndarray, win: np.ndarray, noverlap: int, nfft: int, fs: float):
    """MATLAB spectrogram(x, win, noverlap, nfft, fs) for a REAL vector x.

    ncol = fix((L-noverlap)/(wlen-noverlap)); column c is the nfft-point DFT of
    x[c*hop : c*hop+wlen] .* win (zero-padded); one-sided (nfft/2+1 rows for
    even nfft); T = (c*hop + wlen/2)/fs; F = (0:nfft/2)*fs/nfft;
    P = |S|^2 / (fs * sum(win^2)), doubled except DC and Nyquist ('psd').
    """
    L = len(x); wl = len(win); hop = wl - noverlap
    ncol = (L - noverlap) // hop
    if ncol < 1:
        raise ValueError("spectrogram: signal shorter than the window")
    idx = np.arange(ncol)[:, None] * hop + np.arange(wl)[None, :]
    seg = x[idx] * win[None, :]
    S = np.fft.fft(seg, n=nfft, axis=1)[:, : nfft // 2 + 1].T          # nbins x ncol
    Fv = np.arange(nfft // 2 + 1) * fs / nfft
    T = (np.arange(ncol) * hop + wl / 2) / fs
    P = np.abs(S) ** 2 / (fs * np.sum(win ** 2))
    if nfft % 2 == 0:
        P[1:-1] *= 2
    else:
        P[1:] *= 2
    return S, Fv, T, P


def psd_db(P: np.ndarray) -> np.ndarray:
    """:279-283 (the fftshift of :280 is a row rotation; it is applied and
    undone in ``log_resample``).  20*log10 of a POWER, as the reference does."""
    G = P.max(axis=0)
    return 20 * np.log10(np.abs(P) / G.max())


def log_freq_bins(fs: float, nfft: int, nbins: int = 1024) -> np.ndarray:
    """:293-296; MIN_FREQ = min(F(F>0)) = fs/nfft, MAX_FREQ = fs/2."""
    Fv = np.arange(nfft // 2 + 1) * fs / nfft
    return np.logspace(np.log10(Fv[Fv > 0].min()), np.log10(Fv.max()), nbins)


def log_resample(Fv: np.ndarray, psd: np.ndarray, fq: np.ndarray) -> np.ndarray:
    """:279-280 + :299 interp1(fftshift(F), fftshift(psd,1), fq, 'linear','extrap').
    interp1 sorts non-monotonic sample points (reordering psd rows with them),
    which undoes the fftshift; we therefore interpolate on the sorted axis."""
    Fs_ = np.fft.fftshift(Fv); Ps_ = np.fft.fftshift(psd, axes=0)
    order = np.argsort(Fs_, kind="stable")
    xs = Fs_[order]; ys = Ps_[order]
    i = np.clip(np.searchsorted(xs, fq, side="right") - 1, 0, len(xs) - 2)
    w = (fq - xs[i]) / (xs[i + 1] - xs[i])
    return ys[i] * (1 - w)[:, None] + ys[i + 1] * w[:, None]        # 1024 x nseg


def spectrogram_pipeline(slow: np.ndarray, prt: float, win: np.ndarray, noverlap: int,
                         nfft: int | None = None, nbins: int = 1024):
    """:270-299. nfft=None reproduces the reference rule 2^nextpow2(L)."""
    if nfft is None:
        nfft = 2 ** nextpow2(len(slow))
    fs = 1 / prt
    _, Fv, T, P = spectrogram(slow, win, noverlap, nfft, fs)
    psd = psd_db(P)
    if nbins:
        fq = log_freq_bins(fs, nfft, nbins)
        return dict(time=T, frequency=fq, intensity=log_resample(Fv, psd, fq), nfft=nfft, psd=psd)
    return dict(time=T, frequency=Fv, intensity=psd, nfft=nfft, psd=psd)


# --------------------------------------------------------------------------
# synthetic IQ generator -- same integer hash as csrc/synth.h
# --------------------------------------------------------------------------
_M64 = (1 << 64) - 1


def _splitmix64(z: np.ndarray) -> np.ndarray:
    z = (z + np.uint64(0x9E3779B97F4A7C15)) & np.uint64(_M64)
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def _mix(seed, ctr) -> np.ndarray:
    with np.errstate(over="ignore"):
        return _splitmix64(np.uint64(seed) * np.uint64(0xD1342543DE82EF95) + np.asarray(ctr, np.uint64))


def _u24(h: np.ndarray, shift: int) -> np.ndarray:
    return (((h >> np.uint64(shift)) & np.uint64(0xFFFFFF)).astype(np.float64) + 0.5) / 16777216.0


def synth_cal(nts: int) -> np.ndarray:
    """cal[n] = 0.01*exp(j*2*pi*0.013*n)."""
    n = np.arange(nts)
    return 0.01 * np.exp(2j * np.pi * ((0.013 * n) % 1.0))


def synth_frame_params(f: int, nr: int, nd: int, dist_per_bin: float):
    seed = 0xF3C0 ^ f
    with np.errstate(over="ignore"):
        u = [_u24(_mix(seed, 0x1000 + i), 40) for i in range(6)]
    rlo = int(math.ceil(0.9 / dist_per_bin)) + 2
    rhi = max(rlo, int(math.floor(25.0 / dist_per_bin)) - 2)
    no_target = u[0] < 0.10
    off = 0.37 if u[1] < 0.25 else 0.0
    r = rlo + min(int(u[2] * (rhi - rlo + 1)), rhi - rlo)
    d = -nd // 2 + 1 + min(int(u[3] * (nd - 1)), nd - 2) if nd > 1 else 0
    A = 0.0 if no_target else 0.02 + 0.18 * float(u[4])
    phi = float(u[5])  # in cycles
    return dict(r=r, off=off, d=d, A=A, phi=phi)


def synth_frames(F: int, C: int, S: int, nr: int, nd: int, dist_per_bin: float,
                 frame0: int = 0, sigma: float = 1e-3) -> np.ndarray:
    """x[f,k,n] = cal[n] + A e^{j2pi(n (r+off)/Nr + k d/Nd + phi)} + CN(0, sigma^2)."""
    cal = synth_cal(S)
    out = np.empty((F, C, S), np.complex64)
    n = np.arange(S, dtype=np.int64)[None, :]
    k = np.arange(C, dtype=np.int64)[:, None]
    for i in range(F):
        f = frame0 + i
        fp = synth_frame_params(f, nr, nd, dist_per_bin)
        ph = ((n * fp["r"]) % nr) / nr + (n * fp["off"]) / nr + ((k * (fp["d"] % nd)) % nd) / nd + fp["phi"]
        ph = ph % 1.0
        sig = fp["A"] * np.exp(2j * np.pi * ph)
        idx = (k * S + n).astype(np.uint64)
        with np.errstate(over="ignore"):
            h = _mix(0xF3C0 ^ f, idx + np.uint64(1 << 40))
        u1 = _u24(h, 40); u2 = _u24(h, 16)
        rad = np.sqrt(-2.0 * np.log(u1)) * (sigma / math.sqrt(2.0))
        noise = rad * np.exp(2j * np.pi * u2)
        out[i] = (cal[None, :] + sig + noise).astype(np.complex64)
    return out


def deployed_device(nts: int = 64, pn: int = 16) -> dict:
    """Deployed Infineon 24 GHz module: PRT 0.8 ms, BW 200 MHz, fc 24.125 GHz."""
    return dict(chirpDuration_ns=300000, upperFrequency_kHz=24225000, lowerFrequency_kHz=24025000,
                numAntennasTx=1, numAntennasRx=2, numSamplesPerChirp=nts, numChirpsPerFrame=pn,
                samplerateHz=nts / 300e-6)
