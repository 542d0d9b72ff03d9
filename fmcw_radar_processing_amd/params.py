"""Host-side parameters of the FMCW path.

Mirrors what radar_processing.m computes on the MATLAB host before the loop:
device params from the sXML struct (:94-115), algorithm constants (:117-129),
derived quantities (:131-154), the calibration vector (:166-174) and the
window taps (:138-139, :276).  Nothing here touches the GPU.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from . import windows
from ._lib import Params

C0 = 3e8  # radar_processing.m:67

PARITY = "parity"          # literal constants and quirks of the reference
THROUGHPUT = "throughput"  # configs 2-5 of BASELINE.json


@dataclass
class FmcwConfig:
    prt: float
    bw: float
    fc: float
    nts: int
    pn: int
    nr: int
    nd: int
    n_rx: int = 1
    n_tx: int = 1
    fs_adc: float = 0.0
    mode: str = PARITY
    frame_time: float = 0.15                 # :91
    range_thr: float = 200.0                 # :123
    doppler_thr: float = 50.0                # :124
    min_d: float = 0.9                       # :126
    max_d: float = 25.0                      # :127
    max_targets: int = 1                     # :129
    window_length: int = 20                  # :178
    overlap: int = 19                        # :179
    batch_size: int = 100                    # :189 ('yes' branch)
    extra: dict = field(default_factory=dict)

    # ---- derived (:131-154) ----
    @property
    def if_scale(self) -> float:
        return 16 * 3.3 * self.nr / self.nts           # :121 / :136 (uses the literal Nr)

    @property
    def lam(self) -> float:
        return C0 / self.fc                            # :133

    @property
    def hz_to_mps(self) -> float:
        return self.lam / 2                            # :135

    @property
    def r_max(self) -> float:
        return self.nts * C0 / (2 * self.bw)           # :142

    @property
    def dist_per_bin(self) -> float:
        return self.r_max / self.nr                    # :147

    @property
    def array_bin_range(self) -> np.ndarray:
        return np.arange(self.nr) * self.dist_per_bin  # :149

    @property
    def fd_max(self) -> float:
        return 1 / (2 * self.prt)                      # :152

    @property
    def fd_per_bin(self) -> float:
        return self.fd_max / self.nd                   # :153

    @property
    def array_bin_fd(self) -> np.ndarray:             # :154
        return (np.arange(1, self.nd + 1) - self.nd / 2 - 1) * -self.fd_per_bin * self.hz_to_mps

    @property
    def doppler_fallback_idx(self) -> int:
        # :234 hard-codes 9 (the zero-Doppler bin only when Nd = 16)
        return 9 if self.mode == PARITY else self.nd // 2 + 1

    def speed(self, doppler_idx) -> np.ndarray:
        """:250 (idx - Nd/2 - 1) * -fD_per_bin * Hz_to_mps_constant."""
        return (np.asarray(doppler_idx, dtype=np.float64) - self.nd / 2 - 1) * -self.fd_per_bin * self.hz_to_mps

    def range_m(self, range_idx) -> np.ndarray:
        """:248 (idx - 1) * dist_per_bin."""
        return (np.asarray(range_idx, dtype=np.float64) - 1) * self.dist_per_bin

    def abi(self) -> Params:
        return Params(self.nts, self.pn, self.nr, self.nd, self.max_targets, self.doppler_fallback_idx,
                      self.if_scale, self.range_thr, self.doppler_thr, self.min_d, self.max_d,
                      self.dist_per_bin)

    # ---- window taps (:138-139, :276) ----
    def range_window(self) -> np.ndarray:
        return 2 * windows.blackman(self.nts)

    def doppler_window(self) -> np.ndarray:
        return 2 * windows.chebwin(self.pn, 100.0)

    def stft_window(self) -> np.ndarray:
        if self.mode == PARITY:
            return windows.kaiser(self.window_length, 3.0)   # :276 kaiser(window_length, 3)
        return windows.hann(self.window_length)              # config 4: Hann(20)


def derive_params(device: dict, nr: int = 256, nd: int = 16, mode: str = PARITY, **over) -> FmcwConfig:
    """radar_processing.m:89-115 from the sXML fields.

    ``device`` keys (sXML.Device...Text): chirpDuration_ns, upperFrequency_kHz,
    lowerFrequency_kHz, numAntennasTx, numAntennasRx, numSamplesPerChirp,
    numChirpsPerFrame, samplerateHz.  ``nr``/``nd`` are the literal 256/16 of
    :118-119 in parity mode.
    """
    up = float(device["chirpDuration_ns"]) * 1e-9                                  # :94
    prt = up + 200e-6 + 300e-6                                                     # :95-97
    hi, lo = float(device["upperFrequency_kHz"]), float(device["lowerFrequency_kHz"])
    cfg = FmcwConfig(
        prt=prt, bw=(hi - lo) * 1e3, fc=(hi + lo) / 2 * 1e3,                     # :100, :106
        nts=int(device["numSamplesPerChirp"]), pn=int(device["numChirpsPerFrame"]),  # :109, :112
        nr=int(nr), nd=int(nd), n_rx=int(device.get("numAntennasRx", 1)),
        n_tx=int(device.get("numAntennasTx", 1)), fs_adc=float(device.get("samplerateHz", 0.0)),
        mode=mode)
    for k, v in over.items():
        setattr(cfg, k, v)
    return cfg


def fp16_fp32_bins(cfg: FmcwConfig) -> np.ndarray:
    """Range bins whose hand-off stays fp32 under fp16 storage on the XCD-team schedule: the
    128-bin blocks that hold a bin able to become a detection or slow-time candidate (min_d /
    max_d of :126-127, two bins of margin); the other blocks travel as c32h X / Nr.  Mirror of
    fmcw_api.cpp host_s16mask (float32 parameters as the C-ABI carries them), for checks that
    hold the profile in those blocks, and the target magnitudes, to the fp32 bar."""
    nr = cfg.nr
    dpb = float(np.float32(cfg.dist_per_bin))
    keep = np.ones(nr, bool)
    if not (dpb > 0 and np.isfinite(dpb)) or nr % 128:
        return keep
    lo_d = np.floor(float(np.float32(cfg.min_d)) / dpb) - 2
    hi_d = np.ceil(float(np.float32(cfg.max_d)) / dpb) + 2
    lo = int(max(0.0, min(float(nr), lo_d)))
    hi = int(max(-1.0, min(float(nr - 1), hi_d)))
    for b in range(nr // 128):
        if hi < lo or 128 * b + 127 < lo or 128 * b > hi:
            keep[128 * b: 128 * b + 128] = False
    return keep


def calibration(calib_data: np.ndarray, n_rx: int, nts: int) -> np.ndarray:
    """:166-174 calib_rx1 = (I(1:dec:N_cal) + 1i*Q(1:dec:N_cal)).'"""
    calib_data = np.asarray(calib_data, dtype=np.float64).reshape(-1)
    n_cal = len(calib_data) // (2 * n_rx)
    if n_cal % nts:
        raise ValueError("calibration length is not a multiple of NTS (MATLAB would fail to index)")
    dec = n_cal // nts
    return calib_data[0:n_cal:dec] + 1j * calib_data[n_cal:2 * n_cal:dec]


def deployed_device(nts: int = 64, pn: int = 16) -> dict:
    """The deployed Infineon 24 GHz module: PRT 0.8 ms, BW 200 MHz,
    fc 24.125 GHz; NTS/PN as given (64 x 16 in the field, larger for configs 1-5)."""
    return dict(chirpDuration_ns=300000, upperFrequency_kHz=24225000, lowerFrequency_kHz=24025000,
                numAntennasTx=1, numAntennasRx=2, numSamplesPerChirp=nts, numChirpsPerFrame=pn,
                samplerateHz=nts / 300e-6)


def synth_calibration(nts: int) -> np.ndarray:
    """Calibration used with synthetic frames: 0.01 e^{j 2 pi 0.013 n}."""
    n = np.arange(nts)
    return 0.01 * np.exp(2j * np.pi * ((0.013 * n) % 1.0))


# BASELINE.json configs (geometry only; the device constants are the deployed ones)
CONFIGS = {
    1: dict(nts=256, pn=128, nr=256, nd=16, frames=1, mode=PARITY),
    2: dict(nts=512, pn=128, nr=512, nd=16, frames=4096, mode=THROUGHPUT),
    3: dict(nts=1024, pn=256, nr=1024, nd=256, frames=4096, mode=THROUGHPUT),
    4: dict(nts=1024, pn=256, nr=1024, nd=256, frames=4096, mode=THROUGHPUT, stft_nfft=64),
    5: dict(nts=1024, pn=256, nr=1024, nd=256, frames=65536, mode=THROUGHPUT, stft_nfft=64),
    "deployed": dict(nts=64, pn=16, nr=256, nd=16, frames=115, mode=PARITY),
}


def config(name, **over) -> FmcwConfig:
    c = dict(CONFIGS[name])
    c.update(over)
    cfg = derive_params(deployed_device(c["nts"], c["pn"]), nr=c["nr"], nd=c["nd"], mode=c["mode"])
    cfg.extra = {k: v for k, v in c.items() if k not in ("nts", "pn", "nr", "nd", "mode")}
    return cfg
