"""GPU: fmcw_stft's coarse-to-fine max(P) (fmcw_api.cpp stft_coarse_max), used for the reference
nfft rule at large L (:273 nfft = 2^nextpow2(L) >= 2^18) with the 1024 log bins of :286-299.

max(P) (:282-283) must be the maximum over every bin of every segment; the coarse pass bounds each
segment's maximum from the bins k = m nfft / 16384 (Bernstein's inequality for the degree-19
trigonometric polynomial of a 20-tap segment) and only the 256-segment tiles that can hold it are
evaluated in full.  The outputs must equal the full pass (FMCW_STFT_COARSE=0) bit for bit, for
signals whose maximum sits in one place (a burst), everywhere (a constant: every tile is a
candidate) and in between (noise, a chirp).
"""
import numpy as np
import pytest

from fmcw_radar_processing_amd import params as P
from oracle import oracle as O
from tests.helpers import case

pytestmark = pytest.mark.gpu

L = 140_000                      # nfft 2^18: 139,981 segments x 131,073 bins (coarse step 2^4)


def _signal(kind, L=L):
    n = np.arange(L)
    rng = np.random.default_rng(11)
    if kind == "burst":
        x = np.abs(rng.standard_normal(L)) * 10
        x[L // 2:L // 2 + 40] += 400 * np.hanning(40)
    elif kind == "constant":
        x = np.full(L, 3.0)
    elif kind == "noise":
        x = np.abs(rng.standard_normal(L)) * 100
    elif kind == "signed":       # the bound holds for any sign (a trigonometric polynomial per segment)
        x = rng.standard_normal(L) * 10
        x[L // 3:L // 3 + 30] -= 300 * np.hanning(30)
    else:                        # a slow chirp: the peak bin moves through the spectrum
        x = 50 + 40 * np.cos(2 * np.pi * (1e-6 * n + 2e-11 * n * n))
    return x.astype(np.float32)


# 40,000: nfft 2^16 (step 2^3); 600,001: nfft 2^20 with 599,982 segments, not a multiple of the
# 256-segment tile (the sizes of round 4's GPU fault in the first coarse draft)
@pytest.mark.parametrize("kind,n", [("burst", L), ("constant", L), ("noise", L), ("chirp", L), ("signed", L),
                                    ("burst", 40_000), ("noise", 40_000), ("burst", 600_001)])
def test_coarse_max_is_the_full_max(engine, monkeypatch, capfd, kind, n):
    cfg, p, wr, wd, cal = case(64, 16, 256, 16, P.PARITY)
    engine.set_taps(cfg, cal, wr, wd)
    x = _signal(kind, n)
    win = O.stft_window("kaiser")
    monkeypatch.setenv("FMCW_STFT_COARSE", "0")
    full = engine.stft(x, win, 19, 1 / p["prt"], nfft=0, n_log_bins=1024)
    monkeypatch.setenv("FMCW_STFT_COARSE", "1")
    monkeypatch.setenv("FMCW_STFT_DEBUG", "1")
    capfd.readouterr()
    fast = engine.stft(x, win, 19, 1 / p["prt"], nfft=0, n_log_bins=1024)
    err = capfd.readouterr().err
    assert full["nfft"] == fast["nfft"] == {L: 1 << 18, 40_000: 1 << 16, 600_001: 1 << 20}[n]
    assert "stft_coarse_max" in err, err          # the coarse path ran
    for k in ("time", "frequency", "intensity"):
        np.testing.assert_array_equal(fast[k], full[k], err_msg=k)
    if kind == "burst":                           # the maximum is local: few tiles in full
        used, total = [int(v) for v in err.split("segments, ")[1].split(" tiles")[0].split(" of ")]
        assert used <= 4 and total > n // 300, err
