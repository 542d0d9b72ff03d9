"""GPU: edge inputs of the per-frame loop (radar_processing.m:197-261) and the STFT (:270-299)
through the C-ABI, against the float64 oracle where it has an answer.

  * no frames (F = 0): every call returns empty outputs without touching the device;
  * frames that hold only the calibration tone (every chirp equals calib_rx1): after the :204
    calibration and mean removal they are zero, so the profile, the RD map and the slow-time
    rows are zero and nothing is detected -- for the deployed module, config 2 and config 3/4
    geometry (the XCD-team single pass);
  * one frame of config-3 geometry (seven of the eight XCD teams have no frame);
  * the shortest signal the STFT accepts (exactly one 20-sample window).
"""
import numpy as np
import pytest

from fmcw_radar_processing_amd import params as P
from oracle import oracle as O
from tests.helpers import TOL_FP32_DB, TOL_FP32_REL_L2, case, rd_rel_err, rel_l2

pytestmark = pytest.mark.gpu

GEOMS = [(64, 16, 256, 16, P.PARITY), (512, 128, 512, 16, P.THROUGHPUT), (1024, 256, 1024, 256, P.THROUGHPUT)]
IDS = ["deployed", "cfg2", "cfg3"]


@pytest.mark.parametrize("geom", GEOMS, ids=IDS)
def test_no_frames(engine, geom):
    nts, pn, nr, nd, mode = geom
    cfg, p, wr, wd, cal = case(nts, pn, nr, nd, mode)
    engine.set_taps(cfg, cal, wr, wd)
    got = engine.process(np.zeros((0, pn, nts), np.complex64), want_rd=True)
    assert got["profile"].shape == (0, nr)
    assert got["tgt_count"].shape == (0,)
    assert got["rd"].shape[0] == 0
    cube, prof = engine.range_fft(np.zeros((0, pn, nts), np.complex64))
    assert cube.shape[0] == 0 and prof.shape == (0, nr)


@pytest.mark.parametrize("geom", GEOMS, ids=IDS)
def test_calibration_only_frames_are_empty(engine, geom):
    nts, pn, nr, nd, mode = geom
    cfg, p, wr, wd, cal = case(nts, pn, nr, nd, mode)
    F = 9
    iq = np.broadcast_to(cal.astype(np.complex64), (F, pn, nts)).copy()
    engine.set_taps(cfg, cal, wr, wd)
    got = engine.process(iq, want_rd=True)
    ref = O.process_frames(iq, cal, p, wr, wd, want_rd=True, rd_all_rows=True)
    # what is left is rounding noise: below 1e-4 of the profile peak / RD peak the calibration
    # tone (|cal| = 0.01) would give if it were not removed (|cal| times the windows' gains)
    tone = 0.01 * float(np.sum(wr))
    assert np.abs(got["profile"]).max() <= 1e-4 * tone
    assert np.abs(got["rd"]).max() <= 1e-4 * tone * float(np.sum(wd))
    np.testing.assert_array_equal(got["tgt_count"], ref["tgt_count"])
    assert np.all(got["tgt_count"] == 0)
    assert np.all(got["slow_mag"] == 0)


def test_one_frame_single_pass(engine):
    cfg, p, wr, wd, cal = case(1024, 256, 1024, 256, P.THROUGHPUT)
    iq = O.synth_frames(1, 256, 1024, 1024, 256, p["dist_per_bin"], frame0=4242)
    engine.set_taps(cfg, cal, wr, wd)
    got = engine.process(iq, want_rd=True)
    engine.synchronize()                     # no hand-off wait of the idle teams timed out
    ref = O.process_frames(iq, cal, p, wr, wd, want_cube=True, want_rd=True, rd_all_rows=True)
    assert rd_rel_err(got["rd"], ref["rd"], ref["cube"], wd, cfg.nd).max() <= TOL_FP32_REL_L2
    assert rel_l2(got["profile"], ref["profile"], axis=1).max() <= TOL_FP32_REL_L2
    np.testing.assert_array_equal(got["tgt_count"], ref["tgt_count"])


def test_stft_single_window(engine):
    """L = 20 = the window length: one segment (:276 spectrogram(x, kaiser(20, 3), 19, ...))."""
    cfg, p, wr, wd, cal = case(64, 16, 256, 16, P.PARITY)
    engine.set_taps(cfg, cal, wr, wd)
    x = (np.abs(np.random.default_rng(7).standard_normal(20)) * 10).astype(np.float32).astype(np.float64)
    win = O.stft_window("kaiser")
    got = engine.stft(x, win, 19, 1 / p["prt"], nfft=0, n_log_bins=1024)
    assert got["intensity"].shape[0] == 1
    ref = O.spectrogram_pipeline(x, p["prt"], win, 19, nfft=None, nbins=1024)
    assert got["nfft"] == ref["nfft"] == 32                # 2^nextpow2(20)
    ri = ref["intensity"].T
    sel = ri > -80
    assert sel.any()
    assert np.abs(got["intensity"][sel] - ri[sel]).max() <= TOL_FP32_DB
