"""Golden fixtures (tests/golden/*.npz, made by tests/golden/make_golden.py).

CPU: the oracle still reproduces every committed vector (regression pin).
GPU: libfmcw reproduces them within the SURVEY.md 8d fp32 tolerances -- these
need no oracle run on the box.
"""
import os

import numpy as np
import pytest

from fmcw_radar_processing_amd import params as P
from oracle import oracle as O
from tests.helpers import TOL_FP32_DB, TOL_FP32_REL_L2, rel_l2

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
NAMES = ["deployed_f8", "config1_f1", "config2_f2", "config3_f2"]


def load(name):
    return dict(np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False))


def inputs(g):
    nts, pn, nr, nd, F = (int(g[k]) for k in ("nts", "pn", "nr", "nd", "F"))
    p = O.derive_params(P.deployed_device(nts, pn), nr=nr, nd=nd, parity=bool(g["parity"]))
    iq = g["iq"] if "iq" in g else O.synth_frames(F, pn, nts, nr, nd, p["dist_per_bin"], frame0=int(g["frame0"]))
    assert float(np.abs(iq).astype(np.float64).sum()) == pytest.approx(float(g["iq_checksum"]), rel=1e-12)
    return p, iq


@pytest.mark.parametrize("name", NAMES)
def test_oracle_reproduces_golden(name):
    g = load(name)
    p, iq = inputs(g)
    wr, wd = O.windows(p["nts"], p["pn"])
    out = O.process_frames(iq, O.synth_cal(p["nts"]), p, wr, wd, want_rd=True, rd_all_rows=True)
    for k in ("tgt_count", "tgt_range_idx", "tgt_doppler_idx"):
        np.testing.assert_array_equal(out[k], g[k])
    for k in ("profile", "tgt_range_mag", "slow_mag"):
        np.testing.assert_allclose(out[k], g[k], rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(np.linalg.norm(out["rd"], axis=2), g["rd_row_norms"], rtol=1e-12)
    if "stft_intensity" in g:
        sp = O.spectrogram_pipeline(g["slow_signal"], float(g["prt"]), O.stft_window("kaiser"), 19)
        np.testing.assert_allclose(sp["intensity"], g["stft_intensity"], atol=1e-9)


@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES)
def test_gpu_reproduces_golden(engine, name):
    g = load(name)
    p, iq = inputs(g)
    cfg = P.derive_params(P.deployed_device(p["nts"], p["pn"]), nr=p["nr"], nd=p["nd"],
                          mode=P.PARITY if g["parity"] else P.THROUGHPUT)
    wr, wd = O.windows(p["nts"], p["pn"])
    engine.set_taps(cfg, O.synth_cal(p["nts"]), wr, wd)
    got = engine.process(iq, want_rd=True)
    for k in ("tgt_count", "tgt_range_idx", "tgt_doppler_idx"):
        np.testing.assert_array_equal(got[k], g[k])
    assert rel_l2(got["profile"], g["profile"], axis=1).max() <= TOL_FP32_REL_L2
    has = g["tgt_count"] > 0
    assert rel_l2(got["slow_mag"][has], g["slow_mag"][has], axis=1).max() <= TOL_FP32_REL_L2
    for f in np.nonzero(has)[0]:
        row = got["rd"][f, g["tgt_range_idx"][f, 0] - 1]
        assert rel_l2(row, g["target_rd_rows"][f]) <= TOL_FP32_REL_L2
    if "stft_intensity" in g:
        st = engine.stft(g["slow_signal"], O.stft_window("kaiser"), 19, 1 / float(g["prt"]))
        ref = g["stft_intensity"].T
        sel = ref > -80
        assert np.abs(st["intensity"][sel] - ref[sel]).max() <= TOL_FP32_DB
