"""GPU: the fused XCD-local schedule (kernels_fused.hip) against the oracle and
against the 3-stream schedule.

The two schedules run the same per-frame device functions (frame_ops.h) in
the same arithmetic order, so their outputs must agree bit for bit; the
oracle comparison uses the SURVEY.md 8d fp32 tolerances.
"""
import numpy as np
import pytest

from fmcw_radar_processing_amd import (FMCW_C32H, FMCW_PIPE_AUTO, FMCW_PIPE_FUSED, FMCW_PIPE_STREAMS,
                                       FmcwError)
from fmcw_radar_processing_amd import params as P
from oracle import oracle as O
from tests.helpers import TOL_FP32_REL_L2, case, near_tie_frames, rd_rel_err, rel_l2

pytestmark = pytest.mark.gpu

GEOM = (1024, 256, 1024, 256)      # configs 3/4: the geometry with a fused kernel
KEYS = ("profile", "tgt_count", "tgt_range_idx", "tgt_range_mag", "tgt_doppler_idx", "slow_mag", "probe_mag")


def _frames(F, frame0=0):
    cfg, p, wr, wd, cal = case(*GEOM, P.THROUGHPUT)
    iq = O.synth_frames(F, GEOM[1], GEOM[0], GEOM[2], GEOM[3], p["dist_per_bin"], frame0=frame0)
    return cfg, p, wr, wd, cal, iq


@pytest.fixture
def fused(engine):
    yield engine
    engine.set_pipeline(FMCW_PIPE_AUTO, 0)


# F < 8 leaves XCDs idle; 19 gives them 2 or 3 frames (ragged queues); 37
# runs several slot generations per XCD
@pytest.mark.parametrize("F,nslot", [(3, 2), (19, 2), (37, 2), (37, 3)])
def test_fused_matches_oracle(fused, F, nslot):
    cfg, p, wr, wd, cal, iq = _frames(F, frame0=100)
    fused.set_taps(cfg, cal, wr, wd)
    fused.set_pipeline(FMCW_PIPE_FUSED, nslot)
    probe = min(100 + 256 * (F // 2), F * 256)
    got = fused.process(iq, want_rd=True, probe_column=probe)
    assert fused.pipeline_status() == 0
    ref = O.process_frames(iq, cal, p, wr, wd, want_cube=True, want_rd=True, rd_all_rows=True)
    assert rd_rel_err(got["rd"], ref["rd"], ref["cube"], wd, cfg.nd).max() <= TOL_FP32_REL_L2
    assert rel_l2(got["profile"], ref["profile"], axis=1).max() <= TOL_FP32_REL_L2
    ok = ~near_tie_frames(ref["profile"])
    for k in ("tgt_count", "tgt_range_idx", "tgt_doppler_idx"):
        np.testing.assert_array_equal(got[k][ok], ref[k][ok])
    np.testing.assert_allclose(got["tgt_range_mag"], ref["tgt_range_mag"], rtol=1e-5, atol=0)
    has = ref["tgt_count"] > 0
    if has.any():
        assert rel_l2(got["slow_mag"][has], ref["slow_mag"][has], axis=1).max() <= TOL_FP32_REL_L2
    assert np.all(got["slow_mag"][~has] == 0)
    col = probe - 1
    want = np.abs(ref["cube"][col // 256, col % 256, :])
    assert rel_l2(got["probe_mag"], want) <= TOL_FP32_REL_L2


@pytest.mark.parametrize("want_rd", [True, False])
def test_fused_equals_streams_bitwise(fused, want_rd):
    cfg, p, wr, wd, cal, iq = _frames(21, frame0=7)
    fused.set_taps(cfg, cal, wr, wd)
    fused.set_pipeline(FMCW_PIPE_STREAMS)
    a = fused.process(iq, want_rd=want_rd, probe_column=300)
    fused.set_pipeline(FMCW_PIPE_FUSED)
    b = fused.process(iq, want_rd=want_rd, probe_column=300)
    for k in KEYS + (("rd",) if want_rd else ()):
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)


def test_fused_fp16_equals_streams_bitwise(fused):
    """fp16 IQ in, fp16 RD out (fp32 arithmetic): both schedules agree bit for bit."""
    import torch
    cfg, p, wr, wd, cal, iq = _frames(11, frame0=3)
    fused.set_taps(cfg, cal, wr, wd)
    F = iq.shape[0]
    d_iq = torch.from_numpy(np.stack([iq.real, iq.imag], -1).astype(np.float16)).cuda()
    res = []
    for mode in (FMCW_PIPE_STREAMS, FMCW_PIPE_FUSED):
        fused.set_pipeline(mode)
        outs = dict(profile=torch.empty((F, 1024), device="cuda"),
                    tgt_count=torch.empty(F, dtype=torch.int32, device="cuda"),
                    tgt_range_idx=torch.empty((F, 1), dtype=torch.int32, device="cuda"),
                    tgt_range_mag=torch.empty((F, 1), device="cuda"),
                    tgt_doppler_idx=torch.empty((F, 1), dtype=torch.int32, device="cuda"),
                    slow_mag=torch.empty((F, 256), device="cuda"))
        d_rd = torch.empty((F, 1024, 256, 2), dtype=torch.float16, device="cuda")
        fused.process_device(d_iq, F, FMCW_C32H, outs, d_rd=d_rd, out_dtype=FMCW_C32H,
                             stream=torch.cuda.current_stream())
        torch.cuda.synchronize()
        res.append({k: v.cpu().numpy() for k, v in outs.items()} | {"rd": d_rd.cpu().numpy()})
    assert fused.pipeline_status() == 0
    for k in res[0]:
        np.testing.assert_array_equal(res[0][k], res[1][k], err_msg=k)


def test_fused_rejects_cube_request(fused):
    cfg, p, wr, wd, cal, iq = _frames(2)
    fused.set_taps(cfg, cal, wr, wd)
    fused.set_pipeline(FMCW_PIPE_FUSED)
    with pytest.raises(FmcwError, match="E_ARG"):
        fused.process(iq, want_cube=True)


def test_fused_rejects_unsupported_geometry(fused):
    cfg, p, wr, wd, cal = case(64, 16, 256, 16, P.PARITY)
    iq = O.synth_frames(2, 16, 64, 256, 16, p["dist_per_bin"])
    fused.set_taps(cfg, cal, wr, wd)
    fused.set_pipeline(FMCW_PIPE_FUSED)
    with pytest.raises(FmcwError, match="E_ARG"):
        fused.process(iq)


def test_set_pipeline_validates(fused):
    with pytest.raises(FmcwError, match="E_ARG"):
        fused.set_pipeline(7)
    with pytest.raises(FmcwError, match="E_ARG"):
        fused.set_pipeline(FMCW_PIPE_FUSED, 1)
