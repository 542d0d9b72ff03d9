"""k_rdx beside another resident kernel.

k_rdx's 256 workgroups wait on each other (the XCD-team hand-off of kernels_xcd.hip), so they
must be resident together.  The context checks the grid against the occupancy query once (a
cooperative launch would check it per launch, FMCW_XCD_COOP=1, and is run here too), but a
kernel of ANOTHER stream that holds a CU is outside that check -- the RCCL kernels of a
torchrun job, or another process.  Here a single-wave spin kernel
(torch.cuda._sleep) on a second stream holds one CU while k_rdx runs on the first: one k_rdx
workgroup cannot start until the spin ends (k_rdx's 2 waves x 256 VGPRs fill every SIMD).
The contract: either the outputs equal those of an undisturbed run bit for bit (the blocked
member started before its team's bounded waits ran out), or fmcw_synchronize reports
FMCW_E_HIP ("hand-off timed out") -- never silently wrong data, never a hang.
"""
import time

import numpy as np
import pytest

from fmcw_radar_processing_amd import FMCW_C64, FmcwError
from fmcw_radar_processing_amd import params as P
from fmcw_radar_processing_amd import _lib
from tests.helpers import case

pytestmark = pytest.mark.gpu

F = 48                                   # 6 frames per XCD team


def _run(engine, cfg, d_iq, stream):
    import torch
    M = cfg.max_targets
    outs = dict(profile=torch.empty((F, cfg.nr), device="cuda"),
                tgt_count=torch.empty(F, dtype=torch.int32, device="cuda"),
                tgt_range_idx=torch.empty((F, M), dtype=torch.int32, device="cuda"),
                tgt_range_mag=torch.empty((F, M), device="cuda"),
                tgt_doppler_idx=torch.empty((F, M), dtype=torch.int32, device="cuda"),
                slow_mag=torch.empty((F, cfg.pn), device="cuda"))
    d_rd = torch.empty((F, cfg.nr, cfg.nd, 2), dtype=torch.float32, device="cuda")
    engine.process_device(d_iq, F, FMCW_C64, outs, d_rd=d_rd, out_dtype=FMCW_C64, stream=stream)
    return outs, d_rd


def _host(outs, d_rd):
    return {k: v.cpu().numpy() for k, v in outs.items()} | {"rd": d_rd.cpu().numpy()}


@pytest.mark.parametrize("coop", [False, True])
@pytest.mark.parametrize("hold_s", [0.25, 2.5])
def test_rdx_beside_a_resident_kernel(engine, monkeypatch, hold_s, coop):
    import torch
    monkeypatch.setenv("FMCW_XCD_COOP", "1" if coop else "0")
    cfg, p, wr, wd, cal = case(1024, 256, 1024, 256, P.THROUGHPUT)
    engine.set_taps(cfg, cal, wr, wd)
    engine.set_pipeline(_lib.FMCW_PIPE_XCD)
    try:
        s_main = torch.cuda.Stream()
        s_hog = torch.cuda.Stream()
        d_iq = torch.empty((F, cfg.pn, cfg.nts, 2), dtype=torch.float32, device="cuda")
        engine.synth_device(d_iq, 0, F, FMCW_C64, stream=s_main)
        ref = _run(engine, cfg, d_iq, s_main)
        torch.cuda.synchronize()
        engine.synchronize()
        ref = _host(*ref)
        # the spin kernel holds one CU (one wave) for hold_s; clock64 counts the shader clock
        cycles = int(hold_s * 2.4e9)
        with torch.cuda.stream(s_hog):
            torch.cuda._sleep(cycles)
        time.sleep(0.02)                     # the spin wave is resident before k_rdx is queued
        t0 = time.time()
        got = _run(engine, cfg, d_iq, s_main)
        torch.cuda.synchronize()
        wall = time.time() - t0
        try:
            engine.synchronize()
        except FmcwError as e:
            assert e.status == _lib.FMCW_E_HIP and "timed out" in str(e), e
            print(f"hold {hold_s} s: FMCW_E_HIP after {wall:.2f} s ({e})")
            # the launches after a timed-out one start from clean counters (two counter sets per context,
            # each launch zeroing the other, kernels_xcd.hip): two undisturbed runs equal the reference
            for _ in range(2):
                again = _run(engine, cfg, d_iq, s_main)
                torch.cuda.synchronize()
                engine.synchronize()
                again = _host(*again)
                for k in ref:
                    np.testing.assert_array_equal(again[k], ref[k], err_msg=k)
            return
        got = _host(*got)
        for k in ref:
            np.testing.assert_array_equal(got[k], ref[k], err_msg=k)
        print(f"hold {hold_s} s: outputs bit-identical, {wall:.2f} s")
    finally:
        engine.set_pipeline(_lib.FMCW_PIPE_AUTO)
        torch.cuda.synchronize()
