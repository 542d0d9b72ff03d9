"""Tolerance sweep (BASELINE config 4 "fp32 vs fp16 tolerance sweep"):
the measured error of the GPU path against the float64 oracle at fp32 and at
fp16 storage, on the golden geometries and on config-3 frames.

  python tools/tolerance_sweep.py [--frames 16] > sweep.json     (GPU)

Per case: max over frames of the relative L2 error of the RD map (raw: ||d||/||ref||,
and SURVEY-relaxed: denominator >= a tenth of the pre-cancellation energy, see
tests/helpers.rd_rel_err), of the range profile and of the slow-time rows;
detections that differ; max |dB error| of the spectrogram where psd > -80 dB
(fp32) / > -60 dB (fp16).  Development / DESIGN.md evidence; the pass/fail bars
are the tests'.
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=16)
    a = ap.parse_args()
    import torch
    from fmcw_radar_processing_amd import FMCW_C32H
    from fmcw_radar_processing_amd import params as P
    from fmcw_radar_processing_amd.engine import Engine
    from oracle import oracle as O
    from tests.helpers import rd_rel_err, rel_l2

    eng = Engine(0)
    out = {"note": "max over frames; rel L2 per frame; dB where psd > -80 (fp32) / -60 (fp16)", "cases": {}}
    cases = [("deployed_64x16", 64, 16, 256, 16, True, 115), ("config1_256x128", 256, 128, 256, 16, True, 8),
             ("config2_512x128", 512, 128, 512, 16, False, 8), ("config3_1024x256", 1024, 256, 1024, 256, False, a.frames)]
    for name, nts, pn, nr, nd, parity, F in cases:
        cfg = P.derive_params(P.deployed_device(nts, pn), nr=nr, nd=nd, mode=P.PARITY if parity else P.THROUGHPUT)
        p = O.derive_params(P.deployed_device(nts, pn), nr=nr, nd=nd, parity=parity)
        wr, wd = O.windows(nts, pn)
        cal = O.synth_cal(nts)
        eng.set_taps(cfg, cal, wr, wd)
        iq = O.synth_frames(F, pn, nts, nr, nd, p["dist_per_bin"])
        res = {}
        variants = [("fp32", iq)]
        if nr == 1024 and pn == 256:
            iq16 = np.stack([iq.real, iq.imag], -1).astype(np.float16)
            variants.append(("fp16", iq16))
        for prec, x in variants:
            if prec == "fp32":
                got = eng.process(x, want_rd=True)
                rd = got["rd"]
                xin = x
                slow = got["slow_mag"]
                ridx, cnt = got["tgt_range_idx"], got["tgt_count"]
            else:
                d_iq = torch.from_numpy(x).cuda()
                M = cfg.max_targets
                outs = dict(profile=torch.empty((F, nr), device="cuda"), tgt_count=torch.empty(F, dtype=torch.int32, device="cuda"),
                            tgt_range_idx=torch.empty((F, M), dtype=torch.int32, device="cuda"),
                            tgt_range_mag=torch.empty((F, M), device="cuda"),
                            tgt_doppler_idx=torch.empty((F, M), dtype=torch.int32, device="cuda"),
                            slow_mag=torch.empty((F, pn), device="cuda"))
                d_rd = torch.empty((F, nr, nd, 2), dtype=torch.float16, device="cuda")
                eng.process_device(d_iq, F, FMCW_C32H, outs, d_rd=d_rd, out_dtype=FMCW_C32H,
                                   stream=torch.cuda.current_stream())
                torch.cuda.synchronize()
                rd = d_rd.float().cpu().numpy().view(np.complex64)[..., 0].astype(np.complex128) * (nr * nd)
                got = {k: v.cpu().numpy() for k, v in outs.items()}
                slow, ridx, cnt = got["slow_mag"], got["tgt_range_idx"], got["tgt_count"]
                xin = x.astype(np.float32).view(np.complex64)[..., 0]
            ref = O.process_frames(xin, cal, p, wr, wd, want_cube=True, want_rd=True, rd_all_rows=True)
            raw = rel_l2(rd, ref["rd"], axis=(1, 2))
            relaxed = rd_rel_err(rd, ref["rd"], ref["cube"], wd, nd)
            has = ref["tgt_count"] > 0
            r = {"rd_rel_l2_raw_max": float(raw.max()), "rd_rel_l2_raw_median": float(np.median(raw)),
                 "rd_rel_l2_relaxed_max": float(relaxed.max()),
                 "profile_rel_l2_max": float(rel_l2(got["profile"], ref["profile"], axis=1).max()),
                 "slow_rel_l2_max": float(rel_l2(slow[has], ref["slow_mag"][has], axis=1).max()) if has.any() else None,
                 "detections_differing": int(np.sum(np.any(ridx != ref["tgt_range_idx"], axis=1) | (cnt != ref["tgt_count"]))),
                 "frames": F}
            xs = slow[cnt > 0].reshape(-1).astype(np.float64)
            xr = ref["slow_mag"][ref["tgt_count"] > 0].reshape(-1)
            if len(xs) >= 20 and len(xs) == len(xr):
                floor = -80 if prec == "fp32" else -60
                win = O.stft_window("kaiser")
                st = eng.stft(xs, win, 19, 1 / p["prt"])
                sp = O.spectrogram_pipeline(xr, p["prt"], win, 19)
                ri = sp["intensity"].T
                sel = ri > floor
                r["stft_db_err_max"] = float(np.abs(st["intensity"][sel] - ri[sel]).max())
                r["stft_db_floor"] = floor
            res[prec] = r
        out["cases"][name] = res
        print(name, json.dumps(res), file=sys.stderr, flush=True)
    eng.close()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
