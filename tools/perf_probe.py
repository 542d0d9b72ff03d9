"""Development probe: device timing of the per-frame schedules (not the bench).

usage: python tools/perf_probe.py [streams] [fused:NSLOT ...] [range]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from fmcw_radar_processing_amd import FMCW_C64  # noqa: E402
from fmcw_radar_processing_amd import params as P  # noqa: E402
from fmcw_radar_processing_amd.engine import Engine  # noqa: E402


def _outs(cfg, F, dev):
    M = cfg.max_targets
    return dict(profile=torch.empty((F, cfg.nr), device=dev), tgt_count=torch.empty(F, dtype=torch.int32, device=dev),
                tgt_range_idx=torch.empty((F, M), dtype=torch.int32, device=dev),
                tgt_range_mag=torch.empty((F, M), device=dev),
                tgt_doppler_idx=torch.empty((F, M), dtype=torch.int32, device=dev),
                slow_mag=torch.empty((F, cfg.pn), device=dev))


def per_frame(mode, nslot=0, F=4096, reps=10):
    cfg = P.config(3)
    e = Engine(0)
    e.set_taps(cfg, P.synth_calibration(cfg.nts))
    e.set_pipeline({"streams": 1, "fused": 2}[mode], nslot)
    dev = "cuda"
    d_iq = torch.empty((F, cfg.pn, cfg.nts, 2), dtype=torch.float32, device=dev)
    s = torch.cuda.current_stream()
    e.synth_device(d_iq, 0, F, FMCW_C64, stream=s)
    outs = _outs(cfg, F, dev)
    d_rd = torch.empty((F, cfg.nr, cfg.nd, 2), dtype=torch.float32, device=dev)
    e.process_device(d_iq, F, FMCW_C64, outs, d_rd=d_rd, stream=s)
    torch.cuda.synchronize()
    e.timing(2)
    e.timing_reset()
    for _ in range(reps):
        e.process_device(d_iq, F, FMCW_C64, outs, d_rd=d_rd, stream=s)
    torch.cuda.synchronize()
    tm = e.timing_read()
    span = tm["range_doppler"][0] / reps
    byt = F * (cfg.pn * cfg.nts * 8 + cfg.nr * cfg.nd * 8 + cfg.nr * 4 + cfg.pn * 4)
    print(f"cfg3 {mode} nslot={nslot}: span {span:.3f} ms  {F / span / 1e3:.3f} Mframes/s  "
          f"alg {byt / span / 1e9:.2f} TB/s  status={e.pipeline_status()}", flush=True)
    for k, (ms, n) in tm.items():
        if n and k != "range_doppler":
            print(f"    {k:12s} {ms / reps:8.3f} ms/step  launches/step {n / reps:.0f}  avg {ms / n * 1e3:.1f} us",
                  flush=True)
    e.close()


def range_only(F=4096, reps=10):
    cfg = P.config(2)
    e = Engine(0)
    e.set_taps(cfg, P.synth_calibration(cfg.nts))
    dev = "cuda"
    d_iq = torch.empty((F, cfg.pn, cfg.nts, 2), dtype=torch.float32, device=dev)
    s = torch.cuda.current_stream()
    e.synth_device(d_iq, 0, F, FMCW_C64, stream=s)
    d_cube = torch.empty((F, cfg.pn, cfg.nr, 2), dtype=torch.float32, device=dev)
    d_prof = torch.empty((F, cfg.nr), dtype=torch.float32, device=dev)
    e.range_fft_device(d_iq, F, FMCW_C64, d_cube, d_prof, stream=s)
    torch.cuda.synchronize()
    e.timing(1)
    e.timing_reset()
    for _ in range(reps):
        e.range_fft_device(d_iq, F, FMCW_C64, d_cube, d_prof, stream=s)
    torch.cuda.synchronize()
    ms = e.timing_read()["range_only"][0] / reps
    byt = F * (cfg.pn * cfg.nts * 8 + cfg.pn * cfg.nr * 8 + cfg.nr * 4)
    print(f"cfg2 range-only: {ms:.3f} ms  {F / ms / 1e3:.3f} Mframes/s  alg {byt / ms / 1e9:.2f} TB/s", flush=True)
    e.close()


if __name__ == "__main__":
    args = sys.argv[1:] or ["streams", "fused:2", "fused:3", "range"]
    for a in args:
        if a == "range":
            range_only()
        elif a.startswith("fused"):
            per_frame("fused", int(a.split(":")[1]) if ":" in a else 0)
        else:
            per_frame(a)
