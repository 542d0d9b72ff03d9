"""Device-side timing of the range+Doppler(+detect) path per schedule (development probe).

python tools/onepass_perf.py [F] [reps] [streams,onepass] -> one line per schedule: ms per F frames, frames/s,
algorithmic TB/s (SURVEY 8d config-3 bytes), and the per-kernel event averages.
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from fmcw_radar_processing_amd import FMCW_C32H, FMCW_C64, FMCW_PIPE_ONEPASS, FMCW_PIPE_STREAMS, FMCW_PIPE_XCD  # noqa: E402
from fmcw_radar_processing_amd import params as P  # noqa: E402
from fmcw_radar_processing_amd.engine import Engine  # noqa: E402


def main(F=4096, reps=10, which="streams,onepass"):
    cfg = P.config(3)
    e = Engine(0)
    e.set_taps(cfg, P.synth_calibration(cfg.nts))
    dev = "cuda"
    s = torch.cuda.current_stream()
    fp16 = os.environ.get("FP16", "0") == "1"          # config-4 fp16 storage: c32h in, c32h RD out
    dt = FMCW_C32H if fp16 else FMCW_C64
    tdt = torch.float16 if fp16 else torch.float32
    d_iq = torch.empty((F, cfg.pn, cfg.nts, 2), dtype=tdt, device=dev)
    e.synth_device(d_iq, 0, F, dt, stream=s)
    M = cfg.max_targets
    outs = dict(profile=torch.empty((F, cfg.nr), device=dev), tgt_count=torch.empty(F, dtype=torch.int32, device=dev),
                tgt_range_idx=torch.empty((F, M), dtype=torch.int32, device=dev),
                tgt_range_mag=torch.empty((F, M), device=dev),
                tgt_doppler_idx=torch.empty((F, M), dtype=torch.int32, device=dev),
                slow_mag=torch.empty((F, cfg.pn), device=dev))
    d_rd = torch.empty((F, cfg.nr, cfg.nd, 2), dtype=tdt, device=dev)
    if os.environ.get("NORD", "0") == "1":      # no RD map (row peaks only): the RD stores' share of the time
        d_rd = None
    es = 4 if fp16 else 8
    byt = F * (cfg.pn * cfg.nts * es + cfg.nr * cfg.nd * es + cfg.nr * 4 + cfg.pn * 4)
    modes = {"streams": FMCW_PIPE_STREAMS, "onepass": FMCW_PIPE_ONEPASS, "xcd": FMCW_PIPE_XCD}
    for name in which.split(","):
        mode = modes[name]
        e.set_pipeline(mode)
        e.process_device(d_iq, F, dt, outs, d_rd=d_rd, out_dtype=dt, stream=s)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            e.process_device(d_iq, F, dt, outs, d_rd=d_rd, out_dtype=dt, stream=s)
        torch.cuda.synchronize()
        el = (time.perf_counter() - t0) / reps
        print(f"{name + ('16' if fp16 else ''):8s} F={F}: {el * 1e3:.3f} ms  {F / el / 1e6:.3f} Mframes/s  alg {byt / el / 1e12:.2f} TB/s "
              f"(frac {byt / el / 8e12:.3f})", flush=True)
        e.timing(2)
        e.timing_reset()
        for _ in range(reps):
            e.process_device(d_iq, F, dt, outs, d_rd=d_rd, out_dtype=dt, stream=s)
        tm = e.timing_read()
        e.timing(0)
        if name == "xcd":
            mhz, us = e.rdx_clock()
            print(f"   sclk {mhz:.0f} MHz (last k_rdx, {us:.0f} us stamped)", flush=True)
        for k, (ms, n) in tm.items():
            if n:
                print(f"   {k:14s} {ms / reps:8.3f} ms/step  launches/step {n / reps:.0f}  avg {ms / n * 1e3:.1f} us",
                      flush=True)
    e.close()


if __name__ == "__main__":
    a = sys.argv[1:]
    main(*[int(x) for x in a[:2]], *a[2:3])
