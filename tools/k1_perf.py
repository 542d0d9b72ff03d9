"""Device-side timing of BASELINE config 2 (K1 k_range<512>, range FFT only, cube + profile
written) at 4096 frames (development probe; bench.py's config2_range_fft key times the same)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from fmcw_radar_processing_amd import FMCW_C64  # noqa: E402
from fmcw_radar_processing_amd import params as P  # noqa: E402
from fmcw_radar_processing_amd.engine import Engine  # noqa: E402


def main(F=4096, reps=20):
    cfg = P.config(2)
    e = Engine(0)
    e.set_taps(cfg, P.synth_calibration(cfg.nts))
    d_iq = torch.empty((F, cfg.pn, cfg.nts, 2), dtype=torch.float32, device="cuda")
    s = torch.cuda.current_stream()
    e.synth_device(d_iq, 0, F, FMCW_C64, stream=s)
    d_cube = torch.empty((F, cfg.pn, cfg.nr, 2), dtype=torch.float32, device="cuda")
    d_prof = torch.empty((F, cfg.nr), dtype=torch.float32, device="cuda")
    for _ in range(3):
        e.range_fft_device(d_iq, F, FMCW_C64, d_cube, d_prof, stream=s)
    torch.cuda.synchronize()
    e.timing(1)
    e.timing_reset()
    t0 = time.perf_counter()
    for _ in range(reps):
        e.range_fft_device(d_iq, F, FMCW_C64, d_cube, d_prof, stream=s)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    ms, n = e.timing_read()["range_only"]
    byt = F * (cfg.pn * cfg.nts * 8 + cfg.pn * cfg.nr * 8 + cfg.nr * 4)
    us = ms / n * 1e3
    # the same process's copy of K1's in + cube bytes (bench.py's config-2 copy ceiling, k_copy16)
    nb = d_iq.numel() * d_iq.element_size()
    d_cp = torch.empty(nb // 4, dtype=torch.float32, device="cuda")
    e.copy_device(d_iq, d_cp, nb, stream=s)
    torch.cuda.synchronize()
    ca, cb = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ca.record(s)
    for _ in range(reps):
        e.copy_device(d_iq, d_cp, nb, stream=s)
    cb.record(s)
    torch.cuda.synchronize()
    cus = ca.elapsed_time(cb) / reps * 1e3
    print(f"k1 cfg2 F={F}: {dt * 1e3:.3f} ms/step, K1 {us:.1f} us, {byt / (us * 1e-6) / 1e12:.2f} TB/s "
          f"(frac {byt / (us * 1e-6) / 8e12:.3f}), copy {cus:.1f} us (K1 at {cus / us:.3f} of it)", flush=True)
    e.close()


if __name__ == "__main__":
    main(*[int(x) for x in sys.argv[1:3]])
