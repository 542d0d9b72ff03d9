"""Quick device-side timing of the per-frame path (development probe)."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from fmcw_radar_processing_amd import params as P, FMCW_C64
from fmcw_radar_processing_amd.engine import Engine

def run(cfgname, F, chunk=0, reps=5):
    cfg = P.config(cfgname)
    e = Engine(0)
    e.set_taps(cfg, P.synth_calibration(cfg.nts))
    if chunk: e.set_chunk_frames(chunk)
    dev = "cuda"
    d_iq = torch.empty((F, cfg.pn, cfg.nts, 2), dtype=torch.float32, device=dev)
    s = torch.cuda.current_stream()
    e.synth_device(d_iq, 0, F, FMCW_C64, stream=s)
    M = cfg.max_targets
    outs = dict(profile=torch.empty((F, cfg.nr), device=dev), tgt_count=torch.empty(F, dtype=torch.int32, device=dev),
                tgt_range_idx=torch.empty((F, M), dtype=torch.int32, device=dev), tgt_range_mag=torch.empty((F, M), device=dev),
                tgt_doppler_idx=torch.empty((F, M), dtype=torch.int32, device=dev), slow_mag=torch.empty((F, cfg.pn), device=dev))
    d_rd = torch.empty((F, cfg.nr, cfg.nd, 2), dtype=torch.float32, device=dev)
    e.process_device(d_iq, F, FMCW_C64, outs, d_rd=d_rd, stream=s)
    torch.cuda.synchronize()
    e.timing(2); e.timing_reset()
    t0 = time.perf_counter()
    for _ in range(reps):
        e.process_device(d_iq, F, FMCW_C64, outs, d_rd=d_rd, stream=s)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    tm = e.timing_read()
    byt = F * (cfg.pn * cfg.nts * 8 + cfg.nr * cfg.nd * 8 + cfg.nr * 4 + cfg.pn * 8)
    print(f"{cfgname} F={F} chunk={chunk}: {dt*1e3:.3f} ms/step {F/dt/1e6:.3f} Mframes/s alg {byt/dt/1e12:.2f} TB/s", flush=True)
    for k, (ms, n) in tm.items():
        if n: print(f"   {k:12s} {ms/reps:8.3f} ms/step  launches/step {n/reps:.0f}  avg {ms/n*1e3:.1f} us", flush=True)
    e.timing(0)
    # untimed-events run
    t0 = time.perf_counter()
    for _ in range(reps):
        e.process_device(d_iq, F, FMCW_C64, outs, d_rd=d_rd, stream=s)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    print(f"   no-events: {dt*1e3:.3f} ms/step {F/dt/1e6:.3f} Mframes/s", flush=True)
    e.close()

if __name__ == "__main__":
    import sys as _s
    chunks = [int(c) for c in _s.argv[1:]] or [64, 128, 256]
    for ch in chunks:
        run(3, 4096, chunk=ch)
    run(2, 4096, chunk=256)
