"""A/B of 8-byte vs 16-byte (pair) global access in one process (interleaved rounds)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from fmcw_radar_processing_amd import params as P, FMCW_C64
from fmcw_radar_processing_amd.engine import Engine

def setup(cfgname, F, chunk):
    cfg = P.config(cfgname)
    e = Engine(0); e.set_taps(cfg, P.synth_calibration(cfg.nts)); e.set_chunk_frames(chunk)
    dev = "cuda"; s = torch.cuda.current_stream()
    d_iq = torch.empty((F, cfg.pn, cfg.nts, 2), dtype=torch.float32, device=dev)
    e.synth_device(d_iq, 0, F, FMCW_C64, stream=s)
    M = 1
    outs = dict(profile=torch.empty((F, cfg.nr), device=dev), tgt_count=torch.empty(F, dtype=torch.int32, device=dev),
                tgt_range_idx=torch.empty((F, M), dtype=torch.int32, device=dev), tgt_range_mag=torch.empty((F, M), device=dev),
                tgt_doppler_idx=torch.empty((F, M), dtype=torch.int32, device=dev), slow_mag=torch.empty((F, cfg.pn), device=dev))
    d_rd = torch.empty((F, cfg.nr, cfg.nd, 2), dtype=torch.float32, device=dev)
    return e, d_iq, outs, d_rd, s

def timed(e, d_iq, outs, d_rd, s, F, reps=5, level=0):
    e.process_device(d_iq, F, FMCW_C64, outs, d_rd=d_rd, stream=s); torch.cuda.synchronize()
    e.timing(level); e.timing_reset()
    t0 = time.perf_counter()
    for _ in range(reps): e.process_device(d_iq, F, FMCW_C64, outs, d_rd=d_rd, stream=s)
    torch.cuda.synchronize(); dt = (time.perf_counter() - t0) / reps
    tm = e.timing_read() if level else {}
    e.timing(0)
    return dt, tm

if __name__ == "__main__":
    for cfgname, F, chunk in ((3, 4096, 128), (2, 4096, 256)):
        st = setup(cfgname, F, chunk)
        res = {"0": [], "1": []}
        for rnd in range(4):
            for mode in ("0", "1"):
                os.environ["FMCW_PAIR"] = mode
                dt, tm = timed(*st, F, level=2 if rnd == 3 else 0)
                res[mode].append(dt * 1e3)
                if tm:
                    print(f"cfg{cfgname} pair={mode} per-kernel:", {k: round(v[0]/5, 3) for k, v in tm.items() if v[1]}, flush=True)
        for mode in ("0", "1"):
            print(f"cfg{cfgname} pair={mode} ms/step rounds: {[round(x,3) for x in res[mode]]}  fps {F/min(res[mode])*1e3/1e6:.3f} M", flush=True)
        st[0].close()
