"""Device timing of the config-4 STFT leg alone (development probe).

python tools/stft_perf.py [reps] [forms]  -> per form: us per call (HIP events around `reps` calls)
forms (comma list): max (pass 1, max(P) only), direct (pass 2, dB recomputed), stored (pass 1 with
P written), flat (k_stft_db_flat in place), leg_direct (max + direct), leg_stored (stored + flat).
Input: the bench's own slow-time rows (4096 config-4 frames through process_slow_device).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from fmcw_radar_processing_amd import FMCW_C64  # noqa: E402
from fmcw_radar_processing_amd import params as P  # noqa: E402
from fmcw_radar_processing_amd.engine import Engine  # noqa: E402


def main(reps=50, forms="max,direct,stored,flat,leg_direct,leg_stored"):
    F = 4096
    cfg = P.config(4)
    e = Engine(0)
    e.set_taps(cfg, P.synth_calibration(cfg.nts))
    dev = "cuda"
    s = torch.cuda.Stream()
    torch.cuda.set_stream(s)
    C = cfg.pn
    d_iq = torch.empty((F, C, cfg.nts, 2), dtype=torch.float32, device=dev)
    e.synth_device(d_iq, 0, F, FMCW_C64, stream=s)
    M = cfg.max_targets
    outs = dict(profile=torch.empty((F, cfg.nr), device=dev), tgt_count=torch.empty(F, dtype=torch.int32, device=dev),
                tgt_range_idx=torch.empty((F, M), dtype=torch.int32, device=dev),
                tgt_range_mag=torch.empty((F, M), device=dev),
                tgt_doppler_idx=torch.empty((F, M), dtype=torch.int32, device=dev),
                slow_mag=torch.empty((F, C), device=dev))
    flist = torch.empty(F, dtype=torch.int32, device=dev)
    d_len = torch.zeros(1, dtype=torch.int64, device=dev)
    pmax = torch.zeros(1, dtype=torch.float32, device=dev)
    e.process_slow_device(d_iq, F, FMCW_C64, outs, flist, d_len, d_pmax=pmax, stream=s)
    del d_iq
    win = torch.tensor(cfg.stft_window(), dtype=torch.float32, device=dev)
    fs = 1.0 / cfg.prt
    max_seg = F * C + 19
    d_P = torch.empty((max_seg, 33), dtype=torch.float32, device=dev)
    nseg = torch.zeros(1, dtype=torch.int64, device=dev)
    slow = outs["slow_mag"]

    def f_max():
        e.stft_power_device(slow, flist, d_len, C, win, 20, 19, 64, fs, max_seg, None, pmax, nseg, stream=s)

    def f_direct():
        e.stft_db_direct_device(slow, flist, d_len, C, win, 20, 19, 64, fs, max_seg, pmax, d_P, stream=s)

    def f_stored():
        e.stft_power_device(slow, flist, d_len, C, win, 20, 19, 64, fs, max_seg, d_P, pmax, nseg, stream=s)

    def f_flat():
        e.stft_db_device(d_P, nseg, max_seg, 64, fs, pmax, 0, d_P, stream=s)

    table = {"max": [f_max], "direct": [f_direct], "stored": [f_stored], "flat": [f_flat],
             "leg_direct": [f_max, f_direct], "leg_stored": [f_stored, f_flat]}
    f_stored()
    torch.cuda.synchronize()
    print(f"L = {int(d_len.item())}, nseg = {int(nseg.item())}", flush=True)
    for name in forms.split(","):
        fns = table[name]
        for f in fns:
            f()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        for _ in range(reps):
            for f in fns:
                f()
        b.record(s)
        torch.cuda.synchronize()
        print(f"{name:11s} {a.elapsed_time(b) / reps * 1e3:8.1f} us per call", flush=True)
    e.close()


if __name__ == "__main__":
    a = sys.argv[1:]
    main(int(a[0]) if a else 50, *(a[1:2]))
