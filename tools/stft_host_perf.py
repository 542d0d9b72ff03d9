"""Host-pointer fmcw_stft at the reference nfft rule (1024 log bins): wall clock vs the
kernels' HIP-event stage times.  python tools/stft_host_perf.py [L ...]   (GPU)"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from fmcw_radar_processing_amd import params as P
    from fmcw_radar_processing_amd import windows as W
    from fmcw_radar_processing_amd.engine import Engine
    eng = Engine(0)
    cfg = P.config(3)
    eng.set_taps(cfg, P.synth_calibration(cfg.nts))
    win = W.kaiser(20, 3.0)
    for L in [int(v) for v in sys.argv[1:]] or [1840, 59000]:
        x = np.abs(np.random.default_rng(L).standard_normal(L)).astype(np.float32)
        eng.stft(x, win, 19, 1250.0)
        eng.timing(2)
        eng.timing_reset()
        t = time.perf_counter()
        R = 5
        for _ in range(R):
            r = eng.stft(x, win, 19, 1250.0)
        wall = (time.perf_counter() - t) / R * 1e3
        st = {k: round(v[0] / R, 3) for k, v in eng.timing_read().items() if v[1]}
        eng.timing(0)
        t = time.perf_counter()
        o = np.empty_like(r["intensity"])
        o[...] = 0
        touch = (time.perf_counter() - t) * 1e3
        print(f"L={L} nfft={r['nfft']} out={r['intensity'].shape} wall {wall:.2f} ms  stages(ms) {st}  "
              f"first-touch of an output-sized array {touch:.2f} ms", flush=True)
    eng.close()


if __name__ == "__main__":
    main()
