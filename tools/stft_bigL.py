"""Timing probe: the reference nfft rule (2^nextpow2(L)) at config-3/4 scale through the host API
(fmcw_stft: max(P) over every bin, then P of the 1024 log-bin columns only)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from fmcw_radar_processing_amd import params as P  # noqa: E402
from fmcw_radar_processing_amd import windows as W  # noqa: E402
from fmcw_radar_processing_amd.engine import Engine  # noqa: E402

L = int(sys.argv[1]) if len(sys.argv) > 1 else 940_000
e = Engine(0)
cfg = P.config(3)
e.set_taps(cfg, P.synth_calibration(cfg.nts))
rng = np.random.default_rng(3)
x = (np.abs(rng.standard_normal(L)) * 100 + 50 * np.abs(np.sin(np.arange(L) * 0.01))).astype(np.float32)
win = W.kaiser(20, 3.0)
fs = 1.0 / cfg.prt
e.timing(1)
e.timing_reset()
t = time.perf_counter()
sp = e.stft(x, win, 19, fs)
dt = time.perf_counter() - t
tm = e.timing_read()
print(f"L={L} nfft={sp['nfft']} nseg={sp['intensity'].shape[0]} wall {dt*1e3:.1f} ms; stages "
      + ", ".join(f"{k} {v[0]:.2f} ms" for k, v in tm.items() if v[1]), flush=True)
e.close()
