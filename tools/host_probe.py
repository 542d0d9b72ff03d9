"""Host-path timing probe (development): the deployed module's 115-frame call (fmcw_process +
fmcw_stft on pageable host arrays, radar_processing.m:197-299), repeated; run it under
rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --stats to see where a call's time goes."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from fmcw_radar_processing_amd import FMCW_C64  # noqa: E402
from fmcw_radar_processing_amd import params as P  # noqa: E402
from fmcw_radar_processing_amd import windows as W  # noqa: E402
from fmcw_radar_processing_amd.engine import Engine  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
geom = sys.argv[2] if len(sys.argv) > 2 else "deployed"     # or "3": 256 config-3 frames (bench host_path)
eng = Engine(0)
cfg = P.config("deployed" if geom == "deployed" else int(geom))
eng.set_taps(cfg, P.synth_calibration(cfg.nts))
F = 115 if geom == "deployed" else 256
d = torch.empty((F, cfg.pn, cfg.nts, 2), dtype=torch.float32, device="cuda")
eng.synth_device(d, 0, F, FMCW_C64)
torch.cuda.synchronize()
iq = d.cpu().numpy().view(np.complex64)[..., 0].copy()
win = W.kaiser(20, 3.0)
fs = 1.0 / cfg.prt
out = eng.process(iq)
x = out["slow_mag"][out["tgt_count"] > 0].reshape(-1)
eng.stft(x, win, 19, fs)
tp = ts = 0.0
for _ in range(reps):
    t = time.perf_counter()
    out = eng.process(iq)
    tp += time.perf_counter() - t
    t = time.perf_counter()
    eng.stft(x, win, 19, fs)
    ts += time.perf_counter() - t
print(f"process {tp / reps * 1e3:.3f} ms  stft {ts / reps * 1e3:.3f} ms  calls/s {reps / (tp + ts):.0f}  (L = {len(x)})", flush=True)
eng.close()
