"""Diagnostic for tests/test_gpu_fullsize.py: forward vs reversed frame order at config 4 full size."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from fmcw_radar_processing_amd import FMCW_C64, FMCW_PIPE_XCD
from fmcw_radar_processing_amd import params as P
from fmcw_radar_processing_amd.engine import Engine
from tests.test_gpu_fullsize import _process, F

cfg = P.config(4)
e = Engine(0)
e.set_taps(cfg, P.synth_calibration(cfg.nts))
e.set_pipeline(FMCW_PIPE_XCD)
d = torch.empty((F, cfg.pn, cfg.nts, 2), dtype=torch.float32, device="cuda")
e.synth_device(d, 0, F, FMCW_C64)
a = _process(e, cfg, d, FMCW_C64)
dr = d.flip(0).contiguous()
torch.cuda.synchronize()
print("flip input ok:", torch.equal(dr.flip(0), d))
r = _process(e, cfg, dr, FMCW_C64)
r2 = _process(e, cfg, dr, FMCW_C64)
torch.cuda.synchronize(); e.synchronize()
def rep(name, x, y):
    x = x.float(); y = y.float()
    rows = (x != y).reshape(F, -1).any(1)
    n = int(rows.sum())
    dif = (x - y).abs().reshape(F, -1).max(1).values
    ref = y.abs().reshape(F, -1).max(1).values
    idx = rows.nonzero().flatten()
    print(f"{name}: {n} rows differ; first {idx[:6].tolist()} last {idx[-3:].tolist()}; max abs {float(dif.max()):.3g}, max rel {float((dif/ref.clamp_min(1e-30)).max()):.3g}")
for k in a:
    rep("rev vs fwd " + k, r[k].flip(0), a[k])
for k in a:
    rep("rev run2 " + k, r2[k], r[k])
# second half alone, forward, as its own launch
d2 = d[2048:].contiguous()
from tests import test_gpu_fullsize as T
T.F = 2048
h = _process(e, cfg, d2, FMCW_C64)
torch.cuda.synchronize()
F2 = 2048
for k in ("profile", "rd"):
    x, y = h[k].float(), a[k][2048:].float()
    rows = (x != y).reshape(F2, -1).any(1)
    print(f"half-launch {k}: {int(rows.sum())} of 2048 rows differ; first {rows.nonzero().flatten()[:6].tolist()}")
