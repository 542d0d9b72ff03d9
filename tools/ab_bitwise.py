"""A/B helper: run config-4 frames (fp32 and fp16 storage) through the library named by
FMCW_LIB and save every output, or compare against a saved run (development only)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from fmcw_radar_processing_amd import FMCW_C32H, FMCW_C64  # noqa: E402
from fmcw_radar_processing_amd import params as P  # noqa: E402
from fmcw_radar_processing_amd.engine import Engine  # noqa: E402

mode, path = sys.argv[1], sys.argv[2]
F = 256
cfg = P.config(4)
e = Engine(0)
e.set_taps(cfg, P.synth_calibration(cfg.nts))
res = {}
s = torch.cuda.current_stream()
for h in (False, True):
    dt = FMCW_C32H if h else FMCW_C64
    d = torch.empty((F, cfg.pn, cfg.nts, 2), dtype=torch.float16 if h else torch.float32, device="cuda")
    e.synth_device(d, 77, F, dt, stream=s)
    M = cfg.max_targets
    o = dict(profile=torch.empty((F, cfg.nr), device="cuda"), tgt_count=torch.empty(F, dtype=torch.int32, device="cuda"),
             tgt_range_idx=torch.empty((F, M), dtype=torch.int32, device="cuda"),
             tgt_range_mag=torch.empty((F, M), device="cuda"),
             tgt_doppler_idx=torch.empty((F, M), dtype=torch.int32, device="cuda"),
             slow_mag=torch.empty((F, cfg.pn), device="cuda"))
    rd = torch.empty((F, cfg.nr, cfg.nd, 2), dtype=d.dtype, device="cuda")
    e.process_device(d, F, dt, o, d_rd=rd, out_dtype=dt, stream=s)
    torch.cuda.synchronize()
    e.synchronize()
    for k, v in o.items():
        res[f"{int(h)}_{k}"] = v.cpu().numpy()
    res[f"{int(h)}_rd"] = rd.cpu().numpy()
if mode == "save":
    np.savez(path, **res)
    print("saved", path)
else:
    ref = np.load(path)
    bad = [k for k in res if not np.array_equal(res[k], ref[k])]
    print("bit-identical" if not bad else f"DIFFER: {bad}")
    sys.exit(1 if bad else 0)
