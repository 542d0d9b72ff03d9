"""Development probe: the folded max(P) pass's in-kernel s_memtime stamps (ab/stamps.so built with
-DSTFT_AB_STAMPS; block 0 and the last block, wave 0), printed as cycles from kernel entry."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from fmcw_radar_processing_amd import FMCW_C64  # noqa: E402
from fmcw_radar_processing_amd import params as P  # noqa: E402
from fmcw_radar_processing_amd.engine import Engine  # noqa: E402

F = 4096
cfg = P.config(4)
e = Engine(0)
e.set_taps(cfg, P.synth_calibration(cfg.nts))
s = torch.cuda.Stream()
torch.cuda.set_stream(s)
C = cfg.pn
d_iq = torch.empty((F, C, cfg.nts, 2), dtype=torch.float32, device="cuda")
e.synth_device(d_iq, 0, F, FMCW_C64, stream=s)
M = cfg.max_targets
outs = dict(profile=torch.empty((F, cfg.nr), device="cuda"), tgt_count=torch.empty(F, dtype=torch.int32, device="cuda"),
            tgt_range_idx=torch.empty((F, M), dtype=torch.int32, device="cuda"), tgt_range_mag=torch.empty((F, M), device="cuda"),
            tgt_doppler_idx=torch.empty((F, M), dtype=torch.int32, device="cuda"), slow_mag=torch.empty((F, C), device="cuda"))
flist = torch.empty(F, dtype=torch.int32, device="cuda")
d_len = torch.zeros(1, dtype=torch.int64, device="cuda")
pmax = torch.zeros(1, dtype=torch.float32, device="cuda")
e.process_slow_device(d_iq, F, FMCW_C64, outs, flist, d_len, d_pmax=pmax, stream=s)
del d_iq
win = torch.tensor(cfg.stft_window(), dtype=torch.float32, device="cuda")
max_seg = F * C + 19
nseg = torch.zeros(64 + 3 * 4096 * 4, dtype=torch.int64, device="cuda")
for rep in range(5):
    nseg.zero_()
    e.stft_power_device(outs["slow_mag"], flist, d_len, C, win, 20, 19, 64, 1.0 / cfg.prt, max_seg, None, pmax, nseg, stream=s)
    torch.cuda.synchronize()
    st = nseg.cpu().numpy().view(np.uint64).astype(np.int64)
    for b, o in (("first", 1), ("last", 17)):
        v = st[o:o + 15]
        v = v[v != 0]
        print(rep, b, list(v - st[1]) if len(v) else [], flush=True)
    rt = st[64:].reshape(-1, 3)
    rt = rt[rt[:, 0] != 0]
    t0 = rt[:, 0].min()
    beg, end = (rt[:, 0] - t0) * 10, (rt[:, 1] - t0) * 10       # ns (100 MHz)
    life = end - beg
    print(rep, "waves", len(rt), "start ns: min/p50/p90/max", beg.min(), np.median(beg), np.quantile(beg, 0.9), beg.max(),
          "| end ns p10/p50/max", np.quantile(end, 0.1), np.median(end), end.max(), "| life p50/max", np.median(life), life.max(), flush=True)
    if rep == 4:
        np.save("gpurun_out/stft_rt.npy", rt)
e.close()
