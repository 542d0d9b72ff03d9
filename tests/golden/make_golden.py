"""Generate the committed golden fixtures under tests/golden/ (run from the repo root:
``python tests/golden/make_golden.py``).

Provenance: there is no MATLAB runtime and the reference holds no fixtures or
test vectors, so these vectors are produced by the
float64 oracle (oracle/oracle.py) on the seeded synthetic inputs of SURVEY.md
8d.  They pin the oracle and the GPU path against regressions and make the
on-box GPU tests independent of re-running the oracle; they are NOT MATLAB
outputs (parity against MATLAB stays unpinned).

Fixtures (numpy .npz, no pickles):
  deployed_f8.npz   64 x 16 samples/chirps, Nr 256, Nd 16, 8 frames, parity mode:
                    iq, per-frame outputs, RD rows of the targets, slow signal,
                    reference-rule STFT (kaiser(20,3), nfft 2^nextpow2(L), 1024 log bins)
  config1_f1.npz    256 x 128, Nr 256, Nd 16, 1 frame, parity (Doppler truncation)
  config2_f2.npz    512 x 128, Nr 512, Nd 16, 2 frames, throughput (inputs re-generated
                    from the seed; outputs: profile, detections, slow row)
  config3_f2.npz    1024 x 256, Nr 1024, Nd 256, 2 frames, throughput (ditto + RD rows)
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from fmcw_radar_processing_amd import params as P  # noqa: E402
from oracle import oracle as O  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))

CASES = {
    "deployed_f8": dict(nts=64, pn=16, nr=256, nd=16, F=8, parity=True, store_iq=True, stft=True),
    "config1_f1": dict(nts=256, pn=128, nr=256, nd=16, F=1, parity=True, store_iq=True, stft=False),
    "config2_f2": dict(nts=512, pn=128, nr=512, nd=16, F=2, parity=False, store_iq=False, stft=False),
    "config3_f2": dict(nts=1024, pn=256, nr=1024, nd=256, F=2, parity=False, store_iq=False, stft=False),
}


def build(name, c):
    dev = P.deployed_device(c["nts"], c["pn"])
    p = O.derive_params(dev, nr=c["nr"], nd=c["nd"], parity=c["parity"])
    wr, wd = O.windows(c["nts"], c["pn"])
    cal = O.synth_cal(c["nts"])
    iq = O.synth_frames(c["F"], c["pn"], c["nts"], c["nr"], c["nd"], p["dist_per_bin"], frame0=0)
    out = O.process_frames(iq, cal, p, wr, wd, want_rd=True, rd_all_rows=True)
    rows = np.zeros((c["F"], c["nd"]), np.complex128)
    for f in range(c["F"]):
        if out["tgt_count"][f]:
            rows[f] = out["rd"][f, out["tgt_range_idx"][f, 0] - 1]
    d = dict(nts=c["nts"], pn=c["pn"], nr=c["nr"], nd=c["nd"], F=c["F"], parity=int(c["parity"]),
             frame0=0, seed_rule="0xF3C0 ^ frame", profile=out["profile"], tgt_count=out["tgt_count"],
             tgt_range_idx=out["tgt_range_idx"], tgt_range_mag=out["tgt_range_mag"],
             tgt_doppler_idx=out["tgt_doppler_idx"], slow_mag=out["slow_mag"], target_rd_rows=rows,
             rd_row_norms=np.linalg.norm(out["rd"], axis=2), iq_checksum=float(np.abs(iq).astype(np.float64).sum()))
    if c["store_iq"]:
        d["iq"] = iq
    if c["stft"]:
        x = O.slow_time_signal(out).astype(np.float32).astype(np.float64)   # the GPU STFT input is fp32
        sp = O.spectrogram_pipeline(x, p["prt"], O.stft_window("kaiser"), 19)
        d.update(slow_signal=x, stft_time=sp["time"], stft_freq=sp["frequency"], stft_intensity=sp["intensity"],
                 stft_nfft=sp["nfft"], prt=p["prt"])
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **d)
    print(name, {k: getattr(v, "shape", v) for k, v in d.items() if k != "seed_rule"})


if __name__ == "__main__":
    for n, c in CASES.items():
        build(n, c)
