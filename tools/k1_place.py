"""Config-2 K1 against the placement of its buffers (development probe).

python tools/k1_place.py -> one line per placement: K1 us (HIP events, 20 launches) with the input
cube and the range cube carved out of one allocation at chosen byte offsets, beside the 16-byte copy
of the same bytes.  K1's box-to-box and harness-to-harness spread (profiles/r06_k1_boxes.txt) against a
flat copy suggests its speed depends on where its two 2.1-GB streams sit relative to each other.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from fmcw_radar_processing_amd import FMCW_C64  # noqa: E402
from fmcw_radar_processing_amd import params as P  # noqa: E402
from fmcw_radar_processing_amd.engine import Engine  # noqa: E402


def main(F=4096, reps=20):
    cfg = P.config(2)
    e = Engine(0)
    e.set_taps(cfg, P.synth_calibration(cfg.nts))
    s = torch.cuda.current_stream()
    n_iq = F * cfg.pn * cfg.nts * 2            # floats
    n_cube = F * cfg.pn * cfg.nr * 2
    MB = 1 << 20
    offsets = [(0, 0), (0, 64 << 10), (0, 1 * MB), (0, 2 * MB + (64 << 10)), (0, 3 * MB), (0, 32 * MB + 4096),
               (4096, 0), (1 * MB, 0), (2 * MB + 8192, 64 << 10), (0, 256 * MB)]
    extra = max(a + b for a, b in offsets) // 4 + 1024
    big = torch.empty(n_iq + n_cube + extra, dtype=torch.float32, device="cuda")
    d_prof = torch.empty((F, cfg.nr), dtype=torch.float32, device="cuda")
    d_cp = torch.empty(n_iq, dtype=torch.float32, device="cuda")
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for rnd in range(2):
        for a_off, b_off in offsets:
            i0 = a_off // 4
            c0 = i0 + n_iq + b_off // 4
            d_iq = big[i0:i0 + n_iq].view(F, cfg.pn, cfg.nts, 2)
            d_cube = big[c0:c0 + n_cube].view(F, cfg.pn, cfg.nr, 2)
            e.synth_device(d_iq, 0, F, FMCW_C64, stream=s)
            for _ in range(3):
                e.range_fft_device(d_iq, F, FMCW_C64, d_cube, d_prof, stream=s)
            torch.cuda.synchronize()
            e.timing(1)
            e.timing_reset()
            for _ in range(reps):
                e.range_fft_device(d_iq, F, FMCW_C64, d_cube, d_prof, stream=s)
            torch.cuda.synchronize()
            ms, n = e.timing_read()["range_only"]
            e.timing(0)
            nb = n_iq * 4
            ev[0].record(s)
            for _ in range(reps):
                e.copy_device(d_iq, d_cube, nb, stream=s)
            ev[1].record(s)
            torch.cuda.synchronize()
            cus = ev[0].elapsed_time(ev[1]) / reps * 1e3
            print(f"round {rnd} iq+{a_off:>9d} B  cube gap +{b_off:>9d} B: K1 {ms / n * 1e3:7.1f} us   copy {cus:6.1f} us  "
                  f"(iq 0x{d_iq.data_ptr():x} cube 0x{d_cube.data_ptr():x})", flush=True)
    e.close()


if __name__ == "__main__":
    main()
