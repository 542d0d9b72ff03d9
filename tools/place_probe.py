"""Kernel time against the placement of a kernel's input and output buffers (development probe).

python tools/place_probe.py [k1|rdx] -> one line per byte gap between the end of the input cube and the
start of the output (range cube for K1 / config 2, RD map for k_rdx / config 4), both carved out of one
allocation: the kernel's HIP-event average over `reps` launches.  profiles/r06_k1_place.txt.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from fmcw_radar_processing_amd import FMCW_C64  # noqa: E402
from fmcw_radar_processing_amd import params as P  # noqa: E402
from fmcw_radar_processing_amd.engine import Engine  # noqa: E402

KB, MB = 1 << 10, 1 << 20
GAPS = [0, 4 * KB, 16 * KB, 64 * KB, 128 * KB, 256 * KB, 512 * KB, 1 * MB, 1 * MB + 64 * KB, 2 * MB, 2 * MB + 64 * KB,
        4 * MB, 8 * MB, 16 * MB, 64 * MB, 256 * MB, 256 * MB + 64 * KB, 1024 * MB]


def slots(F=4096, reps=10, rounds=2):
    """k_rdx against the placement of its hand-off slot ring (a library buffer): an ab/ build with
    -DFMCW_XCUBE_PAD_AB puts the ring FMCW_XCUBE_PAD bytes into a 1-GiB-larger allocation."""
    e = Engine(0)
    s = torch.cuda.current_stream()
    cfg = P.config(4)
    e.set_taps(cfg, P.synth_calibration(cfg.nts))
    d_in = torch.empty((F, cfg.pn, cfg.nts, 2), dtype=torch.float32, device="cuda")
    e.synth_device(d_in, 0, F, FMCW_C64, stream=s)
    d_rd = torch.empty((F, cfg.nr, cfg.nd, 2), dtype=torch.float32, device="cuda")
    M = cfg.max_targets
    outs = dict(profile=torch.empty((F, cfg.nr), device="cuda"), tgt_count=torch.empty(F, dtype=torch.int32, device="cuda"),
                tgt_range_idx=torch.empty((F, M), dtype=torch.int32, device="cuda"),
                tgt_range_mag=torch.empty((F, M), device="cuda"),
                tgt_doppler_idx=torch.empty((F, M), dtype=torch.int32, device="cuda"),
                slow_mag=torch.empty((F, cfg.pn), device="cuda"))
    for rnd in range(rounds):
        for pad in [0, 64 * KB, 256 * KB, 1 * MB, 2 * MB, 4 * MB, 16 * MB, 64 * MB, 256 * MB, 512 * MB + 64 * KB]:
            os.environ["FMCW_XCUBE_PAD"] = str(pad)
            for _ in range(2):
                e.process_device(d_in, F, FMCW_C64, outs, d_rd=d_rd, out_dtype=FMCW_C64, stream=s)
            torch.cuda.synchronize()
            e.timing(2)
            e.timing_reset()
            for _ in range(reps):
                e.process_device(d_in, F, FMCW_C64, outs, d_rd=d_rd, out_dtype=FMCW_C64, stream=s)
            torch.cuda.synchronize()
            ms, n = e.timing_read()["onepass"]
            e.timing(0)
            print(f"slots round {rnd} ring pad {pad:>11d} B: k_rdx {ms / n * 1e3:8.1f} us", flush=True)
    e.close()


def main(which="k1", F=4096, reps=10, rounds=2):
    if which == "slots":
        return slots(F, reps, rounds)
    e = Engine(0)
    s = torch.cuda.current_stream()
    cfg = P.config(2 if which == "k1" else 4)
    e.set_taps(cfg, P.synth_calibration(cfg.nts))
    n_in = F * cfg.pn * cfg.nts * 2
    n_out = F * cfg.pn * cfg.nr * 2 if which == "k1" else F * cfg.nr * cfg.nd * 2
    big = torch.empty(n_in + n_out + max(GAPS) // 4 + 1024, dtype=torch.float32, device="cuda")
    d_prof = torch.empty((F, cfg.nr), dtype=torch.float32, device="cuda")
    M = cfg.max_targets
    outs = dict(profile=d_prof, tgt_count=torch.empty(F, dtype=torch.int32, device="cuda"),
                tgt_range_idx=torch.empty((F, M), dtype=torch.int32, device="cuda"),
                tgt_range_mag=torch.empty((F, M), device="cuda"),
                tgt_doppler_idx=torch.empty((F, M), dtype=torch.int32, device="cuda"),
                slow_mag=torch.empty((F, cfg.pn), device="cuda"))
    d_in = big[:n_in].view(F, cfg.pn, cfg.nts, 2)
    e.synth_device(d_in, 0, F, FMCW_C64, stream=s)
    for rnd in range(rounds):
        for gap in GAPS:
            o0 = n_in + gap // 4
            d_out = big[o0:o0 + n_out]
            if which == "k1":
                d_out = d_out.view(F, cfg.pn, cfg.nr, 2)
                run = lambda: e.range_fft_device(d_in, F, FMCW_C64, d_out, d_prof, stream=s)  # noqa: E731
                key = "range_only"
            else:
                d_out = d_out.view(F, cfg.nr, cfg.nd, 2)
                run = lambda: e.process_device(d_in, F, FMCW_C64, outs, d_rd=d_out, out_dtype=FMCW_C64, stream=s)  # noqa: E731
                key = "onepass"
            for _ in range(2):
                run()
            torch.cuda.synchronize()
            e.timing(2)
            e.timing_reset()
            for _ in range(reps):
                run()
            torch.cuda.synchronize()
            tm = e.timing_read()
            e.timing(0)
            ms, n = tm[key]
            print(f"{which} round {rnd} gap {gap:>11d} B (offset in - out {(o0 * 4) % (1 << 30):>11d} mod 1 GiB): "
                  f"{ms / n * 1e3:8.1f} us", flush=True)
    e.close()


if __name__ == "__main__":
    main(*sys.argv[1:2])
