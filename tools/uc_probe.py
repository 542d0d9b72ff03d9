"""k_rdx (and K1) against the allocation kind of the streams it reads once and writes once (probe).

python tools/uc_probe.py [which in out reps] -> one line per combination of the input cube and the output (RD map for k_rdx,
range cube for K1) allocated by torch (default: coarse-grained, cached in the L2) or by
hipExtMallocWithFlags(hipDeviceMallocUncached): uncached lines never enter the XCD's L2, so they cannot
evict k_rdx's hand-off slots (the slots' write-backs are 7.9 of the 16.4 GB written).
"""
import ctypes as ct
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from fmcw_radar_processing_amd import FMCW_C64  # noqa: E402
from fmcw_radar_processing_amd import params as P  # noqa: E402
from fmcw_radar_processing_amd.engine import Engine  # noqa: E402

hip = ct.CDLL("libamdhip64.so")
UNCACHED, CONTIG = 0x3, 0x4


class _Dev:
    def __init__(self, ptr, n):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": "<f4", "data": (ptr, False), "version": 3}


def alloc(n_floats, flag):
    if flag is None:
        return torch.empty(n_floats, dtype=torch.float32, device="cuda"), None
    p = ct.c_void_p()
    rc = hip.hipExtMallocWithFlags(ct.byref(p), ct.c_size_t(n_floats * 4), ct.c_uint(flag))
    if rc != 0:
        raise RuntimeError(f"hipExtMallocWithFlags({flag}) -> {rc}")
    return torch.as_tensor(_Dev(p.value, n_floats), device="cuda"), p


KIND = {"default": None, "uncached": UNCACHED, "contiguous": CONTIG}


def main(F=4096, reps=10, only=None, combos=None):
    """only / combos: one kernel and one (in, out) pair, for a rocprofv3 --pmc pass (tools/uc_pmc.sh)."""
    e = Engine(0)
    s = torch.cuda.current_stream()
    combos = combos or ((None, None), (UNCACHED, None), (None, UNCACHED), (UNCACHED, UNCACHED), (CONTIG, CONTIG))
    for which in (only,) if only else ("rdx", "k1"):
        cfg = P.config(4 if which == "rdx" else 2)
        e.set_taps(cfg, P.synth_calibration(cfg.nts))
        n_in = F * cfg.pn * cfg.nts * 2
        n_out = F * cfg.nr * cfg.nd * 2 if which == "rdx" else F * cfg.pn * cfg.nr * 2
        M = cfg.max_targets
        outs = dict(profile=torch.empty((F, cfg.nr), device="cuda"), tgt_count=torch.empty(F, dtype=torch.int32, device="cuda"),
                    tgt_range_idx=torch.empty((F, M), dtype=torch.int32, device="cuda"),
                    tgt_range_mag=torch.empty((F, M), device="cuda"),
                    tgt_doppler_idx=torch.empty((F, M), dtype=torch.int32, device="cuda"),
                    slow_mag=torch.empty((F, cfg.pn), device="cuda"))
        for rnd in range(1 if only else 2):
            for fin, fout in combos:
                t_in, p_in = alloc(n_in, fin)
                t_out, p_out = alloc(n_out, fout)
                d_in = t_in.view(F, cfg.pn, cfg.nts, 2)
                e.synth_device(d_in, 0, F, FMCW_C64, stream=s)
                if which == "rdx":
                    d_out = t_out.view(F, cfg.nr, cfg.nd, 2)
                    run = lambda: e.process_device(d_in, F, FMCW_C64, outs, d_rd=d_out, out_dtype=FMCW_C64, stream=s)  # noqa: E731
                    key = "onepass"
                else:
                    d_out = t_out.view(F, cfg.pn, cfg.nr, 2)
                    run = lambda: e.range_fft_device(d_in, F, FMCW_C64, d_out, outs["profile"], stream=s)  # noqa: E731
                    key = "range_only"
                for _ in range(2):
                    run()
                torch.cuda.synchronize()
                e.timing(2)
                e.timing_reset()
                for _ in range(reps):
                    run()
                torch.cuda.synchronize()
                ms, n = e.timing_read()[key]
                e.timing(0)
                name = {None: "default", UNCACHED: "uncached", CONTIG: "contiguous"}
                print(f"{which} round {rnd} in {name[fin]:10s} out {name[fout]:10s}: {ms / n * 1e3:8.1f} us", flush=True)
                del d_in, d_out, t_in, t_out
                torch.cuda.synchronize()
                for p in (p_in, p_out):
                    if p is not None:
                        hip.hipFree(p)
    e.close()


if __name__ == "__main__":
    if len(sys.argv) > 1:
        main(reps=int(sys.argv[4]), only=sys.argv[1], combos=((KIND[sys.argv[2]], KIND[sys.argv[3]]),))
    else:
        main()
