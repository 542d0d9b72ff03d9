"""bench.py -- radar frames/s of the MI355X FMCW path (BASELINE.json metric).

One step = the whole hot path over one batch of device-resident synthetic
frames (SURVEY.md 8d generator, seed 0xF3C0 ^ global frame index):
range FFT + Doppler FFT for every range row (RD map written to HBM),
detection, slow-time compaction, hop-1 STFT of the concatenated slow-time
magnitude, global-max dB normalisation -- i.e. BASELINE.json config 4
(config 3 + Hann(20) STFT, nfft 64) at 4096 frames of 256 x 1024 per GPU.
For N > 1 GPUs each rank owns its own 4096-frame shard (weak scaling); the
STFT halo, global max and range_speed gather run as RCCL collectives.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--fp16]

Rank 0 prints one JSON line (contract in the task statement).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "radar frames/sec (range-FFT+Doppler+STFT) + achieved HBM GB/s vs roofline"
HBM_PEAK_GBPS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
STFT_WLEN, STFT_NOVERLAP, STFT_NFFT = 20, 19, 64


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--frames", type=int, default=4096, help="frames per GPU per step")
    ap.add_argument("--fp16", action="store_true", help="config-4 fp16 storage variant")
    ap.add_argument("--chunk", type=int, default=0, help="frames per range/Doppler chunk (0 = library default)")
    ap.add_argument("--pipeline", choices=["auto", "streams", "onepass", "xcd"], default="auto",
                    help="range/Doppler schedule (include/fmcw.h fmcw_set_pipeline)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline budget (0 = skip)")
    ap.add_argument("--no-stage-timing", action="store_true")
    ap.add_argument("--no-fanout", action="store_true")
    ap.add_argument("--no-extras", action="store_true",
                    help="skip the extra single-GPU lines (fp16 storage, config 2, host-pointer path)")
    ap.add_argument("--no-host-path", action="store_true",
                    help="skip the host-pointer path line (profile runs: its small launches share kernel names)")
    return ap.parse_args()


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    from fmcw_radar_processing_amd import FMCW_C32H, FMCW_C64
    from fmcw_radar_processing_amd import dist as fdist
    from fmcw_radar_processing_amd import params as P
    from fmcw_radar_processing_amd.engine import Engine

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    cfg = P.config(4)                       # 1024 samples x 256 chirps, Nr 1024, Nd 256, throughput mode
    F = args.frames
    C, S, NR, ND = cfg.pn, cfg.nts, cfg.nr, cfg.nd
    dt = FMCW_C32H if args.fp16 else FMCW_C64
    tdt = torch.float16 if args.fp16 else torch.float32
    eng = Engine(local)
    eng.set_taps(cfg, P.synth_calibration(S))
    if args.chunk:
        eng.set_chunk_frames(args.chunk)
    eng.set_pipeline({"auto": 0, "streams": 1, "onepass": 3, "xcd": 4}[args.pipeline])
    stream = torch.cuda.current_stream(dev)

    # ---- device-resident input + outputs ------------------------------------------
    d_iq = torch.empty((F, C, S, 2), dtype=tdt, device=dev)
    eng.synth_device(d_iq, rank * F, F, dt, stream=stream)
    M = cfg.max_targets
    outs = dict(profile=torch.empty((F, NR), device=dev), tgt_count=torch.empty(F, dtype=torch.int32, device=dev),
                tgt_range_idx=torch.empty((F, M), dtype=torch.int32, device=dev),
                tgt_range_mag=torch.empty((F, M), device=dev),
                tgt_doppler_idx=torch.empty((F, M), dtype=torch.int32, device=dev),
                slow_mag=torch.empty((F, C), device=dev))
    d_rd = torch.empty((F, NR, ND, 2), dtype=tdt, device=dev)
    win = torch.tensor(cfg.stft_window(), dtype=torch.float32, device=dev)
    fs = 1.0 / cfg.prt
    h = STFT_WLEN - 1
    max_seg = F * C + h
    nb = STFT_NFFT // 2 + 1
    flist = torch.empty(F, dtype=torch.int32, device=dev)
    d_len = torch.zeros(1, dtype=torch.int64, device=dev)
    d_P = torch.empty((max_seg, nb), dtype=torch.float32, device=dev)
    pmax = torch.zeros(1, dtype=torch.float32, device=dev)
    nseg = torch.zeros(1, dtype=torch.int64, device=dev)
    halo = torch.zeros(h, dtype=torch.float32, device=dev)
    halo_len = torch.zeros(1, dtype=torch.int64, device=dev)

    def step():
        eng.process_device(d_iq, F, dt, outs, d_rd=d_rd, out_dtype=dt, stream=stream)
        eng.compact_device(outs["tgt_count"], F, flist, d_len, stream=stream)
        hl, hbuf = None, None
        if world > 1:
            lens = fdist.all_lengths(d_len)
            head = fdist.head_samples(outs["slow_mag"], flist, d_len, h)
            hbuf, hl = fdist.right_halo(head, lens, rank)
        pmax.zero_()
        # two-pass STFT without a stored P: pass 1 forms max(P) only, pass 2 recomputes P and
        # writes 20 log10(P / max) (:276-283) -- P never goes to HBM and back
        eng.stft_power_device(outs["slow_mag"], flist, d_len, C, win, STFT_WLEN, STFT_NOVERLAP, STFT_NFFT, fs,
                              max_seg, None, pmax, nseg, d_halo=hbuf, n_halo=h if world > 1 else 0,
                              d_halo_len=hl, stream=stream)
        if world > 1:
            fdist.global_max_(pmax)
        eng.stft_db_direct_device(outs["slow_mag"], flist, d_len, C, win, STFT_WLEN, STFT_NOVERLAP, STFT_NFFT, fs,
                                  max_seg, pmax, d_P, d_halo=hbuf, n_halo=h if world > 1 else 0, d_halo_len=hl,
                                  stream=stream)
        if world > 1:
            fdist.gather_range_speed(outs["tgt_count"], outs["tgt_range_idx"], outs["tgt_doppler_idx"],
                                     outs["tgt_range_mag"])

    def barrier():
        if world > 1:
            dist.barrier(device_ids=[local])

    # which single-pass kernel the timed step runs (AUTO: k_rdx where the device passes the XCD check)
    xcd_runs = args.pipeline == "xcd" or (args.pipeline == "auto" and
                                          xcd_available(eng, d_iq, dt, outs, d_rd, stream))
    eng.set_pipeline({"auto": 0, "streams": 1, "onepass": 3, "xcd": 4}[args.pipeline])
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    # level 2: HIP events around every K1/K2/K3 launch on its own stream (the
    # per-kernel roofline below) plus the range+Doppler span and STFT launches
    level = 0 if args.no_stage_timing else 2
    eng.timing(level)
    eng.timing_reset()
    barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    barrier()
    elapsed = time.perf_counter() - t0
    stages = eng.timing_read() if level else {}
    eng.timing(0)
    el = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = float(el.item())

    # sanity: the step did real work (detections on most frames)
    det = int((outs["tgt_count"] > 0).sum().item())

    # ---- roofline ----------------------------------------------------------------
    # path: SURVEY.md 8d config-4 algorithmic bytes per frame (input + RD map +
    # profile + slow-time row; the range cube is an intermediate) over the
    # range+Doppler span.  dominant kernel: k_range (K1), whose own algorithmic
    # bytes are its input and the range cube it materialises (the config-2
    # per-frame figure without the profile), over its HIP-event launch time.
    esz = 4 if args.fp16 else 8
    alg_per_frame = C * S * esz + NR * ND * esz + NR * 4 + C * 4
    k1_per_frame = C * S * esz + C * NR * 8          # streams schedule keeps an fp32 cube
    kern = {}
    # k_rd1p (single-pass schedule): input + RD map + profile, no cube
    for name, label, per_frame in (("range", "k_range", k1_per_frame), ("doppler", "k_doppler", C * NR * 8 + NR * ND * esz + NR * 4),
                                   ("onepass", "k_rd1p", C * S * esz + NR * ND * esz + NR * 4),
                                   ("detect", "k_detect", None)):
        ms, n = stages.get(name, (0.0, 0))
        if n:
            fpl = F * args.steps / n
            us = ms / n * 1e3
            kern[label] = {"avg_launch_us": round(us, 2), "frames_per_launch": fpl}
            if per_frame:
                kern[label]["alg_bytes_per_launch"] = int(per_frame * fpl)
                kern[label]["achieved_GBps"] = round(per_frame * fpl / (us * 1e-6) / 1e9, 1)
    roof, path = None, None
    rd_ms, rd_n = stages.get("range_doppler", (0.0, 0))
    if rd_n:
        per_launch_ms = rd_ms / rd_n
        fpl = F * args.steps / rd_n
        ach = alg_per_frame * fpl / (per_launch_ms * 1e-3) / 1e9
        path = {"achieved": round(ach, 1), "frac": round(ach / HBM_PEAK_GBPS, 4), "unit": "GB/s",
                "span_us": round(per_launch_ms * 1e3, 2), "frames_per_span": fpl, "alg_bytes_per_frame": alg_per_frame,
                "what": "range+Doppler span (before first k_range .. after last k_doppler), SURVEY 8d bytes"}
    pmc = load_pmc(os.path.join(ROOT, "profiles"))
    dom = "k_rd1p" if "k_rd1p" in kern else "k_range"
    if dom == "k_rd1p" and xcd_runs:   # the single-pass stage timer covers k_rdx when the XCD schedule runs
        kern["k_rdx"] = kern.pop("k_rd1p")
        dom = "k_rdx"
    if dom in kern:
        k = kern[dom]
        kname = {"k_rd1p": RD1P_NAME[args.fp16], "k_rdx": RDX_NAME[args.fp16]}.get(dom)
        traffic = pmc_traffic(pmc, kname, k["frames_per_launch"]) if kname else None
        roof = {"bound": "hbm", "achieved": k["achieved_GBps"], "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                "frac": round(k["achieved_GBps"] / HBM_PEAK_GBPS, 4), "traffic": traffic,
                "kernel": {"k_rd1p": "k_rd1p (single pass: calibration, mean removal, window, range FFT, profile, Doppler "
                                     "FFT, RD store; one range tile of one frame per workgroup)",
                           "k_rdx": "k_rdx (XCD-team schedule: the 32 CUs of an XCD share each frame; range FFT by chirps, "
                                    "cube handed over through a slot ring, Doppler FFT by range-bin groups; calibration, "
                                    "mean removal, windows, profile, RD store)"}.get(
                              dom, "k_range (K1: calibration, mean removal, window, 1024-pt range FFT, cube store)"),
                "kernel_name": kname,
                "alg_bytes_per_launch": k["alg_bytes_per_launch"], "avg_launch_us": k["avg_launch_us"],
                "frames_per_launch": k["frames_per_launch"],
                "traffic_source": pmc.get("source") if pmc and traffic else None}

    # ---- input fan-out over xGMI from rank 0 (reported separately, not in value) -----
    fanout = None
    if world > 1 and not args.no_fanout:
        nf = 256
        src = torch.empty((world * nf, C, S, 2), dtype=tdt, device=dev) if rank == 0 else None
        dst = torch.empty((nf, C, S, 2), dtype=tdt, device=dev)
        parts = list(src.chunk(world)) if rank == 0 else None
        dist.scatter(dst, parts, src=0)
        torch.cuda.synchronize(dev)
        barrier()
        t1 = time.perf_counter()
        dist.scatter(dst, parts, src=0)
        torch.cuda.synchronize(dev)
        barrier()
        ft = time.perf_counter() - t1
        fanout = {"frames_per_rank": nf, "ms": round(ft * 1e3, 3),
                  "GBps_root_egress": round(world * nf * C * S * esz / ft / 1e9, 1)}
        del src, dst

    extra = {}
    if world == 1 and not args.no_extras and not args.fp16:
        del d_rd, d_P
        extra["fp16_storage"] = bench_fp16(eng, cfg, F, args, dev, stream, pmc)
        extra["config2_range_fft"] = bench_config2(eng, args, dev, stream, pmc)
        if not args.no_host_path:
            extra["host_path"] = bench_host_path(eng)
        eng.set_taps(cfg, P.synth_calibration(S))
    if rank == 0:
        cpu = cpu_baseline(args.cpu_seconds, d_iq, F, dt) if args.cpu_seconds > 0 else None
        total_frames = world * F * args.steps
        value = total_frames / elapsed
        line = {
            "metric": METRIC, "value": round(value, 1), "unit": "frames/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "f16-storage/f32-compute" if args.fp16 else "f32",
            "data": "synthetic (SURVEY.md 8d generator, generated in HBM per rank)",
            "config": {"workload": "BASELINE config 4: per GPU 4096 frames x 256 chirps x 1024 samples; "
                                   "range FFT 1024 + Doppler FFT 256 on every row + detection + "
                                   "Hann(20) hop-1 STFT nfft 64 + dB", "frames_per_gpu": F,
                       "chirps": C, "samples": S, "nr": NR, "nd": ND, "stft_nfft": STFT_NFFT,
                       "parallelism": f"frame-shard dp{world}"},
            "hbm_alg_GBps": round(alg_per_frame * value / world / 1e9, 1),
            "roofline": roof,
            "path_roofline": path,
            "kernels": kern,
            "cpu_baseline": cpu,
            "stages_ms_per_step": {k: round(v[0] / args.steps, 4) for k, v in stages.items() if v[1]},
            "frames_with_target": det,
        }
        if fanout:
            line["input_fanout"] = fanout
        line.update(extra)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


RD1P_NAME = {False: "fmcw::k_rd1p<true, false>", True: "fmcw::k_rd1p<true, true>"}
RDX_NAME = {False: "fmcw::k_rdx<true, false>", True: "fmcw::k_rdx<true, true>"}


def xcd_available(eng, d_iq, dt, outs, d_rd, stream) -> bool:
    """Does this device run the XCD-team schedule (fmcw_set_pipeline(FMCW_PIPE_XCD) accepted on a
    short call)?  AUTO picks it exactly then (include/fmcw.h)."""
    import torch
    from fmcw_radar_processing_amd import FmcwError
    n = 8
    sub = {k: v[:n] for k, v in outs.items()}
    try:
        eng.set_pipeline(4)
        eng.process_device(d_iq[:n], n, dt, sub, d_rd=d_rd[:n], out_dtype=dt, stream=stream)
        torch.cuda.synchronize()
        return True
    except FmcwError:
        return False
K1_NAME = "fmcw::k_range<512, c64, c64, true>"


def load_pmc(pdir: str):
    """Per-launch HBM traffic per kernel from the committed rocprofv3 PMC summary
    of this same command (tools/profile_run.sh -> profiles/bench_pmc.json):
    FETCH_SIZE x 2 (gfx950 read correction, MI355X_MICROARCH.md HBM section) +
    WRITE_SIZE, averaged over the kernel's dispatches, keyed by kernel name."""
    path = os.path.join(pdir, "bench_pmc.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        d = json.load(f)
    d["source"] = os.path.relpath(path, ROOT)
    return d


def pmc_traffic(pmc, name, frames_per_launch):
    """HBM bytes per launch of kernel `name`, if the profile ran the same launch size."""
    if not pmc:
        return None
    pk = (pmc.get("by_name") or {}).get(name)
    if not pk or abs(pk.get("frames_per_launch", 0) - frames_per_launch) >= 0.5:
        return None
    return pk.get("hbm_bytes_per_launch")


def _roof(alg_per_frame, frames_per_launch, avg_us, traffic, name, kernel, pmc):
    ach = alg_per_frame * frames_per_launch / (avg_us * 1e-6) / 1e9
    return {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBPS, 4), "traffic": traffic, "kernel": kernel, "kernel_name": name,
            "alg_bytes_per_launch": int(alg_per_frame * frames_per_launch), "avg_launch_us": round(avg_us, 2),
            "frames_per_launch": frames_per_launch,
            "traffic_source": pmc.get("source") if pmc and traffic else None}


def bench_fp16(eng, cfg, F, args, dev, stream, pmc):
    """BASELINE config 4's fp16-storage variant, same step as the headline (fp16 IQ in,
    fp16 RD map out, fp32 arithmetic), timed the same way on the same GPU."""
    import torch
    from fmcw_radar_processing_amd import FMCW_C32H
    C, S, NR, ND = cfg.pn, cfg.nts, cfg.nr, cfg.nd
    d_iq = torch.empty((F, C, S, 2), dtype=torch.float16, device=dev)
    eng.synth_device(d_iq, 0, F, FMCW_C32H, stream=stream)
    M = cfg.max_targets
    outs = dict(profile=torch.empty((F, NR), device=dev), tgt_count=torch.empty(F, dtype=torch.int32, device=dev),
                tgt_range_idx=torch.empty((F, M), dtype=torch.int32, device=dev),
                tgt_range_mag=torch.empty((F, M), device=dev),
                tgt_doppler_idx=torch.empty((F, M), dtype=torch.int32, device=dev),
                slow_mag=torch.empty((F, C), device=dev))
    d_rd = torch.empty((F, NR, ND, 2), dtype=torch.float16, device=dev)
    win = torch.tensor(cfg.stft_window(), dtype=torch.float32, device=dev)
    max_seg = F * C + STFT_WLEN - 1
    flist = torch.empty(F, dtype=torch.int32, device=dev)
    d_len = torch.zeros(1, dtype=torch.int64, device=dev)
    d_P = torch.empty((max_seg, STFT_NFFT // 2 + 1), dtype=torch.float32, device=dev)
    pmax = torch.zeros(1, dtype=torch.float32, device=dev)
    nseg = torch.zeros(1, dtype=torch.int64, device=dev)
    fs = 1.0 / cfg.prt

    xcd = args.pipeline in ("auto", "xcd") and xcd_available(eng, d_iq, FMCW_C32H, outs, d_rd, stream)
    eng.set_pipeline({"auto": 0, "streams": 1, "onepass": 3, "xcd": 4}[args.pipeline])

    def step():
        eng.process_device(d_iq, F, FMCW_C32H, outs, d_rd=d_rd, out_dtype=FMCW_C32H, stream=stream)
        eng.compact_device(outs["tgt_count"], F, flist, d_len, stream=stream)
        pmax.zero_()
        eng.stft_power_device(outs["slow_mag"], flist, d_len, C, win, STFT_WLEN, STFT_NOVERLAP, STFT_NFFT, fs,
                              max_seg, None, pmax, nseg, stream=stream)
        eng.stft_db_direct_device(outs["slow_mag"], flist, d_len, C, win, STFT_WLEN, STFT_NOVERLAP, STFT_NFFT, fs,
                                  max_seg, pmax, d_P, stream=stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    eng.timing(2)
    eng.timing_reset()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    st = eng.timing_read()
    eng.timing(0)
    ms, n = st["onepass"]
    fpl = F * args.steps / n
    us = ms / n * 1e3
    per = C * S * 4 + NR * ND * 4 + NR * 4
    kname = RDX_NAME[True] if xcd else RD1P_NAME[True]
    out = {"value": round(F * args.steps / el, 1), "unit": "frames/s", "ms_per_step": round(el / args.steps * 1e3, 4),
           "dtype": "f16-storage/f32-compute",
           "what": "BASELINE config 4 fp16-storage variant: the headline step with c32h IQ in and c32h RD out",
           "roofline": _roof(per, fpl, us, pmc_traffic(pmc, kname, fpl), kname,
                             ("k_rdx<fp16 storage> (XCD-team schedule" if xcd else "k_rd1p<fp16 storage> (single pass") +
                             ", c32h in / c32h RD out)", pmc)}
    del d_iq, d_rd, d_P
    torch.cuda.empty_cache()
    return out


def bench_config2(eng, args, dev, stream, pmc):
    """BASELINE config 2: 4096 frames x 128 chirps x 512 samples, range FFT only (K1,
    range cube written, fp32), device-resident; its own roofline on K1's event time."""
    import torch
    from fmcw_radar_processing_amd import FMCW_C64
    from fmcw_radar_processing_amd import params as P
    cfg2 = P.config(2)
    F2, C, S, NR = 4096, cfg2.pn, cfg2.nts, cfg2.nr
    eng.set_taps(cfg2, P.synth_calibration(S))
    d_iq = torch.empty((F2, C, S, 2), dtype=torch.float32, device=dev)
    eng.synth_device(d_iq, 0, F2, FMCW_C64, stream=stream)
    d_cube = torch.empty((F2, C, NR, 2), dtype=torch.float32, device=dev)
    d_prof = torch.empty((F2, NR), dtype=torch.float32, device=dev)
    for _ in range(args.warmup):
        eng.range_fft_device(d_iq, F2, FMCW_C64, d_cube, d_prof, stream=stream)
    torch.cuda.synchronize(dev)
    eng.timing(1)
    eng.timing_reset()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        eng.range_fft_device(d_iq, F2, FMCW_C64, d_cube, d_prof, stream=stream)
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    ms, n = eng.timing_read()["range_only"]
    eng.timing(0)
    us = ms / n * 1e3
    per = C * S * 8 + C * NR * 8 + NR * 4
    out = {"value": round(F2 * args.steps / el, 1), "unit": "frames/s", "ms_per_step": round(el / args.steps * 1e3, 4),
           "dtype": "f32", "what": "BASELINE config 2: 4096 x 128 x 512 IQ, range FFT only, cube + profile written",
           "roofline": _roof(per, F2, us, pmc_traffic(pmc, K1_NAME, F2), K1_NAME,
                             "K1 k_range (calibration, mean, window, 512-pt range FFT, cube + profile store)", pmc)}
    del d_iq, d_cube, d_prof
    torch.cuda.empty_cache()
    return out


def json_timing(sp, python: bool):
    """spectrogram_data.json (:306-321) of one call: libfmcw's native jsonencode writer
     against the Python mirror of jsonencode, same bytes."""
    import tempfile
    from fmcw_radar_processing_amd import json_native
    from fmcw_radar_processing_amd.matlab_json import encode
    obj = {"time": sp["time"], "frequency": sp["frequency"], "intensity": sp["intensity"].T,
           "title": "All Frames - Log-Scaled Spectrogram", "xLabel": "Time (s)", "yLabel": "Frequency (Hz)"}
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "spectrogram_data.json")
        t = time.perf_counter()
        n = json_native.write(path, obj)
        out = {"native_ms": round((time.perf_counter() - t) * 1e3, 2)}
        if python:
            t = time.perf_counter()
            with open(path, "w") as fh:
                fh.write(encode(obj))
            out["python_ms"] = round((time.perf_counter() - t) * 1e3, 2)
    return out, n


def bench_host_path(eng):
    """The path MATLAB calls (MEX -> fmcw_process + fmcw_stft on HOST buffers,
    radar_processing.m:197-299): inputs in pageable host memory, PCIe included,
    at the deployed 64x16 module geometry and at the config-3 geometry."""
    import torch
    from fmcw_radar_processing_amd import FMCW_C64
    from fmcw_radar_processing_amd import params as P
    from fmcw_radar_processing_amd import windows as W
    res = {}
    # one call = one recording, as radar_processing_with_azure.m:50 makes it: the deployed
    # module's 115-frame file, and 256 config-3 frames (512 MiB of IQ, PCIe-bound)
    for name, F, reps in (("deployed_64x16_115_frames", 115, 20), ("config3_256x1024_256_frames", 256, 3)):
        cfg = P.config("deployed" if name.startswith("deployed") else 3)
        eng.set_taps(cfg, P.synth_calibration(cfg.nts))
        d = torch.empty((F, cfg.pn, cfg.nts, 2), dtype=torch.float32, device="cuda")
        eng.synth_device(d, 0, F, FMCW_C64)                # SURVEY 8d frames, then to pageable host memory
        torch.cuda.synchronize()
        iq = d.cpu().numpy().view(np.complex64)[..., 0].copy()
        del d
        win = W.kaiser(20, 3.0)                            # :276 kaiser(window_length, 3)
        fs = 1.0 / cfg.prt
        out = eng.process(iq)                               # warm: slots allocated, code paged in
        x = out["slow_mag"][out["tgt_count"] > 0].reshape(-1)
        if len(x) < 20:
            x = out["slow_mag"].reshape(-1)
        eng.stft(x, win, 19, fs)
        tp = ts = 0.0
        for _ in range(reps):
            t = time.perf_counter()
            out = eng.process(iq)
            tp += time.perf_counter() - t
            x = out["slow_mag"][out["tgt_count"] > 0].reshape(-1)
            if len(x) < 20:
                x = out["slow_mag"].reshape(-1)
            t = time.perf_counter()
            eng.stft(x, win, 19, fs)                        # reference nfft rule + 1024 log bins (:270-299)
            ts += time.perf_counter() - t
        tp /= reps
        ts /= reps
        sp = eng.stft(x, win, 19, fs)
        tj, nbytes = json_timing(sp, python=name.startswith("deployed"))
        res[name] = {"frames": F, "frames_per_s": round(F / (tp + ts), 1), "calls_per_s": round(1.0 / (tp + ts), 2),
                     "spectrogram_json": {"bytes": nbytes, **tj},
                     "process_ms": round(tp * 1e3, 3),
                     "stft_ms": round(ts * 1e3, 3), "h2d_GBps": round(iq.nbytes / tp / 1e9, 2),
                     "what": "fmcw_process (pageable host iq -> pinned 2-slot chunks -> HBM, outputs back) + "
                             "fmcw_stft of the slow-time signal, wall clock"}
    return res


def cpu_baseline(budget_s: float, d_iq, F: int, dt: int):
    """C restatement of radar_processing.m:197-299 (oracle/fmcw_oracle.c, fp64,
    OpenMP over frames) on a bounded sample of the SAME device-resident frames
    (copied back in batches), on this host's cores.  Every row's Doppler FFT is
    computed (as the GPU path does), then the hop-1 STFT of the slow-time signal."""
    import torch
    from fmcw_radar_processing_amd import params as P
    from oracle import coracle as CO
    from oracle import oracle as O
    cores, host = host_cores()
    cfg = P.config(4)
    p = O.derive_params(P.deployed_device(cfg.nts, cfg.pn), nr=cfg.nr, nd=cfg.nd, parity=False)
    wr, wd = O.windows(cfg.nts, cfg.pn)
    cal = P.synth_calibration(cfg.nts)
    win = O.stft_window("hann")
    B = 4 * cores

    def batch(f0):
        x = d_iq[f0:f0 + B].float().cpu().numpy()            # fp16 storage: the same values widened
        return x.view(np.float32).reshape(x.shape[0], cfg.pn, cfg.nts, 2).view(np.complex64)[..., 0]

    def run(threads, budget):
        done, slow, busy = 0, [], 0.0
        rd = np.zeros((B, cfg.nr, cfg.nd), np.complex128)
        f0 = 0
        while busy < budget or done < B:
            iq = batch(f0)                                      # not timed
            t = time.perf_counter()
            out = CO.process_frames(iq, cal, p, wr, wd, rd_out=rd[:iq.shape[0]], nthreads=threads)
            keep = out["tgt_count"] > 0
            slow.append(out["slow_mag"][keep].reshape(-1))
            busy += time.perf_counter() - t
            done += iq.shape[0]
            f0 = (f0 + B) % max(F - B, 1)
        t = time.perf_counter()
        x = np.concatenate(slow)
        if len(x) >= STFT_WLEN:
            CO.spectrogram(x, cfg.prt, win, STFT_NOVERLAP, STFT_NFFT, nbins=0, nthreads=threads)
        return done / (busy + time.perf_counter() - t), done

    v_all, n_all = run(cores, budget_s)
    v_one, n_one = run(1, max(2.0, budget_s / 4))
    return {"value": round(v_all, 2), "unit": "frames/s", "cores": cores, "kind": "port",
            "sample": f"{n_all} config-4 frames (the bench's own device frames, copied back) through "
                      f"oracle/fmcw_oracle.c (fp64, OpenMP {cores} threads, every RD row) + hop-1 STFT nfft 64",
            "single_thread": {"value": round(v_one, 2), "frames": n_one}, "host": host}


def host_cores():
    """Threads for the CPU baseline: every core this process may run on
    (sched_getaffinity), bounded by the host's per-job share when the launcher
    states one (OMP_NUM_THREADS; the GPU pool sets it to the cores it allots
    to one GPU).  Returns (threads, description of the host)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    share = os.environ.get("OMP_NUM_THREADS", "")
    cores = min(aff, int(share)) if share.isdigit() and int(share) > 0 else aff
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    model = ln.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return cores, {"cpu_model": model, "nproc": os.cpu_count(), "affinity_cpus": aff,
                   "omp_num_threads_env": share or None,
                   "threads_used": cores,
                   "rule": "all affinity CPUs, bounded by OMP_NUM_THREADS when the launcher sets it"}


if __name__ == "__main__":
    main()
