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

--gpus N > 1 without a torchrun environment starts N ranks itself (a child
torch.distributed.run, before any GPU call) and exits with its status; under
torchrun the world size must equal --gpus.

Rank 0 prints one JSON line (contract in the task statement).  After every
timed region it checks the launches' sticky error word (fmcw_synchronize) and,
in the oracle leg at the end (CPU baseline), compares every timed frame's
outputs with the float64 C oracle (oracle/fmcw_oracle.c): the "checked" key.
A failed check still prints the line, then exits non-zero.
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
    # the first ~20-30 steps of a process run ~1 % slower (k_rdx 4.38 against 4.34 ms; the same at 200
    # timed steps after 3 warm ones: profiles/r05_bench_warmup.txt), so the default warms up 30 steps
    # and times 100 (0.45 s of a 4096-frame stream per GPU)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=30)
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
    ap.add_argument("--no-check", action="store_true",
                    help="skip the full-size comparison with the C oracle (profile runs)")
    ap.add_argument("--stream-frames", type=int, default=0,
                    help="BASELINE config 5: set --steps so that the run covers exactly this many frames over "
                         "all GPUs (65536 = the config-5 stream: 16 steps on 1 GPU, 2 on 8)")
    ap.add_argument("--stft-form", choices=["direct", "stored"], default="direct",
                    help="dB of the STFT leg: direct = pass 1 max(P) only, pass 2 recomputes P and writes dB, "
                         "P never stored (round 5, the folded k_stft64f: 0.077 ms per step); stored = pass 1 "
                         "writes P and max(P), pass 2 turns P into dB in place (0.084 ms; "
                         "profiles/r05_stft_fold.txt)")
    ap.add_argument("--no-copy-ceiling", action="store_true",
                    help="skip the in-run HBM copy ceiling of k_rdx's bytes (roofline.copy_ceiling_ms)")
    ap.add_argument("--dry-dist", action="store_true",
                    help="launcher test without a GPU: the ranks meet over gloo and rank 0 prints n_gpus")
    ap.add_argument("--dry-empty", default="1",
                    help="--dry-dist: ranks whose slow-time shard is empty at step 0 (comma list)")
    return ap.parse_args()


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def launch_ranks(n: int) -> int:
    """`bench.py --gpus N` outside torchrun: one rank per GPU through a child
    torch.distributed.run on 127.0.0.1 (this process never touches the GPU, so no
    exec of a GPU-initialised process); returns the launcher's exit status."""
    import subprocess
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd, env=env).returncode


CONFIG5_FRAMES = 65536        # BASELINE config 5: the synthetic stream frame-sharded over 8 GPUs


def config_block(world: int, frames: int, steps: int, C: int = 256, S: int = 1024, NR: int = 1024,
                 ND: int = 256) -> dict:
    """`config` of the bench line.  One GPU: BASELINE config 4 (4096 frames per step).  N > 1
    GPUs: BASELINE config 5, the 65,536-frame stream frame-sharded over the ranks (weak
    scaling: each rank keeps config 4's 4096 frames per step); the line states the frames the
    run covered in total and whether that is the whole config-5 stream."""
    total = world * frames * steps
    step = ("range FFT 1024 + Doppler FFT 256 on every row + detection + Hann(20) hop-1 STFT nfft 64 + dB")
    if world > 1:
        wl = (f"BASELINE config 5: {CONFIG5_FRAMES}-frame synthetic stream frame-sharded across {world} GPUs "
              f"(per GPU per step {frames} frames x {C} chirps x {S} samples; {step}); this run: "
              f"{world} x {frames} x {steps} steps = {total} frames")
    else:
        wl = f"BASELINE config 4: per GPU {frames} frames x {C} chirps x {S} samples; {step}"
    return {"workload": wl, "frames_per_gpu": frames, "frames_total_per_run": total,
            "config5_stream_frames": CONFIG5_FRAMES, "covers_config5_stream": total == CONFIG5_FRAMES,
            "chirps": C, "samples": S, "nr": NR, "nd": ND, "stft_nfft": STFT_NFFT,
            "parallelism": f"frame-shard dp{world}"}


def apply_stream_frames(args, world: int) -> None:
    if args.stream_frames:
        per = world * args.frames
        if args.stream_frames % per:
            print(f"bench.py: --stream-frames {args.stream_frames} is not a multiple of {world} x {args.frames}",
                  file=sys.stderr, flush=True)
            sys.exit(2)
        args.steps = args.stream_frames // per


def dry_dist(args, world: int, rank: int) -> None:
    """The launcher path and the step's collectives on CPU (tests/test_bench_harness.py): the ranks
    meet over gloo and run, for every one of the run's steps, exactly the exchange sequence of
    step() (exchange_halo -> the max(P) all_reduce of the STFT leg -> exchange_rows) on CPU tensors
    of the step's shapes (--frames frames of 256 chirps per rank), standing in for the device
    outputs; each rank checks what it received against what every rank must have sent (the
    inputs are seeded by global frame index), and rank 0 prints the config block the GPU run
    would carry."""
    import numpy as np
    import torch
    import torch.distributed as dist

    from fmcw_radar_processing_amd import dist as fdist
    dist.init_process_group("gloo")
    t = torch.ones(1)
    dist.all_reduce(t)
    F, C, h, M = args.frames, 256, STFT_WLEN - 1, 1

    empty = {int(x) for x in args.dry_empty.split(",") if x.strip()}

    def shard(r, step):                 # what rank r's device outputs would hold at this step
        g = np.random.default_rng(1000003 * step + r)
        cnt = (g.random(F) < 0.9).astype(np.int32)
        if r in empty and step == 0:
            cnt[:] = 0                  # an empty slow-time shard: the halo must skip it
        slow = (g.random((F, C)) * 40).astype(np.float32) * cnt[:, None]
        ridx = (g.integers(2, 30, (F, M)) * cnt[:, None]).astype(np.int32)
        didx = (g.integers(1, 257, (F, M)) * cnt[:, None]).astype(np.int32)
        rmag = (g.random((F, M)) * 500).astype(np.float32) * cnt[:, None]
        keep = np.nonzero(cnt)[0]
        return cnt, slow, ridx, didx, rmag, keep

    checks = {"steps": 0, "halo": True, "lengths": True, "max": True, "rows": True}
    for step in range(args.steps):
        cnt, slow, ridx, didx, rmag, keep = shard(rank, step)
        outs = {"tgt_count": torch.from_numpy(cnt), "slow_mag": torch.from_numpy(slow),
                "tgt_range_idx": torch.from_numpy(ridx), "tgt_doppler_idx": torch.from_numpy(didx),
                "tgt_range_mag": torch.from_numpy(rmag)}
        flist = torch.zeros(F, dtype=torch.int32)
        flist[: len(keep)] = torch.from_numpy(keep.astype(np.int32))
        d_len = torch.tensor([len(keep) * C], dtype=torch.int64)
        hbuf, hl = exchange_halo(fdist, world, rank, outs, flist, d_len, h)
        pmax = torch.tensor([float(slow.max()) if len(keep) else 0.0])       # stands in for pass 1's max(P)
        fdist.global_max_(pmax)
        rows = exchange_rows(fdist, world, outs)
        # what the exchange must deliver, from every rank's seeded shard
        allsh = [shard(r, step) for r in range(world)]
        nxt = np.concatenate([a[1][a[5]].reshape(-1) for a in allsh[rank + 1:]] + [np.zeros(0, np.float32)])[:h]
        checks["halo"] &= int(hl.item()) == len(nxt) and np.array_equal(hbuf.numpy()[: len(nxt)], nxt)
        checks["max"] &= float(pmax.item()) == max(float(a[1].max()) if len(a[5]) else 0.0 for a in allsh)
        checks["lengths"] &= int(fdist.all_lengths(d_len).sum().item()) == C * sum(len(a[5]) for a in allsh)
        if rank == 0:
            want = np.concatenate([np.concatenate([a[0].reshape(-1, 1).astype(np.float32), a[2], a[3], a[4]], 1)
                                   for a in allsh], 0)
            checks["rows"] &= rows is not None and np.array_equal(rows.numpy(), want)
        checks["steps"] += 1
    # the fan-out leg of the GPU line (input_fanout), on 2 frames per rank of the step's frame shape
    fan = None
    if not args.no_fanout:
        fan = input_fanout(dist, world, rank, 2, (C, 1024, 2), torch.float32, "cpu",
                           lambda: dist.barrier(), lambda: None)
    ok = torch.tensor([int(all(v for k, v in checks.items() if k != "steps"))])
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    if rank == 0:
        line = {"metric": METRIC, "n_gpus": world, "ranks_reduced": int(t.item()), "dry_dist": True,
                "steps": args.steps, "exchange": {**checks, "all_ranks_ok": bool(ok.item()),
                                                  "empty_shards_step0": sorted(empty)},
                "config": config_block(world, args.frames, args.steps)}
        if fan:
            line["input_fanout"] = dict(fan, dry=True)
        print(json.dumps(line), flush=True)
    dist.destroy_process_group()
    if not ok.item():
        sys.exit(4)


def main():
    args = parse()
    apply_stream_frames(args, args.gpus)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr, flush=True)
        sys.exit(2)
    if args.dry_dist:
        return dry_dist(args, world, rank)
    import torch
    import torch.distributed as dist

    from fmcw_radar_processing_amd import FMCW_C32H, FMCW_C64
    from fmcw_radar_processing_amd import dist as fdist
    from fmcw_radar_processing_amd import params as P
    from fmcw_radar_processing_amd.engine import Engine

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
    # one non-default stream for the engine's calls and torch's own work of the step (pmax.zero_,
    # the RCCL collectives): ordered on one queue, no per-call side-stream joins (engine._sided)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)

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
        # per-frame stages + the slow-time leg's start (compaction, max(P) reset) in one call
        eng.process_slow_device(d_iq, F, dt, outs, flist, d_len, d_pmax=pmax, d_rd=d_rd, out_dtype=dt, stream=stream)
        hbuf, hl = exchange_halo(fdist, world, rank, outs, flist, d_len, h)
        stft_leg(eng, args.stft_form, outs["slow_mag"], flist, d_len, C, win, fs, max_seg, d_P, pmax, nseg,
                 hbuf, hl, h if world > 1 else 0, fdist.global_max_ if world > 1 else None, stream)
        exchange_rows(fdist, world, outs)

    def barrier():
        if world > 1:
            dist.barrier(device_ids=[local])

    eng.set_pipeline({"auto": 0, "streams": 1, "onepass": 3, "xcd": 4}[args.pipeline])
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    sticky_check(eng, "warmup")
    # level 3: HIP events around every launch of the dominant kernel only (k_rdx; the roofline
    # below), on its stream -- each event pair costs the step a few microseconds (round 5: level 2,
    # a pair around every stage, took 43 us of a 4.6-ms step)
    level = 0 if args.no_stage_timing else 3
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
    sticky_check(eng, "timed steps")          # a timed-out k_rdx hand-off invalidates the run
    # the stage breakdown (every launch between event pairs) from a few steps after the timed ones
    breakdown = {}
    if level:
        eng.timing(2)
        eng.timing_reset()
        nb_steps = 5
        for _ in range(nb_steps):
            step()
        torch.cuda.synchronize(dev)
        breakdown = {k: (ms / nb_steps, n) for k, (ms, n) in eng.timing_read().items()}
        eng.timing(0)
        sticky_check(eng, "stage breakdown steps")
    el = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = float(el.item())

    # sanity: the step did real work (detections on most frames)
    det = int((outs["tgt_count"] > 0).sum().item())

    # ---- in-run normalisers of the roofline --------------------------
    # the effective shader clock of the last k_rdx launch (in-kernel stamps) and the HBM copy
    # ceiling of k_rdx's bytes in this process on this box: a 16-byte nontemporal copy of the input
    # cube into an RD-sized buffer (8.6 + 8.6 GB, DESIGN 4.0.1 part A's shape)
    sclk_mhz, _ = eng.rdx_clock()
    copy = None
    if not args.no_copy_ceiling:
        copy = copy_ceiling(eng, d_iq, dev, stream, 5,
                            "16-byte nontemporal copy of the input cube into an RD-sized buffer (k_rdx's in + RD "
                            "bytes), one thread per 16 bytes, HIP events, same process")

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
    # k_rdx (single-pass schedule): input + RD map + profile, no cube
    for name, label, per_frame in (("range", "k_range", k1_per_frame), ("doppler", "k_doppler", C * NR * 8 + NR * ND * esz + NR * 4),
                                   ("onepass", "k_rdx", C * S * esz + NR * ND * esz + NR * 4),
                                   ("detect", "k_detect", None)):
        ms, n = stages.get(name, (0.0, 0))
        steps_of = args.steps
        if not n and name in breakdown:            # stages the timed region does not time (level 3)
            ms, n = breakdown[name]
            ms, steps_of = ms * 5, 5
        if n:
            fpl = F * steps_of / n
            us = ms / n * 1e3
            kern[label] = {"avg_launch_us": round(us, 2), "frames_per_launch": fpl}
            if per_frame:
                kern[label]["alg_bytes_per_launch"] = int(per_frame * fpl)
                kern[label]["achieved_GBps"] = round(per_frame * fpl / (us * 1e-6) / 1e9, 1)
    roof, path = None, None
    rd_ms, rd_n = stages.get("range_doppler", (0.0, 0))
    rd_steps = args.steps
    if not rd_n and "range_doppler" in breakdown:
        rd_ms, rd_n = breakdown["range_doppler"]
        rd_ms, rd_steps = rd_ms * 5, 5
    if rd_n:
        per_launch_ms = rd_ms / rd_n
        fpl = F * rd_steps / rd_n
        ach = alg_per_frame * fpl / (per_launch_ms * 1e-3) / 1e9
        path = {"achieved": round(ach, 1), "frac": round(ach / HBM_PEAK_GBPS, 4), "unit": "GB/s",
                "span_us": round(per_launch_ms * 1e3, 2), "frames_per_span": fpl, "alg_bytes_per_frame": alg_per_frame,
                "what": "range+Doppler span (before first k_range .. after last k_doppler), SURVEY 8d bytes"}
    pmc = load_pmc(os.path.join(ROOT, "profiles"))
    dom = "k_rdx" if "k_rdx" in kern else "k_range"
    if dom in kern:
        k = kern[dom]
        kname = RDX_NAME[args.fp16] if dom == "k_rdx" else None
        traffic = pmc_traffic(pmc, kname, k["frames_per_launch"]) if kname else None
        roof = {"bound": "hbm", "achieved": k["achieved_GBps"], "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                "frac": round(k["achieved_GBps"] / HBM_PEAK_GBPS, 4), "traffic": traffic,
                "kernel": {"k_rdx": "k_rdx (XCD-team schedule: the 32 CUs of an XCD share each frame; range FFT by chirps, "
                                    "cube handed over through a slot ring, Doppler FFT by range-bin groups; calibration, "
                                    "mean removal, windows, profile, RD store)"}.get(
                              dom, "k_range (K1: calibration, mean removal, window, 1024-pt range FFT, cube store)"),
                "kernel_name": kname,
                "alg_bytes_per_launch": k["alg_bytes_per_launch"], "avg_launch_us": k["avg_launch_us"],
                "frames_per_launch": k["frames_per_launch"],
                "traffic_source": pmc.get("source") if pmc and traffic else None}
        if dom == "k_rdx":
            roof["sclk_mhz"] = round(sclk_mhz, 1) if sclk_mhz else None
            if copy:
                copy_ms_launch = copy["ms"] * (k["alg_bytes_per_launch"] / copy["bytes"])
                roof["copy_ceiling_ms"] = round(copy_ms_launch, 4)
                roof["frac_of_copy_ceiling"] = round(copy_ms_launch / (k["avg_launch_us"] * 1e-3), 4)
                roof["copy_ceiling"] = copy

    # ---- input fan-out over xGMI from rank 0 (reported separately, not in value) -----
    fanout = None
    if world > 1 and not args.no_fanout:
        fanout = input_fanout(dist, world, rank, 256, (C, S, 2), tdt, dev, barrier,
                              lambda: torch.cuda.synchronize(dev))

    extra, legs = {}, []
    if rank == 0 and not args.no_check:
        legs.append(dict(name="config4_f32" if not args.fp16 else "config4_fp16", cfg=cfg, d_iq=d_iq, outs=outs,
                         d_rd=d_rd, d_db=d_P, d_nseg=nseg, fp16=args.fp16, world=world))
    if world == 1 and not args.no_extras and not args.fp16:
        extra["fp16_storage"], leg16 = bench_fp16(eng, cfg, F, args, dev, stream, pmc)
        extra["config2_range_fft"], leg2 = bench_config2(eng, args, dev, stream, pmc)
        if not args.no_check:
            legs += [leg16, leg2]
        if not args.no_host_path:
            extra["host_path"] = bench_host_path(eng)
        eng.set_taps(cfg, P.synth_calibration(S))
    checked, ok = None, True
    if rank == 0:
        # oracle leg, after every timed region: the CPU baseline on this run's own frames and the
        # full-size comparison of every timed frame's outputs with the float64 C oracle
        cpu = cpu_baseline(args.cpu_seconds, d_iq, F, dt) if args.cpu_seconds > 0 and not legs else None
        if legs:
            checked, cpu = oracle_leg(legs, args.cpu_seconds)
            ok = all(v.get("pass", False) for v in checked.values())
        total_frames = world * F * args.steps
        value = total_frames / elapsed
        line = {
            "metric": METRIC, "value": round(value, 1), "unit": "frames/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "f16-storage/f32-compute" if args.fp16 else "f32",
            "data": "synthetic (SURVEY.md 8d generator, generated in HBM per rank)",
            "config": dict(config_block(world, F, args.steps, C, S, NR, ND), stft_form=args.stft_form),
            "hbm_alg_GBps": round(alg_per_frame * value / world / 1e9, 1),
            "roofline": roof,
            "path_roofline": path,
            "kernels": kern,
            "cpu_baseline": cpu,
            "checked": checked,
            "stages_ms_per_step": {k: round(v[0], 4) for k, v in breakdown.items() if v[1]},
            "stages_note": "HIP-event pairs around every launch, 5 steps after the timed ones (the timed steps carry "
                           "k_rdx's pair only)",
            "frames_with_target": det,
        }
        if fanout:
            line["input_fanout"] = fanout
        line.update(extra)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier(device_ids=[local])
        dist.destroy_process_group()
    if not ok:
        print("bench.py: the full-size check against the oracle FAILED (see \"checked\")", file=sys.stderr, flush=True)
        sys.exit(1)


def input_fanout(dist, world, rank, nf, frame_shape, tdt, dev, barrier, sync) -> dict:
    """SURVEY 8e collective 1: the host-staged input scattered from rank 0 (nf frames per rank), timed
    on its own after one untimed scatter; not part of `value` (each rank generates its frames in
    HBM).  The same call runs over gloo on CPU tensors in --dry-dist."""
    import torch
    src = torch.empty((world * nf,) + tuple(frame_shape), dtype=tdt, device=dev) if rank == 0 else None
    dst = torch.empty((nf,) + tuple(frame_shape), dtype=tdt, device=dev)
    parts = list(src.chunk(world)) if rank == 0 else None
    dist.scatter(dst, parts, src=0)
    sync()
    barrier()
    t1 = time.perf_counter()
    dist.scatter(dst, parts, src=0)
    sync()
    barrier()
    ft = time.perf_counter() - t1
    nbytes = world * nf * dst[0].numel() * dst.element_size()
    return {"frames_per_rank": nf, "ms": round(ft * 1e3, 3), "GBps_root_egress": round(nbytes / ft / 1e9, 1)}


def exchange_halo(fdist, world, rank, outs, flist, d_len, h):
    """The step's collectives before the STFT (dist.py): every shard's compacted
    length, then the right halo -- the first wlen-1 samples of the following shards.  (None, None)
    on one GPU.  The same calls run over gloo on CPU tensors in --dry-dist."""
    if world == 1:
        return None, None
    lens = fdist.all_lengths(d_len)
    head = fdist.head_samples(outs["slow_mag"], flist, d_len, h)
    return fdist.right_halo(head, lens, rank)


def exchange_rows(fdist, world, outs):
    """The step's collective after the STFT: the per-frame range_speed rows
    gathered to rank 0 (:386-389).  Returns them on rank 0, None elsewhere or on one GPU."""
    if world == 1:
        return None
    return fdist.gather_range_speed(outs["tgt_count"], outs["tgt_range_idx"], outs["tgt_doppler_idx"],
                                    outs["tgt_range_mag"])


def stft_leg(eng, form, slow, flist, d_len, C, win, fs, max_seg, d_P, pmax, nseg, hbuf, hl, n_halo, gmax, stream):
    """The STFT leg of a step (:270-283) over the compacted slow-time rows; d_P ends as the dB map.
    stored: pass 1 writes P (:276) and max(P), pass 2 turns P into 20 log10(P / max) in place;
    direct: pass 1 forms max(P) only, pass 2 recomputes P and writes the dB.  gmax: the
    all_reduce(MAX) of max(P) across ranks (dist.py), between the passes.  pmax was zeroed by the
    step's process_slow_device call (the detection kernel's last workgroup)."""
    stored = form == "stored"
    eng.stft_power_device(slow, flist, d_len, C, win, STFT_WLEN, STFT_NOVERLAP, STFT_NFFT, fs, max_seg,
                          d_P if stored else None, pmax, nseg, d_halo=hbuf, n_halo=n_halo, d_halo_len=hl,
                          stream=stream)
    if gmax is not None:
        gmax(pmax)
    if stored:
        eng.stft_db_device(d_P, nseg, max_seg, STFT_NFFT, fs, pmax, 0, d_P, stream=stream)
    else:
        eng.stft_db_direct_device(slow, flist, d_len, C, win, STFT_WLEN, STFT_NOVERLAP, STFT_NFFT, fs, max_seg,
                                  pmax, d_P, d_halo=hbuf, n_halo=n_halo, d_halo_len=hl, stream=stream)


def sticky_check(eng, where: str) -> None:
    """fmcw_synchronize: raises when a k_rdx hand-off wait of any launch since the
    last check timed out (its outputs are invalid); the bench then exits non-zero."""
    from fmcw_radar_processing_amd import FmcwError
    try:
        eng.synchronize()
    except FmcwError as e:
        print(f"bench.py: {where}: {e}", file=sys.stderr, flush=True)
        sys.exit(3)


# the headline instantiations: full 1024-sample chirps, RD map written
RDX_NAME = {False: "fmcw::k_rdx<true, false, true>", True: "fmcw::k_rdx<true, true, true>"}


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

    eng.set_pipeline({"auto": 0, "streams": 1, "onepass": 3, "xcd": 4}[args.pipeline])

    def step():
        eng.process_slow_device(d_iq, F, FMCW_C32H, outs, flist, d_len, d_pmax=pmax, d_rd=d_rd, out_dtype=FMCW_C32H,
                                stream=stream)
        stft_leg(eng, args.stft_form, outs["slow_mag"], flist, d_len, C, win, fs, max_seg, d_P, pmax, nseg,
                 None, None, 0, None, stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    sticky_check(eng, "fp16 warmup")
    eng.timing(3)
    eng.timing_reset()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    st = eng.timing_read()
    eng.timing(0)
    sticky_check(eng, "fp16 timed steps")
    ms, n = st["onepass"]
    fpl = F * args.steps / n
    us = ms / n * 1e3
    per = C * S * 4 + NR * ND * 4 + NR * 4
    kname = RDX_NAME[True]
    out = {"value": round(F * args.steps / el, 1), "unit": "frames/s", "ms_per_step": round(el / args.steps * 1e3, 4),
           "dtype": "f16-storage/f32-compute",
           "what": "BASELINE config 4 fp16-storage variant: the headline step with c32h IQ in and c32h RD out",
           "roofline": _roof(per, fpl, us, pmc_traffic(pmc, kname, fpl), kname,
                             "k_rdx<fp16 storage> (XCD-team schedule, c32h in / c32h RD out)", pmc)}
    leg = dict(name="config4_fp16", cfg=cfg, d_iq=d_iq, outs=outs, d_rd=d_rd, d_db=d_P, d_nseg=nseg, fp16=True,
               world=1)
    return out, leg


def copy_ceiling(eng, src, dev, stream, reps, what):
    """The HBM copy ceiling of a kernel's bytes in this process on this box:
    src (a device tensor) copied into a fresh buffer of its size by k_copy16, HIP events over reps."""
    import torch
    nbytes = src.numel() * src.element_size()
    d_cp = torch.empty(nbytes // 4, dtype=torch.float32, device=dev)
    eng.copy_device(src, d_cp, nbytes, stream=stream)
    torch.cuda.synchronize(dev)
    ca, cb = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ca.record(stream)
    for _ in range(reps):
        eng.copy_device(src, d_cp, nbytes, stream=stream)
    cb.record(stream)
    torch.cuda.synchronize(dev)
    cms = ca.elapsed_time(cb) / reps
    del d_cp
    return {"ms": round(cms, 4), "bytes": 2 * nbytes, "GBps": round(2 * nbytes / (cms * 1e-3) / 1e9, 1), "what": what}


def bench_config2(eng, args, dev, stream, pmc):
    """BASELINE config 2: 4096 frames x 128 chirps x 512 samples, range FFT only (K1,
    range cube written, fp32), device-resident; its own roofline on K1's event time."""
    import torch
    from fmcw_radar_processing_amd import FMCW_C64
    from fmcw_radar_processing_amd import params as P
    cfg2 = P.config(2)
    F2, C, S, NR = 4096, cfg2.pn, cfg2.nts, cfg2.nr
    eng.set_taps(cfg2, P.synth_calibration(S))
    # K1 reads the input and writes the cube at the same time, and its time depends on where the two
    # 2-GiB streams sit relative to each other in HBM: 748-860 us on one box for ten byte gaps between
    # the input's end and the cube (profiles/r06_k1_place.txt; the copy of the same bytes 680-705 us,
    # k_rdx flat).  So the harness places them the way a caller should (include/fmcw.h,
    # fmcw_range_fft_device): one allocation, the cube 64 KiB past the input's end; K1's time on two
    # separate default allocations is reported beside it (`default_alloc_us`).
    gap = 64 << 10
    n_in, n_cube = F2 * C * S * 2, F2 * C * NR * 2
    arena = torch.empty(n_in + gap // 4 + n_cube, dtype=torch.float32, device=dev)
    d_iq = arena[:n_in].view(F2, C, S, 2)
    eng.synth_device(d_iq, 0, F2, FMCW_C64, stream=stream)
    d_cube = arena[n_in + gap // 4:].view(F2, C, NR, 2)
    d_prof = torch.empty((F2, NR), dtype=torch.float32, device=dev)
    # a K1 launch is < 1 ms: time at least 100 of them (after 10 warm ones) so that the
    # extra key is not one clock ramp (20 launches varied 846-870 us between boxes)
    warm2, reps2 = max(args.warmup, 10), max(args.steps, 100)
    for _ in range(warm2):
        eng.range_fft_device(d_iq, F2, FMCW_C64, d_cube, d_prof, stream=stream)
    torch.cuda.synchronize(dev)
    eng.timing(3)
    eng.timing_reset()
    t0 = time.perf_counter()
    for _ in range(reps2):
        eng.range_fft_device(d_iq, F2, FMCW_C64, d_cube, d_prof, stream=stream)
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    ms, n = eng.timing_read()["range_only"]
    eng.timing(0)
    us = ms / n * 1e3
    # the same launches on a default torch allocation of the cube (placed wherever the allocator puts it)
    d_cube_def = torch.empty((F2, C, NR, 2), dtype=torch.float32, device=dev)
    for _ in range(3):
        eng.range_fft_device(d_iq, F2, FMCW_C64, d_cube_def, d_prof, stream=stream)
    torch.cuda.synchronize(dev)
    eng.timing(3)
    eng.timing_reset()
    for _ in range(20):
        eng.range_fft_device(d_iq, F2, FMCW_C64, d_cube_def, d_prof, stream=stream)
    torch.cuda.synchronize(dev)
    ms_d, n_d = eng.timing_read()["range_only"]
    eng.timing(0)
    del d_cube_def
    # (the cube of the timed launches is rewritten for the full-size check below)
    eng.range_fft_device(d_iq, F2, FMCW_C64, d_cube, d_prof, stream=stream)
    torch.cuda.synchronize(dev)
    per = C * S * 8 + C * NR * 8 + NR * 4
    out = {"value": round(F2 * reps2 / el, 1), "unit": "frames/s", "ms_per_step": round(el / reps2 * 1e3, 4),
           "launches_timed": reps2,
           "placement": {"cube_gap_after_input_bytes": gap, "one_allocation": True,
                         "default_alloc_us": round(ms_d / n_d * 1e3, 2),
                         "default_alloc_frac": round(per * F2 / (ms_d / n_d * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
                         "sweep": "profiles/r06_k1_place.txt (748-860 us over 18 gaps, one box)"},
           "dtype": "f32", "what": "BASELINE config 2: 4096 x 128 x 512 IQ, range FFT only, cube + profile written",
           "roofline": _roof(per, F2, us, pmc_traffic(pmc, K1_NAME, F2), K1_NAME,
                             "K1 k_range (calibration, mean, window, 512-pt range FFT, cube + profile store)", pmc)}
    if not args.no_copy_ceiling:   # K1's own in-run ceiling: its input copied into a cube-sized buffer
        cc = copy_ceiling(eng, d_iq, dev, stream, 10,
                          "16-byte nontemporal copy of the config-2 input into a cube-sized buffer (K1's in + cube "
                          "bytes), HIP events, same process")
        out["roofline"]["copy_ceiling_ms"] = cc["ms"]
        out["roofline"]["frac_of_copy_ceiling"] = round(cc["ms"] / (us * 1e-3), 4)
        out["roofline"]["copy_ceiling"] = cc
    leg = dict(name="config2", cfg=cfg2, d_iq=d_iq, d_cube=d_cube, d_prof=d_prof)
    return out, leg


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


def bench_host_path(eng0):
    """The path MATLAB calls (MEX -> fmcw_process + fmcw_stft on HOST buffers,
    radar_processing.m:197-299): inputs in pageable host memory, PCIe included,
    at the deployed 64x16 module geometry and at the config-3 geometry, on the context the
    MATLAB drop-in creates (matlab/radar_processing.m: FMCW_DEVICES, else every visible device;
    frames / STFT segments sharded over its devices)."""
    import torch
    from fmcw_radar_processing_amd import FMCW_C64
    from fmcw_radar_processing_amd import params as P
    from fmcw_radar_processing_amd import windows as W
    from fmcw_radar_processing_amd.engine import Engine
    eng = Engine(None)
    info = eng.device_info()
    res = {"context_devices": info["devices"], "rccl": info["rccl"]}
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
    eng.close()
    return res


def _oracle_setup(cfg):
    """The float64 oracle's parameters, windows and calibration for a bench config
    (the same taps the bench gave the device: cfg windows, SURVEY 8d calibration)."""
    from fmcw_radar_processing_amd import params as P
    from oracle import oracle as O
    p = O.derive_params(P.deployed_device(cfg.nts, cfg.pn), nr=cfg.nr, nd=cfg.nd, parity=False)
    wr, wd = O.windows(cfg.nts, cfg.pn)
    return p, wr, wd, P.synth_calibration(cfg.nts)


def _host_frames(d_iq, f0: int, f1: int, C: int, S: int):
    """Frames f0..f1 of a device IQ tensor as complex64 (fp16 storage: the same values widened)."""
    x = d_iq[f0:f1].float().cpu().numpy()
    return x.view(np.float32).reshape(f1 - f0, C, S, 2).view(np.complex64)[..., 0]


def _rel_rows(got, ref):
    got = np.asarray(got, np.float64)
    num = np.sqrt(np.sum((got - ref) ** 2, axis=1))
    return num / np.maximum(np.sqrt(np.sum(ref ** 2, axis=1)), 1e-300)


def check_rd_leg(leg, threads: int):
    """Every frame of a config-4 step (radar_processing.m:203-219, :257-283) against the C
    oracle: RD map per-frame relative L2 (raw, and relaxed as tests/helpers.rd_rel_err),
    profile, detections (exact except near-ties), slow-time rows, and the hop-1 STFT dB.
    Returns (result dict, seconds of oracle_process, frames, seconds of the oracle STFT)."""
    from fmcw_radar_processing_amd import params as P
    from oracle import coracle as CO
    from oracle import oracle as O
    cfg, fp16, world = leg["cfg"], leg["fp16"], leg.get("world", 1)
    C, S, NR, ND = cfg.pn, cfg.nts, cfg.nr, cfg.nd
    d_iq = leg["d_iq"]
    F = d_iq.shape[0]
    p, wr, wd, cal = _oracle_setup(cfg)
    B = max(16, 4 * threads)
    rd_buf = np.zeros((B, NR, ND), np.complex128)
    keys = ("profile", "tgt_count", "tgt_range_idx", "tgt_range_mag", "tgt_doppler_idx", "slow_mag")
    per = {k: [] for k in keys}
    raw, rlx = np.zeros(F), np.zeros(F)
    busy = 0.0
    for f0 in range(0, F, B):
        f1 = min(F, f0 + B)
        n = f1 - f0
        iq = _host_frames(d_iq, f0, f1, C, S)
        t = time.perf_counter()
        out = CO.process_frames(iq, cal, p, wr, wd, rd_out=rd_buf[:n], nthreads=threads, want_pre=True)
        busy += time.perf_counter() - t
        g = leg["d_rd"][f0:f1]
        unscale = 1.0
        if fp16:                       # c32h RD holds D / (Nr Nd) (include/fmcw.h)
            g, unscale = g.float(), float(NR * ND)
        num, den = CO.err2(rd_buf[:n], g.cpu().numpy(), unscale, threads)
        raw[f0:f1] = np.sqrt(num / np.maximum(den, 1e-300))
        rlx[f0:f1] = np.sqrt(num) / np.maximum(np.maximum(np.sqrt(den), 0.1 * np.sqrt(out["pre"])), 1e-300)
        for k in keys:
            per[k].append(out[k])
    ref = {k: np.concatenate(v) for k, v in per.items()}
    got = {k: leg["outs"][k].cpu().numpy() for k in keys}
    srt = np.sort(ref["profile"], axis=1)
    row_tol, row16_tol = 1e-5, 3e-3          # fp32 rel L2 1e-5; fp16 storage 3e-3 (c32h hand-off blocks)
    tie = (srt[:, -1] - srt[:, -2]) <= (1e-3 if fp16 else 1e-5) * srt[:, -1]   # top-2 bins within rounding
    differ = np.zeros(F, bool)
    for k in ("tgt_count", "tgt_range_idx", "tgt_doppler_idx"):
        a, b = got[k].reshape(F, -1), ref[k].reshape(F, -1)
        differ |= np.any(a != b, axis=1)
    bad_det = int(np.sum(differ & ~tie))
    has = ref["tgt_count"] > 0
    # fp16 storage hands the 128-bin blocks that cannot hold a candidate over as c32h: the profile
    # there is held to the fp16 bar, the blocks around the detection window (fp32 hand-off), the
    # slow-time rows and the target magnitudes to the fp32 bar
    keep = P.fp16_fp32_bins(cfg) if fp16 else np.ones(NR, bool)
    prof_err = float(_rel_rows(got["profile"][:, keep], ref["profile"][:, keep]).max())
    prof16_err = float(_rel_rows(got["profile"][:, ~keep], ref["profile"][:, ~keep]).max()) if (~keep).any() else 0.0
    slow_err = float(_rel_rows(got["slow_mag"][has], ref["slow_mag"][has]).max()) if has.any() else 0.0
    slow_zero = bool(np.all(got["slow_mag"][~has & ~differ] == 0))
    m = ref["tgt_count"][:, None] > np.arange(ref["tgt_range_mag"].shape[1])[None, :]
    mag_err = float(np.max(np.abs(got["tgt_range_mag"][m] - ref["tgt_range_mag"][m]) / ref["tgt_range_mag"][m])) \
        if m.any() else 0.0
    # :270-283 STFT dB of the concatenated slow-time signal, on the native nfft/2+1 bins
    x = ref["slow_mag"][has].reshape(-1)
    t = time.perf_counter()
    sp = CO.spectrogram(x, cfg.prt, O.stft_window("hann"), STFT_NOVERLAP, STFT_NFFT, nbins=0, nthreads=threads)
    t_stft = time.perf_counter() - t
    nref = sp["intensity"].shape[0]
    nc = min(int(leg["d_nseg"].item()), nref)
    if differ.any():                   # compare the segments before the first frame whose detection differs
        fd = int(np.argmax(differ))
        nc = min(nc, C * int(np.sum(has[:fd])) - (STFT_WLEN - 1))
    db_tol, db_floor = (0.05, -60.0) if fp16 else (1e-3, -80.0)
    stft_err = None
    if nc > 0:
        g = leg["d_db"][:nc].cpu().numpy().astype(np.float64)
        r = sp["intensity"][:nc]
        if world > 1:                  # rank 0's dB is normalised by the global max(P): renormalise both locally
            g, r = g - g.max(), r - r.max()
        sel = r > db_floor
        stft_err = float(np.max(np.abs(g[sel] - r[sel]))) if sel.any() else 0.0
    rd_tol = 3e-3 if fp16 else 1e-5
    res = {"frames": F, "what": "every frame of the last timed step vs oracle/fmcw_oracle.c (fp64)",
           "rd_rel_l2_raw_max": float(raw.max()), "rd_rel_l2_raw_median": float(np.median(raw)),
           "rd_rel_l2_relaxed_max": float(rlx.max()), "rd_tol": rd_tol,
           "profile_rel_l2_max": prof_err, "slow_rows_rel_l2_max": slow_err, "range_mag_rel_max": mag_err,
           "row_tol": row_tol, "profile_c32h_blocks_rel_l2_max": prof16_err if fp16 else None,
           "profile_c32h_blocks_tol": row16_tol if fp16 else None,
           "profile_fp32_bins": int(keep.sum()), "detections_differing": bad_det, "near_tie_frames": int(tie.sum()),
           "frames_with_target": int(has.sum()), "no_target_rows_zero": slow_zero,
           "stft_segments_compared": int(max(nc, 0)), "stft_segments_ref": int(nref),
           "stft_max_abs_db": stft_err, "stft_tol_db": db_tol, "stft_db_floor": db_floor}
    res["pass"] = bool(raw.max() <= rd_tol and prof_err <= row_tol and prof16_err <= row16_tol and
                       slow_err <= row_tol and mag_err <= row_tol and
                       bad_det == 0 and slow_zero and stft_err is not None and stft_err <= db_tol and
                       nc >= 0.99 * nref - world * STFT_WLEN)
    return res, busy, F, t_stft


def check_cube_leg(leg, threads: int):
    """Config 2 (range FFT only, :203-207, :210): every frame's range cube (per-frame
    relative L2) and profile against the C oracle."""
    from oracle import coracle as CO
    cfg = leg["cfg"]
    C, S, NR = cfg.pn, cfg.nts, cfg.nr
    d_iq = leg["d_iq"]
    F = d_iq.shape[0]
    p, wr, wd, cal = _oracle_setup(cfg)
    B = max(16, 4 * threads)
    cube_buf = np.zeros((B, C, NR), np.complex128)
    err, prof = np.zeros(F), []
    for f0 in range(0, F, B):
        f1 = min(F, f0 + B)
        n = f1 - f0
        out = CO.process_frames(_host_frames(d_iq, f0, f1, C, S), cal, p, wr, wd, cube_out=cube_buf[:n],
                                nthreads=threads)
        num, den = CO.err2(cube_buf[:n], leg["d_cube"][f0:f1].cpu().numpy(), 1.0, threads)
        err[f0:f1] = np.sqrt(num / np.maximum(den, 1e-300))
        prof.append(out["profile"])
    perr = float(_rel_rows(leg["d_prof"].cpu().numpy(), np.concatenate(prof)).max())
    res = {"frames": F, "what": "every frame of the last timed launch vs oracle/fmcw_oracle.c (fp64)",
           "cube_rel_l2_max": float(err.max()), "cube_rel_l2_median": float(np.median(err)),
           "profile_rel_l2_max": perr, "tol": 1e-5}
    res["pass"] = bool(err.max() <= 1e-5 and perr <= 1e-5)
    return res


def oracle_leg(legs, budget_s: float):
    """After every timed region (rank 0): the full-size check of each leg, and the CPU
    baseline, whose first pass is the headline leg's own check pass."""
    cores, _ = host_cores()
    checked, cpu = {}, None
    for leg in legs:
        if "d_cube" in leg:
            checked[leg["name"]] = check_cube_leg(leg, cores)
            continue
        res, busy, nfr, t_stft = check_rd_leg(leg, cores)
        checked[leg["name"]] = res
        if cpu is None and budget_s > 0:
            cpu = cpu_baseline(budget_s, leg["d_iq"], leg["d_iq"].shape[0], None, prior=(nfr, busy + t_stft))
    return checked, cpu


def cpu_baseline(budget_s: float, d_iq, F: int, dt, prior=None):
    """C restatement of radar_processing.m:197-299 (oracle/fmcw_oracle.c, fp64,
    OpenMP over frames) on a bounded sample of the SAME device-resident frames
    (copied back in batches), on this host's cores.  Every row's Doppler FFT is
    computed (as the GPU path does), then the hop-1 STFT of the slow-time signal.
    prior = (frames, seconds) already measured on all cores (the check pass)."""
    from oracle import coracle as CO
    from oracle import oracle as O
    from fmcw_radar_processing_amd import params as P
    cores, host = host_cores()
    cfg = P.config(4)
    p, wr, wd, cal = _oracle_setup(cfg)
    win = O.stft_window("hann")
    B = 4 * cores

    def run(threads, budget, done=0, busy=0.0):
        slow = []
        rd = np.zeros((B, cfg.nr, cfg.nd), np.complex128)
        f0 = 0
        while busy < budget or done < B:
            iq = _host_frames(d_iq, f0, min(F, f0 + B), cfg.pn, cfg.nts)      # not timed
            t = time.perf_counter()
            out = CO.process_frames(iq, cal, p, wr, wd, rd_out=rd[:iq.shape[0]], nthreads=threads)
            keep = out["tgt_count"] > 0
            slow.append(out["slow_mag"][keep].reshape(-1))
            busy += time.perf_counter() - t
            done += iq.shape[0]
            f0 = (f0 + B) % max(F - B, 1)
        t = time.perf_counter()
        x = np.concatenate(slow) if slow else np.zeros(0)
        if len(x) >= STFT_WLEN:
            CO.spectrogram(x, cfg.prt, win, STFT_NOVERLAP, STFT_NFFT, nbins=0, nthreads=threads)
        return done / (busy + time.perf_counter() - t), done

    n0, s0 = prior if prior else (0, 0.0)
    v_all, n_all = run(cores, budget_s, done=n0, busy=s0)
    v_one, n_one = run(1, max(2.0, budget_s / 4))
    return {"value": round(v_all, 2), "unit": "frames/s", "cores": cores, "kind": "port",
            "sample": f"{n_all} config-4 frames (the bench's own device frames, copied back) through "
                      f"oracle/fmcw_oracle.c (fp64, OpenMP {cores} threads, every RD row) + hop-1 STFT nfft 64"
                      + (f"; the first {n0} are the full-size check pass" if n0 else ""),
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
