"""CPU: the bench harness itself (bench.py), without a GPU.

* ``bench.py --gpus 2`` outside torchrun starts two ranks through its own child
  launcher; they meet over gloo (``--dry-dist``) and rank 0 reports n_gpus 2.
  A world size that disagrees with --gpus is an error.
* The full-size check of the oracle leg (check_rd_leg / check_cube_leg) passes
  on outputs that agree with the oracle to fp32 rounding and fails on a
  perturbed RD map, range cube, detection or STFT.  The "device" outputs here
  are the Python oracle's own, rounded to float32, held in CPU tensors.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from fmcw_radar_processing_amd import params as P  # noqa: E402
from oracle import oracle as O  # noqa: E402


def _run_bench(args, env_extra=None, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, cwd=ROOT,
                          capture_output=True, text=True, timeout=timeout)


def test_gpus_2_launches_two_ranks():
    r = _run_bench(["--gpus", "2", "--dry-dist"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout             # rank 0 alone prints
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["ranks_reduced"] == 2


def test_gpus_2_names_config5_and_the_frame_total():
    """with N > 1 ranks the line names BASELINE config 5 and the frames the
    run covered; --stream-frames 65536 makes the run the whole config-5 stream (8 steps on 2)."""
    r = _run_bench(["--gpus", "2", "--dry-dist", "--stream-frames", "65536"])
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    c = d["config"]
    assert c["workload"].startswith("BASELINE config 5") and "65536-frame" in c["workload"]
    assert d["steps"] == 8 and c["frames_total_per_run"] == 65536 and c["covers_config5_stream"]
    assert c["parallelism"] == "frame-shard dp2" and c["frames_per_gpu"] == 4096
    one = bench.config_block(1, 4096, 20)
    assert one["workload"].startswith("BASELINE config 4") and one["frames_total_per_run"] == 81920
    assert bench.config_block(8, 4096, 2)["covers_config5_stream"]


@pytest.mark.parametrize("args", [["--gpus", "2", "--stream-frames", "65536"],
                                  ["--gpus", "3", "--frames", "512", "--steps", "2"],
                                  ["--gpus", "8", "--stream-frames", "65536"],
                                  ["--gpus", "8", "--frames", "256", "--steps", "2", "--dry-empty", "3,4"]],
                         ids=["2_ranks_config5", "3_ranks_empty_middle", "8_ranks_config5", "8_ranks_two_empty"])
def test_dry_dist_runs_the_step_exchange(args):
    """the ranks run exactly the step's collective sequence (bench.exchange_halo
    -> the STFT leg's max(P) all_reduce -> bench.exchange_rows) on CPU tensors of the step's
    shapes, every step of the run (65,536 frames over 2 ranks: 8 steps of 4096 frames; 3 ranks
    with an empty slow-time shard in the middle at step 0), and each rank checks what it received
    (halo, lengths, max, the range_speed rows on rank 0)."""
    r = _run_bench(args + ["--dry-dist"])
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    ex = d["exchange"]
    assert ex["all_ranks_ok"] and ex["halo"] and ex["lengths"] and ex["max"] and ex["rows"], ex
    n = int(args[1])
    assert ex["steps"] == d["steps"] and d["n_gpus"] == n
    if "--stream-frames" in args:                    # the whole config-5 stream: 65,536 / (n x 4096) steps
        assert d["config"]["covers_config5_stream"] and d["steps"] == 65536 // (n * 4096)
        assert d["config"]["workload"].startswith("BASELINE config 5")
        assert d["config"]["parallelism"] == f"frame-shard dp{n}"
    if "--dry-empty" in args:                        # two adjacent empty shards: rank 2's halo comes from rank 5
        assert ex["empty_shards_step0"] == [3, 4]
    fo = d["input_fanout"]                           # the fan-out leg's fields
    assert fo["dry"] and fo["frames_per_rank"] == 2 and fo["ms"] > 0 and fo["GBps_root_egress"] > 0


def test_stream_frames_must_divide():
    r = _run_bench(["--gpus", "2", "--dry-dist", "--stream-frames", "65537"])
    assert r.returncode == 2 and "not a multiple" in r.stderr


def test_world_size_must_match_gpus():
    r = _run_bench(["--gpus", "2", "--dry-dist"], env_extra={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2
    assert "WORLD_SIZE 1" in r.stderr


def _config_small():
    # a throughput-mode geometry small enough for the pure-Python oracle
    cfg = P.derive_params(P.deployed_device(256, 64), nr=256, nd=64, mode=P.THROUGHPUT)
    return cfg


def _rd_leg(F=6, fp16=False):
    cfg = _config_small()
    p, wr, wd, cal = bench._oracle_setup(cfg)
    iq = O.synth_frames(F, cfg.pn, cfg.nts, cfg.nr, cfg.nd, p["dist_per_bin"], frame0=40)
    if fp16:
        iq = iq.astype(np.complex64)
        h = np.stack([iq.real, iq.imag], -1).astype(np.float16)
        iq = (h[..., 0].astype(np.float32) + 1j * h[..., 1].astype(np.float32)).astype(np.complex64)
    ref = O.process_frames(iq, cal, p, wr, wd, want_rd=True, rd_all_rows=True)
    d_iq = torch.from_numpy(np.stack([iq.real, iq.imag], -1).astype(np.float16 if fp16 else np.float32))
    outs = {k: torch.from_numpy(np.asarray(ref[k]).astype(np.int32 if "idx" in k or "count" in k else np.float32))
            for k in ("profile", "tgt_count", "tgt_range_idx", "tgt_range_mag", "tgt_doppler_idx", "slow_mag")}
    rd = ref["rd"]
    if fp16:
        rd = rd / (cfg.nr * cfg.nd)
        d_rd = torch.from_numpy(np.stack([rd.real, rd.imag], -1).astype(np.float16))
    else:
        d_rd = torch.from_numpy(np.stack([rd.real, rd.imag], -1).astype(np.float32))
    x = O.slow_time_signal(ref)
    _, _, _, Pw = O.spectrogram(x.astype(np.float32).astype(np.float64), O.stft_window("hann"),
                                bench.STFT_NOVERLAP, bench.STFT_NFFT, 1.0 / cfg.prt)
    db = O.psd_db(Pw).T.astype(np.float32)                  # [nseg][nfft/2+1]
    leg = dict(name="t", cfg=cfg, d_iq=d_iq, outs=outs, d_rd=d_rd, d_db=torch.from_numpy(db.copy()),
               d_nseg=torch.tensor([db.shape[0]]), fp16=fp16, world=1)
    return leg


@pytest.mark.parametrize("fp16", [False, True])
def test_check_rd_leg_passes_on_agreeing_outputs(fp16):
    leg = _rd_leg(fp16=fp16)
    res, busy, nfr, _ = bench.check_rd_leg(leg, 2)
    assert res["pass"], res
    assert nfr == leg["d_iq"].shape[0] and busy > 0
    assert res["stft_segments_compared"] == res["stft_segments_ref"] > 0
    assert res["detections_differing"] == 0


def test_check_rd_leg_fails_on_errors():
    leg = _rd_leg()
    leg["d_rd"][2, 17, 5, 0] += 1e-2 * float(leg["d_rd"][2].abs().max())
    res, *_ = bench.check_rd_leg(leg, 2)
    assert not res["pass"] and res["rd_rel_l2_raw_max"] > 1e-5
    leg = _rd_leg()
    has = np.nonzero(leg["outs"]["tgt_count"].numpy() > 0)[0]
    leg["outs"]["tgt_doppler_idx"][has[0], 0] += 1
    res, *_ = bench.check_rd_leg(leg, 2)
    assert not res["pass"] and res["detections_differing"] == 1
    leg = _rd_leg()
    leg["d_db"][3, 4] += 0.01
    res, *_ = bench.check_rd_leg(leg, 2)
    assert not res["pass"] and res["stft_max_abs_db"] >= 0.009


def test_check_cube_leg():
    cfg = P.derive_params(P.deployed_device(128, 32), nr=128, nd=16, mode=P.THROUGHPUT)
    p, wr, wd, cal = bench._oracle_setup(cfg)
    iq = O.synth_frames(5, cfg.pn, cfg.nts, cfg.nr, cfg.nd, p["dist_per_bin"])
    ref = O.process_frames(iq, cal, p, wr, wd, want_cube=True)
    cube = ref["cube"]
    leg = dict(name="c2", cfg=cfg, d_iq=torch.from_numpy(np.stack([iq.real, iq.imag], -1).astype(np.float32)),
               d_cube=torch.from_numpy(np.stack([cube.real, cube.imag], -1).astype(np.float32)),
               d_prof=torch.from_numpy(ref["profile"].astype(np.float32)))
    res = bench.check_cube_leg(leg, 2)
    assert res["pass"], res
    leg["d_cube"][1, 3, 7, 1] += 1e-2 * float(leg["d_cube"][1].abs().max())
    res = bench.check_cube_leg(leg, 2)
    assert not res["pass"]
