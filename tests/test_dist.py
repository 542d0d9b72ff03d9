"""CPU, multi-process (gloo): the frame-sharded slow-time path of
fmcw_radar_processing_amd/dist.py reproduces the single-process result.

Each rank owns a contiguous frame shard.  The per-frame stages are independent,
so what must be right is the exchange: global lengths, the right halo taken
from the following ranks (also when a rank has fewer than wlen-1 samples or
none), the global max(P), and the range_speed gather.  Per-rank spectrogram
segments are evaluated with the oracle here (no GPU in this container).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

WLEN, NOV, NFFT, PRT = 20, 19, 64, 8e-4


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _scenario(F, C, seed):
    g = np.random.default_rng(seed)
    count = (g.random(F) > 0.3).astype(np.int32)
    if F > 4:
        count[F // 3: F // 3 + 4] = 0        # a run of empty frames (a shard may see none)
    slow = np.abs(g.standard_normal((F, C))) * count[:, None]
    ridx = (g.integers(5, 100, F) * count).astype(np.int32)[:, None]
    didx = (g.integers(1, 17, F) * count).astype(np.int32)[:, None]
    rmag = (g.random(F) * 1000 * count)[:, None]
    return count, slow, ridx, didx, rmag


def _worker(rank, world, port, F, C, seed, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from fmcw_radar_processing_amd import dist as fd
        from oracle import oracle as O
        count, slow, ridx, didx, rmag = _scenario(F, C, seed)
        f0, n = fd.shard_range(F, rank, world)
        c_l, s_l = count[f0:f0 + n], slow[f0:f0 + n]
        flist = np.nonzero(c_l > 0)[0].astype(np.int32)                # what k_compact produces
        L = torch.tensor([len(flist) * C], dtype=torch.int64)
        lens = fd.all_lengths(L)
        fl_t = torch.from_numpy(np.r_[flist, np.zeros(max(0, n - len(flist)), np.int32)])
        head = fd.head_samples(torch.from_numpy(s_l), fl_t, L, WLEN - 1)
        halo, hl = fd.right_halo(head, lens, rank)
        local = s_l[flist].reshape(-1)
        ext = np.r_[local, halo[: int(hl.item())].double().numpy()]
        win = O.stft_window("hann")
        nseg = max(0, (len(ext) - NOV) // (WLEN - NOV))
        if nseg:
            _, _, _, P = O.spectrogram(ext, win, NOV, NFFT, 1 / PRT)
        else:
            P = np.zeros((NFFT // 2 + 1, 0))
        pmax = torch.tensor([P.max() if P.size else 0.0], dtype=torch.float64)
        fd.global_max_(pmax)
        psd = 20 * np.log10(P / pmax.item()) if P.size else P
        parts = [None] * world
        dist.all_gather_object(parts, psd)
        rs = fd.gather_range_speed(torch.from_numpy(c_l), torch.from_numpy(ridx[f0:f0 + n]),
                                   torch.from_numpy(didx[f0:f0 + n]), torch.from_numpy(rmag[f0:f0 + n]), F_total=F)
        if rank == 0:
            q.put((np.concatenate([p for p in parts if p.size], axis=1), rs.numpy() if rs is not None else None,
                   [int(v) for v in lens.tolist()]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,F,C", [(2, 13, 8), (3, 12, 4), (4, 17, 4),
                                        (4, 3, 32)])   # F < world: rank 3 owns no frame at all
def test_sharded_stft_equals_single_process(world, F, C):
    from oracle import oracle as O
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, F, C, 7 + world, q)) for r in range(world)]
    for p in procs:
        p.start()
    got, rs, lens = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    count, slow, ridx, didx, rmag = _scenario(F, C, 7 + world)
    x = slow[count > 0].reshape(-1)
    ref = O.spectrogram_pipeline(x, PRT, O.stft_window("hann"), NOV, nfft=NFFT, nbins=0)
    assert got.shape == ref["intensity"].shape
    np.testing.assert_allclose(got, ref["intensity"], atol=1e-9)
    assert sum(lens) == len(x)
    np.testing.assert_array_equal(rs[:, 0], count)               # every frame, in order
    np.testing.assert_array_equal(rs[:, 1], ridx[:, 0])
    np.testing.assert_allclose(rs[:, 3], rmag[:, 0], rtol=1e-6)


def test_shard_range_covers_in_order():
    from fmcw_radar_processing_amd.dist import shard_range
    for F in (1, 7, 4096, 65536):
        for w in (1, 2, 3, 8):
            spans = [shard_range(F, r, w) for r in range(w)]
            assert spans[0][0] == 0
            assert all(spans[i][0] + spans[i][1] == spans[i + 1][0] for i in range(w - 1))
            assert sum(s[1] for s in spans) == F
