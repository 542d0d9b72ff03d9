"""Frame-sharded multi-GPU path: one process per GPU.

Frames are independent through stages a4-a12, so rank g owns the contiguous
frame range [g*F, (g+1)*F) of the stream and generates / receives only those.
The only cross-frame step is the slow-time STFT over the concatenated signal
(radar_processing.m:259, :276).  Its exchange steps, all tiny, run as RCCL
collectives (torch.distributed "nccl" = RCCL over xGMI) on device tensors:

  1. all_gather of each rank's compacted length L_g (int64): global offsets
  2. all_gather of each rank's first (wlen-1) slow-time samples: the right halo,
     so segments that straddle a shard boundary are computed by their left rank
  3. all_reduce(MAX) of the local max(P): the global normalisation of :282-283
  4. gather to rank 0 of (count, range idx, Doppler idx, magnitude) per frame:
     the range_speed concatenation of :386-389

The collective helpers take and return torch tensors and work unchanged on the
gloo backend with CPU tensors (tests/test_dist.py).
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard_range(F_total: int, rank: int, world: int):
    """Contiguous frame shard [f0, f0+n) of rank (keeps the :259 concatenation order)."""
    base, rem = divmod(F_total, world)
    f0 = rank * base + min(rank, rem)
    return f0, base + (1 if rank < rem else 0)


def all_lengths(L_local: torch.Tensor) -> torch.Tensor:
    """[world] int64 of every rank's compacted slow-time length."""
    world = dist.get_world_size()
    out = torch.empty(world, dtype=L_local.dtype, device=L_local.device)
    dist.all_gather_into_tensor(out, L_local.reshape(1))
    return out


def head_samples(slow_mag: torch.Tensor, frame_list: torch.Tensor, L_local: torch.Tensor, h: int) -> torch.Tensor:
    """First h samples of this rank's compacted signal (zeros past L), on device, no host sync."""
    pn = slow_mag.shape[1]
    if frame_list.numel() == 0 or slow_mag.shape[0] == 0:       # empty shard (F_total < world)
        return torch.zeros(h, dtype=slow_mag.dtype, device=slow_mag.device)
    q = torch.arange(h, device=slow_mag.device)
    fi = torch.clamp(q // pn, max=frame_list.numel() - 1)
    fr = frame_list[fi].long().clamp(0, slow_mag.shape[0] - 1)
    vals = slow_mag[fr, q % pn]
    return torch.where(q < L_local.reshape(()), vals, torch.zeros_like(vals))


def right_halo(head_local: torch.Tensor, lens: torch.Tensor, rank: int):
    """Halo = the first samples of the following ranks' signals, in order, up to h.

    Returns (halo [h] float32, halo_len [1] int64), both on device; no host sync.
    """
    world = lens.numel()
    h = head_local.numel()
    heads = torch.empty(world * h, dtype=head_local.dtype, device=head_local.device)
    dist.all_gather_into_tensor(heads, head_local.contiguous())
    heads = heads.reshape(world, h)
    avail = torch.clamp(lens, max=h)
    avail = torch.where(torch.arange(world, device=lens.device) > rank, avail, torch.zeros_like(avail))
    ends = torch.cumsum(avail, 0)
    starts = ends - avail
    j = torch.arange(h, device=lens.device)
    r = torch.searchsorted(ends, j, right=True).clamp(max=world - 1)
    src = (j - starts[r]).clamp(0, h - 1)
    halo = heads[r, src]
    total = ends[-1].clamp(max=h)
    halo = torch.where(j < total, halo, torch.zeros_like(halo))
    return halo.contiguous(), total.reshape(1).to(torch.int64)


def global_max_(pmax: torch.Tensor) -> torch.Tensor:
    dist.all_reduce(pmax, op=dist.ReduceOp.MAX)
    return pmax


def gather_range_speed(count: torch.Tensor, ridx: torch.Tensor, didx: torch.Tensor, rmag: torch.Tensor,
                       F_total: int | None = None, dst: int = 0):
    """range_speed concatenation (:386-389): per-frame rows (count, ridx.., didx.., rmag..)
    of every rank, in frame order, on rank ``dst`` as one float32 tensor; None on
    the other ranks.  Shards may differ by one frame (shard_range): rows are
    padded to ceil(F_total/world) for the collective and trimmed on ``dst``."""
    rows = torch.cat([count.reshape(-1, 1).float(), ridx.float(), didx.float(), rmag.float()], 1)
    world, rank = dist.get_world_size(), dist.get_rank()
    F_total = F_total if F_total is not None else rows.shape[0] * world
    cap = -(-F_total // world)
    if rows.shape[0] < cap:
        rows = torch.cat([rows, rows.new_zeros(cap - rows.shape[0], rows.shape[1])], 0)
    rows = rows.contiguous()
    if rank == dst:
        bufs = [torch.empty_like(rows) for _ in range(world)]
        dist.gather(rows, gather_list=bufs, dst=dst)
        return torch.cat([b[: shard_range(F_total, r, world)[1]] for r, b in enumerate(bufs)], 0)
    dist.gather(rows, dst=dst)
    return None
