"""Probe: can two ranks share one GPU under RCCL (torch.distributed 'nccl')?  Development only."""
import os
import torch
import torch.distributed as dist

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", device_id=dev)
r = dist.get_rank()
t = torch.full((4,), float(r + 1), device=dev)
dist.all_reduce(t)
torch.cuda.synchronize()
print(f"rank {r}: all_reduce -> {t.tolist()}", flush=True)
dist.destroy_process_group()
