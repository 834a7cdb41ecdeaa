#!/usr/bin/env python3
"""Probe: can two RCCL ranks share one GPU on this box?  (torchrun --nproc-per-node 2)
Prints the outcome of an all_reduce and a send/recv between the two ranks on cuda:0."""
import datetime
import os

import torch
import torch.distributed as dist

rank = int(os.environ["RANK"])
torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
try:
    dist.init_process_group("nccl", rank=rank, world_size=2,
                            timeout=datetime.timedelta(seconds=60), device_id=dev)
    t = torch.full((4,), float(rank + 1), device=dev)
    dist.all_reduce(t)
    torch.cuda.synchronize()
    print(f"rank {rank}: all_reduce -> {t.tolist()}", flush=True)
    x = torch.full((1 << 20,), float(rank), device=dev)
    y = torch.empty_like(x)
    ops = [dist.P2POp(dist.isend, x, 1 - rank), dist.P2POp(dist.irecv, y, 1 - rank)]
    for w in dist.batch_isend_irecv(ops):
        w.wait()
    torch.cuda.synchronize()
    print(f"rank {rank}: send/recv -> {y[0].item()}", flush=True)
    dist.destroy_process_group()
except Exception as e:  # noqa: BLE001
    print(f"rank {rank}: FAILED {type(e).__name__}: {str(e)[:300]}", flush=True)
