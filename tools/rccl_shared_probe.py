#!/usr/bin/env python3
"""Probe: can two RCCL ranks share the one GPU of a gpurun box? (all-reduce
and a grouped send/recv, the two collectives the MPIAIJ path uses). Launch:
  python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 tools/rccl_shared_probe.py
"""
import os

import torch
import torch.distributed as dist

rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
dist.init_process_group("nccl", device_id=dev)
t = torch.full((4,), float(rank + 1), device=dev)
dist.all_reduce(t)
torch.cuda.synchronize()
send = torch.full((8,), float(rank), device=dev)
recv = torch.empty(8, device=dev)
peer = (rank + 1) % world
ops = [dist.P2POp(dist.isend, send, peer), dist.P2POp(dist.irecv, recv, (rank - 1) % world)]
for w in dist.batch_isend_irecv(ops):
    w.wait()
torch.cuda.synchronize()
print(f"rank {rank}: all_reduce {t[0].item()} recv {recv[0].item()}", flush=True)
dist.destroy_process_group()
