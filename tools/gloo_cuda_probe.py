"""Probe: which torch.distributed gloo collectives accept GPU tensors here
(used to decide how the multi-rank GPU tests run on a one-GPU box)."""
import os
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def work(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda:0")
    res = {}
    t = torch.full((4,), float(rank + 1), device=dev)
    for name, fn in [
        ("all_reduce", lambda: dist.all_reduce(t)),
        ("all_gather_into_tensor", lambda: dist.all_gather_into_tensor(torch.empty(8, device=dev), t)),
        ("batch_isend_irecv", lambda: [w.wait() for w in dist.batch_isend_irecv(
            [dist.P2POp(dist.isend, t, 1 - rank), dist.P2POp(dist.irecv, torch.empty(4, device=dev), 1 - rank)])]),
    ]:
        try:
            fn()
            torch.cuda.synchronize()
            res[name] = "ok"
        except Exception as e:  # noqa: BLE001
            res[name] = f"{type(e).__name__}: {str(e)[:120]}"
    print(rank, res, flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    mp.spawn(work, args=(2, 29755), nprocs=2)
    sys.exit(0)
