#!/usr/bin/env python3
"""The distributed CG iteration replayed from a captured HIP graph vs launched
directly, at one rank over a real RCCL communicator.

One rank holds the N = 8 strong-scaling slab of the 300^3 operand (38 of 300
z-planes, 3.42 M rows); its two boundary planes are made ghosts of itself
(the self-halo of tests/test_rccl_selfhalo_gpu.py: A_o holds the entries in
those columns, the p2p plan sends and receives them through ncclSend /
ncclRecv to itself), so every iteration pays an N = 8 rank's exchange and its
host enqueue. CG + Jacobi, rtol = 0 (a fixed iteration count), the same
solve with graph=False and graph=True in alternating rounds; the solutions
must be bit-identical. One JSON line per round on stdout.

    python tools/graph_probe.py [--grid 300] [--planes 38] [--its 400] [--rounds 3]
"""
import argparse
import importlib
import json
import os
import sys
import time
from pathlib import Path

if int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0) < 8:
    os.environ["GPU_MAX_HW_QUEUES"] = "8"
ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", type=int, default=300)
    ap.add_argument("--planes", type=int, default=38)
    ap.add_argument("--its", type=int, default=400)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--ghosts", type=int, default=1, help="1: the boundary planes as self-ghosts (RCCL in the batch)")
    ap.add_argument("--overlap", type=int, default=-1, help="exchange placement: -1 automatic, 0 serial, 1 side stream")
    a = ap.parse_args()
    import numpy as np
    import torch
    import torch.distributed as dist
    from test_rccl_selfhalo_gpu import split_self
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29531")
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=0, world_size=1)
    pkg = importlib.import_module("petsc-openacc_amd")
    C = importlib.import_module("petsc-openacc_amd.comm")
    dev = torch.device("cuda:0")
    comm = C.Comm.rccl(device=0, timeout_s=120)
    G, nz = a.grid, a.planes
    ai, aj, aa = pkg.poisson_csr(G, G, nz)
    m = G * G * nz
    if a.ghosts:
        ghosts = np.concatenate([np.arange(0, G * G), np.arange(m - G * G, m)])
        (dai, daj, daa), (oai, oaj, oaa) = split_self(ai, aj, aa, ghosts)
        Ad = pkg.SeqAIJHIP(dai, daj, daa, ncols=m)
        Ao = pkg.SeqAIJHIP(oai, oaj, oaa, ncols=len(ghosts))
        op = C.NativeMPIAIJ(comm, Ad, Ao, "p2p", [(0, ghosts)], [(0, 0, len(ghosts))], 0)
    else:  # no exchange: the batch is kernels only
        ghosts = np.zeros(0, np.int64)
        Ad, Ao = pkg.SeqAIJHIP(ai, aj, aa, ncols=m), None
        op = C.NativeMPIAIJ(comm, Ad, None, "p2p", [], [], 0)
    if a.overlap >= 0:
        op.set_overlap(bool(a.overlap))
    rhs, _ = pkg.poisson_vectors(G, G, nz)
    b = torch.from_numpy(rhs).to(dev)
    sols = {}
    for rnd in range(a.rounds):
        for graph in (False, True):
            x = torch.zeros_like(b)
            with C.KSPCGMPINative(op, rtol=0.0, atol=0.0, max_it=a.its, pc="jacobi", graph=graph) as k:
                print(f"round {rnd} graph {graph}: warm-up solve", file=sys.stderr, flush=True)
                k.solve(b, x)  # warm-up (and the capture)
                torch.cuda.synchronize()
                print(f"round {rnd} graph {graph}: timed solve", file=sys.stderr, flush=True)
                t0 = time.perf_counter()
                k.solve(b, x)
                torch.cuda.synchronize()
                dt = time.perf_counter() - t0
                rec = {"round": rnd, "graph": graph, "its": k.its, "us_per_iter": round(dt / k.its * 1e6, 2),
                       "batches": k.graph_batches, "host_syncs": k.host_syncs, "rows": m,
                       "ghosts": int(len(ghosts)), "overlap": op.overlap()}
            sols[graph] = x.cpu().numpy()
            print(json.dumps(rec), flush=True)
    same = bool(np.array_equal(sols[False].view(np.uint64), sols[True].view(np.uint64)))
    print(json.dumps({"bitwise_equal": same}), flush=True)
    op.destroy()
    Ad.destroy()
    if Ao is not None:
        Ao.destroy()
    comm.destroy()
    dist.destroy_process_group()
    if not same:
        sys.exit(1)


if __name__ == "__main__":
    main()
