#!/usr/bin/env python3
"""The parts of one rank's work at N = 8 strong scaling (300^3 over 8 GPUs:
37-38 z-planes, 3.33-3.42 M rows per rank), measured on one GPU, for the
N = 8 projection (profiles/r03/n8_projection/):

  - the diagonal block's SpMV (STREAM, HIP events, median of 100 launches);
  - the off-diagonal block (2 boundary planes, one entry per row,
    compressed rows) as MatMultAdd;
  - the halo pack of two 300^2 planes;
  - CG+Jacobi per iteration on the slab-sized operator (single-GPU solver,
    fused SpMV + p.w: what a rank computes per iteration besides the two
    all-reduces);
  - the same rank's slab at N = 1 through aijhip_mpiaij over RCCL with no
    ghosts (world size 1), against its A_d alone: the zero-ghost overhead.

    python tools/slab_probe.py [--planes 37] [--grid 300]
"""
from __future__ import annotations

import argparse
import importlib
import json
import os
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def med_us(fn, stream, reps=100, warm=5):
    for _ in range(warm):
        fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record(stream)
        fn()
        b.record(stream)
    torch.cuda.synchronize()
    us = np.array([a.elapsed_time(b) for a, b in ev]) * 1e3
    return float(np.median(us)), float(np.mean(us))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", type=int, default=300)
    ap.add_argument("--planes", type=int, default=37)
    args = ap.parse_args()
    pkg = importlib.import_module("petsc-openacc_amd")
    K = importlib.import_module("petsc-openacc_amd.ksp")
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream()
    G, pz = args.grid, args.planes
    z0 = G // 2 - pz // 2  # an interior slab: ghosts on both sides
    ai, aj, aa = pkg.poisson_csr(G, G, G, z0, z0 + pz)
    lo, hi = z0 * G * G, (z0 + pz) * G * G
    (dai, daj, daa), (oai, oaj, oaa), garray = pkg.split_rows(ai, aj, aa, lo, hi)
    m = hi - lo
    out = {"grid": G, "planes": pz, "rows": m, "nnz_d": int(len(daj)), "nnz_o": int(len(oaj)),
           "ghosts": int(len(garray))}
    A_d = pkg.SeqAIJHIP(dai, daj, daa, ncols=m)
    A_o = pkg.SeqAIJHIP(oai, oaj, oaa, ncols=len(garray))
    x = torch.from_numpy(pkg.splitmix_uniform(m, 42)).to(dev)
    y = torch.empty_like(x)
    g = torch.from_numpy(pkg.splitmix_uniform(len(garray), 7)).to(dev)
    med, mean = med_us(lambda: A_d.mult(x, y, s), s)
    nb = pkg.algorithmic_bytes(m, m, len(daj))
    out["A_d_us"] = {"median": round(med, 2), "mean": round(mean, 2), "GBs": round(nb / (med * 1e-6) / 1e9, 1)}
    med, mean = med_us(lambda: A_o.mult_add(g, y, y, s), s)
    out["A_o_multadd_us"] = {"median": round(med, 2), "mean": round(mean, 2), "info": {k: v for k, v in A_o.info().items() if k in ("m", "nz", "kernel", "n_blocks")}}
    idx = torch.from_numpy(np.concatenate([np.arange(G * G), np.arange(m - G * G, m)])).to(dev)
    buf = torch.empty(2 * G * G, dtype=torch.float64, device=dev)
    med, mean = med_us(lambda: torch.index_select(x, 0, idx, out=buf), s)
    out["pack_2_planes_us"] = {"median": round(med, 2), "note": "torch index_select as a stand-in for k_pack"}
    # CG+Jacobi per iteration on a slab-sized operator (no coupling: the
    # single-GPU solver's kernels, which the distributed CG shares)
    rhs = torch.from_numpy(pkg.splitmix_uniform(m, 3)).to(dev)
    xs = torch.zeros_like(rhs)
    with K.KSPCG(A_d, rtol=0.0, atol=0.0, max_it=5) as ksp:
        ksp.solve(rhs, xs)
        ksp.set_tolerances(0.0, 0.0, 1e5, 200)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        ksp.solve(rhs, xs)
        e1.record(s)
        torch.cuda.synchronize()
        out["cg_jacobi_us_per_iter"] = round(e0.elapsed_time(e1) * 1e3 / max(ksp.its, 1), 2)
    # zero-ghost overhead over RCCL at world size 1
    if os.environ.get("MASTER_ADDR"):
        import torch.distributed as dist
        C = importlib.import_module("petsc-openacc_amd.comm")
        dist.init_process_group("nccl", device_id=dev)
        comm = C.Comm.rccl(device=0, timeout_s=60)
        op = C.NativeMPIAIJ(comm, A_d, None, "p2p", [], [])
        med_op, _ = med_us(lambda: op.mult(x, y, s), s)
        med_d, _ = med_us(lambda: A_d.mult(x, y, s), s)
        med_op2, _ = med_us(lambda: op.mult(x, y, s), s)
        out["rccl_world1_no_ghosts"] = {"mpiaij_us": round(med_op, 2), "A_d_us": round(med_d, 2),
                                        "mpiaij_again_us": round(med_op2, 2),
                                        "overhead_us": round(min(med_op, med_op2) - med_d, 2)}
        op.destroy()
        comm.destroy()
        dist.destroy_process_group()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
