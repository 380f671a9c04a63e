#!/usr/bin/env python3
"""One workload per process, for `rocprofv3 --kernel-trace --stats -- python3
tools/prof_case.py CASE`: the per-kernel breakdown of a case the bench line
only reports as a total.

    gamg      CG + GAMG solve at --grid^3 (reference options), after set-up
    jacobi    --its CG + Jacobi iterations at --grid^3
    skewed    --its SpMVs of the Flan_1565 stand-in (default kernel)
"""
from __future__ import annotations

import argparse
import importlib
import sys
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("case", choices=["gamg", "jacobi", "skewed", "skewed_nohub", "poisson", "fem_hex"])
    ap.add_argument("--exact", type=int, default=0)
    ap.add_argument("--grid", type=int, default=300)
    ap.add_argument("--its", type=int, default=50)
    ap.add_argument("--solves", type=int, default=1, help="solves timed after the set-up (gamg / jacobi)")
    ap.add_argument("--kernel", default="auto")
    ap.add_argument("--opt", action="append", default=[], help="set_option NAME=VALUE (repeatable)")
    ap.add_argument("--gamg-opt", action="append", default=[],
                    help="GAMG parameter NAME=VALUE (aijhip_gamg_params_t field, repeatable), e.g. coarsen=1")
    args = ap.parse_args()
    pkg = importlib.import_module("petsc-openacc_amd")
    K = importlib.import_module("petsc-openacc_amd.ksp")
    dev = torch.device("cuda:0")
    if args.case in ("skewed", "skewed_nohub", "poisson", "fem_hex"):
        if args.case == "poisson":
            ai, aj, aa = pkg.poisson_csr(args.grid)
        elif args.case == "fem_hex":
            ai, aj, aa = pkg.fem_hex_csr()
        else:
            ai, aj, aa = pkg.skewed_csr()
        if args.case == "skewed_nohub":  # hub rows emptied (tools/tune.py)
            import numpy as np
            ln = np.diff(ai)
            keep = np.repeat(ln <= 1000, ln)
            ai = np.concatenate([[0], np.cumsum(np.where(ln <= 1000, ln, 0))]).astype(np.int32)
            aj, aa = aj[keep], aa[keep]
        A = pkg.SeqAIJHIP(ai, aj, aa, kernel=args.kernel, exact=args.exact)
        for o in args.opt:
            k, v = o.split("=")
            A.set_option(k, int(v))
        x = torch.from_numpy(pkg.splitmix_uniform(A.n, 42)).to(dev)
        y = torch.empty(A.m, dtype=torch.float64, device=dev)
        for _ in range(args.its):
            A.mult(x, y)
        torch.cuda.synchronize()
        print(args.case, A.info())
        return
    G = args.grid
    ai, aj, aa = pkg.poisson_csr(G)
    A = pkg.SeqAIJHIP(ai, aj, aa)
    rhs, _ = pkg.poisson_vectors(G)
    b = torch.from_numpy(rhs).to(dev)
    x = torch.zeros_like(b)
    gp = {k: (float(v) if "." in v else int(v)) for k, v in (o.split("=") for o in args.gamg_opt)} or None
    if args.case == "gamg":
        # a first set-up in this process pays one-time costs (code objects of
        # the set-up kernels loaded on first launch); time a second one too
        warm = K.KSPCG(A, rtol=1e-14, atol=1e-12, pc="gamg", gamg=gp)
        t0 = time.perf_counter()
        warm.set_up()
        torch.cuda.synchronize()
        print(f"gamg: first set-up in process {time.perf_counter() - t0:.3f} s")
        warm.destroy()
        ksp = K.KSPCG(A, rtol=1e-14, atol=1e-12, pc="gamg", gamg=gp)
    else:
        ksp = K.KSPCG(A, rtol=0.0, atol=0.0, max_it=args.its)
    t0 = time.perf_counter()
    ksp.set_up()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    ksp.solve(b, x)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"{args.case}: set-up {t1 - t0:.3f} s, solve {t2 - t1:.4f} s, its {ksp.its}, reason {ksp.reason}, "
          f"x bits {int(x.view(torch.int64).sum()) & 0xffffffffffff:012x}")
    for _ in range(args.solves - 1):  # the same solve again from x = 0
        x.zero_()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        ksp.solve(b, x)
        torch.cuda.synchronize()
        print(f"{args.case}: solve again {time.perf_counter() - t1:.4f} s")
    ksp.destroy()
    A.destroy()


if __name__ == "__main__":
    main()
