#!/usr/bin/env python3
"""DIAGNOSTIC: A/B of the non-temporal store hint in the CG vector kernels and
the fused V-cycle smoothers (AIJHIP_VEC_NT read at KSPCreate), interleaved
in one process on the 300^3 operand: CG+Jacobi iterations/s and the CG+GAMG
solve time, each setting timed `--rounds` times alternately."""
from __future__ import annotations

import argparse
import importlib
import json
import os
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", type=int, default=300)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--its", type=int, default=200)
    args = ap.parse_args()
    pkg = importlib.import_module("petsc-openacc_amd")
    K = importlib.import_module("petsc-openacc_amd.ksp")
    dev = torch.device("cuda:0")
    G = args.grid
    ai, aj, aa = pkg.poisson_csr(G)
    A = pkg.SeqAIJHIP(ai, aj, aa)
    rhs, _ = pkg.poisson_vectors(G)
    b = torch.from_numpy(rhs).to(dev)
    x = torch.zeros_like(b)
    solvers = {}
    for nt in (0, 1):
        os.environ["AIJHIP_VEC_NT"] = str(nt)
        jac = K.KSPCG(A, rtol=0.0, atol=0.0, max_it=args.its)
        jac.set_up()
        gam = K.KSPCG(A, rtol=1e-14, atol=1e-12, pc="gamg")
        gam.set_up()
        solvers[nt] = (jac, gam)
    torch.cuda.synchronize()
    res = {f"{kind}_nt{nt}": [] for nt in (0, 1) for kind in ("jacobi_its_per_s", "gamg_solve_s")}
    its = {}
    for rnd in range(args.rounds):
        for nt in (0, 1):
            jac, gam = solvers[nt]
            x.zero_()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            jac.solve(b, x)
            torch.cuda.synchronize()
            res[f"jacobi_its_per_s_nt{nt}"].append(jac.its / (time.perf_counter() - t0))
            x.zero_()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            gam.solve(b, x)
            torch.cuda.synchronize()
            res[f"gamg_solve_s_nt{nt}"].append(time.perf_counter() - t0)
            its[nt] = gam.its
    for k, v in res.items():
        print(json.dumps({"variant": k, "median": round(float(np.median(v)), 4), "all": [round(a, 4) for a in v]}))
    print(json.dumps({"gamg_its": its}))


if __name__ == "__main__":
    main()
