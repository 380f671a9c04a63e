#!/usr/bin/env python3
"""A/B of the STREAM phase-1 forms on PETSc's CSR (row patterns and column
codes off) in ONE process, interleaved per round: the predicated form (the
default) and the buffer-load form (AIJHIP_STREAM_BUF=1: range-checked
buffer loads, no branches, trash-slot stores). Bitwise equality checked.

    python tools/ab_buf.py [--grid 300] [--rounds 7] [--launches 30] [--matrix poisson|fem_hex|skewed]
"""
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", type=int, default=300)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--launches", type=int, default=30)
    ap.add_argument("--matrix", default="poisson", choices=["poisson", "fem_hex", "skewed"])
    args = ap.parse_args()
    pkg = importlib.import_module("petsc-openacc_amd")
    if args.matrix == "poisson":
        ai, aj, aa = pkg.poisson_csr(args.grid)
    elif args.matrix == "fem_hex":
        ai, aj, aa = pkg.fem_hex_csr()
    else:
        ai, aj, aa = pkg.skewed_csr()
    m = len(ai) - 1
    A = pkg.SeqAIJHIP(ai, aj, aa, ncols=m, kernel="stream")
    for o in ("row_patterns", "column_codes", "gather_sort"):
        A.set_option(o, 0)
    info = A.info()
    nbytes = info["mult_layout_bytes"]
    s = torch.cuda.current_stream()
    x = torch.from_numpy(pkg.splitmix_uniform(m, 42)).cuda()
    ys = {v: torch.empty_like(x) for v in ("pred", "buf")}
    res = {v: [] for v in ys}
    for r in range(args.rounds + 1):
        for v in ("pred", "buf") if r % 2 == 0 else ("buf", "pred"):
            os.environ["AIJHIP_STREAM_BUF"] = "1" if v == "buf" else "0"
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                  for _ in range(args.launches)]
            for a, b in ev:
                a.record(s)
                A.mult(x, ys[v], s)
                b.record(s)
            torch.cuda.synchronize()
            if r > 0:
                res[v] += [a.elapsed_time(b) * 1e3 for a, b in ev]
    out = {"matrix": args.matrix, "grid": args.grid, "rows": m, "nnz": len(aj), "bytes": nbytes,
           "blocks": info["n_blocks"], "geometry": info["stream_geometry"],
           "bitwise_equal": bool(torch.equal(ys["pred"], ys["buf"]))}
    for v, us in res.items():
        us = np.array(us)
        out[v] = {"us_median": round(float(np.median(us)), 2), "us_min": round(float(us.min()), 2),
                  "frac_median": round(nbytes / (np.median(us) * 1e-6) / 8e12, 4)}
    print(json.dumps(out), flush=True)
    A.destroy()


if __name__ == "__main__":
    main()
