#!/usr/bin/env python3
"""A/B of AIJHIP_OPT_PIPELINE (two row blocks in flight per workgroup) on the
headline operand: 300^3 Poisson in the CSR layout (row patterns and column
codes off — the kernel `value` times), interleaved rounds of launches timed
with HIP events, every variant's y checked bit for bit against the default
one-block-per-workgroup kernel. One JSON line per variant to stdout.

    python3 tools/ab_pipe.py [--grid 300] [--rounds 30] [--per 10]
"""
from __future__ import annotations

import argparse
import importlib
import json
import statistics
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", type=int, default=300)
    ap.add_argument("--rounds", type=int, default=30)
    ap.add_argument("--per", type=int, default=10)
    ap.add_argument("--variants", default="0:6,1:6,2:6,3:6,2:8,4:8,5:8",
                    help="pipe:geometry pairs (pipe 0 = the default kernel)")
    args = ap.parse_args()
    pkg = importlib.import_module("petsc-openacc_amd")
    dev = torch.device("cuda:0")
    ai, aj, aa = pkg.poisson_csr(args.grid)
    x = torch.from_numpy(pkg.splitmix_uniform(len(ai) - 1, 42)).to(dev)
    variants = [tuple(int(v) for v in s.split(":")) for s in args.variants.split(",")]
    mats, ys = {}, {}
    for pipe, geom in variants:
        A = pkg.SeqAIJHIP(ai, aj, aa)
        A.set_option("row_patterns", 0)
        A.set_option("column_codes", 0)
        if geom != 6:
            A.set_option("geometry", geom)
        if pipe:
            A.set_option("pipeline", pipe)
        mats[(pipe, geom)] = A
        ys[(pipe, geom)] = torch.empty(A.m, dtype=torch.float64, device=dev)
        print(f"ab_pipe: variant pipe {pipe} geometry {geom}: {A.info()}", file=sys.stderr, flush=True)
    ref = (0, 6)
    for k, A in mats.items():  # warm-up + bitwise check
        A.mult(x, ys[k])
    torch.cuda.synchronize()
    yb = ys[ref].view(torch.int64)
    equal = {k: bool(torch.equal(ys[k].view(torch.int64), yb)) for k in mats}
    times = {k: [] for k in mats}
    s = torch.cuda.current_stream()
    for r in range(args.rounds):
        for k, A in mats.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(args.per):
                A.mult(x, ys[k])
            e1.record(s)
            e1.synchronize()
            times[k].append(e0.elapsed_time(e1) * 1e3 / args.per)
        if r % 10 == 0:
            print(f"ab_pipe: round {r}", file=sys.stderr, flush=True)
    nbytes = 12 * len(aj) + 4 * len(ai) + 16 * (len(ai) - 1)
    for k in mats:
        med = statistics.median(times[k])
        print(json.dumps({"pipe": k[0], "geometry": k[1], "median_us": round(med, 2),
                          "min_us": round(min(times[k]), 2), "GBs": round(nbytes / med / 1e3, 1),
                          "frac_8TBs": round(nbytes / med / 1e3 / 8000, 4), "bitwise_equal": equal[k]}), flush=True)
    for A in mats.values():
        A.destroy()


if __name__ == "__main__":
    main()
