#!/usr/bin/env python3
"""Interleaved A/B of STREAM option sets on one operand: every variant built
first, then rounds of launches of each in turn (HIP events per launch), y
checked bit for bit against the first variant. One JSON line per variant.

    python3 tools/ab_opts.py [--case poisson|skewed|fem_hex] [--grid 300]
        [--variant '{"row_patterns": 0, "column_codes": 0}' ...]
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
    ap.add_argument("--case", default="poisson", choices=["poisson", "skewed", "skewed_nohub", "fem_hex"])
    ap.add_argument("--grid", type=int, default=300)
    ap.add_argument("--rounds", type=int, default=30)
    ap.add_argument("--per", type=int, default=10)
    ap.add_argument("--variant", action="append", default=[], help="JSON dict of set_option NAME: VALUE")
    ap.add_argument("--dummy-streams", type=int, default=0,
                    help="HIP streams created (and kept) before the matrices: moves the side stream's hardware queue")
    args = ap.parse_args()
    pkg = importlib.import_module("petsc-openacc_amd")
    dev = torch.device("cuda:0")
    dummies = [torch.cuda.Stream(device=dev) for _ in range(args.dummy_streams)]  # noqa: F841 (kept alive)
    if args.case == "poisson":
        ai, aj, aa = pkg.poisson_csr(args.grid)
    elif args.case.startswith("skewed"):
        ai, aj, aa = pkg.skewed_csr()
        if args.case == "skewed_nohub":  # the hub rows emptied (tools/prof_case.py)
            import numpy as np
            ln = np.diff(ai)
            keep = np.repeat(ln <= 1000, ln)
            ai = np.concatenate([[0], np.cumsum(np.where(ln <= 1000, ln, 0))]).astype(np.int32)
            aj, aa = aj[keep], aa[keep]
    else:
        ai, aj, aa = pkg.fem_hex_csr()
    m = len(ai) - 1
    x = torch.from_numpy(pkg.splitmix_uniform(m, 42)).to(dev)
    variants = [json.loads(v) for v in args.variant] or [{}]
    mats, ys = [], []
    import os
    for opts in variants:
        env = opts.get("_env", {})  # planner environment knobs, e.g. AIJHIP_ISOLATE_ROW_NNZ, for this matrix only
        saved = {k: os.environ.get(k) for k in env}
        os.environ.update({k: str(v) for k, v in env.items()})
        A = pkg.SeqAIJHIP(ai, aj, aa, ncols=m, kernel="stream")
        for k, v in opts.items():
            if k != "_env":
                A.set_option(k, int(v))
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        mats.append(A)
        ys.append(torch.empty(A.m, dtype=torch.float64, device=dev))
        print(f"ab_opts: {opts}: {A.info()}", file=sys.stderr, flush=True)
    for A, y in zip(mats, ys):
        A.mult(x, y)
    torch.cuda.synchronize()
    equal = [bool(torch.equal(y.view(torch.int64), ys[0].view(torch.int64))) for y in ys]
    times = [[] for _ in mats]
    s = torch.cuda.current_stream()
    for r in range(args.rounds):
        for i, (A, y) in enumerate(zip(mats, ys)):
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.per)]
            for a, b in ev:
                a.record(s)
                A.mult(x, y)
                b.record(s)
            torch.cuda.synchronize()
            times[i].extend(a.elapsed_time(b) * 1e3 for a, b in ev)
        if r % 10 == 0:
            print(f"ab_opts: round {r}", file=sys.stderr, flush=True)
    nbytes = pkg.algorithmic_bytes(m, m, len(aj))
    for opts, A, t, eq in zip(variants, mats, times, equal):
        med = statistics.median(t)
        lb = A.info()["mult_layout_bytes"]
        print(json.dumps({"case": args.case, "options": opts, "us_median": round(med, 2),
                          "us_mean": round(statistics.mean(t), 2), "us_min": round(min(t), 2),
                          "layout_frac_8TBs": round(lb / med / 1e3 / 8000, 4),
                          "csr_frac_8TBs": round(nbytes / med / 1e3 / 8000, 4), "bitwise_equal": eq}), flush=True)
    for A in mats:
        A.destroy()


if __name__ == "__main__":
    main()
