#!/usr/bin/env python3
"""Cache-state probe for the 300^3 SpMV: the same launch timed (HIP events
around the SpMV only) back to back, after a 1 GiB write that evicts the
Infinity Cache, and after the eviction plus a fresh write of x (the state x
is in inside CG, where p = z + b p was just written)."""
from __future__ import annotations

import importlib
import json
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    pkg = importlib.import_module("petsc-openacc_amd")
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream()
    ai, aj, aa = pkg.poisson_csr(300)
    A = pkg.SeqAIJHIP(ai, aj, aa)
    m = len(ai) - 1
    x = torch.from_numpy(pkg.splitmix_uniform(m, 42)).to(dev)
    x2 = x.clone()
    y = torch.empty_like(x)
    junk = torch.empty(1 << 27, dtype=torch.float64, device=dev)  # 1 GiB

    def run(pre, n=30):
        ts = []
        for _ in range(n):
            pre()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            A.mult(x, y, s)
            b.record(s)
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b) * 1e3)
        return float(np.median(ts))

    cases = {
        "back_to_back": lambda: None,
        "after_1GiB_write": lambda: junk.fill_(1.0),
        "after_1GiB_write_then_x_rewritten": lambda: (junk.fill_(1.0), x.copy_(x2)),
        "x_rewritten": lambda: x.copy_(x2),
    }
    for rnd in range(2):
        for k, f in cases.items():
            print(json.dumps({"case": k, "round": rnd, "us_median": round(run(f), 1)}), flush=True)
    A.destroy()


if __name__ == "__main__":
    main()
