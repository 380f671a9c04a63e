#!/usr/bin/env python3
"""Calibrates STREAM phase 2 (one lane per row vs L lanes per row) against
the row length: banded synthetic CSR with every row holding `len` entries in
3-column runs inside a +-2100-column band (the skewed stand-in's shape), about
120 M entries each; exact=1 (sequential rows) vs exact=0 (multi-lane when the
block's mean row exceeds kSplitMinMean) for the default and 1024-lane
geometries, interleaved A/B in one process (tools/tune.py's method)."""
from __future__ import annotations

import importlib
import json
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
from tools.tune import time_launches  # noqa: E402


def banded(m, length, seed=7):
    rng = np.random.default_rng(seed)
    runs = length // 3
    node = np.arange(m) // 3
    nn = m // 3
    starts = node[:, None] + rng.integers(-700, 701, size=(m, runs))
    starts = np.clip(starts, 0, nn - 1)
    starts.sort(axis=1)
    cols = (3 * starts[:, :, None] + np.arange(3)).reshape(m, -1)
    aj = cols.astype(np.int32).ravel()
    ai = (np.arange(m + 1, dtype=np.int64) * cols.shape[1]).astype(np.int32)
    aa = rng.uniform(-1, 1, size=aj.size)
    return ai, aj, aa


def main():
    pkg = importlib.import_module("petsc-openacc_amd")
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream()
    for length in (12, 24, 48, 96, 192, 384):
        m = (120_000_000 // length) // 3 * 3
        ai, aj, aa = banded(m, length)
        A = pkg.SeqAIJHIP(ai, aj, aa)
        x = torch.from_numpy(pkg.splitmix_uniform(m, 42)).to(dev)
        y = torch.empty(m, dtype=torch.float64, device=dev)
        nbytes = pkg.algorithmic_bytes(m, m, len(aj))
        res = {}
        for rnd in range(3):
            for geom in (1, 6, 7):
                for exact in (0, 1):
                    A.set_option("geometry", geom)
                    A.set_option("exact", exact)
                    fn = lambda: A.mult(x, y, s)  # noqa: E731
                    time_launches(fn, 3, s)
                    res.setdefault((geom, exact), []).append(float(np.median(time_launches(fn, 15, s))))
        for (geom, exact), v in sorted(res.items(), key=lambda kv: np.median(kv[1])):
            us = float(np.median(v))
            print(json.dumps({"row_len": length, "geometry": geom, "exact": exact, "us": round(us, 1),
                              "GBs": round(nbytes / us / 1e3, 1)}), flush=True)
        A.destroy()


if __name__ == "__main__":
    main()
