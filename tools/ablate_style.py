#!/usr/bin/env python3
"""DIAGNOSTIC: load-style study of the STREAM kernel (tools/ablate.hip
k_style), interleaved in one process with the product's MatMult."""
from __future__ import annotations

import ctypes
import importlib
import json
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

CONFIGS = [(1024, 5, 0), (1024, 5, 1), (1024, 5, 2), (1024, 4, 0), (1024, 4, 1), (1024, 4, 2),
           (512, 4, 0), (512, 4, 1), (512, 4, 2), (512, 5, 1), (256, 4, 0), (256, 4, 1), (256, 4, 2)]


def main(grid=300, rounds=5, launches=20):
    pkg = importlib.import_module("petsc-openacc_amd")
    L = ctypes.CDLL(str(ROOT / "tools" / "libablate.so"))
    L.ablate_style.argtypes = [ctypes.c_int] * 4 + [ctypes.c_void_p] * 7
    dev = torch.device("cuda:0")
    ai, aj, aa = pkg.poisson_csr(grid)
    m, nz = len(ai) - 1, len(aj)
    A = pkg.SeqAIJHIP(ai, aj, aa)
    p_ai, p_aj, p_aa = A.device_csr()
    x = torch.from_numpy(pkg.splitmix_uniform(m, 42)).to(dev)
    y = torch.empty(m, dtype=torch.float64, device=dev)
    s = torch.cuda.current_stream()
    tables = {}
    for R in (1024, 512, 256):
        row0 = np.arange(0, m, R)
        nrows = np.minimum(R, m - row0)
        k0 = ai[row0]
        nk = ai[row0 + nrows] - k0
        tables[R] = (torch.from_numpy(np.stack([row0, nrows, k0, nk], 1).astype(np.int32).copy()).to(dev), len(row0))
    ref = None

    def mk(tt, it, st):
        blk, nb = tables[tt]

        def f():
            assert L.ablate_style(tt, it, st, nb, blk.data_ptr(), p_ai, p_aj, p_aa, x.data_ptr(), y.data_ptr(),
                                  s.cuda_stream) == 0
        return f

    variants = [(f"T{tt}_IT{it}_style{st}", mk(tt, it, st)) for tt, it, st in CONFIGS]
    variants.append(("product_mult", lambda: A.mult(x, y, s)))
    res = {n: [] for n, _ in variants}
    for rnd in range(rounds):
        for name, fn in variants:
            for _ in range(3):
                fn()
            if rnd == 0:
                torch.cuda.synchronize()
                yy = y.cpu().numpy()
                if ref is None:
                    ref = yy
                assert np.array_equal(yy.view(np.uint64), ref.view(np.uint64)), name
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(launches)]
            for a, b in ev:
                a.record(s)
                fn()
                b.record(s)
            torch.cuda.synchronize()
            res[name].append(float(np.median([a.elapsed_time(b) * 1e3 for a, b in ev])))
    nb = pkg.algorithmic_bytes(m, m, nz)
    for name, v in sorted(res.items(), key=lambda kv: np.median(kv[1])):
        us = float(np.median(v))
        print(json.dumps({"variant": name, "us": round(us, 1), "GBs": round(nb / us / 1e3, 1)}), flush=True)


if __name__ == "__main__":
    main()
