#!/usr/bin/env python3
"""DIAGNOSTIC: time the ablations of tools/ablate.hip on the 300^3 operand,
interleaved in one process (rounds x launches, median per variant), next to
the product's own MatMult and the ablation's `full` kernel run on the
product handle's device arrays (separates code effects from allocation).

    hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/ablate.hip -o tools/libablate.so
    python tools/ablate.py [--grid 300]
"""
from __future__ import annotations

import argparse
import ctypes
import importlib
import json
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
NAMES = ["full", "no_gather", "no_reduce", "matrix_only", "flat_matrix", "flat_read_aa", "flat4_matrix",
         "block4_matrix"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", type=int, default=300)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--launches", type=int, default=20)
    args = ap.parse_args()
    pkg = importlib.import_module("petsc-openacc_amd")
    L = ctypes.CDLL(str(ROOT / "tools" / "libablate.so"))
    L.ablate_launch.argtypes = [ctypes.c_int, ctypes.c_int] + [ctypes.c_void_p] * 6 + [ctypes.c_int64, ctypes.c_void_p]
    dev = torch.device("cuda:0")
    ai, aj, aa = pkg.poisson_csr(args.grid)
    m, nz = len(ai) - 1, len(aj)
    row0 = np.arange(0, m, 1024)
    nrows = np.minimum(1024, m - row0)
    k0 = ai[row0]
    nk = ai[row0 + nrows] - k0
    assert nk.max() <= 8192
    blk = torch.from_numpy(np.stack([row0, nrows, k0, nk], axis=1).astype(np.int32).copy()).to(dev)
    d_ai = torch.from_numpy(ai).to(dev)
    d_aj = torch.from_numpy(np.concatenate([aj, np.zeros(2, np.int32)])).to(dev)
    d_aa = torch.from_numpy(np.concatenate([aa, np.zeros(2)])).to(dev)
    x = torch.from_numpy(pkg.splitmix_uniform(m, 42)).to(dev)
    y = torch.empty(max(m, 256 * 8 * 256), dtype=torch.float64, device=dev)
    s = torch.cuda.current_stream()
    nblk = len(row0)
    A = pkg.SeqAIJHIP(ai, aj, aa)
    p_ai, p_aj, p_aa = A.device_csr()
    full = pkg.algorithmic_bytes(m, m, nz)
    traffic = [full, full - 8 * m, full, 12 * nz + 4 * (m + 1) + 8 * m, 12 * nz, 8 * nz, 12 * nz,
               12 * nz + 4 * (m + 1) + 8 * m]

    def abl(mode, pai=None, paj=None, paa=None):
        def f():
            rc = L.ablate_launch(mode, nblk, blk.data_ptr(), pai or d_ai.data_ptr(), paj or d_aj.data_ptr(),
                                 paa or d_aa.data_ptr(), x.data_ptr(), y.data_ptr(), nz, s.cuda_stream)
            assert rc == 0
        return f

    variants = [(NAMES[i], abl(i), traffic[i]) for i in range(8)]
    variants.append(("full_on_product_arrays", abl(0, p_ai, p_aj, p_aa), full))
    variants.append(("product_mult", lambda: A.mult(x, y[:m], s), full))
    res = {v[0]: [] for v in variants}
    for _ in range(args.rounds):
        for name, fn, _ in variants:
            for _ in range(3):
                fn()
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                  for _ in range(args.launches)]
            for a, b in ev:
                a.record(s)
                fn()
                b.record(s)
            torch.cuda.synchronize()
            res[name].append(float(np.median([a.elapsed_time(b) * 1e3 for a, b in ev])))
    for name, _, nb in variants:
        us = float(np.median(res[name]))
        print(json.dumps({"variant": name, "us": round(us, 1), "bytes": nb, "GBs": round(nb / us / 1e3, 1)}),
              flush=True)


if __name__ == "__main__":
    main()
