#!/usr/bin/env python3
"""DIAGNOSTIC: time the ablations of tools/ablate.hip on the 300^3 operand,
interleaved in one process (5 rounds x 20 launches, median per variant).

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
NAMES = ["full", "no_gather", "no_reduce", "matrix_only", "flat_matrix", "flat_read_aa", "flat4_matrix", "block4_matrix"]


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
    bytes_full = pkg.algorithmic_bytes(m, m, nz)
    traffic = {0: bytes_full, 1: bytes_full - 8 * m, 2: bytes_full, 3: 12 * nz + 4 * (m + 1) + 8 * m,
               4: 12 * nz, 5: 8 * nz, 6: 12 * nz, 7: 12 * nz + 4 * (m + 1) + 8 * m}

    def launch(mode):
        rc = L.ablate_launch(mode, nblk, blk.data_ptr(), d_ai.data_ptr(), d_aj.data_ptr(), d_aa.data_ptr(),
                             x.data_ptr(), y.data_ptr(), nz, s.cuda_stream)
        assert rc == 0

    res = {k: [] for k in range(8)}
    for _ in range(args.rounds):
        for mode in range(8):
            for _ in range(3):
                launch(mode)
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                  for _ in range(args.launches)]
            for a, b in ev:
                a.record(s)
                launch(mode)
                b.record(s)
            torch.cuda.synchronize()
            res[mode].append(float(np.median([a.elapsed_time(b) * 1e3 for a, b in ev])))
    for mode in range(8):
        us = float(np.median(res[mode]))
        print(json.dumps({"variant": NAMES[mode], "us": round(us, 1), "bytes": traffic[mode],
                          "GBs": round(traffic[mode] / us / 1e3, 1)}), flush=True)


if __name__ == "__main__":
    main()
