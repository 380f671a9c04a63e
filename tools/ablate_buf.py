#!/usr/bin/env python3
"""DIAGNOSTIC: block-shape / load-form study of the STREAM SpMV
(tools/ablate_buf.hip), interleaved in one process with the product's
MatMult on the same device arrays; every variant is checked bit for bit
against the product's y first.

    hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -shared -fPIC tools/ablate_buf.hip -o tools/libablate_buf.so
    python tools/ablate_buf.py [--grid 300]
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


def block_table(ai, rows_per_block, slots):
    m = len(ai) - 1
    row0 = np.arange(0, m, rows_per_block, dtype=np.int64)
    nrows = np.minimum(rows_per_block, m - row0)
    k0 = ai[row0].astype(np.int64)
    nk = ai[row0 + nrows].astype(np.int64) - k0
    assert int((nk + (k0 & 1)).max()) <= slots, "block exceeds its entry slots"
    return np.stack([row0, nrows, k0, nk], 1).astype(np.int32)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", type=int, default=300)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--launches", type=int, default=20)
    args = ap.parse_args()
    pkg = importlib.import_module("petsc-openacc_amd")
    L = ctypes.CDLL(str(ROOT / "tools" / "libablate_buf.so"))
    L.ablate_buf.argtypes = [ctypes.c_int] * 6 + [ctypes.c_void_p] * 5 + [ctypes.c_int32] + [ctypes.c_void_p] * 2
    buf = (ctypes.c_int * 400)()
    ncfg = L.ablate_buf_configs(buf, 400)
    configs = [tuple(buf[5 * i:5 * i + 5]) for i in range(ncfg)]
    dev = torch.device("cuda:0")
    ai, aj, aa = pkg.poisson_csr(args.grid)
    m, nz = len(ai) - 1, len(aj)
    maxlen = int(np.diff(ai).max())
    A = pkg.SeqAIJHIP(ai, aj, aa)
    p_ai, p_aj, p_aa = A.device_csr()
    x = torch.from_numpy(pkg.splitmix_uniform(m, 42)).to(dev)
    y = torch.empty(m, dtype=torch.float64, device=dev)
    s = torch.cuda.current_stream()
    A.mult(x, y, s)
    torch.cuda.synchronize()
    ref = y.cpu().numpy().copy()

    def mk(tt, it, rpt, mode, nty):
        slots = 2 * tt * it
        R = min(rpt * tt, (slots - 1) // maxlen)
        tab = torch.from_numpy(block_table(ai, R, slots)).to(dev)
        nb = tab.shape[0]

        def f():
            assert L.ablate_buf(tt, it, rpt, mode, nty, nb, tab.data_ptr(), p_ai, p_aj, p_aa, x.data_ptr(), m,
                                y.data_ptr(), s.cuda_stream) == 0
        return f, R

    variants = []
    for c in configs:
        f, R = mk(*c)
        variants.append((f"T{c[0]}_IT{c[1]}_RPT{c[2]}_R{R}_mode{c[3]}_nty{c[4]}", f))
    variants.append(("product_mult", lambda: A.mult(x, y, s)))
    res = {n: [] for n, _ in variants}
    for rnd in range(args.rounds):
        for name, fn in variants:
            if rnd == 0:
                y.zero_()
            for _ in range(3):
                fn()
            if rnd == 0:
                torch.cuda.synchronize()
                yy = y.cpu().numpy()
                assert np.array_equal(yy.view(np.uint64), ref.view(np.uint64)), name
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                  for _ in range(args.launches)]
            for a, b in ev:
                a.record(s)
                fn()
                b.record(s)
            torch.cuda.synchronize()
            res[name].append(float(np.median([a.elapsed_time(b) * 1e3 for a, b in ev])))
        print(f"round {rnd} done", file=sys.stderr, flush=True)
    nbytes = pkg.algorithmic_bytes(m, m, nz)
    for name, v in sorted(res.items(), key=lambda kv: np.median(kv[1])):
        us = float(np.median(v))
        print(json.dumps({"variant": name, "us": round(us, 1), "us_min_round": round(min(v), 1),
                          "GBs": round(nbytes / us / 1e3, 1)}), flush=True)


if __name__ == "__main__":
    main()
