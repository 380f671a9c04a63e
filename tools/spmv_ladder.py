#!/usr/bin/env python3
"""Drive tools/spmv_ladder.hip on the 300^3 Poisson operand (measurement
tool, not product code): the product's CSR MatMult beside rungs 0-3 of the
ladder, every variant timed by HIP events (median of --reps launches) over
--rounds interleaved rounds, one JSON line per (variant, round).

    python tools/spmv_ladder.py [--grid 300] [--reps 50] [--rounds 3]
"""
from __future__ import annotations

import argparse
import ctypes
import importlib
import json
import subprocess
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
SO = ROOT / "tools" / "libspmv_ladder.so"


def build():
    src = ROOT / "tools" / "spmv_ladder.hip"
    if not SO.exists() or SO.stat().st_mtime < src.stat().st_mtime:
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-ffp-contract=off", "-std=c++17",
                        "-shared", "-fPIC", "-o", str(SO), str(src)], check=True)
    return ctypes.CDLL(str(SO))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", type=int, default=300)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    L = build()
    P = ctypes.c_void_p
    L.ladder_launch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int32, ctypes.c_int64, P, P, P, P,
                                P, P]
    L.ladder_flat.argtypes = [ctypes.c_int, ctypes.c_int64, P, P, ctypes.c_int64, P]
    pkg = importlib.import_module("petsc-openacc_amd")
    dev = torch.device("cuda:0")
    ai, aj, aa = pkg.poisson_csr(args.grid)
    m, nnz = len(ai) - 1, len(aj)
    nbytes = pkg.algorithmic_bytes(m, m, nnz)
    A = pkg.SeqAIJHIP(ai, aj, aa, row_patterns=0, column_codes=0)
    d_ai, d_aj, d_aa = A.device_csr()
    x = torch.from_numpy(pkg.splitmix_uniform(m, 42)).to(dev)
    y = torch.empty(m, dtype=torch.float64, device=dev)
    flat = torch.rand((nbytes - 8 * m) // 8 // 2 * 2, dtype=torch.float64, device=dev)
    s = torch.cuda.current_stream()
    sh = s.cuda_stream

    def run(name):
        if name == "product":
            A.mult(x, y, s)
        elif name.startswith("flat"):
            rc = L.ladder_flat(int(name.endswith("nt")), flat.numel(), flat.data_ptr(), y.data_ptr(), m, sh)
            assert rc == 0
        else:  # rungR[_256][_nt], multi[_nt]
            rung = 9 if name.startswith("multi") else int(name[4])
            nt, rows = int(name.endswith("nt")), 256 if "_256" in name else 512
            rc = L.ladder_launch(rung, nt, rows, m, nnz, d_ai, d_aj, d_aa, x.data_ptr(), y.data_ptr(), sh)
            assert rc == 0, rc

    variants = ["product", "flat", "flat_nt", "multi", "multi_nt", "rung1", "rung1_nt", "rung1_256", "rung1_256_nt",
                "rung2", "rung2_nt", "rung2_256_nt", "rung3", "rung3_nt", "rung3_256", "rung3_256_nt"]
    ref = torch.empty_like(y)
    A.mult(x, ref, s)
    for chk in ("rung3", "rung3_256_nt"):
        run(chk)
        torch.cuda.synchronize()
        print(json.dumps({"check": f"{chk} equals the product bit for bit", "equal": bool(torch.equal(ref, y))}),
              flush=True)
    print(json.dumps({"m": m, "nnz": nnz, "bytes": nbytes, "flat_bytes": flat.numel() * 8 + 8 * m}), flush=True)
    for rnd in range(args.rounds):
        for v in variants:
            for _ in range(5):
                run(v)
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                  for _ in range(args.reps)]
            for a, b in ev:
                a.record(s)
                run(v)
                b.record(s)
            torch.cuda.synchronize()
            us = np.array([a.elapsed_time(b) for a, b in ev]) * 1e3
            med = float(np.median(us))
            print(json.dumps({"round": rnd, "variant": v, "us_median": round(med, 2),
                              "us_mean": round(float(us.mean()), 2), "TBs": round(nbytes / med / 1e6, 3),
                              "frac": round(nbytes / med / 1e6 / 8.0, 4)}), flush=True)
    A.destroy()


if __name__ == "__main__":
    main()
