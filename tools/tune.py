#!/usr/bin/env python3
"""Interleaved A/B timing of SpMV variants in ONE process (cdna guide §5.4
rule 24): every round times every variant once, and the report gives the
median and min per variant. Also times torch read/copy kernels on buffers of
the same size as a measured-bandwidth reference, and checks that every
variant's y is bit-identical to the first STREAM variant's.

    python tools/tune.py [--grid 300] [--rounds 5] [--launches 20] [--variants all|stream]
"""
from __future__ import annotations

import argparse
import importlib
import itertools
import json
import os
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def time_launches(fn, n, stream):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for a, b in ev:
        a.record(stream)
        fn()
        b.record(stream)
    torch.cuda.synchronize()
    return np.array([a.elapsed_time(b) * 1e3 for a, b in ev])  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", type=int, default=300)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--launches", type=int, default=20)
    ap.add_argument("--variants", default="stream")
    ap.add_argument("--matrix", default="poisson", choices=["poisson", "skewed", "skewed_nohub", "skewed_localx", "skewed_blocksort", "fem_hex", "banded"])
    ap.add_argument("--file", default=None, help="a MatrixMarket (.mtx) or PETSc binary operand, e.g. Flan_1565.mtx")
    args = ap.parse_args()
    pkg = importlib.import_module("petsc-openacc_amd")
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream()
    t0 = time.time()
    if args.file:
        matio = importlib.import_module("petsc-openacc_amd.matio")
        load = matio.load_mtx if args.file.endswith(".mtx") else matio.load_petsc_binary
        ai, aj, aa, ncols = load(args.file)
        if ncols != len(ai) - 1:
            raise SystemExit("tune.py times square operands (x and y share a length)")
    elif args.matrix == "poisson":
        ai, aj, aa = pkg.poisson_csr(args.grid)
    elif args.matrix == "fem_hex":  # Flan_1565's structure: hexahedral mesh, 3 dofs per node
        ai, aj, aa = pkg.fem_hex_csr()
    elif args.matrix == "banded":  # 3 M rows of ~30 random columns within +-20000 (GAMG-coarse-like scatter)
        rng = np.random.default_rng(5)
        m, w = 3_000_000, 30
        c = np.sort(np.clip(np.arange(m)[:, None] + rng.integers(-20000, 20001, (m, w)), 0, m - 1), axis=1)
        keep = np.ones_like(c, dtype=bool)
        keep[:, 1:] = c[:, 1:] != c[:, :-1]
        ai = np.concatenate([[0], np.cumsum(keep.sum(axis=1))]).astype(np.int32)
        aj = c[keep].astype(np.int32)
        aa = rng.uniform(-1, 1, len(aj))
    else:
        ai, aj, aa = pkg.skewed_csr()
        if args.matrix in ("skewed_nohub", "skewed_localx", "skewed_blocksort"):  # the FEM-like rows only (hub rows emptied)
            ln = np.diff(ai)
            keep = np.repeat(ln <= 1000, ln)
            ai = np.concatenate([[0], np.cumsum(np.where(ln <= 1000, ln, 0))]).astype(np.int32)
            aj, aa = aj[keep], aa[keep]
        if args.matrix == "skewed_localx":  # experiment: same stream, x gathers confined to 32 KiB
            aj = (aj & 4095).astype(np.int32)
        if args.matrix == "skewed_blocksort":  # experiment: each ~4096-entry row block's columns sorted
            # across the block (the gather pattern a column-sorted in-block
            # layout would give; the rows' sums change, the stream does not)
            ln = np.diff(ai)
            aj = aj.copy()
            r0 = 0
            while r0 < len(ln):
                r1, nk = r0, 0
                while r1 < len(ln) and r1 - r0 < 512 and nk + ln[r1] <= 4096:
                    nk += ln[r1]
                    r1 += 1
                r1 = max(r1, r0 + 1)
                a, b = ai[r0], ai[r1]
                aj[a:b] = np.sort(aj[a:b])
                r0 = r1
    m = len(ai) - 1
    nbytes = pkg.algorithmic_bytes(m, m, len(aj))
    x = torch.from_numpy(pkg.splitmix_uniform(m, 42)).to(dev)
    y = torch.empty(m, dtype=torch.float64, device=dev)
    A = pkg.SeqAIJHIP(ai, aj, aa)
    print(f"# setup {time.time() - t0:.1f}s m={m} nnz={len(aj)} bytes={nbytes}", flush=True)

    variants = []
    if args.variants in ("stream", "all"):
        for g, nt in itertools.product(range(10), (0, 1)):
            variants.append(("stream", dict(geometry=g, nt_loads=nt)))
    if args.variants in ("kernels", "all"):
        variants += [("scalar", {}), ("vector", {"lanes": 8}), ("vector", {"lanes": 4})]
    if args.variants == "default":  # the product's defaults only
        variants.append(("stream", {}))
    if args.variants == "rowsum":  # default plus the small geometries (medium-length rows)
        variants += [("stream", {})] + [("stream", dict(geometry=g)) for g in (0, 1, 6, 8)]
    if args.variants == "ntlong":  # non-temporal matrix loads for long-row operands, both automatic geometries
        for g, nt in itertools.product((1, 6), (0, 1)):
            variants.append(("stream", dict(geometry=g, nt_loads=nt)))
    if args.variants == "ntgeom":  # non-temporal matrix loads x load depth (tools/read_sweep.hip: nt reads 6.8 TB/s)
        for g, nt in itertools.product((6, 11, 8, 0), (0, 1)):
            variants.append(("stream", dict(geometry=g, nt_loads=nt)))
    if args.variants == "longxcd":
        for g, lx in itertools.product((1, 6), (0, 1)):
            variants.append(("stream", dict(geometry=g, long_xcd=lx)))
    if args.variants == "skewgeom":
        for g, ex in itertools.product(range(9), (0, 1)):
            variants.append(("stream", dict(geometry=g, exact=ex)))
    if args.variants == "gsort":  # gather-ordered row blocks (AIJHIP_OPT_GATHER_SORT) against the unsorted
        for g, gs, nt in ((-1, -1, -1), (-1, 0, -1), (6, 1, 0), (1, 1, 0), (6, 1, 1), (6, 0, 0), (1, 0, 1)):
            variants.append(("stream", dict(geometry=g, gather_sort=gs, nt_loads=nt)))
    if args.variants == "codes":  # 16-bit column codes (AIJHIP_OPT_COLUMN_CODES) against aj, gather order off/on
        for gs, cc, nt in ((0, 0, 0), (0, 1, 0), (0, 1, 1), (-1, 0, -1), (0, 0, 1)):
            variants.append(("stream", dict(geometry=6, gather_sort=gs, column_codes=cc, nt_loads=nt)))
    if args.variants == "codesgeom":  # column codes at the geometries the coded launch is built for
        for g, cc, nt in ((6, 1, 0), (6, 1, 1), (7, 1, 0), (7, 1, 1), (9, 1, 0), (9, 1, 1), (6, 0, 0)):
            variants.append(("stream", dict(geometry=g, gather_sort=0, column_codes=cc, nt_loads=nt)))
    if args.variants == "layouts":  # the automatic layout (row patterns / codes) against codes and aj
        for rp, cc, nt in ((-1, -1, 0), (0, 1, 0), (0, 0, 0), (1, 0, 1)):
            variants.append(("stream", dict(geometry=6, gather_sort=0, row_patterns=rp, column_codes=cc, nt_loads=nt)))
    if args.variants == "patnt":  # row patterns: plain vs non-temporal aa loads
        for nt in (0, 1, 0, 1):
            variants.append(("stream", dict(row_patterns=1, nt_loads=nt)))
    if args.variants == "overlap":  # hub segments + wide blocks after the row blocks or on a side stream
        for ov in (0, 1, 0, 1):
            variants.append(("stream", dict(long_overlap=ov)))
    if args.variants == "bf":  # branch-free STREAM phase 1 (AIJHIP_STREAM_BF) against the predicated form, aj layout
        for bf in ("0", "1", "0", "1"):
            variants.append(("stream", dict(row_patterns=0, column_codes=0, env={"AIJHIP_STREAM_BF": bf})))
    if args.variants == "geoms":  # the default plan at the geometries of 256 / 512 lanes and 2 / 4 pair-iterations
        for g in (6, 8, 11, 0, 6, 8, 11, 0):
            variants.append(("stream", dict(geometry=g)))
    if args.variants == "exact":  # PETSc's sequential row order in every block (exact) against the split sums
        for ex in (0, 1, 0, 1):
            variants.append(("stream", dict(exact=ex)))
    if args.variants == "bfauto":  # branch-free phase 1 against the predicated form, the library's automatic layout
        for bf in ("0", "1", "0", "1"):
            variants.append(("stream", dict(env={"AIJHIP_STREAM_BF": bf})))
    if args.variants == "gslong":  # hub-row segments beside the gather-ordered blocks: XCD placement on / off
        for lx in (1, 0):
            variants.append(("stream", dict(long_xcd=lx)))
    if args.variants == "geo16":  # the two automatic geometries
        for g in (1, 6):
            variants.append(("stream", dict(geometry=g)))
    if args.variants == "skewgeom2":  # the geometry the skewgeom sweep left out (9) against 1
        for g, nt in itertools.product((1, 9), (0, 1)):
            variants.append(("stream", dict(geometry=g, nt_loads=nt)))
    if args.variants == "skewed":
        for g in (0, 1, 4, 6, 7, 8):
            variants.append(("stream", dict(geometry=g, nt_loads=0)))
        for g in (1, 6):
            variants.append(("stream", dict(geometry=g, exact=1)))
        variants += [("vector", {"lanes": 16}), ("vector", {"lanes": 32}), ("vector", {"lanes": 64}),
                     ("scalar", {})]

    def configure(kind, opts):
        for k, v in opts.get("env", {}).items():  # read by the planner (the set_option calls below re-plan)
            os.environ[k] = v
        A.set_kernel(kind, opts.get("lanes", 0))
        A.set_option("geometry", opts.get("geometry", -1))  # -1: the library's choice
        A.set_option("exact", opts.get("exact", 0))
        A.set_option("long_xcd", opts.get("long_xcd", 1))
        A.set_option("long_overlap", opts.get("long_overlap", -1))
        A.set_option("gather_sort", opts.get("gather_sort", -1))
        A.set_option("column_codes", opts.get("column_codes", -1))
        A.set_option("row_patterns", opts.get("row_patterns", -1))
        for k in ("geometry", "nt_loads"):
            if k in opts:
                A.set_option(k, opts[k])

    # reference bandwidth: torch streaming kernels over the same byte count
    buf = torch.empty(nbytes // 8, dtype=torch.float64, device=dev).uniform_()
    half = torch.empty(nbytes // 16, dtype=torch.float64, device=dev)
    refs = {
        "torch_sum_read": (lambda: buf.sum(), nbytes),
        "torch_copy": (lambda: half.copy_(buf[: nbytes // 16]), nbytes),
    }

    ref_y = None
    results = {name: [] for name in [json.dumps([k, o]) for k, o in variants] + list(refs)}
    for rnd in range(args.rounds):
        for kind, opts in variants:
            key = json.dumps([kind, opts])
            configure(kind, opts)
            fn = lambda: A.mult(x, y, stream)  # noqa: E731
            time_launches(fn, 3, stream)
            us = time_launches(fn, args.launches, stream)
            results[key].append(float(np.median(us)))
            if rnd == 0:
                yy = y.cpu().numpy()
                if ref_y is None:
                    ref_y = yy
                same = bool(np.array_equal(yy.view(np.uint64), ref_y.view(np.uint64)))
                maxdiff = float(np.max(np.abs(yy - ref_y)))
                inf = A.info()
                print(json.dumps({"variant": key, "bitwise_equal_first": same, "max_abs_diff": maxdiff,
                                  "geometry": inf["stream_geometry"],
                                  "n_blocks": inf["n_blocks"]}), flush=True)
        for name, (fn, nb) in refs.items():
            time_launches(fn, 2, stream)
            results[name].append(float(np.median(time_launches(fn, args.launches, stream))))
    rows = []
    for key, v in results.items():
        nb = refs[key][1] if key in refs else nbytes
        med, mn = float(np.median(v)), float(np.min(v))
        rows.append({"variant": key, "us_median": round(med, 2), "us_min": round(mn, 2),
                     "GBs_median": round(nb / med / 1e3, 1), "frac_8TBs": round(nb / med / 1e3 / 8000, 4)})
    rows.sort(key=lambda r: r["us_median"])
    for r in rows:
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
