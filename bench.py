#!/usr/bin/env python3
"""Benchmark: CSR SpMV effective HBM GB/s on the 300^3 7-point Poisson operand.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--grid 300] [--layout csr|auto]

A step is one MatMult (y = A x) of the whole operand, inputs resident in HBM.
The workload at every N is BASELINE.json configs[1]: 300^3 Poisson CSR (27 M
rows, 188.46 M entries, fp64 values, int32 indices).
N = 1: MatMult_SeqAIJ on one MI355X.
N > 1: the SAME operand row-partitioned over N GPUs in balanced whole
z-planes (strong scaling — the reference's own sweep, runs/single-node-
scaling.pbs:56-67, `aprun -n 16/8/4/2/1 ... -da_grid_x 300`), one rank per
GPU over RCCL: MatMult_MPIAIJ, the halo planes exchanged while the diagonal
block multiplies (csrc/ksp_mpi.hip). Launched by torch.distributed.run, or by
this script itself: `python bench.py --gpus N` with no WORLD_SIZE in the
environment starts the N rank processes (before any GPU call) and prints rank
0's line. Beside `value`, the `weak` block is BASELINE configs[3]: every rank
a 300^3-row z-slab of a grid that doubles one axis per factor 2 of N (N = 8:
the 600^3 grid), and per rank the halo cost of every exchange form.

The headline MatMult reads PETSc's CSR as stored (ai / aj / aa; --layout
csr, the default): the metric is a CSR SpMV. The library's automatic layout
(row patterns for a stencil: no aj at all) is timed beside it in the
`effective` block, on its own bytes, and is never `value`.

value  = algorithmic bytes of the whole operand x K / (max-over-ranks wall
         time of the K timed steps), bytes per SpMV = 12 nnz + 4 (m+1) + 8 n
         + 8 m (x and the matrix read once, y written once).
roofline.achieved = the compulsory bytes of the layout rank 0's timed launch
         reads (aijhip_info_t.mult_layout_bytes: the CSR bytes above for
         --layout csr) / the mean duration of the launch, from HIP events
         recorded around every launch on the stream it runs on; peak 8 TB/s
         (MI355X_MICROARCH.md). Every `frac` in the line is bytes the timed
         kernel moves / its time / 8 TB/s.
cpu_baseline = the C restatement of PETSc's MatMult_SeqAIJ (oracle/, a port:
         the reference cannot be built here) on 1 host core and on all the
         process's threads, bounded samples of the whole 300^3 operand, rank
         0 at every N.
Every leg beside the headline has a wall budget (Legs): a leg that cannot
fit in what is left of --wall-budget is recorded as {"error": "budget"}, and
a leg still running at the deadline is cut the same way; the line is always
printed.
"""
from __future__ import annotations

import argparse
import ctypes
import importlib
import json
import os
import sys
import threading
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

# HIP maps streams onto GPU_MAX_HW_QUEUES hardware queues (4 by default)
# round-robin: with the library's exchange and side streams, torch's and
# RCCL's, a fifth stream shares a queue with the compute stream and its
# "concurrent" work runs behind it. Measured (profiles/r05/e/): the skewed
# stand-in's side-stream overlap 344 us at 4 queues (slower than serial, 325)
# vs 313 us at 8; the halo's empty fork / join 29.5 vs 13.5 us. Set before
# HIP initialises (the rank children inherit it); at least 8, a larger value stays.
if int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0) < 8:
    os.environ["GPU_MAX_HW_QUEUES"] = "8"

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md §Chip-level parameters (spec)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--grid", type=int, default=300, help="per-rank grid edge (N^3 rows per rank)")
    p.add_argument("--kernel", default="auto", choices=["auto", "stream", "scalar", "vector"])
    p.add_argument("--geometry", type=int, default=None, help="STREAM geometry 0..11 (default: the library's)")
    p.add_argument("--nt", type=int, default=None, help="STREAM non-temporal matrix loads 0/1")
    p.add_argument("--layout", default="csr", choices=["csr", "auto"],
                   help="what the headline MatMult reads: csr = PETSc's aj/aa (the metric's CSR SpMV; default), "
                        "auto = the library's automatic layout (row patterns / column codes where they fit)")
    p.add_argument("--codes", type=int, default=None,
                   help="STREAM column codes -1 (library default: automatic) / 0 (aj) / 1")
    p.add_argument("--patterns", type=int, default=None,
                   help="STREAM row patterns -1 (library default: automatic) / 0 / 1")
    p.add_argument("--templates", type=int, default=None,
                   help="row templates (the patterns with the values) -1 (library default: automatic) / 0 / 1")
    p.add_argument("--halo", default="p2p", choices=["p2p", "allgather"])
    p.add_argument("--x", default="uniform", choices=["uniform", "exact"], help="x = splitmix(42) or generateExt")
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="bound of the CPU baseline sample")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-cg", action="store_true")
    p.add_argument("--no-gamg", action="store_true", help="skip the CG+GAMG solve (BASELINE configs[2])")
    p.add_argument("--cg-iters", type=int, default=200, help="CG iterations timed for cg.iters_per_s")
    p.add_argument("--no-host-vec", action="store_true", help="skip the host-vector MatMult timing")
    p.add_argument("--no-flan", action="store_true", help="skip the configs[4] Flan_1565 stand-in legs")
    p.add_argument("--no-pmc", action="store_true",
                   help="skip the live rocprofv3 --pmc passes for roofline.traffic (use the committed record)")
    p.add_argument("--roofline-reps", type=int, default=50,
                   help="launches timed by HIP events for roofline.achieved (at least this many, SURVEY §8d)")
    p.add_argument("--no-weak", action="store_true", help="N > 1: skip the weak-scaling block (BASELINE configs[3])")
    p.add_argument("--weak-grid", type=int, default=None,
                   help="per-rank edge of the weak-scaling block (default: --grid; N = 8 -> 600^3)")
    p.add_argument("--wall-budget", type=float, default=420.0,
                   help="seconds from the start barrier after which no leg starts and a running leg is cut "
                        "(the line is still printed; per-leg budgets in leg_budgets)")
    p.add_argument("--mpi", action="store_true",
                   help="take the multi-GPU code path (MPIAIJ, RCCL, distributed CG) even at N = 1 "
                        "(launch with torch.distributed.run): a one-GPU rehearsal of the N > 1 run")
    p.add_argument("--comm-timeout", type=float, default=300.0,
                   help="seconds before a stuck collective aborts the run (process group and RCCL waits)")
    p.add_argument("--rehearse-one-gpu", action="store_true",
                   help="N > 1 control-flow rehearsal on a one-GPU box: every rank on cuda:0 over gloo "
                        "(RCCL refuses two ranks on one device); timings are not scaling numbers")
    return p.parse_args()


def weak_grid(G: int, world: int):
    """Global grid (nx, ny, nz) with G^3 rows per rank in whole z-planes:
    each factor 2 of the world size doubles z, then y, then x (N = 8 from
    G = 300 is 600^3); any odd factor multiplies z. Falls back to
    G x G x G*world when the planes do not divide evenly."""
    dims, axis, w = [G, G, G], 2, world
    while w % 2 == 0:
        dims[axis] *= 2
        axis = (axis - 1) % 3
        w //= 2
    dims[2] *= w
    nx, ny, nz = dims
    if nz % world or nx * ny * (nz // world) != G ** 3:
        return G, G, G * world
    return nx, ny, nz


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def rank_plan(n: int, argv, port: int, child=None, env=None):
    """The N rank processes `python bench.py --gpus N` starts when no launcher
    set WORLD_SIZE (the driver may run the bench plainly at every N): one per
    GPU, the torch.distributed env contract of torch.distributed.run (RANK,
    LOCAL_RANK, WORLD_SIZE, LOCAL_WORLD_SIZE, MASTER_ADDR 127.0.0.1,
    MASTER_PORT), the same arguments. Returns [(cmd, env)] in rank order."""
    cmd = list(child) if child is not None else [sys.executable, "-u", str(Path(__file__).resolve())] + list(argv)
    base = dict(os.environ if env is None else env)
    out = []
    for r in range(n):
        e = dict(base)
        e.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0",
                 MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        out.append((cmd, e))
    return out


def launch_ranks(n: int, argv, child=None, poll_s: float = 0.2) -> int:
    """Start the N ranks (rank_plan) as child processes of this one — no exec,
    and nothing here has touched the GPU — and wait for them. Rank 0's stdout
    is this process's stdout (its one JSON line); the other ranks' stdout goes
    to stderr, so exactly one line reaches the driver. If a rank fails, the
    others are stopped (by their own Popen handles) and its exit code is
    returned."""
    import subprocess
    plan = rank_plan(n, argv, free_port(), child)
    procs = []
    for r, (cmd, env) in enumerate(plan):
        procs.append(subprocess.Popen(cmd, env=env, stdout=None if r == 0 else sys.stderr.fileno()))
    rc = 0
    t0 = last = time.perf_counter()
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                rc = bad[0]
                break
            if all(c == 0 for c in codes):
                break
            time.sleep(poll_s)
            if time.perf_counter() - last >= 30.0:  # a heartbeat while the ranks start up (torch import, HIP init)
                last = time.perf_counter()
                running = sum(c is None for c in codes)
                print(f"bench: {running} of {n} ranks running, {last - t0:.0f} s", file=sys.stderr, flush=True)
    finally:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=30)
            except Exception:  # noqa: BLE001
                p.kill()
                p.wait()
    return rc


def rank_record(rank, device, pci_bus, rows, nnz, ghosts, spmv_ms, diag_ms, paired=None):
    """One rank's entry of the N > 1 line: where it ran and how much of its
    distributed SpMV the exchange (+ the A_o product) adds on top of the
    diagonal block alone. paired: the interleaved timing of halo_forms
    (median per-round differences) — then
    halo_exposed_us is that median, else the difference of the means."""
    rec = {"rank": rank, "device": device, "pci_bus": pci_bus, "rows": rows, "nnz": nnz, "ghosts": ghosts,
           "spmv_us_mean": round(spmv_ms * 1e3, 2), "diag_block_us_mean": round(diag_ms * 1e3, 2),
           "halo_exposed_us": round((spmv_ms - diag_ms) * 1e3, 2)}
    if paired is not None:
        rec.update(spmv_us_median=round(paired["spmv_us_median"], 2),
                   diag_block_us_median=round(paired["diag_us_median"], 2),
                   halo_exposed_us=round(paired["diff_us_median"], 2),
                   halo_exposed_iqr_us=[round(v, 2) for v in paired["diff_us_iqr"]],
                   rounds=paired["rounds"])
    return rec


def distributed_block(world, backend, comm_info, timeout_s, ranks):
    """The `distributed` object of the N > 1 line: world
    size, backends, RCCL version, the collective timeout and every rank's
    record, slowest exposed halo first in `worst_rank`."""
    worst = max(ranks, key=lambda r: r["halo_exposed_us"]) if ranks else None
    return {"world_size": world, "backend": backend, "comm": comm_info["kind"],
            "rccl_version": comm_info["version"] or None, "comm_timeout_s": timeout_s, "ranks": ranks,
            "worst_rank": None if worst is None else worst["rank"],
            "halo_hidden": "per rank, A_d alone and the distributed SpMV launched in turn (interleaved rounds): the "
                           "exchange runs on a second stream while A_d multiplies; halo_exposed_us is the median "
                           "per-round difference, what it adds (A_o product and the fork / join included)"}


def cpu_baseline(ai, aj, aa, x, seconds, all_cores=False):
    """Time the oracle (C restatement of MatMult_SeqAIJ) on 1 core — PETSc's
    1 rank = 1 core — or, with all_cores, its OpenMP static-row-block form on
    every host thread this process may use; repeated
    whole-operand SpMVs until `seconds` elapse (bounded sample). Returns
    (seconds per SpMV, reps, threads)."""
    build = importlib.import_module("petsc-openacc_amd.build")
    L = ctypes.CDLL(str(build.build_oracle()))
    P = ctypes.c_void_p
    fn = L.oracle_matmult_seqaij_omp if all_cores else L.oracle_matmult_seqaij
    fn.argtypes = [ctypes.c_int32, P, P, P, P, P]
    fn.restype = None
    threads = 1
    if all_cores:
        L.oracle_omp_threads.restype = ctypes.c_int
        threads = L.oracle_omp_threads()
    m = len(ai) - 1
    y = np.empty(m)
    args = (m, ai.ctypes.data, aj.ctypes.data, aa.ctypes.data, x.ctypes.data, y.ctypes.data)
    fn(*args)  # warm-up (page-in)
    reps, t0 = 0, time.perf_counter()
    while True:
        fn(*args)
        reps += 1
        el = time.perf_counter() - t0
        if el >= seconds or reps >= 50:
            break
    return el / reps, reps, threads


def cpu_cg_baseline(ai, aj, aa, pkg, nx, ny, nz, iters=8):
    """The oracle's KSPSolve_CG restatement (numpy vector ops + the C
    MatMult_SeqAIJ loop) on the host, a fixed small number of iterations."""
    from oracle import ksp_cg
    build = importlib.import_module("petsc-openacc_amd.build")
    L = ctypes.CDLL(str(build.build_oracle()))
    P = ctypes.c_void_p
    L.oracle_matmult_seqaij.argtypes = [ctypes.c_int32, P, P, P, P, P]
    L.oracle_matmult_seqaij.restype = None
    m = len(ai) - 1

    def mm(v):
        v = np.ascontiguousarray(v)
        y = np.empty(m)
        L.oracle_matmult_seqaij(m, ai.ctypes.data, aj.ctypes.data, aa.ctypes.data, v.ctypes.data, y.ctypes.data)
        return y

    rhs, _ = pkg.poisson_vectors(nx, ny, nz)
    t0 = time.perf_counter()
    _, its, _, _ = ksp_cg.cg(ai, aj, aa, rhs, rtol=0.0, atol=0.0, max_it=iters, matmult=mm)
    dt = time.perf_counter() - t0
    return {"iters_per_s": round(its / dt, 3), "cores": 1, "kind": "port",
            "sample": f"{its} CG+Jacobi iterations, oracle/ksp_cg.py + oracle/matmult_seqaij.c, 1 core"}


def cpu_cg_gamg_baseline(ai, aj, aa, pkg, nx, ny, nz, small=100):
    """The reference's CPU configuration, measured: CG + GAMG to rtol 1e-14 /
    atol 1e-12 from x = 0 on the host (oracle/cg_gamg.c: OpenMP row blocks,
    the library's host hierarchy builder), (i) on every host thread this
    process may use at the benchmark operand — the analogue of the reference's
    16-rank node run (/root/reference/runs/single-node-scaling.pbs:56-67) —
    and (ii) on 1 core at {small}^3 (BASELINE configs[0], the reference's
    plumbing configuration: 1 rank)."""
    from oracle import host_cg_gamg
    rhs, exact = pkg.poisson_vectors(nx, ny, nz)
    h = host_cg_gamg.solve(ai, aj, aa, rhs)
    out = {"time_to_solution_s": round(h["setup_s"] + h["solve_s"], 3), "setup_s": round(h["setup_s"], 3),
           "solve_s": round(h["solve_s"], 3), "its": h["its"], "reason": h["reason"],
           "max_err": float(np.abs(h["x"] - exact).max()), "cores": h["threads"], "cpu": cpu_model(),
           "kind": "port",
           "sample": f"full solve at {nx}x{ny}x{nz}: oracle/cg_gamg.c (CG + V-cycle, OpenMP, {h['threads']} threads) "
                     f"over the library's host GAMG hierarchy (built with the same threads)"}
    del h
    s_ai, s_aj, s_aa = pkg.poisson_csr(small)
    s_rhs, s_exact = pkg.poisson_vectors(small)
    h1 = host_cg_gamg.solve(s_ai, s_aj, s_aa, s_rhs, threads=1)
    out["one_core_configs0"] = {
        "workload": f"{small}^3 Poisson CG+GAMG (BASELINE configs[0])", "cores": 1,
        "time_to_solution_s": round(h1["setup_s"] + h1["solve_s"], 3), "setup_s": round(h1["setup_s"], 3),
        "solve_s": round(h1["solve_s"], 3), "its": h1["its"], "reason": h1["reason"],
        "max_err": float(np.abs(h1["x"] - s_exact).max()), "kind": "port"}
    return out


def host_vec_mult(A, x_h, reps=10):
    """MatMult with HOST x and y (aijhip_mat_mult_host: the path an unchanged
    PETSc caller with host Vecs takes), PCIe included: the
    serial step-2 form, the pipelined step-3/4 analogue from pageable arrays
    (copied directly: one H2D stream, and a second host thread issuing the D2H
    of y chunks) and from pinned arrays (direct DMA). The
    three results must be bit-identical."""
    import torch
    out, ys = {}, []
    for name, chunk, pin in (("serial_pageable", 0, False), ("pipelined_pageable", -1, False),
                             ("pipelined_pinned", -1, True)):
        A.set_option("host_pipeline", chunk)
        if pin:
            xp = torch.from_numpy(x_h).pin_memory().numpy()
            yp = torch.empty(A.m, dtype=torch.float64).pin_memory().numpy()
        else:
            xp, yp = x_h, np.empty(A.m)
        A.mult_host(xp, out=yp)  # warm-up (builds the pipeline)
        t0 = time.perf_counter()
        for _ in range(reps):
            A.mult_host(xp, out=yp)
        dt = (time.perf_counter() - t0) / reps
        out[name] = {"ms": round(dt * 1e3, 3), "pcie_GBs": round((8 * A.n + 8 * A.m) / dt / 1e9, 2)}
        ys.append(np.array(yp, copy=True))
    A.set_option("host_pipeline", -1)
    out["bitwise_equal"] = bool(all(np.array_equal(ys[0].view(np.uint64), y.view(np.uint64)) for y in ys[1:]))
    out["speedup_pipelined_pageable"] = round(out["serial_pageable"]["ms"] / out["pipelined_pageable"]["ms"], 3)
    out["note"] = "ms per MatMult with x, y in host memory (x H2D + product + y D2H), whole-call wall time"
    return out


def read_ceiling(nbytes, dev, reps=20):
    """The achievable HBM read rate on this box, timed in the same run:
    aijhip_read_probe over a buffer of the SpMV's byte count, each byte read
    once per launch; mean of `reps` launches by HIP events. Returns
    {mode: (GB/s, us)} for mode 0 (the fastest shape measured: non-temporal
    16-B loads, two per lane) and mode 1 (the STREAM kernel's shape: plain
    loads, four per lane)."""
    import torch
    ksp = importlib.import_module("petsc-openacc_amd.ksp")
    L = ksp._veclib()
    buf = torch.rand(nbytes // 8, dtype=torch.float64, device=dev)
    s = torch.cuda.current_stream()
    out = {}
    for mode in (0, 1):
        for _ in range(3):
            L.aijhip_read_probe(buf.data_ptr(), buf.numel(), mode, s.cuda_stream)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
        for a, b in ev:
            a.record(s)
            L.aijhip_read_probe(buf.data_ptr(), buf.numel(), mode, s.cuda_stream)
            b.record(s)
        torch.cuda.synchronize()
        ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
        out[mode] = (round(nbytes / (ms / 1e3) / 1e9, 1), round(ms * 1e3, 2))
    del buf
    return out


def pmc_traffic(rows, nnz, block):
    """HBM bytes per launch from the committed rocprofv3 PMC record
    (profiles/pmc_latest.json, written from tools/gpu_pmc_case.sh), used only
    when it was measured on the same operand with the same block geometry;
    bench.py itself runs without the profiler, so it cannot count bytes."""
    p = ROOT / "profiles" / "pmc_latest.json"
    try:
        rec = json.loads(p.read_text())
    except (OSError, ValueError):
        return None, None
    if rec.get("rows") != rows or rec.get("nnz") != nnz or rec.get("block") != block:
        return None, None
    return rec.get("hbm_traffic_bytes_per_launch"), rec.get("source")


def live_pmc_traffic(grid, timeout_s=150, case="poisson", opts=("row_patterns=0", "column_codes=0"), its=10):
    """HBM bytes per MatMult counted in THIS run: two rocprofv3 --pmc passes
    (FETCH_SIZE, then WRITE_SIZE: one counter group each, no other tracing)
    over a child process that launches the same kernels on the same operand
    (tools/prof_case.py CASE: `poisson` in the CSR layout — the headline —
    or a Flan stand-in in its default layout; `its` MatMults), corrected as
    MI355X_MICROARCH.md's HBM section prescribes for gfx950 (read bytes =
    2 x FETCH_SIZE KiB, write bytes = WRITE_SIZE KiB; tools/pmc_summary.py),
    summed over the MatMult's dispatches (row blocks, long-row segments and
    their finish) and divided by `its`. The child runs in its own process
    group, killed (SIGKILL) at the time limit. Returns (bytes, detail) or
    (None, reason)."""
    import csv
    import shutil
    import signal
    import subprocess
    import tempfile
    exe = shutil.which("rocprofv3")
    if not exe:
        return None, "rocprofv3 not on PATH"
    got = {}
    with tempfile.TemporaryDirectory(prefix="bench_pmc_", dir=os.environ.get("TMPDIR", "/tmp")) as td:
        for counter in ("FETCH_SIZE", "WRITE_SIZE"):
            out_dir = Path(td) / counter
            cmd = [exe, "--pmc", counter, "--output-format", "csv", "-d", str(out_dir), "-o", "run", "--",
                   sys.executable, str(ROOT / "tools" / "prof_case.py"), case, "--grid", str(grid), "--its", str(its)]
            for o in opts:
                cmd += ["--opt", o]
            with open(Path(td) / f"{counter}.log", "w") as log:
                proc = subprocess.Popen(cmd, stdout=log, stderr=subprocess.STDOUT, start_new_session=True)
                try:
                    proc.wait(timeout=timeout_s)
                except subprocess.TimeoutExpired:
                    os.killpg(proc.pid, signal.SIGKILL)
                    proc.wait()
                    return None, f"{counter} pass exceeded {timeout_s} s (killed)"
            if proc.returncode != 0:
                return None, f"{counter} pass exited {proc.returncode}"
            vals = []
            for f in out_dir.rglob("*counter_collection.csv"):
                with open(f) as fh:
                    for row in csv.DictReader(fh):
                        k = row.get("Kernel_Name", "")
                        spmv = ("k_spmv_stream" in k or "k_spmv_pattern" in k) and "OpMult<false>" in k
                        if (spmv or "k_long_partial" in k or "k_long_finish" in k) and row.get("Counter_Name") == counter:
                            vals.append(float(row["Counter_Value"]))
            if not vals:
                return None, f"{counter}: no MatMult dispatch in the record"
            got[counter] = (float(np.sum(vals)) / its, len(vals))
    rd = 2.0 * got["FETCH_SIZE"][0] * 1024
    wr = got["WRITE_SIZE"][0] * 1024
    return int(rd + wr), {"read_bytes": int(rd), "write_bytes": int(wr),
                          "dispatches": [got["FETCH_SIZE"][1], got["WRITE_SIZE"][1]], "matmults": its}


def launch_times(fn, stream, reps):
    """Per-launch HIP events on `stream` around `reps` calls of fn(): the
    launch times in us."""
    import torch
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record(stream)
        fn()
        b.record(stream)
    torch.cuda.synchronize()
    return [a.elapsed_time(b) * 1e3 for a, b in ev]


def time_launches(fn, stream, reps):
    """Per-launch HIP events on `stream` around `reps` calls of fn():
    (mean us, median us, min us)."""
    import torch
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record(stream)
        fn()
        b.record(stream)
    torch.cuda.synchronize()
    us = np.array([a.elapsed_time(b) for a, b in ev]) * 1e3
    return float(np.mean(us)), float(np.median(us)), float(np.min(us))


def flan_standins(pkg, dev, reps, cpu_sample):
    """BASELINE configs[4] (SuiteSparse Flan_1565, absent offline) through its
    two stand-ins at full size, each timed like the headline kernel (HIP events
    on the launch stream, `reps` launches after warm-up) beside a flat read of
    the same byte count in the same run:
      skewed — 1,564,794 rows of 45-99 banded entries plus 1e-4 hub rows of
               1e3-2e5 scattered entries (seed 1565): the merge-path
               load-balance stress; STREAM (default: gather-ordered row
               blocks, hub rows as 4096-entry segments after them;
               stream_side: the segments on a side stream beside them), STREAM exact
               (PETSc's order in every row that fits a block) and STREAM on
               PETSc's aj as stored (stream_csr);
      fem_hex — Flan_1565's own structure: a hexahedral mesh of 81x80x80
               nodes, 3 dofs per node, 81-entry interior rows.
    Parity is the -m gpu tests' job (tests/test_flan_standins_gpu.py)."""
    import torch
    stream = torch.cuda.current_stream()
    out = {}
    for name, make, kernels in (("skewed", lambda: pkg.skewed_csr(),
                                 ("stream", "stream_side", "stream_exact", "stream_csr")),
                                ("fem_hex", lambda: pkg.fem_hex_csr(), ("stream",))):
        ai, aj, aa = make()
        m, nnz = len(ai) - 1, len(aj)
        nbytes = pkg.algorithmic_bytes(m, m, nnz)
        x = torch.from_numpy(pkg.splitmix_uniform(m, 42)).to(dev)
        y = torch.empty_like(x)
        rec = {"rows": m, "nnz": nnz, "max_row": int(np.diff(ai).max()), "bytes_per_spmv": nbytes}
        # every variant built first, then timed in interleaved rounds (10
        # launches of each per round): a leg timed alone after another leg
        # read up to 6 % apart from the same code (r05 records, skewed
        # stream vs stream_exact)
        mats, infos, times = {}, {}, {}
        try:
            for kern in kernels:
                A = pkg.SeqAIJHIP(ai, aj, aa, ncols=m, kernel="stream")
                mats[kern] = A
                if kern == "stream_exact":
                    A.set_option("exact", 1)
                if kern == "stream_csr":  # aj as stored: no gather order
                    A.set_option("gather_sort", 0)
                if kern == "stream_side":  # the long rows on a side stream beside the row blocks
                    A.set_option("long_overlap", 1)
                infos[kern] = A.info()
                times[kern] = []
                # warm-up of >= 50 ms of launches: the first leg follows the
                # PCIe-bound host-vector leg, and after 5 launches it read 6-8 %
                # slow (profiles/r04/bench_r04e.json vs s3/skewed_exact.jsonl)
                t_w = time.perf_counter()
                while time.perf_counter() - t_w < 0.05:
                    for _ in range(10):
                        A.mult(x, y, stream)
                    torch.cuda.synchronize()
            for _ in range(max(8, reps // 10)):
                for kern, A in mats.items():
                    times[kern].extend(launch_times(lambda: A.mult(x, y, stream), stream, 10))
        finally:
            for A in mats.values():
                A.destroy()
        for kern in kernels:
            info, us = infos[kern], np.array(times[kern])
            mean, med, mn = float(np.mean(us)), float(np.median(us)), float(np.min(us))
            lb = info["mult_layout_bytes"]
            rec[kern] = {"us_mean": round(mean, 2), "us_median": round(med, 2), "us_min": round(mn, 2),
                         "launches": int(len(us)),
                         "layout_bytes": lb, "GBs": round(lb / (mean * 1e-6) / 1e9, 1),
                         "frac": round(lb / (mean * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
                         "csr_effective_GBs": round(nbytes / (mean * 1e-6) / 1e9, 1),
                         "geometry": info.get("stream_geometry"), "long_rows": info.get("n_long_rows"),
                         "column_codes": info.get("column_codes"), "gather_sorted": info.get("gather_sorted"),
                         "row_patterns": info.get("row_patterns"), "long_overlap": info.get("long_overlap"),
                         "exact": info.get("exact")}
        del x, y
        flat = read_ceiling(nbytes, dev)
        rec["ceiling_flat_read"] = {"GBs": flat[0][0], "us": flat[0][1],
                                    "frac_of_ceiling": round(rec["stream"]["csr_effective_GBs"] / flat[0][0], 4),
                                    "note": "the CSR byte count read once by aijhip_read_probe (mode 0); "
                                            "frac_of_ceiling = the flat read's time / the stream launch's time "
                                            "(the CSR bytes over both)"}
        if cpu_sample:
            t_cpu, reps_cpu, _ = cpu_baseline(ai, aj, aa, pkg.splitmix_uniform(m, 42), 3.0)
            rec["cpu_baseline"] = {"value": round(nbytes / t_cpu / 1e9, 3), "unit": "GB/s", "cores": 1,
                                   "kind": "port", "sample": f"{reps_cpu} SpMVs on 1 core, oracle/matmult_seqaij.c"}
        out[name] = rec
        del ai, aj, aa
    out["note"] = ("Flan_1565 itself is not in the image (no network); matio.load_mtx reads it when present. "
                   "GBs / frac = the bytes of the layout the launch reads (layout_bytes: column codes 10 B per "
                   "coded entry, the gather-ordered copy 12 B, CSR 12 B) / mean HIP-event launch time, of 8 TB/s; "
                   "csr_effective_GBs = SURVEY §8d's CSR bytes / the same time")
    return out


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def halo_forms(op, x, stream, reps, rank, dev, m_loc, nnz_loc):
    """Per rank, what each exchange form adds on top of the diagonal block:
    distributed SpMVs through the all-gather operator (op.native, built with
    halo="allgather") and through its p2p twin (op.p2p_native(): same A_d,
    ghost-numbered A_o, ncclSend/ncclRecv to the slab neighbours), that twin
    with the exchange in order on the compute stream (p2p_serial: no fork /
    join events, aijhip_mpiaij_set_overlap 0), and A_d alone, INTERLEAVED — one launch of each in turn for max(reps, 200) rounds,
    HIP events on the compute stream around every launch, a 1.5 ms device
    delay queued ahead of each round so the events time device work rather
    than host enqueue overhead — so box drift hits the three alike; halo_exposed_us = the median over rounds of (form − A_d)
    in the same round (two sequential means differed by
    10 µs for the same operator). Returns {form: this rank's record}."""
    import torch
    rounds = max(reps, 200)
    y = torch.empty(op.mloc, dtype=torch.float64, device=dev)
    fns = {"diag": lambda: op.A_d.mult(x, y, stream)}
    for form, nat in (("p2p", op.p2p_native()), ("allgather", op.native)):
        fns[form] = (lambda n: lambda: n.mult(x, y, stream))(nat)
    p2p = op.p2p_native()

    def p2p_serial():  # the p2p plan in order on the compute stream (no fork / join)
        p2p.set_overlap(False)
        p2p.mult(x, y, stream)
        p2p.set_overlap(None)  # back to the library's automatic choice
    fns["p2p_serial"] = p2p_serial
    for _ in range(3):
        for f in fns.values():
            f()
    ev = {k: [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(rounds)]
          for k in fns}
    # a device delay ahead of every round: the round is fully enqueued before
    # it runs, so the events time device work (fork / join included), not the
    # host's launch overhead (RCCL's enqueue alone is tens of µs)
    VL = importlib.import_module("petsc-openacc_amd.ksp")._veclib()
    for i in range(rounds):
        VL.aijhip_delay_probe(1500.0, stream.cuda_stream)
        for k, f in fns.items():
            a, b = ev[k][i]
            a.record(stream)
            f()
            b.record(stream)
    torch.cuda.synchronize()
    us = {k: np.array([a.elapsed_time(b) for a, b in ev[k]]) * 1e3 for k in fns}
    out = {}
    for form in ("p2p", "allgather", "p2p_serial"):
        d = us[form] - us["diag"]
        paired = {"spmv_us_median": float(np.median(us[form])), "diag_us_median": float(np.median(us["diag"])),
                  "diff_us_median": float(np.median(d)),
                  "diff_us_iqr": [float(np.percentile(d, 25)), float(np.percentile(d, 75))], "rounds": rounds}
        out[form] = rank_record(rank, torch.cuda.current_device(),
                                getattr(torch.cuda.get_device_properties(dev), "pci_bus_id", None), m_loc, nnz_loc,
                                op.n_ghost, float(np.mean(us[form])) / 1e3, float(np.mean(us["diag"])) / 1e3, paired)
    del y
    return out


def gather_forms(mine, world):
    """All ranks' halo_forms records, per form, worst exposed rank named."""
    import torch.distributed as dist
    allr = [None] * world
    dist.all_gather_object(allr, mine)
    res = {}
    for form in ("p2p", "allgather", "p2p_serial"):
        ranks = [r[form] for r in allr]
        worst = max(ranks, key=lambda q: q["halo_exposed_us"])
        res[form] = {"ranks": ranks, "worst_rank": worst["rank"], "worst_halo_exposed_us": worst["halo_exposed_us"]}
    return res


class Legs:
    """Per-leg wall budgets and a hard deadline.

    Every leg beside the headline runs through run(name, budget_s, fn): it
    starts only if every rank still has at least budget_s of the run's wall
    budget (--wall-budget, counted from the start barrier) left — the ranks
    agree on the minimum, so all skip or all start — else it is recorded as
    {"error": "budget"} and not started. A leg that is still running at the
    deadline is cut by the watchdog: rank 0 writes the line built so far with
    that leg as {"error": "budget"}, and every rank exits (the ranks share the
    deadline, so none is left waiting in a collective). A heartbeat line on
    stderr every 60 s names the leg each rank is in."""

    def __init__(self, total_s, rank, world, distributed, dev, progress, line_fd):
        self.total_s, self.rank, self.world, self.distributed, self.dev = total_s, rank, world, distributed, dev
        self.progress, self.line_fd = progress, line_fd
        self.t0 = time.time()
        self.deadline = self.t0 + total_s
        self.log = {}
        self.current = None
        self.out = None  # rank 0: the line built so far
        self.headline_done = False
        self._lock = threading.Lock()
        self._written = False
        self._timer = None

    def remaining(self) -> float:
        return self.deadline - time.time()

    def _all_min(self, v: float) -> float:
        if not self.distributed:
            return v
        import torch
        import torch.distributed as dist
        t = torch.tensor([v], dtype=torch.float64, device=self.dev)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return float(t.item())

    def run(self, name, budget_s, fn, collective=True):
        """collective=False: a leg one rank runs alone (no agreement)."""
        rem = self._all_min(self.remaining()) if collective else self.remaining()
        if rem < budget_s:
            self.log[name] = {"budget_s": budget_s, "status": "skipped", "remaining_s": round(rem, 1)}
            self.progress(f"{name}: skipped, {rem:.0f} s of the wall budget left < its {budget_s} s")
            res = {"error": "budget", "budget_s": budget_s, "remaining_s": round(rem, 1),
                   "note": "not started: less than this leg's budget was left of the run's --wall-budget"}
        else:
            self.current = name
            t = time.perf_counter()
            res = guarded_leg(name, fn, self.distributed and collective, self.dev, self.progress)
            took = time.perf_counter() - t
            self.current = None
            self.log[name] = {"budget_s": budget_s, "took_s": round(took, 1),
                              "status": "ok" if took <= budget_s else "over"}
        if self.out is not None:
            self.out[name] = res
        return res

    def summary(self, cut=None) -> dict:
        d = {"wall_budget_s": self.total_s, "elapsed_s": round(time.time() - self.t0, 1), "legs": dict(self.log)}
        if cut is not None:
            d["legs"][cut] = {"status": "cut at the deadline"}
        return d

    def emit(self, obj) -> bool:
        """Write the line (rank 0, exactly once)."""
        with self._lock:
            if self._written:
                return False
            self._written = True
        os.write(self.line_fd, (json.dumps(obj) + "\n").encode())
        return True

    def arm(self):
        """Start the watchdog and the heartbeat (daemon threads)."""
        def fire():
            cut = self.current
            self.progress(f"wall budget ({self.total_s:.0f} s) reached in leg {cut!r}: writing the line and exiting")
            if self.rank == 0:
                if self.out is not None:
                    part = dict(self.out)
                    if cut is not None:
                        part[cut] = {"error": "budget", "note": "cut at the run's --wall-budget deadline"}
                    part["budget"] = self.summary(cut)
                else:
                    part = {"metric": METRIC, "value": None, "unit": "GB/s", "n_gpus": self.world,
                            "error": "budget: the wall budget ran out before the headline was measured",
                            "budget": self.summary(cut)}
                self.emit(part)
            sys.stderr.flush()
            os._exit(0 if self.headline_done else 1)

        self._timer = threading.Timer(max(0.0, self.remaining()), fire)
        self._timer.daemon = True
        self._timer.start()

        def beat():
            while True:
                time.sleep(60.0)
                self.progress(f"heartbeat: in {self.current or 'the headline / between legs'}")
        threading.Thread(target=beat, daemon=True).start()

    def disarm(self):
        if self._timer is not None:
            self._timer.cancel()


def guarded_leg(name, fn, distributed, dev, progress):
    """Run one leg; an exception raised alike on every rank (a bug, an
    allocation failure) is recorded in the line instead of discarding the
    headline measurement, and every rank learns whether any rank failed, so
    none waits on a peer that gave up."""
    progress(name)
    try:
        res, ok = fn(), 1.0
    except Exception as e:  # noqa: BLE001
        print(f"bench: {name} failed: {e!r}", file=sys.stderr, flush=True)
        res, ok = {"error": f"{type(e).__name__}: {e}"[:300]}, 0.0
    if distributed:
        import torch
        import torch.distributed as dist
        flag = torch.tensor([ok], dtype=torch.float64, device=dev)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        if float(flag.item()) < 1.0 and ok:
            res = {"error": "failed on another rank"}
    return res


METRIC = "CSR SpMV effective HBM GB/s (300^3 7-pt Poisson, fp64 MatMult_SeqAIJ)"


def slab_row_starts(mpiaij, dims, world):
    """Balanced whole z-planes (DMDA PETSC_DECIDE over z, helper.cpp:31-36
    with a 1x1xP process grid): (row_starts[world + 1], [(z0, z1)] per rank)."""
    nx, ny, nz = dims
    bounds = [mpiaij.slab_bounds(nz, world, r) for r in range(world)]
    starts = np.array([b[0] * nx * ny for b in bounds] + [nx * ny * nz], dtype=np.int64)
    return starts, bounds


def headline_line(*, world, dims, nnz_global, K, warmup, elapsed_s, launch_us, layout_bytes, info, distributed,
                  halo, x_kind, planes=None):
    """The contract fields of the one JSON line (pure: tests/test_bench.py
    checks it without a GPU). value = the whole operand's algorithmic bytes x
    K / the max-over-ranks wall time of the K timed steps. At N > 1 the
    operand is the same G^3 one row-partitioned over the N GPUs — strong
    scaling, the reference's own sweep (runs/single-node-scaling.pbs:56-67:
    aprun -n 1..16 ... -da_grid_x 300): `value` at every N is the metric's
    300^3 MatMult, comparable across N. roofline = the layout bytes rank 0's
    launch moves / the mean HIP-event time of its launches."""
    nx, ny, nz = dims
    n_global = nx * ny * nz
    bytes_global = 12 * nnz_global + 4 * (n_global + 1) + 8 * n_global + 8 * n_global
    launch_us = np.asarray(launch_us, dtype=np.float64)
    mean_s = float(np.mean(launch_us)) * 1e-6
    achieved = layout_bytes / mean_s / 1e9
    value = bytes_global * K / elapsed_s / 1e9
    csr = not (info.get("row_patterns") or info.get("column_codes"))
    if distributed:
        workload = (f"{nx}x{ny}x{nz} Poisson CSR MatMult row-partitioned over {world} GPU"
                    f"{'s' if world > 1 else ''} in z-slabs of {planes} planes (BASELINE configs[1] strong-scaled, "
                    f"the reference's 1-16 rank sweep at 300^3)")
    else:
        workload = f"{nx}x{ny}x{nz} Poisson CSR MatMult_SeqAIJ (BASELINE configs[1])"
    if nx == ny == nz:
        workload = f"{nx}^3" + workload[len(f"{nx}x{ny}x{nz}"):]
    block = {k: info.get(k) for k in ("stream_threads", "stream_nnz_cap", "stream_rows", "nt_loads", "column_codes",
                                      "row_patterns")}
    return {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": K,
        "warmup": warmup,
        "ms_per_step": round(elapsed_s / K * 1e3, 4),
        "ms_per_step_median_launch": round(float(np.median(launch_us[:K])) / 1e3, 4),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": ("synthetic (generated 7-pt Poisson operand of helper.cpp; x = splitmix64 uniform[-1,1))"
                 if x_kind == "uniform" else "synthetic (helper.cpp operand; x = generateExt field)"),
        "config": {
            "workload": workload, "rows": n_global, "nnz": nnz_global, "index": "int32", "values": "fp64",
            "kernel": info.get("kernel"), "layout": layout_name(info), "halo": halo if distributed else None,
            "block": block, "bytes_per_spmv": bytes_global, "flops_per_spmv_petsc": 2 * nnz_global - n_global,
        },
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": None,
            "traffic_source": None,
            "traffic_detail": None,
            "kernel": ("k_spmv_stream (CSR: aj / aa pairs, x gathered, LDS row sums)" if csr else layout_name(info)),
            "kernel_us_mean": round(mean_s * 1e6, 2),
            "kernel_us_median": round(float(np.median(launch_us)), 2),
            "kernel_us_min": round(float(np.min(launch_us)), 2),
            "launches_timed": int(len(launch_us)),
            "achieved_from_median": round(layout_bytes / (float(np.median(launch_us)) * 1e-6) / 1e9, 1),
            "bytes_per_launch": layout_bytes,
            "layout": layout_name(info),
            "note": ("rank 0's distributed MatMult (exchange + A_d + A_o) on rank 0's bytes"
                     if distributed else "bytes the timed kernel moves / mean HIP-event launch time"),
        },
    }


def cpu_spmv_baselines(pkg, G, seconds):
    """cpu_baseline (1 core) and cpu_baseline_all_cores (the OpenMP form on
    every thread this process may use) of the oracle's MatMult_SeqAIJ loop on
    the whole G^3 operand, x = the headline's splitmix x (a port: the
    reference cannot be built here). Rank 0 only, at every N."""
    ai, aj, aa = pkg.poisson_csr(G)
    m = len(ai) - 1
    x = pkg.splitmix_uniform(m, 42)
    nbytes = pkg.algorithmic_bytes(m, m, len(aj))
    t1, reps1, _ = cpu_baseline(ai, aj, aa, x, seconds)
    tn, repsn, threads = cpu_baseline(ai, aj, aa, x, seconds / 2, all_cores=True)
    one = {"value": round(nbytes / t1 / 1e9, 3), "unit": "GB/s", "cores": 1, "kind": "port",
           "sample": f"{reps1} whole-operand {G}^3 SpMVs on 1 core ({cpu_model()}), {t1 * 1e3:.1f} ms each; "
                     f"oracle/matmult_seqaij.c"}
    alln = {"value": round(nbytes / tn / 1e9, 3), "unit": "GB/s", "cores": threads, "kind": "port",
            "sample": f"{repsn} whole-operand {G}^3 SpMVs, OpenMP static row blocks on {threads} threads, "
                      f"{tn * 1e3:.1f} ms each; oracle/matmult_seqaij.c oracle_matmult_seqaij_omp"}
    return one, alln


def build_dist_operator(pkg, mpiaij, make_local, dims, world, rank, dev, comm):
    """This rank's z-slab of the nx x ny x nz operand as the native MPIAIJ
    (built with the all-gather halo; its p2p twin shares A_d, so both exchange
    forms run on one diagonal block). Returns (op, slab record)."""
    import torch
    import torch.distributed as dist
    row_starts, bounds = slab_row_starts(mpiaij, dims, world)
    z0, z1 = bounds[rank]
    ai, aj, aa = pkg.poisson_csr(*dims, z0, z1)
    op = mpiaij.MPIAIJ(ai, aj, aa, row_starts, make_local, pkg.split_rows, dev, halo="allgather", comm=comm)
    nnz_t = torch.tensor([len(aj)], dtype=torch.float64, device=dev)
    dist.all_reduce(nnz_t)
    slab = {"z0": z0, "z1": z1, "row_starts": row_starts, "nnz_local": len(aj), "nnz_global": int(nnz_t.item()),
            "csr": (ai, aj, aa)}
    return op, slab


def destroy_dist_operator(op):
    op.native.destroy()
    if op._twin is not None:
        op._twin[1].destroy()
        if op._twin[0] is not None:
            op._twin[0].destroy()
    op.A_d.destroy()
    if op.A_o is not None:
        op.A_o.destroy()


def weak_block(pkg, mpiaij, make_local, Gw, world, rank, dev, args, comm):
    """BASELINE configs[3] (beside the headline, not
    `value`): weak scaling, every rank a Gw^3-row z-slab of weak_grid(Gw, N)
    (N = 8, Gw = 300: the 600^3 grid), timed like the headline — K
    distributed MatMults between barriers, max over ranks — with both halo
    forms per rank."""
    import torch
    import torch.distributed as dist
    dims = weak_grid(Gw, world)
    op, slab = build_dist_operator(pkg, mpiaij, make_local, dims, world, rank, dev, comm)
    try:
        nat = op.native if args.halo == "allgather" else op.p2p_native()
        layout_local = op.A_d.info()["mult_layout_bytes"]
        stream = torch.cuda.current_stream()
        x = torch.from_numpy(pkg.splitmix_uniform(op.mloc, 42, int(slab["row_starts"][rank]))).to(dev)
        y = torch.empty(op.mloc, dtype=torch.float64, device=dev)
        for _ in range(args.warmup):
            nat.mult(x, y, stream)
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            nat.mult(x, y, stream)
        torch.cuda.synchronize()
        dist.barrier()
        el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        dt = float(el.item()) / args.steps
        forms = gather_forms(halo_forms(op, x, stream, max(args.steps, 20), rank, dev, op.mloc, slab["nnz_local"]),
                             world)
        lt = torch.tensor([float(layout_local)], dtype=torch.float64, device=dev)
        dist.all_reduce(lt)
        del x, y
    finally:
        destroy_dist_operator(op)
    n = dims[0] * dims[1] * dims[2]
    nbytes = pkg.algorithmic_bytes(n, n, slab["nnz_global"])
    return {"workload": f"{dims[0]}x{dims[1]}x{dims[2]} Poisson CSR, {slab['z1'] - slab['z0']}-plane z-slab "
                        f"({op.mloc} rows) per GPU (BASELINE configs[3] at N = 8)",
            "scaling": "weak", "value": round(nbytes / dt / 1e9, 2), "unit": "GB/s",
            "frac": round(float(lt.item()) / dt / 1e9 / (HBM_PEAK_GBS * world), 4),
            "ms_per_step": round(dt * 1e3, 4), "rows": n, "nnz": slab["nnz_global"], "halo": args.halo,
            "halo_forms": forms}


def layout_name(info) -> str:
    if info.get("row_templates"):
        return (f"row templates ({info['row_patterns']} distinct rows, offsets and values, a 1-byte id per row: "
                "the MatMult reads neither aj nor aa — a constant-coefficient stencil) — not CSR")
    if info.get("row_patterns"):
        return (f"row patterns ({info['row_patterns']} column - row offset lists, a 1-byte id per row, aa "
                "verbatim, no column per entry; cf. PETSc's inode rows) — not CSR")
    if info.get("column_codes"):
        return "column codes (a 16-bit code per entry in aj's place, aa verbatim) — not CSR"
    if info.get("gather_sorted"):
        return "gather-ordered copy of the CSR row blocks"
    return "CSR (PETSc's ai / aj / aa as stored)"


def leg_budgets(distributed):
    """Seconds each leg may need (a leg starts only with this much of the
    wall budget left). Measured on MI355X (profiles/r05, r06): the N = 1 legs
    take 2-25 s each; the distributed CG + GAMG set-up at 27 M rows per rank
    is the largest (profiles/r06)."""
    if distributed:
        return {"cg": 60, "weak": 150, "cg_gamg": 240, "cpu_baseline": 60}
    return {"cg": 60, "cg_gamg": 180, "host_vec": 60, "read_ceiling": 30, "flan_standin": 120, "pmc": 200,
            "pmc_skewed": 120, "pmc_fem_hex": 120, "cpu_baseline": 60}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no launcher: start the N ranks here, before anything touches the GPU
        raise SystemExit(launch_ranks(args.gpus, sys.argv[1:]))
    # Exactly one line reaches stdout: everything else any layer prints there
    # (gloo's "[Gloo] Rank 0 is connected ...", RCCL / HIP runtime notices)
    # goes to stderr, and the JSON line is written to the saved descriptor.
    sys.stdout.flush()
    line_fd = os.dup(1)
    os.dup2(2, 1)
    import torch
    import torch.distributed as dist

    pkg = importlib.import_module("petsc-openacc_amd")
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    t_start = time.perf_counter()

    def progress(msg):
        """A line per leg on stderr (every rank): a long multi-rank run keeps
        writing, and a stuck rank shows where it stopped."""
        print(f"bench[{rank}/{world}] {time.perf_counter() - t_start:7.1f} s: {msg}", file=sys.stderr, flush=True)
    if args.gpus != world:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs a GPU (the HIP path has no CPU fallback)")
    if args.rehearse_one_gpu:
        local_rank = 0
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    distributed = world > 1 or args.mpi
    csr_forced = args.layout == "csr"

    def set_layout(mat, csr):
        """csr: the MatMult reads PETSc's aj (row patterns and column codes
        off); else the library's automatic layout (or what --codes /
        --patterns / --templates force)."""
        mat.set_option("column_codes", 0 if csr else (-1 if args.codes is None else args.codes))
        mat.set_option("row_templates", -1 if args.templates is None else args.templates)
        mat.set_option("row_patterns", 0 if csr else (-1 if args.patterns is None else args.patterns))

    def configure(mat, csr=csr_forced):
        for opt, val in (("geometry", args.geometry), ("nt_loads", args.nt)):
            if val is not None:
                mat.set_option(opt, val)
        set_layout(mat, csr)
        return mat

    comm = None
    if distributed:
        from datetime import timedelta
        to = timedelta(seconds=args.comm_timeout)
        if args.rehearse_one_gpu:
            dist.init_process_group("gloo", timeout=to)
        else:
            dist.init_process_group("nccl", device_id=dev, timeout=to)
        # the library's own communicator (include/aijhip_mpi.h): RCCL, or the
        # host transport when the ranks share one GPU (RCCL refuses that)
        C = importlib.import_module("petsc-openacc_amd.comm")
        comm = (C.Comm.host(device=local_rank, timeout_s=args.comm_timeout) if args.rehearse_one_gpu
                else C.Comm.rccl(device=local_rank, timeout_s=args.comm_timeout))
        dist.barrier()
    legs = Legs(args.wall_budget, rank, world, distributed, dev, progress, line_fd)
    legs.arm()
    budget = leg_budgets(distributed)

    G = args.grid
    dims = (G, G, G)
    stream = torch.cuda.current_stream()
    t_setup = time.perf_counter()
    if distributed:
        from importlib import import_module
        mpiaij = import_module("petsc-openacc_amd.mpiaij")

        def make_local(a_i, a_j, a_a, ncols):
            return configure(pkg.SeqAIJHIP(a_i, a_j, a_a, ncols=ncols, device=local_rank, kernel=args.kernel))

        op, slab = build_dist_operator(pkg, mpiaij, make_local, dims, world, rank, dev, comm)
        z0, z1 = slab["z0"], slab["z1"]
        progress(f"operand {G}^3 strong-scaled, planes {z0}..{z1}")
        ai, aj, aa = slab.pop("csr")
        m_loc, nnz_loc, nnz_global = op.mloc, slab["nnz_local"], slab["nnz_global"]
        x_off = int(slab["row_starts"][rank])
        nat = op.native if args.halo == "allgather" else op.p2p_native()
        info = op.A_d.info()
        # what the timed launch moves: A_d's layout + A_o as CSR (its rows, ghosts)
        layout_bytes = info["mult_layout_bytes"] + (pkg.algorithmic_bytes(m_loc, m_loc, op.nz_o) - 4 * (m_loc + 1)
                                                     - 16 * m_loc + 8 * op.n_ghost if op.nz_o else 0)
    else:
        z0, z1 = 0, G
        progress(f"operand {G}^3")
        ai, aj, aa = pkg.poisson_csr(G)
        m_loc = len(ai) - 1
        nnz_loc = nnz_global = len(aj)
        x_off = 0
        A = configure(pkg.SeqAIJHIP(ai, aj, aa, ncols=m_loc, device=local_rank, kernel=args.kernel))
        info = A.info()
        layout_bytes = info["mult_layout_bytes"]
    planes = z1 - z0
    if args.x == "exact":
        _, x_h = pkg.poisson_vectors(G, G, G, z0, z1)
    else:
        x_h = pkg.splitmix_uniform(m_loc, 42, x_off)
    xd = torch.from_numpy(x_h).to(dev)
    yd = torch.empty(m_loc, dtype=torch.float64, device=dev)
    step = (lambda: nat.mult(xd, yd, stream)) if distributed else (lambda: A.mult(xd, yd, stream))
    torch.cuda.synchronize()
    t_setup = time.perf_counter() - t_setup
    bytes_local = pkg.algorithmic_bytes(m_loc, m_loc, nnz_loc)

    progress("operator ready; warm-up")
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    progress("timed steps")

    # per-launch HIP events on the stream the SpMV kernel runs on
    K = args.steps
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(K):
        ev[i][0].record(stream)
        step()
        ev[i][1].record(stream)
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    el_t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if distributed:
        dist.all_reduce(el_t, op=dist.ReduceOp.MAX)
    elapsed = float(el_t.item())
    launch_ms = np.array([a.elapsed_time(b) for a, b in ev])

    # roofline sample: at least --roofline-reps launches (SURVEY §8d asks
    # for the median of >= 50), the K timed ones plus more if K is smaller
    extra = max(0, args.roofline_reps - K)
    if extra:
        launch_ms = np.concatenate([launch_ms, np.array(launch_times(step, stream, extra)) / 1e3])

    # correctness spot-check of the timed output against a fresh multiply
    y_chk = yd.clone()
    step()
    torch.cuda.synchronize()
    stable = bool(torch.equal(y_chk, yd))
    out = headline_line(world=world, dims=dims, nnz_global=nnz_global, K=K, warmup=args.warmup, elapsed_s=elapsed,
                        launch_us=launch_ms * 1e3, layout_bytes=layout_bytes, info=info, distributed=distributed,
                        halo=args.halo, x_kind=args.x, planes=planes)
    out["result_stable"] = stable
    out["setup_s"] = round(t_setup, 2)
    legs.headline_done = True
    if rank == 0:
        legs.out = out

    forms = None
    if distributed:
        # Evidence the exchange hides behind the diagonal block: both halo
        # forms against the same launches of A_d alone, per rank
        progress("halo forms")
        forms = gather_forms(halo_forms(op, xd, stream, K, rank, dev, m_loc, nnz_loc), world)
        out["aggregate_frac"] = round(out["value"] / (HBM_PEAK_GBS * world), 4)
        out["distributed"] = distributed_block(world, dist.get_backend(), comm.info(), args.comm_timeout,
                                               forms[args.halo]["ranks"])
        out["distributed"]["halo_forms"] = forms
        if args.rehearse_one_gpu:
            out["rehearsal"] = f"{world} ranks sharing cuda:0 over gloo: control flow only, not a scaling number"

    # The library's automatic layout (row patterns for the stencil: no aj)
    # timed beside the CSR headline in the same run, on ITS bytes; its y must
    # be the headline's bits. It is not a CSR measurement and never `value`.
    if not distributed and csr_forced:
        def effective_layout():
            set_layout(A, False)
            inf = A.info()
            if inf["mult_layout_bytes"] == bytes_local and not inf.get("row_patterns") and \
                    not inf.get("column_codes"):
                return {"layout": layout_name(inf), "note": "the automatic layout is CSR here"}
            y_e = torch.empty_like(yd)
            for _ in range(5):
                A.mult(xd, y_e, stream)
            mean, med, mn = time_launches(lambda: A.mult(xd, y_e, stream), stream, max(args.roofline_reps, 50))
            same = bool(torch.equal(y_e, y_chk))
            del y_e
            lb = inf["mult_layout_bytes"]
            return {"layout": layout_name(inf), "bytes_per_launch": lb,
                    "us_mean": round(mean, 2), "us_median": round(med, 2), "us_min": round(mn, 2),
                    "achieved": round(lb / (mean * 1e-6) / 1e9, 1),
                    "frac": round(lb / (mean * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
                    "csr_equivalent_GBs": round(bytes_local / (mean * 1e-6) / 1e9, 1),
                    "bitwise_equal_csr": same,
                    "note": "NOT a CSR SpMV: this layout does not read aj (the bytes it moves are bytes_per_launch; "
                            "frac is on those). csr_equivalent_GBs = the CSR bytes over the same time, for "
                            "comparison only. The CG / CG+GAMG legs below run on this layout."}
        out["effective"] = effective_layout()

    # the solver legs run on the automatic layout (what a caller gets)
    if distributed and csr_forced:
        set_layout(op.A_d, False)
    elif not distributed:
        set_layout(A, False)
    solver_layout = layout_name((op.A_d if distributed else A).info())

    def single_cg():
        ksp = importlib.import_module("petsc-openacc_amd.ksp")
        res = ksp.bench_cg(pkg, A, G, G, G, dev, iters=args.cg_iters)
        res["layout"] = solver_layout
        if not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_cg_baseline(ai, aj, aa, pkg, G, G, G)
        return res

    def distributed_cg():
        # row-partitioned CG+Jacobi: dots all-reduced over RCCL
        # aijhip_kspmpi: scalar steps on the device, RCCL all-reduces of device
        # doubles on the compute stream, host polls every 8 iterations
        rhs_h, _ = pkg.poisson_vectors(G, G, G, z0, z1)
        b = torch.from_numpy(rhs_h).to(dev)
        xs = torch.zeros_like(b)
        cgm = C.KSPCGMPINative(nat, rtol=0.0, atol=0.0, max_it=5)
        cgm.solve(b, xs)  # warm-up
        cgm.set_tolerances(0.0, 0.0, 1e5, args.cg_iters)
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        cgm.solve(b, xs)
        torch.cuda.synchronize()
        el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        dt = float(el.item())
        its = cgm.its
        res = {"iters": its, "seconds": round(dt, 4), "iters_per_s": round(its / dt, 2),
               "ms_per_iter": round(dt / its * 1e3, 4), "pc": "jacobi (bjacobi+jacobi per rank)",
               "reductions": "2 all-reduces per iteration (" + ("host transport over gloo" if args.rehearse_one_gpu
                                                                 else "RCCL, device doubles") +
                             ("; skipped at one rank" if world == 1 else "") + ")",
               "host_syncs": cgm.host_syncs, "halo": args.halo, "solver": "aijhip_kspmpi (native)",
               "layout": solver_layout,
               "workload": f"{G}^3 Poisson, {planes}-plane z-slab on rank 0 of {world}"}
        cgm.destroy()
        return res

    def distributed_cg_gamg():
        # CG + PCGAMG across the ranks (csrc/gamg_mpi.hip: one distributed
        # hierarchy, as PETSc's agg GAMG on MPIAIJ), the reference's
        # tolerances, from x = 0; the hierarchy's level halos are p2p plans
        rhs_h, exact_h = pkg.poisson_vectors(G, G, G, z0, z1)
        b = torch.from_numpy(rhs_h).to(dev)
        xs = torch.zeros_like(b)
        kg = C.KSPCGMPINative(op.p2p_native(), rtol=1e-14, atol=1e-12, max_it=10000, pc="gamg")
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        kg.solve(b, xs)  # first solve: includes the GAMG set-up
        torch.cuda.synchronize()
        t_first = time.perf_counter() - t0
        xs.zero_()
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        kg.solve(b, xs)
        torch.cuda.synchronize()
        t_solve = time.perf_counter() - t0
        rows_l, nnz_l = kg.pc_levels()  # collective
        syncs = kg.host_syncs
        tt = torch.tensor([t_first, t_solve], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        err = torch.tensor([float((xs.cpu() - torch.from_numpy(exact_h)).abs().max())], dtype=torch.float64,
                           device=dev)
        dist.all_reduce(err, op=dist.ReduceOp.MAX)
        res = {"its": kg.its, "reason": kg.reason, "rnorm": kg.rnorm, "max_err": float(err.item()),
               "setup_s": round(float(tt[0].item()) - float(tt[1].item()), 3), "solve_s": round(float(tt[1].item()), 4),
               "time_to_solution_s": round(float(tt[0].item()), 3),
               "ms_per_iter": round(float(tt[1].item()) / max(kg.its, 1) * 1e3, 3), "host_syncs": syncs,
               "levels": [{"rows": int(r), "nnz": int(z)} for r, z in zip(rows_l, nnz_l)],
               "pc": ("PCGAMG across ranks (aggregates per rank, P and Galerkin products over the MPIAIJ "
                      "operator, csrc/gamg_mpi.hip)" if world > 1 or os.environ.get("AIJHIP_GAMG_DIST") == "1"
                      else "PCGAMG (single-GPU set-up)"),
               "options": "rtol 1e-14 atol 1e-12", "workload": f"{G}^3 Poisson over {world} GPU(s)",
               "layout": solver_layout, "halo": "p2p (the p2p twin of the operator; shares A_d)"}
        kg.destroy()
        return res

    def single_cg_gamg():
        ksp = importlib.import_module("petsc-openacc_amd.ksp")
        res = ksp.bench_cg_gamg(pkg, A, G, G, G, dev)
        res["layout"] = solver_layout
        res["hierarchy"] = ("PETSc 3.7 agg restated (the default since round 5): MIS of the squared graph "
                            "(finest level) in a hashed random order, smoothAggs, then MIS of the graph; emax "
                            "from CG's Lanczos tridiagonal (coarsen 1, eig_ksp 1)")
        # the greedy hierarchy beside it (the default through round 4; VERDICT
        # r04 item 5: both measured, the faster is the default)
        greedy = ksp.bench_cg_gamg(pkg, A, G, G, G, dev, gamg=dict(coarsen=0, eig_ksp=0), light=True)
        greedy["hierarchy"] = "greedy aggregation in natural order, power-iteration emax (coarsen 0, eig_ksp 0)"
        res["greedy_hierarchy"] = greedy
        if "error" not in greedy:  # like for like: each hierarchy's second set-up in the process + its solve
            res["hierarchy_comparison"] = {
                "default_mis_s": round(res["setup_again_s"] + res["solve_s"], 4),
                "greedy_s": round(greedy["setup_again_s"] + greedy["solve_s"], 4),
                "note": "set-up again (warm: the first set-up of the process also pays one-time costs, and the "
                        "greedy leg runs after the default one) + solve, seconds"}
        print(f"bench: CG+GAMG {res['its']} its, solve {res['solve_s']} s, set-up {res['setup_s']} s",
              file=sys.stderr, flush=True)
        # BASELINE configs[0] (100^3) on the device as well, beside its 1-core host solve
        s_ai, s_aj, s_aa = pkg.poisson_csr(100)
        with pkg.SeqAIJHIP(s_ai, s_aj, s_aa, device=local_rank) as A100:
            small = ksp.bench_cg_gamg(pkg, A100, 100, 100, 100, dev)
        res["configs0_device"] = {k: small[k] for k in ("its", "reason", "max_err", "setup_s", "solve_s",
                                                        "time_to_solution_s")}
        if not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_cg_gamg_baseline(ai, aj, aa, pkg, G, G, G)
        return res

    if not args.no_cg:
        legs.run("cg", budget["cg"], distributed_cg if distributed else single_cg)
    if distributed and world > 1 and not args.no_weak:
        legs.run("weak", budget["weak"],
                 lambda: weak_block(pkg, mpiaij, make_local, args.weak_grid or G, world, rank, dev, args, comm))
    if not args.no_gamg:
        legs.run("cg_gamg", budget["cg_gamg"], distributed_cg_gamg if distributed else single_cg_gamg)
    ceiling = flan = live_pmc = None
    if not distributed:
        if not args.no_host_vec:
            legs.run("host_vec", budget["host_vec"], lambda: host_vec_mult(A, x_h))
        ceiling = legs.run("read_ceiling", budget["read_ceiling"], lambda: read_ceiling(bytes_local, dev))
        out.pop("read_ceiling", None)
        if not args.no_flan:
            flan = legs.run("flan_standin", budget["flan_standin"],
                            lambda: flan_standins(pkg, dev, max(args.roofline_reps, 50), not args.no_cpu_baseline))
        under_profiler = any(k.startswith("ROCPROF") for k in os.environ)  # (never nest a profiler)
        if rank == 0 and not args.no_pmc and not args.no_cpu_baseline and not under_profiler:
            progress("roofline.traffic: two rocprofv3 --pmc passes of the headline kernel")
            live_pmc = legs.run("pmc", budget["pmc"], lambda: live_pmc_traffic(G))
            out.pop("pmc", None)
            if isinstance(flan, dict) and "error" not in flan:  # the stand-ins' default MatMult
                for name in ("skewed", "fem_hex"):
                    if isinstance(flan.get(name), dict) and "stream" in flan[name]:
                        t = legs.run(f"pmc_{name}", budget[f"pmc_{name}"],
                                     lambda n=name: live_pmc_traffic(G, case=n, opts=(), its=10))
                        out.pop(f"pmc_{name}", None)
                        rec = flan[name]["stream"]
                        if isinstance(t, tuple) and t[0] is not None:
                            rec["traffic"], rec["traffic_detail"] = t
                            rec["traffic_vs_layout_bytes"] = round(t[0] / rec["layout_bytes"], 4)
                        else:
                            rec["traffic"] = None
                            rec["traffic_detail"] = {"live_pmc_failed": str(t[1] if isinstance(t, tuple) else t)}

    progress("done; writing the line")
    if distributed:
        dist.barrier()
    if rank == 0 and not distributed:
        r = out["roofline"]
        block = out["config"]["block"]
        r["traffic"], r["traffic_source"] = pmc_traffic(G ** 3, nnz_global, block)
        if isinstance(live_pmc, tuple) and live_pmc[0] is not None and not info.get("row_patterns") \
                and not info.get("column_codes"):
            r["traffic"], r["traffic_detail"] = live_pmc
            r["traffic_source"] = ("this run: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (one counter group "
                                   "each) of tools/prof_case.py poisson in the CSR layout, gfx950-corrected "
                                   "(2 x FETCH_SIZE KiB + WRITE_SIZE KiB), mean over the kernel's dispatches")
        elif live_pmc is not None:
            r["traffic_detail"] = {"live_pmc_failed": str(live_pmc[1] if isinstance(live_pmc, tuple) else live_pmc)}
        if isinstance(ceiling, dict) and "error" not in ceiling:  # same-run flat reads of the same bytes
            achieved = r["achieved"]
            r["ceiling_flat_read"] = {
                "GBs": ceiling[0][0], "us": ceiling[0][1], "frac_of_ceiling": round(achieved / ceiling[0][0], 4),
                "probe": "aijhip_read_probe mode 0: the SpMV's CSR byte count read once, non-temporal 16-B loads, "
                         "512-lane workgroups of two loads per lane (the fastest shape, tools/read_sweep.hip); "
                         "frac_of_ceiling = roofline.achieved / this rate",
                "stream_shape_read": {"GBs": ceiling[1][0], "us": ceiling[1][1],
                                      "frac": round(achieved / ceiling[1][0], 4),
                                      "probe": "mode 1: plain loads, four per lane (the STREAM kernel's shape)"}}
    # the host baselines last: at N > 1 the other ranks are done with the GPU
    # by now, and rank 0 times the oracle on the whole G^3 operand
    if rank == 0 and not args.no_cpu_baseline:
        del ai, aj, aa
        base = legs.run("cpu_baseline", budget["cpu_baseline"],
                        lambda: cpu_spmv_baselines(pkg, G, args.cpu_seconds), collective=False)
        if isinstance(base, tuple):
            out["cpu_baseline"], out["cpu_baseline_all_cores"] = base
    if rank == 0:
        out["budget"] = legs.summary()
        legs.emit(out)
    legs.disarm()
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
