#!/usr/bin/env python3
"""What the release scope of the library's fork / join events costs
(AIJHIP_EVENT_FENCE = system | device | none, read when an operator creates
them). One process, one GPU, interleaved rounds, a device delay queued ahead
of every round (device-only timing, tools/halo_probe.py).

--per-process: ONE fence mode per process (the environment's), one operator
of each kind — several operators each with its own exchange / side stream in
one process share HIP's hardware queues (GPU_MAX_HW_QUEUES, 4 by default)
round-robin, so a stream may land on the compute stream's queue and
serialise behind it (r05d's in-process comparison was confounded by that).

  halo   the one-rank RCCL operators of tools/halo_probe.py: the all-gather
         operator with no ghosts (fork + count-1 collective + join) and the
         self-halo p2p operator (both boundary planes as ghosts), each built
         under every fence mode, against the diagonal block alone;
  skewed the Flan_1565 skewed stand-in: hub segments on the side stream
         (fork / join per MatMult) under every fence mode, and serial.

Every variant's y is compared bit for bit with its reference.

    python3 tools/fence_probe.py [--planes 38 300] [--reps 100]
"""
import argparse
import importlib
import json
import os
import socket
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tools"))
MODES = ("system", "device", "none")


def timed(variants, reps, stream, VL, preload_us):
    import torch
    ev = {k: [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
          for k in variants}
    for f in variants.values():
        f()
    torch.cuda.synchronize()
    for i in range(reps):
        VL.aijhip_delay_probe(preload_us, stream.cuda_stream)
        for k, f in variants.items():
            a, b = ev[k][i]
            a.record(stream)
            f()
            b.record(stream)
    torch.cuda.synchronize()
    return {k: np.array([a.elapsed_time(b) for a, b in ev[k]]) * 1e3 for k in variants}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", type=int, default=300)
    ap.add_argument("--planes", type=int, nargs="+", default=[38, 300])
    ap.add_argument("--reps", type=int, default=100)
    ap.add_argument("--no-skewed", action="store_true")
    ap.add_argument("--per-process", action="store_true",
                    help="only the fence mode of AIJHIP_EVENT_FENCE (default system), one operator of each kind")
    args = ap.parse_args()
    import torch
    import torch.distributed as dist
    from halo_probe import free_port, split_self
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", str(free_port()))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=0, world_size=1)
    pkg = importlib.import_module("petsc-openacc_amd")
    C = importlib.import_module("petsc-openacc_amd.comm")
    VL = importlib.import_module("petsc-openacc_amd.ksp")._veclib()
    comm = C.Comm.rccl(device=0, timeout_s=60)
    stream = torch.cuda.current_stream()
    dev = torch.device("cuda:0")
    G = args.grid
    modes = MODES
    if args.per_process:
        modes = (os.environ.get("AIJHIP_EVENT_FENCE", "system"),)

    def local(a_i, a_j, a_a, ncols):
        A = pkg.SeqAIJHIP(a_i, a_j, a_a, ncols=ncols)
        A.set_option("column_codes", 0)
        A.set_option("row_patterns", 0)
        return A

    for planes in args.planes:
        ai, aj, aa = pkg.poisson_csr(G, G, planes)
        m = len(ai) - 1
        x = torch.from_numpy(pkg.splitmix_uniform(m, 42)).to(dev)
        Ad = local(ai, aj, aa, m)
        Gh = np.concatenate([np.arange(0, G * G), np.arange(m - G * G, m)])
        (dai, daj, daa), (oai, oaj, oaa) = split_self(ai, aj, aa, Gh)
        Ad_s = local(dai, daj, daa, m)
        Ao_s = local(oai, oaj, oaa, len(Gh))
        ops, keep = {}, []
        env0 = os.environ.get("AIJHIP_EVENT_FENCE")
        for mode in modes:
            os.environ["AIJHIP_EVENT_FENCE"] = mode
            Ao0 = None
            ops["ag_empty_" + mode] = C.NativeMPIAIJ(comm, Ad, Ao0, "allgather", [(-1, np.zeros(1, np.int64))], [], 1)
            ops["p2p_self_" + mode] = C.NativeMPIAIJ(comm, Ad_s, Ao_s, "p2p", [(0, Gh)], [(0, 0, len(Gh))], 0)
        os.environ.pop("AIJHIP_EVENT_FENCE", None)
        if env0 is not None:
            os.environ["AIJHIP_EVENT_FENCE"] = env0
        ys = {k: torch.empty(m, dtype=torch.float64, device=dev) for k in list(ops) + ["diag", "diag_s"]}
        variants = {"diag": lambda: Ad.mult(x, ys["diag"], stream), "diag_s": lambda: Ad_s.mult(x, ys["diag_s"], stream)}
        for k, op in ops.items():
            variants[k] = (lambda o, y: lambda: o.mult(x, y, stream))(op, ys[k])
        us = timed(variants, args.reps, stream, VL, 1500.0 if planes < 100 else 8000.0)
        rec = {"case": "halo", "grid": G, "planes": planes, "rows": m, "reps": args.reps}
        for k, v in us.items():
            base = "diag" if k.startswith("ag_empty") or k == "diag" else "diag_s"
            rec[k] = {"us_median": round(float(np.median(v)), 2),
                      "minus_" + base + "_us_median": round(float(np.median(v - us[base])), 2)}
        ref_p2p = "p2p_self_" + modes[0]
        rec["bitwise"] = {k: bool(torch.equal(ys[k], ys[ref_p2p] if k.startswith("p2p") else ys["diag"]))
                          for k in ops}
        rec["hw_queues"] = os.environ.get("GPU_MAX_HW_QUEUES")
        print(json.dumps(rec), flush=True)
        for op in ops.values():
            op.destroy()
        for A in (Ad, Ad_s, Ao_s):
            A.destroy()
        del x, ys
        torch.cuda.empty_cache()
    if not args.no_skewed:
        ai, aj, aa = pkg.skewed_csr()
        m = len(ai) - 1
        x = torch.from_numpy(pkg.splitmix_uniform(m, 42)).to(dev)
        mats = {}
        env0 = os.environ.get("AIJHIP_EVENT_FENCE")
        for mode in modes:
            os.environ["AIJHIP_EVENT_FENCE"] = mode
            mats["stream_" + mode] = pkg.SeqAIJHIP(ai, aj, aa, ncols=m, kernel="stream")
        os.environ.pop("AIJHIP_EVENT_FENCE", None)
        if env0 is not None:
            os.environ["AIJHIP_EVENT_FENCE"] = env0
        mats["serial"] = pkg.SeqAIJHIP(ai, aj, aa, ncols=m, kernel="stream")
        mats["serial"].set_option("long_overlap", 0)
        ys = {k: torch.empty(m, dtype=torch.float64, device=dev) for k in mats}
        variants = {k: (lambda A, y: lambda: A.mult(x, y, stream))(A, ys[k]) for k, A in mats.items()}
        us = timed(variants, args.reps, stream, VL, 3000.0)
        rec = {"case": "skewed", "rows": m, "nnz": len(aj), "bytes": mats["serial"].info()["mult_layout_bytes"]}
        for k, v in us.items():
            rec[k] = {"us_median": round(float(np.median(v)), 2), "us_min": round(float(v.min()), 2)}
        rec["bitwise"] = {k: bool(torch.equal(ys[k], ys["serial"])) for k in mats}
        rec["hw_queues"] = os.environ.get("GPU_MAX_HW_QUEUES")
        print(json.dumps(rec), flush=True)
        for A in mats.values():
            A.destroy()
    comm.destroy()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
