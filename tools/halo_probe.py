#!/usr/bin/env python3
"""Where does the distributed MatMult's fixed cost go at one rank (VERDICT r04
item 1)?  One process, one GPU, a real RCCL communicator of one rank (a rank
may send to and receive from itself; tests/test_rccl_selfhalo_gpu.py).

Variants, timed INTERLEAVED (one launch of each in turn, `--reps` rounds, HIP
events on the compute stream around every launch) so box drift and clock
ramps hit every variant alike; each variant's cost is reported as the median
of its per-round difference to the diagonal block launched in the same round:

  diag        A_d.mult alone (the operand's slab, --planes of --grid^2 rows)
  forkjoin    A_d.mult with an empty fork/join to a second stream around it
              (torch events: what the halo's two event edges cost by themselves)
  rec_only / fork_only / join_done / join_fresh   its parts: an event record
              on the compute stream; the fork alone; a wait on an event long
              complete; a wait on one the idle side stream records now
  ag_empty    the MPIAIJ all-gather operator bench.py --mpi builds at N = 1
              (no ghosts; the count-0 ncclAllGather on the exchange stream)
  p2p_empty   its p2p twin (no ghosts: no exchange at all)
  p2p_self    a self-halo: the slab's two boundary planes are "ghosts" sent by
              ncclSend/ncclRecv to this rank (A_o holds their entries)
  ag_self     the same ghost set through ncclAllGather
  p2p_selfd   p2p_self's own A_d alone (p2p_self / ag_self are differenced to it)

Two timings per variant:
  device     --preload-us of device delay (aijhip_delay_probe) queued ahead
             of every round, so the round is fully enqueued before it runs and
             the events time device work only (fork / join packets included,
             host launch overhead excluded);
  pipelined  --burst back-to-back launches of the variant between two events
             (no preload): per-launch time when the host feeds the queue —
             host-bound if the host's enqueue is slower than the device;
             host_us = the host's wall time per call in that burst.

Prints one JSON line per --planes value.

    python3 tools/halo_probe.py --grid 300 --planes 300 38 --reps 200
"""
from __future__ import annotations

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


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def split_self(ai, aj, aa, G):
    """A_d: the entries outside columns G (diagonal kept); A_o: the entries in
    columns G (off the diagonal), columns renumbered to their position in G."""
    m = len(ai) - 1
    pos = np.full(m, -1, np.int64)
    pos[G] = np.arange(len(G))
    rows = np.repeat(np.arange(m), np.diff(ai))
    off = (pos[aj] >= 0) & (aj != rows)
    d_cnt = np.bincount(rows[~off], minlength=m)
    o_cnt = np.bincount(rows[off], minlength=m)
    dai = np.concatenate([[0], np.cumsum(d_cnt)]).astype(np.int32)
    oai = np.concatenate([[0], np.cumsum(o_cnt)]).astype(np.int32)
    return (dai, aj[~off].astype(np.int32), aa[~off]), (oai, pos[aj[off]].astype(np.int32), aa[off])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", type=int, default=300)
    ap.add_argument("--planes", type=int, nargs="+", default=[300, 38])
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--layout", default="csr", choices=["csr", "auto"])
    ap.add_argument("--only", default=None, help="comma-separated variant subset (trace runs)")
    ap.add_argument("--preload-us", type=float, default=1500.0)
    ap.add_argument("--burst", type=int, default=100)
    ap.add_argument("--graphs", type=int, default=0,
                    help="also time HIP-graph replays of diag / p2p_self / ag_self (torch's capture_end segfaulted "
                         "on them in round 5, profiles/r05/c/graph_diag.err)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", str(free_port()))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=0, world_size=1)
    pkg = importlib.import_module("petsc-openacc_amd")
    C = importlib.import_module("petsc-openacc_amd.comm")
    mpiaij = importlib.import_module("petsc-openacc_amd.mpiaij")
    dev = torch.device("cuda:0")
    comm = C.Comm.rccl(device=0, timeout_s=60)
    K = importlib.import_module("petsc-openacc_amd.ksp")
    VL = K._veclib()
    import time
    stream = torch.cuda.current_stream()
    G = args.grid

    def local(a_i, a_j, a_a, ncols):
        A = pkg.SeqAIJHIP(a_i, a_j, a_a, ncols=ncols)
        if args.layout == "csr":
            A.set_option("column_codes", 0)
            A.set_option("row_patterns", 0)
        return A

    for planes in args.planes:
        ai, aj, aa = pkg.poisson_csr(G, G, planes)
        m = len(ai) - 1
        x = torch.from_numpy(pkg.splitmix_uniform(m, 42)).to(dev)
        ys = {}
        # the bench's N = 1 operator (all-gather native + p2p twin, no ghosts)
        op = mpiaij.MPIAIJ(ai, aj, aa, np.array([0, m], np.int64), local, pkg.split_rows, dev, halo="allgather",
                           comm=comm)
        p2p0 = op.p2p_native()
        # the self-halo: both boundary planes are ghosts
        Gh = np.concatenate([np.arange(0, G * G), np.arange(m - G * G, m)])
        (dai, daj, daa), (oai, oaj, oaa) = split_self(ai, aj, aa, Gh)
        Ad_s = local(dai, daj, daa, m)
        Ao_s = local(oai, oaj, oaa, len(Gh))
        p2p_s = C.NativeMPIAIJ(comm, Ad_s, Ao_s, "p2p", [(0, Gh)], [(0, 0, len(Gh))], 0)
        Ao_g = local(oai, oaj, oaa, len(Gh))
        ag_s = C.NativeMPIAIJ(comm, Ad_s, Ao_g, "allgather", [(-1, Gh)], [], len(Gh))
        side = torch.cuda.Stream()
        e_fork, e_join = torch.cuda.Event(), torch.cuda.Event()

        def forkjoin(y):
            e_fork.record(stream)
            side.wait_event(e_fork)
            op.A_d.mult(x, y, stream)
            e_join.record(side)
            stream.wait_event(e_join)

        e_rec, e_pre = torch.cuda.Event(), torch.cuda.Event()
        e_pre.record(side)  # recorded once on the idle side stream: complete
        torch.cuda.synchronize()

        def rec_only(y):  # an event recorded on the compute stream, nobody waits
            e_rec.record(stream)
            op.A_d.mult(x, y, stream)

        def fork_only(y):
            e_fork.record(stream)
            side.wait_event(e_fork)
            op.A_d.mult(x, y, stream)

        def join_done(y):  # the compute stream waits on an event long complete
            op.A_d.mult(x, y, stream)
            stream.wait_event(e_pre)

        def join_fresh(y):  # ... on one the idle side stream records now
            op.A_d.mult(x, y, stream)
            e_join.record(side)
            stream.wait_event(e_join)

        variants = {
            "diag": lambda y: op.A_d.mult(x, y, stream),
            "forkjoin": forkjoin,
            "rec_only": rec_only,
            "fork_only": fork_only,
            "join_done": join_done,
            "join_fresh": join_fresh,
            "ag_empty": lambda y: op.native.mult(x, y, stream),
            "p2p_empty": lambda y: p2p0.mult(x, y, stream),
            "p2p_selfd": lambda y: Ad_s.mult(x, y, stream),
            "p2p_self": lambda y: p2p_s.mult(x, y, stream),
            "ag_self": lambda y: ag_s.mult(x, y, stream),
        }
        # the same launches captured once into a HIP graph and replayed
        # (hipGraphLaunch: one host call instead of RCCL's enqueue per call)
        graphs, gerr = {}, {}
        if args.graphs:
            for gname, base in (("diag", "diag"), ("p2p_self", "p2p_self"), ("ag_self", "ag_self")):
                yg = torch.empty(m, dtype=torch.float64, device=dev)
                try:
                    g = torch.cuda.CUDAGraph()
                    gs = torch.cuda.Stream()
                    gs.wait_stream(stream)
                    with torch.cuda.stream(gs):
                        fn = {"diag": lambda y, st: op.A_d.mult(x, y, st),
                              "p2p_self": lambda y, st: p2p_s.mult(x, y, st),
                              "ag_self": lambda y, st: ag_s.mult(x, y, st)}[base]
                        fn(yg, gs)  # warm-up outside the capture
                        torch.cuda.synchronize()
                        with torch.cuda.graph(g, stream=gs):
                            fn(yg, torch.cuda.current_stream())
                    torch.cuda.synchronize()
                    graphs[gname + "_graph"] = (g, yg)
                except Exception as e:  # noqa: BLE001
                    gerr[gname + "_graph"] = repr(e)[:300]
                    torch.cuda.synchronize()
            for k, (g, yg) in graphs.items():
                variants[k] = (lambda gg: lambda y: gg.replay())(g)
        if args.only:
            keep = set(args.only.split(","))
            variants = {k: v for k, v in variants.items() if k in keep}
        for k in variants:
            ys[k] = torch.empty(m, dtype=torch.float64, device=dev)
        for _ in range(5):
            for k, f in variants.items():
                f(ys[k])
        torch.cuda.synchronize()
        R = args.reps
        ev = {k: [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(R)]
              for k in variants}
        for i in range(R):
            VL.aijhip_delay_probe(args.preload_us, stream.cuda_stream)
            for k, f in variants.items():
                a, b = ev[k][i]
                a.record(stream)
                f(ys[k])
                b.record(stream)
        torch.cuda.synchronize()
        pipe = {}
        for k, f in variants.items():
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            a.record(stream)
            t0 = time.perf_counter()
            for _ in range(args.burst):
                f(ys[k])
            th = time.perf_counter() - t0
            b.record(stream)
            torch.cuda.synchronize()
            pipe[k] = (a.elapsed_time(b) * 1e3 / args.burst, th * 1e6 / args.burst)
        us = {k: np.array([a.elapsed_time(b) for a, b in ev[k]]) * 1e3 for k in variants}
        rec = {"grid": G, "planes": planes, "rows": m, "reps": R, "layout": args.layout,
               "preload_us": args.preload_us, "burst": args.burst,
               "ghosts_self": int(len(Gh))}
        for k in variants:
            rec[k] = {"us_median": round(float(np.median(us[k])), 2), "us_mean": round(float(np.mean(us[k])), 2),
                      "pipelined_us": round(pipe[k][0], 2), "host_us": round(pipe[k][1], 2)}
        for k, base in (("forkjoin", "diag"), ("rec_only", "diag"), ("fork_only", "diag"), ("join_done", "diag"),
                        ("join_fresh", "diag"), ("ag_empty", "diag"), ("p2p_empty", "diag"),
                        ("p2p_self", "p2p_selfd"), ("ag_self", "p2p_selfd")):
            if k in us and base in us:
                d = us[k] - us[base]
                rec[k]["minus_" + base + "_us_median"] = round(float(np.median(d)), 2)
                rec[k]["minus_" + base + "_us_iqr"] = [round(float(np.percentile(d, 25)), 2),
                                                      round(float(np.percentile(d, 75)), 2)]
        for k, base in (("diag_graph", "diag"), ("p2p_self_graph", "p2p_self"), ("ag_self_graph", "ag_self")):
            if k in us and base in us:
                rec[k]["minus_" + base + "_us_median"] = round(float(np.median(us[k] - us[base])), 2)
        if gerr:
            rec["graph_errors"] = gerr
        for k, (g, yg) in graphs.items():
            base = k[: -len("_graph")]
            if base in ys:
                rec[k]["bitwise_equal_" + base] = bool(torch.equal(yg, ys[base]))
        # bitwise: every distributed form against its diagonal block + A_o
        if "p2p_self" in ys and "ag_self" in ys:
            rec["self_forms_bitwise_equal"] = bool(torch.equal(ys["p2p_self"], ys["ag_self"]))
        if "diag" in ys and "ag_empty" in ys:
            rec["empty_forms_bitwise_equal"] = bool(torch.equal(ys["diag"], ys["ag_empty"]))
        print(json.dumps(rec), flush=True)
        for h in (p2p_s, ag_s):
            h.destroy()
        for A in (Ad_s, Ao_s, Ao_g):
            A.destroy()
        op.native.destroy()
        if op._twin is not None:
            op._twin[1].destroy()
            if op._twin[0] is not None:
                op._twin[0].destroy()
        op.A_d.destroy()
        if op.A_o is not None:
            op.A_o.destroy()
        del x, ys
    comm.destroy()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
