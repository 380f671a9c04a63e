#!/usr/bin/env python3
"""CG iterations of the distributed GAMG (pc gamg) and of block Jacobi + GAMG
(pc bjacobi_gamg) for one global Poisson grid split into k z-slabs, the k
ranks sharing cuda:0 over the host transport (a control-flow and iteration
rehearsal: one GPU, not a timing of the multi-GPU path). Strong partition:
the same global problem at every k, so the counts compare directly with the
single-GPU solve's.

    python tools/gamg_its_ranks.py --grid 300 300 300 --ranks 2 4
"""
from __future__ import annotations

import argparse
import importlib
import json
import os
import socket
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def worker(rank, world, port, dims, pcs, q):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        pkg = importlib.import_module("petsc-openacc_amd")
        mp_mod = importlib.import_module("petsc-openacc_amd.mpiaij")
        C = importlib.import_module("petsc-openacc_amd.comm")
        dev = torch.device("cuda:0")
        nx, ny, nz = dims
        bounds = [mp_mod.slab_bounds(nz, world, r) for r in range(world)]
        row_starts = np.array([b[0] * nx * ny for b in bounds] + [nx * ny * nz], dtype=np.int64)
        z0, z1 = bounds[rank]
        ai, aj, aa = pkg.poisson_csr(nx, ny, nz, z0, z1)
        comm = C.Comm.host(device=0, timeout_s=600)
        op = mp_mod.MPIAIJ(ai, aj, aa, row_starts, lambda a, b, c, n: pkg.SeqAIJHIP(a, b, c, ncols=n),
                           pkg.split_rows, dev, comm=comm)
        del ai, aj, aa
        rhs, exact = pkg.poisson_vectors(nx, ny, nz, z0, z1)
        b = torch.from_numpy(rhs).to(dev)
        out = {}
        for pc in pcs:
            x = torch.zeros_like(b)
            with C.KSPCGMPINative(op.native, rtol=1e-14, atol=1e-12, max_it=2000, pc=pc) as k:
                t0 = time.perf_counter()
                k.solve(b, x)
                torch.cuda.synchronize()
                t = time.perf_counter() - t0
                rows, _ = k.pc_levels()
                err = float(np.abs(x.cpu().numpy() - exact).max())
                out[pc] = {"its": k.its, "reason": k.reason, "levels": rows, "seconds_incl_setup": round(t, 2),
                           "setup_s": round(k.setup_seconds, 2), "max_err": err}
        q.put((rank, out))
    except Exception as e:  # noqa: BLE001
        q.put((rank, {"error": repr(e)}))
    finally:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", type=int, nargs=3, default=[300, 300, 300])
    ap.add_argument("--ranks", type=int, nargs="+", default=[2, 4])
    ap.add_argument("--pcs", nargs="+", default=["gamg", "bjacobi_gamg"])
    args = ap.parse_args()
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    for k in args.ranks:
        q = ctx.Queue()
        port = _free_port()
        procs = [ctx.Process(target=worker, args=(r, k, port, tuple(args.grid), args.pcs, q)) for r in range(k)]
        for p in procs:
            p.start()
        got = {}
        for _ in range(k):
            r, out = q.get(timeout=1200)
            got[r] = out
        for p in procs:
            p.join(timeout=300)
        rec = {"grid": args.grid, "ranks": k}
        if any("error" in got[r] for r in got):
            rec["error"] = [got[r].get("error") for r in sorted(got)]
        else:
            for pc in args.pcs:
                rec[pc] = got[0][pc]
                rec[pc]["max_err"] = max(got[r][pc]["max_err"] for r in got)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
