"""The multi-GPU code path on one GPU: k ranks as k
processes sharing cuda:0, torch.distributed over gloo (which takes GPU
tensors for the halo send/recv, all-gather and all-reduce), the per-rank
operators the product's SeqAIJHIP handles (HIP kernels), the exchange and
the distributed CG the product's (mpiaij.py, ksp.py KSPCGMPI with the device
vector kernels). RCCL itself runs only in the driver's multi-GPU bench."""
import importlib
import os
import socket

import numpy as np
import pytest

from oracle import ksp_cg, seqaij


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, dims, halo, q):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        pkg = importlib.import_module("petsc-openacc_amd")
        mp_mod = importlib.import_module("petsc-openacc_amd.mpiaij")
        K = importlib.import_module("petsc-openacc_amd.ksp")
        dev = torch.device("cuda:0")
        nx, ny, nz = dims
        bounds = [mp_mod.slab_bounds(nz, world, r) for r in range(world)]
        row_starts = np.array([b[0] * nx * ny for b in bounds] + [nx * ny * nz], dtype=np.int64)
        z0, z1 = bounds[rank]
        ai, aj, aa = pkg.poisson_csr(nx, ny, nz, z0, z1)

        def make_local(a_i, a_j, a_a, ncols):
            return pkg.SeqAIJHIP(a_i, a_j, a_a, ncols=ncols)

        op = mp_mod.MPIAIJ(ai, aj, aa, row_starts, make_local, pkg.split_rows, dev, halo=halo)
        C = importlib.import_module("petsc-openacc_amd.comm")
        comm = C.Comm.host(device=0, timeout_s=120)
        op_n = mp_mod.MPIAIJ(ai, aj, aa, row_starts, make_local, pkg.split_rows, dev, halo=halo, comm=comm)
        lo, hi = int(row_starts[rank]), int(row_starts[rank + 1])
        xg = seqaij.splitmix_uniform(nx * ny * nz, 42)
        x = torch.from_numpy(xg[lo:hi].copy()).to(dev)
        y = torch.empty(hi - lo, dtype=torch.float64, device=dev)
        op.mult(x, y)
        y_n = torch.full_like(y, float("nan"))
        op_n.mult(x, y_n)
        op_n.mult(x, y_n)  # twice: the ghost buffer is reused
        torch.cuda.synchronize()
        same = bool(torch.equal(y, y_n))
        rhs, _ = pkg.poisson_vectors(nx, ny, nz, z0, z1)
        b = torch.from_numpy(rhs).to(dev)
        dinv = torch.empty_like(b)
        K.DeviceVecOps.jacobi_inverse(op.A_d, dinv)
        cg = K.KSPCGMPI(op, op.mloc, dinv=dinv, rtol=1e-10, max_it=1000, device=dev)
        xs = torch.zeros_like(b)
        cg.solve(b, xs)
        torch.cuda.synchronize()
        xn = torch.full_like(b, float("nan"))
        with C.KSPCGMPINative(op_n.native, rtol=1e-10, max_it=1000, poll=3) as kn:
            kn.solve(b, xn)
            native = (xn.cpu().numpy(), kn.its, kn.reason, kn.hist.tolist())
        xg = torch.full_like(b, float("nan"))  # CG + bjacobi/GAMG (one hierarchy per diagonal block)
        with C.KSPCGMPINative(op_n.native, rtol=1e-10, max_it=1000, pc="bjacobi_gamg") as kg:
            kg.solve(b, xg)
            native_gamg = (xg.cpu().numpy(), kg.its, kg.reason, kg.hist.tolist())
        q.put((rank, y.cpu().numpy(), xs.cpu().numpy(), cg.its, cg.reason, list(cg.hist), same, native,
               native_gamg))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("world,dims,halo", [(2, (12, 10, 16), "p2p"), (3, (9, 8, 13), "allgather"),
                                             (3, (10, 10, 12), "p2p")])
def test_gpu_mpiaij_and_cg_on_k_ranks(world, dims, halo):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, dims, halo, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(world):
        r = q.get(timeout=300)
        got[r[0]] = r[1:]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    nx, ny, nz = dims
    ai, aj, aa, rhs, _ = seqaij.create_system(nx, ny, nz)
    y_ref = seqaij.matmult(ai, aj, aa, seqaij.splitmix_uniform(nx * ny * nz, 42))
    y = np.concatenate([got[r][0] for r in range(world)])
    # each block's sums keep PETSc's order; the off-diagonal entries of a row
    # are added after its diagonal-block part (MatMult_MPIAIJ), so compare to
    # rounding
    np.testing.assert_allclose(y, y_ref, rtol=1e-12, atol=1e-12 * np.abs(y_ref).max())
    xo, its_o, reason_o, hist_o = ksp_cg.cg(ai, aj, aa, rhs, rtol=1e-10, max_it=1000)
    assert len({got[r][2] for r in range(world)}) == 1
    assert abs(got[0][2] - its_o) <= 1 and got[0][3] == reason_o
    np.testing.assert_allclose(got[0][4][:10], hist_o[:10], rtol=1e-9)
    x = np.concatenate([got[r][1] for r in range(world)])
    assert np.linalg.norm(x - xo) <= 1e-8 * np.linalg.norm(xo)
    # the native path (aijhip_mpiaij / aijhip_kspmpi over the host transport)
    assert all(got[r][5] for r in range(world)), "native MatMult_MPIAIJ differs from the stream-ordered path"
    nat = [got[r][6] for r in range(world)]
    assert len({n[1] for n in nat}) == 1 and len({n[2] for n in nat}) == 1  # every rank took the same path
    assert abs(nat[0][1] - its_o) <= 1 and nat[0][2] == reason_o
    np.testing.assert_allclose(nat[0][3][:10], hist_o[:10], rtol=1e-9)
    xn = np.concatenate([n[0] for n in nat])
    assert np.linalg.norm(xn - xo) <= 1e-8 * np.linalg.norm(xo)
    # CG + bjacobi/GAMG against the oracle CG preconditioned by one oracle
    # V-cycle per rank's diagonal block (PETSc -pc_type bjacobi -sub_pc_type gamg)
    import importlib
    import scipy.sparse as sp
    from oracle import gamg as ogamg
    pkg = importlib.import_module("petsc-openacc_amd")
    mp_mod = importlib.import_module("petsc-openacc_amd.mpiaij")
    bounds = [mp_mod.slab_bounds(nz, world, r) for r in range(world)]
    starts = [b[0] * nx * ny for b in bounds] + [nx * ny * nz]
    blocks = []
    for r in range(world):
        lo, hi = starts[r], starts[r + 1]
        (dai, daj, daa), _, _ = pkg.split_rows(*pkg.poisson_csr(nx, ny, nz, *bounds[r]), lo, hi)
        blocks.append((lo, hi, ogamg.build(sp.csr_matrix((daa, daj, dai), shape=(hi - lo, hi - lo)))))

    def bjacobi(rv):
        return np.concatenate([ogamg.vcycle(lv, rv[lo:hi]) for lo, hi, lv in blocks])

    xg_o, its_g, reason_g, hist_g = ksp_cg.cg(ai, aj, aa, rhs, rtol=1e-10, max_it=1000, pc=bjacobi)
    gm = [got[r][7] for r in range(world)]
    assert len({g[1] for g in gm}) == 1 and len({g[2] for g in gm}) == 1
    print(f"\nbjacobi/GAMG: {gm[0][1]} its (oracle {its_g}), CG/Jacobi {nat[0][1]} its")
    assert abs(gm[0][1] - its_g) <= 1 and gm[0][2] == reason_g
    np.testing.assert_allclose(gm[0][3][:10], hist_g[:10], rtol=1e-7)
    xgm = np.concatenate([g[0] for g in gm])
    assert np.linalg.norm(xgm - xg_o) <= 1e-8 * np.linalg.norm(xg_o)


def _unfused_worker(rank, world, port, dims, q):
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
        rhs, _ = pkg.poisson_vectors(nx, ny, nz, z0, z1)
        b = torch.from_numpy(rhs).to(dev)
        comm = C.Comm.host(device=0, timeout_s=120)
        out = {}
        for kernel in ("stream", "vector"):
            def make_local(a_i, a_j, a_a, ncols, kernel=kernel):
                return pkg.SeqAIJHIP(a_i, a_j, a_a, ncols=ncols, kernel=kernel)

            op = mp_mod.MPIAIJ(ai, aj, aa, row_starts, make_local, pkg.split_rows, dev, comm=comm)
            x = torch.full_like(b, float("nan"))
            with C.KSPCGMPINative(op.native, rtol=1e-10, max_it=1000) as k:
                k.solve(b, x)
                torch.cuda.synchronize()
                out[kernel] = (x.cpu().numpy(), k.its, k.reason, k.hist.tolist(), op.A_d.info()["kernel"])
        q.put((rank, out))
    except Exception as e:  # noqa: BLE001
        q.put((rank, {"error": repr(e)}))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_gpu_kspmpi_unfused_dot_matches_fused_and_oracle():
    """with a diagonal block the STREAM epilogue cannot carry p.w
    (here the VECTOR kernel), the distributed CG takes the unfused dot, which
    must not add the off-diagonal correction a second time: same iterations
    and residual history as the fused run and the oracle CG."""
    import torch.multiprocessing as mp
    world, dims = 2, (12, 10, 16)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_unfused_worker, args=(r, world, port, dims, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(world):
        r, out = q.get(timeout=300)
        got[r] = out
    for p in procs:
        p.join(timeout=120)
    for r in range(world):
        assert "error" not in got[r], got[r]["error"]
    nx, ny, nz = dims
    ai, aj, aa, rhs, _ = seqaij.create_system(nx, ny, nz)
    xo, its_o, reason_o, hist_o = ksp_cg.cg(ai, aj, aa, rhs, rtol=1e-10, max_it=1000)
    fused, unfused = got[0]["stream"], got[0]["vector"]
    assert fused[4] == "stream" and unfused[4] == "vector"
    assert unfused[2] == reason_o and abs(unfused[1] - its_o) <= 1 and abs(unfused[1] - fused[1]) <= 1
    np.testing.assert_allclose(unfused[3][:10], hist_o[:10], rtol=1e-9)
    np.testing.assert_allclose(unfused[3][:10], fused[3][:10], rtol=1e-9)
    x = np.concatenate([got[r]["vector"][0] for r in range(world)])
    assert np.linalg.norm(x - xo) <= 1e-8 * np.linalg.norm(xo)
