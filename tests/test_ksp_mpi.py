"""Row-partitioned CG (petsc-openacc_amd/ksp.py KSPCGMPI): the
dots all-reduced across ranks. CPU: world size 2 and 3 over gloo, the
MPIAIJ exchange and the CG driver are the product's, the per-rank SpMV and
vector kernels are test doubles (numpy), checked against the single-process
oracle CG. GPU: the device vector kernels (aijhip_vec.h) with world size 1,
against the device KSP."""
import importlib
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import ksp_cg, seqaij


class NumpyVecOps:
    """CPU test double for DeviceVecOps (same formulas, numpy order)."""

    def __init__(self):
        self.red = torch.zeros(3, dtype=torch.float64)

    def aypx(self, beta, x, y):
        y.copy_(x + beta * y)

    def dot(self, x, y):
        self.red[0] = float(np.dot(x.numpy(), y.numpy()))
        return self.red[:1]

    def jacobi(self, r, dinv, z):
        z.copy_(dinv * r if dinv is not None else r)
        zn, rn = z.numpy(), r.numpy()
        self.red.copy_(torch.tensor([zn @ zn, zn @ rn, rn @ rn]))
        return self.red

    def cg_update(self, a, x, p, r, w, z, dinv):
        x.add_(a * p)
        r.copy_(r + (-a) * w)
        return self.jacobi(r, dinv, z)


class OracleLocal:
    def __init__(self, ai, aj, aa, ncols):
        self.ai, self.aj, self.aa = ai, aj, aa

    def mult(self, x, y, stream=None):
        y.copy_(torch.from_numpy(seqaij.matmult(self.ai, self.aj, self.aa, x.numpy())))

    def mult_add(self, x, z, w, stream=None):
        w.copy_(torch.from_numpy(seqaij.matmult_add(self.ai, self.aj, self.aa, x.numpy(), z.numpy())))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, dims, halo, norm, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        pkg = importlib.import_module("petsc-openacc_amd")
        mp_mod = importlib.import_module("petsc-openacc_amd.mpiaij")
        K = importlib.import_module("petsc-openacc_amd.ksp")
        nx, ny, nz = dims
        bounds = [mp_mod.slab_bounds(nz, world, r) for r in range(world)]
        row_starts = np.array([b[0] * nx * ny for b in bounds] + [nx * ny * nz], dtype=np.int64)
        z0, z1 = bounds[rank]
        ai, aj, aa = pkg.poisson_csr(nx, ny, nz, z0, z1)
        rhs, _ = pkg.poisson_vectors(nx, ny, nz, z0, z1)
        op = mp_mod.MPIAIJ(ai, aj, aa, row_starts, OracleLocal, pkg.split_rows, torch.device("cpu"), halo=halo)
        lo = int(row_starts[rank])
        dinv = torch.from_numpy(ksp_cg.jacobi_inverse(*_diag_block(ai, aj, aa, lo, op.mloc)))
        ksp = K.KSPCGMPI(op, op.mloc, dinv=dinv, ops=NumpyVecOps(), rtol=1e-10, max_it=500, norm=norm,
                         device=torch.device("cpu"))
        x = torch.zeros(op.mloc, dtype=torch.float64)
        ksp.solve(torch.from_numpy(rhs), x)
        q.put((rank, x.numpy().copy(), ksp.its, ksp.reason, list(ksp.hist)))
    finally:
        dist.destroy_process_group()


def _diag_block(ai, aj, aa, lo, m):
    """Local rows with local column numbering of the diagonal entries only
    (enough for jacobi_inverse: it reads the entry with column == row)."""
    aj_loc = aj.astype(np.int64) - lo
    keep = (aj_loc >= 0) & (aj_loc < m)
    rows = np.repeat(np.arange(m), np.diff(ai))
    k_ai = np.concatenate([[0], np.cumsum(np.bincount(rows[keep], minlength=m))]).astype(np.int32)
    return k_ai, aj_loc[keep].astype(np.int32), aa[keep]


@pytest.mark.parametrize("world,dims,halo,norm", [(2, (6, 5, 8), "p2p", "preconditioned"),
                                                  (3, (5, 4, 9), "allgather", "unpreconditioned")])
def test_cg_mpi_matches_oracle(world, dims, halo, norm):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, dims, halo, norm, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict((r[0], r[1:]) for r in (q.get(timeout=180) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    nx, ny, nz = dims
    ai, aj, aa, rhs, _ = seqaij.create_system(nx, ny, nz)
    xo, its_o, reason_o, hist_o = ksp_cg.cg(ai, aj, aa, rhs, rtol=1e-10, max_it=500, norm=norm)
    x = np.concatenate([got[r][0] for r in range(world)])
    its = {got[r][1] for r in range(world)}
    assert len(its) == 1 and abs(its.pop() - its_o) <= 1  # every rank took the same path
    assert {got[r][2] for r in range(world)} == {reason_o}
    np.testing.assert_allclose(got[0][3][:10], hist_o[:10], rtol=1e-9)
    assert np.linalg.norm(x - xo) <= 1e-8 * np.linalg.norm(xo)


@pytest.mark.gpu
@pytest.mark.parametrize("norm", ["preconditioned", "natural"])
def test_gpu_cg_mpi_world1_matches_device_ksp(pkg, norm):
    """The device vector kernels under the host-driven CG give the device
    KSP's iterations and residual history (world size 1: no exchange)."""
    assert torch.cuda.is_available()
    K = importlib.import_module("petsc-openacc_amd.ksp")
    N = 24
    ai, aj, aa = pkg.poisson_csr(N)
    rhs, _ = pkg.poisson_vectors(N)
    A = pkg.SeqAIJHIP(ai, aj, aa)
    b = torch.from_numpy(rhs).cuda()
    dinv = torch.empty_like(b)
    K.DeviceVecOps.jacobi_inverse(A, dinv)
    np.testing.assert_array_equal(dinv.cpu().numpy(), ksp_cg.jacobi_inverse(ai, aj, aa))
    cg = K.KSPCGMPI(A, A.m, dinv=dinv, rtol=1e-12, max_it=2000, norm=norm, device=b.device)
    x1 = torch.zeros_like(b)
    cg.solve(b, x1)
    x2 = torch.zeros_like(b)
    with K.KSPCG(A, rtol=1e-12, max_it=2000, norm=norm) as ksp:
        ksp.solve(b, x2)
        assert cg.reason == ksp.reason and abs(cg.its - ksp.its) <= 1
        np.testing.assert_allclose(np.array(cg.hist[:20]), ksp.history()[:20], rtol=1e-10)
    assert torch.linalg.norm(x1 - x2) <= 1e-9 * torch.linalg.norm(x2)
    A.destroy()
