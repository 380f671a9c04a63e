"""Distributed row-block SpMV (MatMult_MPIAIJ analogue) on CPU: world_size 2
and 3 over gloo. The exchange logic is the product's (petsc-openacc_amd/
mpiaij.py); only the per-rank local multiply is the oracle here, because
this container has no GPU. The GPU form of the same class is exercised by
bench.py --gpus N on the box."""
import importlib
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import seqaij


class OracleLocal:
    """CPU stand-in for SeqAIJHIP (tests only)."""

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


def _operand(kind, dims):
    """Global (ai, aj, aa) of a general test operand (not z-slab aligned)."""
    pkg = importlib.import_module("petsc-openacc_amd")
    if kind == "skewed":  # hub rows: ghosts from every rank, non-contiguous send lists
        return pkg.skewed_csr(dims[0], seed=7)
    return pkg.fem_hex_csr(*dims)


def _general_worker(rank, world, port, kind, dims, row_starts, halo, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        pkg = importlib.import_module("petsc-openacc_amd")
        mp_mod = importlib.import_module("petsc-openacc_amd.mpiaij")
        ai, aj, aa = _operand(kind, dims)
        lo, hi = int(row_starts[rank]), int(row_starts[rank + 1])
        lai = (ai[lo:hi + 1] - ai[lo]).astype(np.int32)
        op = mp_mod.MPIAIJ(lai, aj[ai[lo]:ai[hi]].copy(), aa[ai[lo]:ai[hi]].copy(), row_starts, OracleLocal,
                           pkg.split_rows, torch.device("cpu"), halo=halo)
        xg = seqaij.splitmix_uniform(len(ai) - 1, 3)
        x = torch.from_numpy(xg[lo:hi].copy())
        y = torch.empty(hi - lo, dtype=torch.float64)
        op.mult(x, y)
        op.mult(x, y)
        q.put((rank, y.numpy().copy(), {p: op.plan.send_slices[p] is None for p in op.plan.send}))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("kind,dims,fracs,halo", [("skewed", (30000,), (0.0, 0.21, 0.64, 1.0), "p2p"),
                                                  ("skewed", (30000,), (0.0, 0.5, 1.0), "allgather"),
                                                  ("fem_hex", (7, 6, 9), (0.0, 0.3, 0.55, 1.0), "p2p"),
                                                  ("fem_hex", (7, 6, 9), (0.0, 0.3, 0.55, 1.0), "allgather")])
def test_mpiaij_general_operands(kind, dims, fracs, halo):
    """Uneven row blocks of unstructured operands: ghosts owned by several
    ranks, gathered (non-contiguous) send lists; against the global multiply
    within the fp64 reorder bound."""
    ai, aj, aa = _operand(kind, dims)
    m = len(ai) - 1
    row_starts = np.array([int(f * m) for f in fracs], dtype=np.int64)
    world = len(row_starts) - 1
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_general_worker, args=(r, world, port, kind, dims, row_starts, halo, q))
             for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(world):
        r, y, sends = q.get(timeout=120)
        got[r] = (y, sends)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    y_ref = seqaij.matmult(ai, aj, aa, seqaij.splitmix_uniform(m, 3))
    y = np.concatenate([got[r][0] for r in range(world)])
    absax = seqaij.matmult(ai, aj, np.abs(aa), np.abs(seqaij.splitmix_uniform(m, 3)))
    assert np.all(np.abs(y - y_ref) <= 4 * np.diff(ai) * 2.0 ** -53 * absax + 1e-300)
    # the gathered (non-contiguous) send path was taken somewhere
    assert any(any(g[1].values()) for g in got.values())


def _worker(rank, world, port, dims, halo, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        pkg = importlib.import_module("petsc-openacc_amd")
        mp_mod = importlib.import_module("petsc-openacc_amd.mpiaij")
        nx, ny, nz = dims
        bounds = [mp_mod.slab_bounds(nz, world, r) for r in range(world)]
        row_starts = np.array([b[0] * nx * ny for b in bounds] + [nx * ny * nz], dtype=np.int64)
        z0, z1 = bounds[rank]
        ai, aj, aa = pkg.poisson_csr(nx, ny, nz, z0, z1)
        op = mp_mod.MPIAIJ(ai, aj, aa, row_starts, OracleLocal, pkg.split_rows, torch.device("cpu"), halo=halo)
        n = nx * ny * nz
        xg = seqaij.splitmix_uniform(n, 42)
        lo, hi = row_starts[rank], row_starts[rank + 1]
        x = torch.from_numpy(xg[lo:hi].copy())
        y = torch.empty(hi - lo, dtype=torch.float64)
        op.mult(x, y)
        op.mult(x, y)  # a second exchange reuses the buffers
        q.put((rank, y.numpy().copy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,dims,halo", [(2, (6, 5, 8), "p2p"), (3, (4, 4, 10), "p2p"),
                                             (2, (6, 5, 8), "allgather"), (3, (5, 4, 7), "allgather")])
def test_mpiaij_matches_global_matmult(world, dims, halo):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, dims, halo, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    nx, ny, nz = dims
    ai, aj, aa, _, _ = seqaij.create_system(nx, ny, nz)
    y_ref = seqaij.matmult(ai, aj, aa, seqaij.splitmix_uniform(nx * ny * nz, 42))
    y = np.concatenate([got[r] for r in range(world)])
    # diagonal-then-off-diagonal order differs from the global row order only
    # on the slab boundary rows: fp64 reorder bound
    np.testing.assert_allclose(y, y_ref, rtol=0, atol=1e-12 * np.max(np.abs(aa)))


def test_slab_bounds_cover():
    mp_mod = importlib.import_module("petsc-openacc_amd.mpiaij")
    for nz, world in [(300, 8), (7, 3), (600, 8), (10, 4)]:
        b = [mp_mod.slab_bounds(nz, world, r) for r in range(world)]
        assert b[0][0] == 0 and b[-1][1] == nz
        assert all(b[i][1] == b[i + 1][0] for i in range(world - 1))
        assert max(e - s for s, e in b) - min(e - s for s, e in b) <= 1
