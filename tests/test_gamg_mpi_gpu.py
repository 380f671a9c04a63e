"""PCGAMG across ranks on the GPU (csrc/gamg_mpi.hip through aijhip_kspmpi):
k ranks as processes sharing cuda:0 over the host transport (gloo), the
distributed hierarchy and its V-cycle the product's, checked against
oracle/gamg_mpi.py — the same distributed hierarchy restated globally with
scipy (aggregates per rank's diagonal block, P and the Galerkin products over
the whole operator) — preconditioning oracle/ksp_cg.py's CG.

The reference's multi-rank runs are CG + PETSc's parallel agg GAMG
(/root/reference/runs/single-node-scaling.pbs:56-67,
/root/reference/configs/PETSc_SolverOptions_GAMG.info:6-21); block Jacobi
with a hierarchy per rank (pc "bjacobi_gamg") loses the slab coupling and its
iterations grow with the rank count, which the distributed hierarchy must
not.
"""
import importlib
import os
import socket

import numpy as np
import pytest
import scipy.sparse as sp

from oracle import gamg_mpi as ogm
from oracle import ksp_cg, seqaij

TOL = dict(rtol=1e-14, atol=1e-12)  # PETSc_SolverOptions_GAMG.info:2-4


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, dims, pcs, env, q, halo="p2p"):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ.update(env)
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

        def make_local(a_i, a_j, a_a, ncols):
            return pkg.SeqAIJHIP(a_i, a_j, a_a, ncols=ncols)

        comm = C.Comm.host(device=0, timeout_s=120)
        op = mp_mod.MPIAIJ(ai, aj, aa, row_starts, make_local, pkg.split_rows, dev, halo=halo, comm=comm)
        rhs, _ = pkg.poisson_vectors(nx, ny, nz, z0, z1)
        b = torch.from_numpy(rhs).to(dev)
        out = {}
        if halo == "allgather" and world > 1:  # PCGAMG on the all-gather operator itself: refused at PCSetType
            try:
                C.KSPCGMPINative(op.native, max_it=10, pc="gamg", **TOL).destroy()
                out["refused"] = None
            except pkg.AIJHIPError as e:
                out["refused"] = str(e)
        for pc in pcs:
            x = torch.full_like(b, float("nan"))
            with C.KSPCGMPINative(op.p2p_native() if pc == "gamg" else op.native, max_it=1000, pc=pc, **TOL) as k:
                k.solve(b, x)
                torch.cuda.synchronize()
                rows, nnz = k.pc_levels()
                out[pc] = dict(x=x.cpu().numpy(), its=k.its, reason=k.reason, hist=k.hist.tolist(), rows=rows,
                               nnz=nnz, syncs=k.host_syncs)
                if pc == "gamg" and (world > 1 or env):
                    out[pc]["A"] = [k.pc_level(l, "A") for l in range(len(rows))]
                    out[pc]["P"] = [k.pc_level(l, "P") for l in range(len(rows) - 1)]
        q.put((rank, out))
    except Exception as e:  # noqa: BLE001
        q.put((rank, {"error": repr(e)}))
    finally:
        dist.destroy_process_group()


def _run(world, dims, pcs, env=None, halo="p2p"):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, dims, pcs, env or {}, q, halo)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(world):
        r, out = q.get(timeout=600)
        got[r] = out
    for p in procs:
        p.join(timeout=120)
    for r in range(world):
        assert "error" not in got[r], got[r]["error"]
    for p in procs:
        assert p.exitcode == 0
    return got


def _oracle(dims, world):
    mp_mod = importlib.import_module("petsc-openacc_amd.mpiaij")
    nx, ny, nz = dims
    ai, aj, aa, rhs, _ = seqaij.create_system(nx, ny, nz)
    A = sp.csr_matrix((aa, aj, ai), shape=(len(ai) - 1,) * 2)
    bounds = [mp_mod.slab_bounds(nz, world, r) for r in range(world)]
    starts = [b[0] * nx * ny for b in bounds] + [nx * ny * nz]
    levels = ogm.build(A, starts)
    xo, its, reason, hist = ksp_cg.cg(ai, aj, aa, rhs, max_it=1000, pc=lambda r: ogm.vcycle(levels, r), **TOL)
    return levels, xo, its, reason, hist


@pytest.mark.gpu
@pytest.mark.parametrize("world,dims", [(2, (16, 14, 20)), (3, (12, 12, 18)), (4, (12, 10, 24))])
def test_gpu_gamg_across_ranks_matches_oracle(world, dims):
    """The distributed hierarchy's global level sizes equal the oracle's, and
    CG preconditioned by it takes the oracle's iterations (+-1), residual
    history and solution to rounding; block Jacobi + GAMG on the same ranks
    for contrast (its iterations grow)."""
    got = _run(world, dims, ("gamg", "bjacobi_gamg"))
    levels, xo, its_o, reason_o, hist_o = _oracle(dims, world)
    g = [got[r]["gamg"] for r in range(world)]
    assert len({x["its"] for x in g}) == 1 and len({x["reason"] for x in g}) == 1  # every rank alike
    assert g[0]["rows"] == [L["A"].shape[0] for L in levels], (g[0]["rows"], [L["A"].shape[0] for L in levels])
    # (entries: the product keeps the structural zeros of the Galerkin sums,
    # as the single-GPU set-up does, where scipy's products drop exact zeros;
    # the values are compared level by level below)
    # the hierarchy itself, level by level, against the oracle's operators
    def glue(parts, shape):
        rows, cols, vals = [], [], []
        for r0, ai, aj, aa in parts:
            rows.append(r0 + np.repeat(np.arange(len(ai) - 1), np.diff(ai)))
            cols.append(aj)
            vals.append(aa)
        return sp.csr_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(cols))), shape=shape)

    # Level by level: the oracle coarsens the device's own level-l operator
    # over the device's row ownership, and its P_l and A_{l+1} must equal the
    # device's to rounding. (Coarsening the oracle's own A_l instead can pick
    # other aggregates where phase 2 compares strengths that are equal in
    # exact arithmetic and differ in their last bit.)
    nl = len(g[0]["rows"])
    B = None  # the near-null space the device coarsens level l with (ones, then the Bc chain)
    for l in range(nl):
        parts = [got[r]["gamg"]["A"][l] for r in range(world)]
        n_l = g[0]["rows"][l]
        Al = glue(parts, (n_l, n_l))
        if l == 0:
            assert abs(Al - levels[0]["A"]).max() == 0.0
        if l + 1 == nl:
            break
        starts = [p[0] for p in parts] + [n_l]
        sub = ogm.build(Al, starts, max_levels=2, coarse_eq_limit=0, B=B, level0=l)  # (MIS keys and squaring by level)
        B = sub[0]["Bc"]
        n_c = g[0]["rows"][l + 1]
        assert sub[1]["A"].shape[0] == n_c, (l, sub[1]["A"].shape, n_c)
        Pg = glue([got[r]["gamg"]["P"][l] for r in range(world)], (n_l, n_c))
        Ac = glue([got[r]["gamg"]["A"][l + 1] for r in range(world)], (n_c, n_c))
        dP = abs(Pg - sub[0]["P"]).max()
        dA = abs(Ac - sub[1]["A"]).max()
        print(f"level {l}: |dP| {dP:.2e} |dA_c| {dA:.2e}")
        assert dP <= 1e-12 * abs(sub[0]["P"]).max(), (l, "P", dP)
        assert dA <= 1e-12 * abs(sub[1]["A"]).max(), (l, "A_c", dA)
    bj = got[0]["bjacobi_gamg"]["its"]
    print(f"\n{world} ranks {dims}: GAMG across ranks {g[0]['its']} its (oracle {its_o}), levels {g[0]['rows']}, "
          f"bjacobi+GAMG {bj} its, host syncs {g[0]['syncs']}")
    assert g[0]["reason"] == reason_o and g[0]["reason"] > 0
    assert abs(g[0]["its"] - its_o) <= 1
    # the oracle's own hierarchy may differ in tie-broken aggregates on the
    # coarse levels (above): the same convergence, not the same digits
    k = min(len(g[0]["hist"]), len(hist_o), 10)
    np.testing.assert_allclose(g[0]["hist"][:k], hist_o[:k], rtol=0.05)
    x = np.concatenate([got[r]["gamg"]["x"] for r in range(world)])
    assert np.linalg.norm(x - xo) <= 1e-7 * np.linalg.norm(xo)
    assert g[0]["its"] <= bj


@pytest.mark.gpu
def test_gpu_gamg_distributed_setup_at_one_rank_matches_pcgamg():
    """AIJHIP_GAMG_DIST=1 forces the distributed set-up at one rank: the same
    hierarchy as the single-GPU PCGAMG (level sizes and entries), the same
    iterations and residual history to rounding (the dots are summed in a
    different order)."""
    dims = (20, 20, 20)
    dist_run = _run(1, dims, ("gamg",), env={"AIJHIP_GAMG_DIST": "1"})[0]["gamg"]
    single = _run(1, dims, ("gamg",))[0]["gamg"]
    assert dist_run["rows"] == single["rows"] and dist_run["nnz"] == single["nnz"]
    assert dist_run["its"] == single["its"]
    np.testing.assert_allclose(dist_run["hist"], single["hist"], rtol=1e-6, atol=1e-15 * single["hist"][0])
    np.testing.assert_allclose(dist_run["x"], single["x"], rtol=1e-9, atol=1e-12)


@pytest.mark.gpu
def test_gpu_gamg_on_allgather_operator():
    """An operator with the north star's all-gather halo: CG + Jacobi runs on
    it as built, PCGAMG across ranks on its p2p twin (MPIAIJ.p2p_native, which
    shares A_d); both equal the p2p operator's solves bit for bit."""
    dims = (12, 12, 16)
    ag = _run(2, dims, ("gamg", "jacobi"), halo="allgather")
    pp = _run(2, dims, ("gamg", "jacobi"))
    for r in range(2):  # the plain all-gather handle is refused early, pointing at the p2p twin
        assert ag[r]["refused"] and "p2p" in ag[r]["refused"], ag[r].get("refused")
    for r in range(2):
        for pc in ("gamg", "jacobi"):
            assert ag[r][pc]["its"] == pp[r][pc]["its"], (r, pc)
            assert np.array_equal(ag[r][pc]["x"].view(np.uint64), pp[r][pc]["x"].view(np.uint64)), (r, pc)


@pytest.mark.gpu
def test_gpu_gamg_mpi_fused_smoothers_within_tolerance_of_petsc_order():
    """The fused distributed smoothers (the default) add A_o's share after the
    A_d epilogue — r = (b - A_d x) - A_o g, x = [t + D^-1 (b - A_d t)] +
    D^-1 (-A_o g) — where PETSc's MatResidual forms A_d x + A_o g first
    (AIJHIP_MG_UNFUSED=1 keeps that order). Only the boundary rows' rounding
    differs: the same iterations, the residual history to 1e-10 relative and
    the solution to 1e-10 (the reordering is documented and
    pinned, not claimed bit-exact)."""
    dims = (12, 12, 16)
    fused = _run(2, dims, ("gamg",))
    petsc_order = _run(2, dims, ("gamg",), env={"AIJHIP_MG_UNFUSED": "1"})
    for r in range(2):
        a, b = fused[r]["gamg"], petsc_order[r]["gamg"]
        assert a["its"] == b["its"]
        h0 = b["hist"][0]
        np.testing.assert_allclose(a["hist"], b["hist"], rtol=1e-10, atol=1e-14 * h0)
        np.testing.assert_allclose(a["x"], b["x"], rtol=1e-10, atol=1e-12)


@pytest.mark.gpu
def test_gpu_gamg_across_ranks_is_partition_independent():
    """PETSc's parallel MIS exchanges ghost states every round (VERDICT r05
    item 4); restated as the global MIS by global keys, the device's
    hierarchy at 2, 3 and 4 ranks has the one-rank distributed set-up's level
    sizes and entry counts and CG takes the same iterations (no extra
    aggregates along the slab boundaries)."""
    dims = (12, 12, 24)
    one = _run(1, dims, ("gamg",), env={"AIJHIP_GAMG_DIST": "1"})[0]["gamg"]
    for world in (2, 3, 4):
        g = _run(world, dims, ("gamg",))[0]["gamg"]
        print(f"{world} ranks: levels {g['rows']} its {g['its']} (1 rank: {one['rows']} {one['its']})")
        assert g["rows"] == one["rows"] and g["nnz"] == one["nnz"], world
        assert g["its"] == one["its"], world
