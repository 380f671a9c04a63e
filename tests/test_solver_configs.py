"""BASELINE.json's solver configurations at their full sizes, on the GPU.

configs[2]: 3-D Poisson 300^3, the full KSP CG+GAMG solve with the
reference's options (/root/reference/configs/PETSc_SolverOptions_GAMG.info,
driven as /root/reference/src/main_ksp.cpp:92-129 drives it), on 1 MI355X.
configs[0]: the same solver at 100^3 (the reference's plumbing case).

At 300^3 the oracle cannot rerun the solve in test time, so the solve is
checked through size-independent facts plus the pieces the oracle can
afford: the true residual b - A x with the C restatement of MatMult_SeqAIJ,
the discretisation error against generateExt (helper.cpp:148-151) at O(h^2),
the iteration count pinned, and the device-built hierarchy compared entry for
entry with the host builder (itself bit-identical to oracle/gamg.py) at this
size, including whichever device product classes fire. At 100^3 the oracle's
CG + V-cycle reruns the whole solve on the product's host hierarchy.
"""
import importlib

import numpy as np
import pytest
import scipy.sparse as sp

from oracle import gamg as ogamg
from oracle import ksp_cg

TOL = dict(rtol=1e-14, atol=1e-12, max_it=10000)  # PETSc_SolverOptions_GAMG.info:2-4
# Iteration counts of this build's CG+GAMG at the BASELINE sizes with the
# default hierarchy (PETSc 3.7 agg's MIS + CG emax since round 5: 53 at 300^3
# measured on MI355X, profiles/r05/m/; 52 at 100^3 from the oracle CG over the
# host hierarchy; the greedy hierarchy took 57 and 47); +-1 allows a
# reordered dot at the tolerance boundary.
PINNED_ITS = {300: 53, 100: 52}
# Linf(x - exact) <= C_H2 * h^2: the 7-point scheme is second order; the
# measured constant is ~6.6 at 300^3 and ~6.6 at 100^3.
C_H2 = 8.0


def _bits(x):
    return np.ascontiguousarray(x).view(np.uint64)


def _levels_as_oracle(ai, aj, aa, lv):
    """The product's host hierarchy in oracle/gamg.py's level format."""
    m = len(ai) - 1
    out = [dict(A=sp.csr_matrix((aa, aj, ai), shape=(m, m)))]
    for l in range(1, len(lv)):
        mc = lv[l]["m"]
        pai, paj, paa = lv[l - 1]["P"]
        out[l - 1]["P"] = sp.csr_matrix((paa, paj, pai), shape=(lv[l - 1]["m"], mc))
        cai, caj, caa = lv[l]["A"]
        out.append(dict(A=sp.csr_matrix((caa, caj, cai), shape=(mc, mc))))
    return out


def _solve(pkg, ai, aj, aa, rhs, dev="cuda"):
    import torch
    K = importlib.import_module("petsc-openacc_amd.ksp")
    A = pkg.SeqAIJHIP(ai, aj, aa)
    b = torch.from_numpy(rhs).to(dev)
    x = torch.empty_like(b)
    ksp = K.KSPCG(A, pc="gamg", **TOL)
    ksp.solve(b, x)
    torch.cuda.synchronize()
    return A, ksp, x.cpu().numpy()


@pytest.mark.gpu
def test_gpu_cg_gamg_300_configs2(pkg, coracle):
    """configs[2]: converged (reason > 0) in the pinned iteration count, the
    true residual small, Linf against the analytic solution O(h^2)."""
    torch = pytest.importorskip("torch")
    assert torch.cuda.is_available()
    N = 300
    ai, aj, aa = pkg.poisson_csr(N)
    rhs, exact = pkg.poisson_vectors(N)
    A, ksp, x = _solve(pkg, ai, aj, aa, rhs)
    try:
        its, reason, rnorm = ksp.its, ksp.reason, ksp.rnorm
        hist = ksp.history()
        path, overflow = ksp.setup_path()
        syncs = ksp.host_syncs
    finally:
        ksp.destroy()
        A.destroy()
    r = rhs - coracle.matmult(ai, aj, aa, x, omp=True)
    rel = np.linalg.norm(r) / np.linalg.norm(rhs)
    err = float(np.max(np.abs(x - exact)))
    print(f"\n300^3 CG+GAMG: its {its} reason {reason} rnorm {rnorm:.3e} "
          f"|b-Ax|/|b| {rel:.3e} Linf {err:.3e} (h^2 x {err * N * N:.2f}) path {path} overflow {overflow}")
    assert reason > 0, reason
    assert abs(its - PINNED_ITS[N]) <= 1, its
    # KSPConvergedDefault: the last preconditioned norm is under rtol * the first
    assert hist[-1] <= max(TOL["rtol"] * hist[0], TOL["atol"])
    assert np.all(np.isfinite(x))
    assert rel <= 1e-11, rel
    assert err <= C_H2 / (N * N), err
    assert all(p == "device" for p, _ in path[:2]), path  # the two big levels are built on the GPU
    # the V-cycle honours the device stop flag: iterations go out in batches
    # of 8 between host polls (53 iterations -> 7 polls + the final read)
    assert syncs <= 10, syncs


@pytest.mark.gpu
@pytest.mark.parametrize("pc", ["gamg", "jacobi"])
def test_gpu_batched_polling_is_bitwise(pkg, pc, monkeypatch):
    """Polling the stop flag every 8 iterations (default) or every iteration
    (AIJHIP_KSP_POLL=1) gives the same residual history and x bit for bit:
    kernels launched past convergence return at once."""
    torch = pytest.importorskip("torch")
    K = importlib.import_module("petsc-openacc_amd.ksp")
    N = 48
    ai, aj, aa = pkg.poisson_csr(N)
    rhs, _ = pkg.poisson_vectors(N)
    out = {}
    A = pkg.SeqAIJHIP(ai, aj, aa)
    try:
        with K.KSPCG(A, pc=pc, **TOL) as ksp:
            for poll in ("1", "8"):
                monkeypatch.setenv("AIJHIP_KSP_POLL", poll)
                b = torch.from_numpy(rhs).cuda()
                x = torch.empty_like(b)
                ksp.solve(b, x)
                torch.cuda.synchronize()
                out[poll] = (ksp.its, ksp.history(), x.cpu().numpy(), ksp.host_syncs)
    finally:
        A.destroy()
    (i1, h1, x1, s1), (i8, h8, x8, s8) = out["1"], out["8"]
    assert i1 == i8 and i1 > 8
    assert np.array_equal(_bits(h1), _bits(h8)) and np.array_equal(_bits(x1), _bits(x8))
    assert s1 >= i1 and s8 <= i8 // 8 + 3, (s1, s8, i1)


@pytest.mark.gpu
def test_gpu_gamg_setup_300_matches_host_bitwise(pkg):
    """configs[2]'s hierarchy: the device set-up (aijhip_ksp_set_up) against
    the host builder (aijhip_gamg_build_host, pinned to oracle/gamg.py at the
    sizes the oracle can run) at 300^3, every level's A and P entry for
    entry, and the device product classes that fired on the way."""
    torch = pytest.importorskip("torch")
    assert torch.cuda.is_available()
    K = importlib.import_module("petsc-openacc_amd.ksp")
    G = importlib.import_module("petsc-openacc_amd.gamg")
    N = 300
    ai, aj, aa = pkg.poisson_csr(N)
    lv = G.build_host(ai, aj, aa)
    A = pkg.SeqAIJHIP(ai, aj, aa)
    try:
        with K.KSPCG(A, pc="gamg") as ksp:
            ksp.set_up()
            rows, nnz, _ = ksp.pc_levels()
            path, overflow = ksp.setup_path()
            print(f"\n300^3 hierarchy rows {rows} nnz {nnz} path {path} overflow {overflow}")
            assert rows == [L["m"] for L in lv]
            assert len(rows) >= 4 and rows[1] < rows[0] // 4
            for l in range(1, len(lv)):
                dai, daj, daa, _ = ksp.pc_level(l, "A")
                hai, haj, haa = lv[l]["A"]
                assert np.array_equal(dai, hai) and np.array_equal(daj, haj), l
                assert np.array_equal(_bits(daa), _bits(haa)), l
            for l in range(len(lv) - 1):
                pai, paj, paa, pn = ksp.pc_level(l, "P")
                hai, haj, haa = lv[l]["P"]
                assert pn == lv[l + 1]["m"]
                assert np.array_equal(pai, hai) and np.array_equal(paj, haj), l
                assert np.array_equal(_bits(paa), _bits(haa)), l
            assert path[0] == ("device", path[0][1]) and path[1][0] == "device", path
    finally:
        A.destroy()


@pytest.mark.gpu
def test_gpu_mis_gamg_setup_100_matches_host_and_solves(pkg):
    """PETSc 3.7's coarsening (coarsen 1 + the CG emax, eig_ksp 1) at 100^3:
    the device set-up equals the host builder level for level, and CG + that
    hierarchy converges to the reference's tolerances."""
    torch = pytest.importorskip("torch")
    assert torch.cuda.is_available()
    K = importlib.import_module("petsc-openacc_amd.ksp")
    G = importlib.import_module("petsc-openacc_amd.gamg")
    N = 100
    ai, aj, aa = pkg.poisson_csr(N)
    rhs, exact = pkg.poisson_vectors(N)
    prm = dict(coarsen=1, eig_ksp=1)
    lv = G.build_host(ai, aj, aa, **prm)
    A = pkg.SeqAIJHIP(ai, aj, aa)
    try:
        with K.KSPCG(A, pc="gamg", gamg=prm, rtol=1e-14, atol=1e-12) as ksp:
            ksp.set_up()
            rows, nnz, _ = ksp.pc_levels()
            print(f"\n100^3 MIS hierarchy rows {rows} nnz {nnz}")
            assert rows == [L["m"] for L in lv] and rows[1] < rows[0] // 6
            for l in range(1, len(lv)):
                dai, daj, daa, _ = ksp.pc_level(l, "A")
                hai, haj, haa = lv[l]["A"]
                assert np.array_equal(dai, hai) and np.array_equal(daj, haj), l
                assert np.array_equal(_bits(daa), _bits(haa)), l
            b = torch.from_numpy(rhs).cuda()
            x = torch.empty_like(b)
            ksp.solve(b, x)
            assert ksp.reason > 0 and ksp.its < 100, (ksp.its, ksp.reason)
            assert np.abs(x.cpu().numpy() - exact).max() <= C_H2 / N ** 2
    finally:
        A.destroy()


@pytest.mark.gpu
def test_gpu_cg_gamg_100_configs0_vs_oracle(pkg):
    """configs[0] (100^3): the device solve against the oracle's CG
    (oracle/ksp_cg.py) preconditioned by the oracle's V-cycle
    (oracle/gamg.py vcycle) over the product's host hierarchy — iterations
    +-1, residual history to 1e-7, solution to 1e-8; and O(h^2) accuracy."""
    torch = pytest.importorskip("torch")
    assert torch.cuda.is_available()
    G = importlib.import_module("petsc-openacc_amd.gamg")
    N = 100
    ai, aj, aa = pkg.poisson_csr(N)
    rhs, exact = pkg.poisson_vectors(N)
    lv = G.build_host(ai, aj, aa)
    levels = _levels_as_oracle(ai, aj, aa, lv)
    xo, its_o, reason_o, hist_o = ksp_cg.cg(ai, aj, aa, rhs, pc=lambda r: ogamg.vcycle(levels, r), **TOL)
    A, ksp, x = _solve(pkg, ai, aj, aa, rhs)
    try:
        its, reason, hist = ksp.its, ksp.reason, ksp.history()
        rows, _, _ = ksp.pc_levels()
    finally:
        ksp.destroy()
        A.destroy()
    err = float(np.max(np.abs(x - exact)))
    print(f"\n100^3 CG+GAMG: its {its} (oracle {its_o}) reason {reason} Linf {err:.3e} "
          f"(h^2 x {err * N * N:.2f}) levels {rows}")
    assert rows == [L["m"] for L in lv]
    assert reason == reason_o and reason > 0
    assert abs(its - its_o) <= 1 and abs(its - PINNED_ITS[N]) <= 1, (its, its_o)
    k = min(len(hist), len(hist_o))
    np.testing.assert_allclose(hist[:min(k, 10)], hist_o[:min(k, 10)], rtol=1e-7)
    # (the last norms sit at ~1e-14 of the first, where the device's and the
    # oracle's dot orders differ in the last bits: an absolute floor there)
    np.testing.assert_allclose(hist[:k], hist_o[:k], rtol=1e-4, atol=1e-15 * hist_o[0])
    assert np.linalg.norm(x - xo) <= 1e-8 * np.linalg.norm(xo)
    assert err <= C_H2 / (N * N), err
