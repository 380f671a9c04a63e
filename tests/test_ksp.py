"""CG (KSPSolve_CG restatement): oracle sanity on CPU, device CG vs oracle on
the GPU. CG reorders dot products relative to PETSc's BLAS, so the bar is
rounding-level agreement: same converged reason, iteration count within 1,
residual history within rtol 1e-8 over the first 30 iterations, and the
solutions within 1e-9 relative."""
import importlib

import numpy as np
import pytest

from conftest import golden
from oracle import ksp_cg, seqaij


def test_oracle_cg_solves_poisson():
    ai, aj, aa, rhs, exact = seqaij.create_system(6, 6, 6)
    x, its, reason, hist = ksp_cg.cg(ai, aj, aa, rhs, rtol=1e-14, atol=1e-12, max_it=10000)
    assert reason in (ksp_cg.CONVERGED_RTOL, ksp_cg.CONVERGED_ATOL)
    assert its < 6 ** 3
    r = rhs - seqaij.matmult(ai, aj, aa, x)
    assert np.linalg.norm(r) <= 1e-8 * np.linalg.norm(rhs)
    assert len(hist) == its + 1


def test_oracle_cg_exact_in_n_steps():
    rng = np.random.default_rng(3)
    n = 12
    M = rng.standard_normal((n, n))
    A = M @ M.T + n * np.eye(n)
    ai = np.arange(0, n * n + 1, n, dtype=np.int32)
    aj = np.tile(np.arange(n, dtype=np.int32), n)
    aa = A.ravel()
    b = rng.standard_normal(n)
    x, its, reason, _ = ksp_cg.cg(ai, aj, aa, b, rtol=1e-12, max_it=100, pc="none")
    assert its <= n + 1 and reason == ksp_cg.CONVERGED_RTOL
    np.testing.assert_allclose(x, np.linalg.solve(A, b), rtol=1e-9)


def test_oracle_cg_max_it():
    ai, aj, aa, rhs, _ = seqaij.create_system(5, 5, 5)
    _, its, reason, hist = ksp_cg.cg(ai, aj, aa, rhs, rtol=0.0, atol=0.0, max_it=7)
    assert reason == ksp_cg.DIVERGED_ITS and its == 7 and len(hist) == 8


# ------------------------------------------------------------------- GPU
def _gpu(pkg):
    torch = pytest.importorskip("torch")
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    return torch, importlib.import_module("petsc-openacc_amd.ksp")


@pytest.mark.gpu
@pytest.mark.parametrize("N,kernel,pc,norm", [
    (16, "auto", "jacobi", "preconditioned"),
    (16, "scalar", "jacobi", "preconditioned"),      # unfused SpMV + dot path
    (24, "auto", "none", "unpreconditioned"),
    (30, "auto", "jacobi", "natural"),
])
def test_gpu_cg_matches_oracle(pkg, N, kernel, pc, norm):
    torch, K = _gpu(pkg)
    ai, aj, aa = pkg.poisson_csr(N)
    rhs, exact = pkg.poisson_vectors(N)
    tol = dict(rtol=1e-14, atol=1e-12, max_it=10000)  # PETSc_SolverOptions_GAMG.info:2-4
    xo, its_o, reason_o, hist_o = ksp_cg.cg(ai, aj, aa, rhs, pc=pc, norm=norm, **tol)
    A = pkg.SeqAIJHIP(ai, aj, aa, kernel=kernel)
    b = torch.from_numpy(rhs).cuda()
    x = torch.empty_like(b)
    with K.KSPCG(A, pc=pc, norm=norm, **tol) as ksp:
        ksp.solve(b, x)
        torch.cuda.synchronize()
        assert ksp.fused == (kernel == "auto")
        assert ksp.reason == reason_o, (ksp.reason, reason_o)
        assert abs(ksp.its - its_o) <= 1, (ksp.its, its_o)
        h = ksp.history()
        k = min(30, len(h), len(hist_o))
        np.testing.assert_allclose(h[:k], hist_o[:k], rtol=1e-8)
        xg = x.cpu().numpy()
        assert np.linalg.norm(xg - xo) <= 1e-9 * np.linalg.norm(xo)
        r = rhs - seqaij.matmult(ai, aj, aa, xg)
        assert np.linalg.norm(r) <= 1e-8 * np.linalg.norm(rhs)
    A.destroy()


@pytest.mark.gpu
def test_gpu_cg_edge_cases(pkg):
    torch, K = _gpu(pkg)
    ai, aj, aa = pkg.poisson_csr(8)
    A = pkg.SeqAIJHIP(ai, aj, aa)
    b = torch.zeros(A.m, dtype=torch.float64, device="cuda")
    x = torch.full_like(b, 3.0)
    with K.KSPCG(A, rtol=1e-10) as ksp:  # zero rhs: converged at iteration 0, x = 0
        ksp.solve(b, x)
        assert ksp.its == 0 and ksp.reason == 3 and torch.count_nonzero(x).item() == 0
    rhs, _ = pkg.poisson_vectors(8)
    b = torch.from_numpy(rhs).cuda()
    with K.KSPCG(A, rtol=0.0, atol=0.0, max_it=13) as ksp:  # max_it reached
        ksp.solve(b, x)
        assert ksp.its == 13 and ksp.reason == -3 and len(ksp.history()) == 14
        _, its_o, reason_o, hist_o = ksp_cg.cg(ai, aj, aa, rhs, rtol=0.0, atol=0.0, max_it=13)
        np.testing.assert_allclose(ksp.history(), hist_o, rtol=1e-8)
    # nonzero initial guess
    x0 = pkg.splitmix_uniform(A.m, 5)
    xo, its_o, reason_o, hist_o = ksp_cg.cg(ai, aj, aa, rhs, x0=x0, rtol=1e-10)
    x = torch.from_numpy(x0.copy()).cuda()
    with K.KSPCG(A, rtol=1e-10, guess_nonzero=True) as ksp:
        ksp.solve(b, x)
        assert ksp.reason == reason_o and abs(ksp.its - its_o) <= 1
        np.testing.assert_allclose(ksp.history()[:10], hist_o[:10], rtol=1e-8)
    A.destroy()


@pytest.mark.gpu
def test_gpu_cg_deterministic(pkg):
    torch, K = _gpu(pkg)
    g = golden("poisson16")
    A = pkg.SeqAIJHIP(g["ai"], g["aj"], g["aa"])
    b = torch.from_numpy(g["rhs"]).cuda()
    xs = []
    with K.KSPCG(A, rtol=1e-12) as ksp:
        for _ in range(2):
            x = torch.empty_like(b)
            ksp.solve(b, x)
            xs.append(x.cpu().numpy())
    assert np.array_equal(xs[0].view(np.uint64), xs[1].view(np.uint64))
    A.destroy()


@pytest.mark.gpu
@pytest.mark.parametrize("pc,guess", [("gamg", False), ("jacobi", False), ("jacobi", True)])
def test_gpu_solve_host_vectors_equals_device_solve(pkg, pc, guess):
    """KSPSolve with host b / x (aijhip_ksp_solve_host: the solve-level
    offload a registered PETSc KSP type uses, b up and x down once per
    solve) is the device solve bit for bit, iterations and history too, with a
    zero and with a nonzero initial guess."""
    import torch
    K = importlib.import_module("petsc-openacc_amd.ksp")
    N = 20
    ai, aj, aa = pkg.poisson_csr(N)
    rhs, _ = pkg.poisson_vectors(N)
    x0 = pkg.splitmix_uniform(len(rhs), 3) if guess else np.zeros(len(rhs))
    with pkg.SeqAIJHIP(ai, aj, aa) as A:
        with K.KSPCG(A, rtol=1e-12, atol=1e-14, pc=pc, guess_nonzero=guess) as ksp:
            b = torch.from_numpy(rhs).cuda()
            xd = torch.from_numpy(x0.copy()).cuda()
            ksp.solve(b, xd)
            torch.cuda.synchronize()
            its_d, hist_d, xdev = ksp.its, np.array(ksp.history()), xd.cpu().numpy()
            xh = x0.copy()
            ksp.solve_host(rhs, xh)
            assert ksp.its == its_d
            assert np.array_equal(np.array(ksp.history()).view(np.uint64), hist_d.view(np.uint64))
            assert np.array_equal(xh.view(np.uint64), xdev.view(np.uint64))


@pytest.mark.gpu
@pytest.mark.parametrize("pc", ["gamg", "jacobi"])
def test_gpu_replanned_operator_sets_up_again(pkg, pc):
    """PCSetUp semantics on a changed operator: re-planning the handle
    (set_option, MatAssemblyEnd) changes its plan generation, and the next
    KSPSolve sets the KSP up again (Jacobi diagonal, the GAMG hierarchy, the
    partial buffers sized by the new plan) instead of reading a stale plan:
    the solve is a fresh KSP's bit for bit."""
    import torch
    K = importlib.import_module("petsc-openacc_amd.ksp")
    N = 24
    ai, aj, aa = pkg.poisson_csr(N)
    rhs, _ = pkg.poisson_vectors(N)
    b = torch.from_numpy(rhs).cuda()

    def run(ksp):
        x = torch.zeros_like(b)
        ksp.solve(b, x)
        torch.cuda.synchronize()
        return ksp.its, np.array(ksp.history()), x.cpu().numpy()

    with pkg.SeqAIJHIP(ai, aj, aa, geometry=6) as A:
        with K.KSPCG(A, rtol=1e-12, atol=1e-14, pc=pc) as ksp:
            run(ksp)
            A.set_option("geometry", 8)  # 256-row blocks instead of 512: a new plan, twice the partials
            got = run(ksp)
        with K.KSPCG(A, rtol=1e-12, atol=1e-14, pc=pc) as fresh:
            ref = run(fresh)
    assert got[0] == ref[0]
    assert np.array_equal(got[1].view(np.uint64), ref[1].view(np.uint64))
    assert np.array_equal(got[2].view(np.uint64), ref[2].view(np.uint64))
