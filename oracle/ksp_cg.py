"""ORACLE — TEST INFRASTRUCTURE ONLY.

numpy restatement of PETSc 3.7.6's KSPSolve_CG [ext] (src/ksp/ksp/impls/cg/
cg.c, not in the image) with KSPConvergedDefault [ext] and PCApply_Jacobi,
as the reference drives it (/root/reference/src/main_ksp.cpp:92-103,
/root/reference/configs/PETSc_SolverOptions_GAMG.info:1-4). Used only by
tests/ and bench.py's cpu_baseline leg.

Parity unpinned: PETSc is absent, so this restatement is checked against the
analytic facts of CG (exact convergence in n steps on tiny SPD systems,
A-orthogonality) and the GPU path against it to rounding. PETSc's BLAS ddot /
dnrm2 summation orders are not reproduced (np.dot), so iteration counts may
differ by one at a tolerance boundary.
"""
from __future__ import annotations

import math

import numpy as np

from . import seqaij

CONVERGED_RTOL, CONVERGED_ATOL = 2, 3
DIVERGED_ITS, DIVERGED_DTOL, DIVERGED_INDEFINITE_PC, DIVERGED_NANORINF, DIVERGED_INDEFINITE_MAT = -3, -4, -8, -9, -10


def jacobi_inverse(ai, aj, aa):
    """PCSetUp_Jacobi [ext]: first stored diagonal entry, 0 -> 1, reciprocal."""
    m = len(ai) - 1
    d = np.zeros(m)
    for i in range(m):
        for k in range(ai[i], ai[i + 1]):
            if aj[k] == i:
                d[i] = aa[k]
                break
    d[d == 0.0] = 1.0
    return 1.0 / d


def cg(ai, aj, aa, b, x0=None, rtol=1e-5, atol=1e-50, dtol=1e5, max_it=10000, pc="jacobi",
       norm="preconditioned", matmult=None):
    """Returns (x, its, reason, history)."""
    mm = matmult or (lambda v: seqaij.matmult(ai, aj, aa, v))
    if callable(pc):  # e.g. oracle.gamg.vcycle bound to a hierarchy
        apply_pc = pc
    else:
        dinv = jacobi_inverse(ai, aj, aa) if pc == "jacobi" else None
        apply_pc = (lambda r: dinv * r) if dinv is not None else (lambda r: r.copy())
    guess_zero = x0 is None
    x = np.zeros_like(b) if guess_zero else x0.copy()
    r = b.copy() if guess_zero else b - mm(x)
    z = apply_pc(r)

    def nrm(z, r):
        if norm == "preconditioned":
            return math.sqrt(float(np.dot(z, z)))
        if norm == "unpreconditioned":
            return math.sqrt(float(np.dot(r, r)))
        return math.sqrt(abs(float(np.dot(z, r))))

    dp = nrm(z, r)
    hist = [dp]
    snorm = dp
    if not guess_zero:
        sb = apply_pc(b) if norm != "unpreconditioned" else b
        snorm = math.sqrt(float(np.dot(sb, sb)))
    ttol = max(rtol * snorm, atol)

    def test(rn):
        if math.isnan(rn) or math.isinf(rn):
            return DIVERGED_NANORINF
        if rn <= ttol:
            return CONVERGED_ATOL if rn < atol else CONVERGED_RTOL
        if rn >= dtol * snorm:
            return DIVERGED_DTOL
        return 0

    reason = test(dp)
    if reason:
        return x, 0, reason, hist
    beta = float(np.dot(z, r))
    p = np.zeros_like(b)
    betaold = dpi = 0.0
    i = 0
    its = 0
    while i < max_it:
        its = i + 1
        if beta == 0.0:
            return x, its, CONVERGED_ATOL, hist
        if i > 0 and beta * betaold < 0.0:
            return x, its, DIVERGED_INDEFINITE_PC, hist
        if i == 0:
            p = z.copy()
        else:
            p = z + (beta / betaold) * p
        w = mm(p)
        dpiold, dpi = dpi, float(np.dot(p, w))
        betaold = beta
        if dpi == 0.0 or (i > 0 and dpi * dpiold <= 0.0):
            return x, its, DIVERGED_INDEFINITE_MAT, hist
        a = beta / dpi
        x = x + a * p
        r = r + (-a) * w
        z = apply_pc(r)
        dp = nrm(z, r)
        hist.append(dp)
        reason = test(dp)
        if reason:
            return x, its, reason, hist
        beta = float(np.dot(z, r))
        i += 1
    return x, its, DIVERGED_ITS, hist
