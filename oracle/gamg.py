"""ORACLE — TEST INFRASTRUCTURE ONLY.

numpy/scipy restatement of the smoothed-aggregation hierarchy of
include/aijhip_gamg.h (PETSc 3.7.6 PCGAMG agg [ext], as configured by
/root/reference/configs/PETSc_SolverOptions_GAMG.info:6-21) and of the
multiplicative V-cycle PCMG applies with those options (Richardson(1) +
Jacobi smoothing on every level, preonly + Jacobi on the coarsest).

Parity unpinned w.r.t. PETSc (absent; its MIS aggregation order is not
reproduced). This restatement pins the product's C++ set-up and device
V-cycle: aggregates identical, operators to rounding.
"""
from __future__ import annotations

import math

import numpy as np
import scipy.sparse as sp


def first_diagonal(A: sp.csr_matrix) -> np.ndarray:
    """MatGetDiagonal: first stored diagonal entry per row (0 if none)."""
    rows = np.repeat(np.arange(A.shape[0]), np.diff(A.indptr))
    hit = np.flatnonzero(A.indices == rows)
    r, first = np.unique(rows[hit], return_index=True)  # first stored hit per row
    d = np.zeros(A.shape[0])
    d[r] = A.data[hit[first]]
    return d


def strength_graph(A, d, theta):
    rows = np.repeat(np.arange(A.shape[0]), np.diff(A.indptr))
    cols = A.indices
    v = np.abs(A.data)
    keep = (rows != cols) & (v > theta * np.sqrt(np.abs(d[rows] * d[cols])))
    S = sp.csr_matrix((np.ones(keep.sum()), (rows[keep], cols[keep])), shape=A.shape)
    S = ((S + S.T) != 0).astype(np.int8).tocsr()
    S.sort_indices()
    return S


def aggregate(A, S):
    m = A.shape[0]
    agg = -np.ones(m, dtype=np.int64)
    na = 0
    for i in range(m):
        nb = S.indices[S.indptr[i]:S.indptr[i + 1]]
        if agg[i] != -1 or len(nb) == 0:
            continue
        if np.all(agg[nb] == -1):
            agg[i] = na
            agg[nb] = na
            na += 1
    phase1 = agg.copy()
    for i in range(m):
        if phase1[i] != -1:
            continue
        nbset = set(S.indices[S.indptr[i]:S.indptr[i + 1]].tolist())
        best, bv = -1, -1.0
        for k in range(A.indptr[i], A.indptr[i + 1]):
            j = A.indices[k]
            if j == i or phase1[j] == -1 or j not in nbset:
                continue
            v = abs(A.data[k])
            if v > bv or (v == bv and j < best):
                bv, best = v, j
        if best >= 0:
            agg[i] = phase1[best]
    for i in range(m):
        if agg[i] != -1:
            continue
        agg[i] = na
        for j in S.indices[S.indptr[i]:S.indptr[i + 1]]:
            if agg[j] == -1:
                agg[j] = na
        na += 1
    return agg, na


def _mix64(z):
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9 & 0xFFFFFFFFFFFFFFFF
    z = (z ^ (z >> 27)) * 0x94D049BB133111EB & 0xFFFFFFFFFFFFFFFF
    return z ^ (z >> 31)


def _blockdot(a, b, block=256):
    """The C++ set-up's dot: left to right inside fixed 256-entry blocks,
    then the block sums left to right (np.cumsum accumulates sequentially;
    np.dot is pairwise). The aggregation of the next level is sensitive to the
    last bit of every coarse entry (ties, zero threshold), so the restatement
    keeps the order."""
    p = np.asarray(a, dtype=np.float64) * np.asarray(b, dtype=np.float64)
    n = len(p)
    if n == 0:
        return 0.0
    full = (n // block) * block  # block sums left to right, vectorised over blocks
    parts = np.cumsum(p[:full].reshape(-1, block), axis=1)[:, -1] if full else np.zeros(0)
    if full < n:
        parts = np.concatenate([parts, [np.cumsum(p[full:])[-1]]])
    return float(np.cumsum(parts)[-1])


def estimate_emax(A, dinv, its):
    """Power iteration on D^-1 A from the same counter-based start."""
    m = A.shape[0]
    v = np.array([2.0 * ((_mix64((0x5EED + (i + 1) * 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF) >> 11)
                         * (1.0 / 9007199254740992.0)) - 1.0 for i in range(m)])
    v /= math.sqrt(_blockdot(v, v))
    lam = 1.0
    for _ in range(its):
        w = dinv * (A @ v)
        nw = math.sqrt(_blockdot(w, w))
        if not nw > 0.0:
            break
        lam = nw
        v = w / nw
    return lam


def build(A, threshold=0.0, coarse_eq_limit=50, max_levels=10, nsmooths=1, smooth_scale=1.4, eig_its=10):
    """Returns a list of levels: dict(A, P, agg, emax) (P/agg absent on the coarsest)."""
    A = sp.csr_matrix(A)
    levels = []
    B = np.ones(A.shape[0])
    while len(levels) + 1 < max_levels and A.shape[0] > coarse_eq_limit:
        d = first_diagonal(A)
        dinv = 1.0 / np.where(d == 0.0, 1.0, d)
        S = strength_graph(A, d, threshold)
        agg, na = aggregate(A, S)
        if na >= A.shape[0] or na == 0:
            break
        emax = estimate_emax(A, dinv, eig_its) if nsmooths > 0 else 1.0
        Bc = np.sqrt(np.bincount(agg, weights=B * B, minlength=na))
        p0 = np.where(Bc[agg] > 0, B / np.where(Bc[agg] > 0, Bc[agg], 1.0), 0.0)
        P0 = sp.csr_matrix((p0, (np.arange(A.shape[0]), agg)), shape=(A.shape[0], na))
        P = P0
        if nsmooths > 0:
            T = A @ P0
            P = (-smooth_scale / emax) * (sp.diags(dinv) @ T) + P0
        P = sp.csr_matrix(P)
        P.sort_indices()
        PT = sp.csr_matrix(P.T)  # rows list fine rows ascending, as the C++ transpose
        PT.sort_indices()
        AP = sp.csr_matrix(A @ P)
        AP.sort_indices()
        Ac = sp.csr_matrix(PT @ AP)  # csr x csr: scipy's csr_matmat order = the C++ spgemm's
        Ac.sort_indices()
        levels.append(dict(A=A, P=P, agg=agg, emax=emax))
        A, B = Ac, Bc
    levels.append(dict(A=A))
    return levels


def vcycle(levels, b):
    """PCApply_MG, multiplicative V-cycle: Richardson(1)+Jacobi down (zero
    guess) and up (nonzero guess), P^T restriction, P interpolation, coarse
    preonly + Jacobi. The Jacobi inverses are cached in the level dicts."""
    for L in levels:
        if "dinv" not in L:
            d = first_diagonal(L["A"])
            L["dinv"] = 1.0 / np.where(d == 0.0, 1.0, d)

    def cycle(l, bl):
        A, dinv = levels[l]["A"], levels[l]["dinv"]
        x = dinv * bl
        if l == len(levels) - 1:
            return x
        r = bl - A @ x
        xc = cycle(l + 1, levels[l]["P"].T @ r)
        x = x + levels[l]["P"] @ xc
        x = x + dinv * (bl - A @ x)
        return x

    return cycle(0, np.asarray(b, dtype=np.float64))
