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


# ---------------------------------------------------------------------------
# PETSc 3.7's own agg coarsening (the reference's options leave
# -pc_gamg_square_graph at its default 1; /root/reference/configs/
# PETSc_SolverOptions_GAMG.info:6-9). Restated from PETSc 3.7.6's published
# src/ksp/pc/impls/gamg/agg.c (PCGAMGCoarsen_AGG, smoothAggs) and
# src/mat/coarsen/impls/mis/mis.c (maxIndSetAgg) — sources ABSENT from
# /root/reference (PETSc is fetched by scripts/petsc.sh:37-41), so parity
# with PETSc's hierarchy is unpinned:
#   graph G1   = the filtered graph (|a_ij| > threshold * sqrt|a_ii a_jj|,
#                the diagonal kept; our strength graph S plus the diagonal);
#   G2         = G1's square (distance <= 2) on the first `square_graph`
#                levels, else G1;
#   order      = PETSc shuffles the natural order with PetscRandom swaps;
#                its rand48 stream is not reproducible here, so the order is
#                the ascending order of a counter-based 64-bit hash (mis_keys);
#   MIS        = one pass in that order: an undone node with a G2 neighbour
#                becomes a root and takes every undone G2 neighbour (strict
#                aggregates); a node alone in its G2 row is removed (no
#                aggregate: a zero row of P0 — the reference point row 0 of
#                helper.cpp:264-274 has only explicit zeros off the diagonal);
#   smoothAggs = squared levels only: the roots in natural order each take
#                every G1 neighbour that sits in another root's aggregate.
# Coarse points are numbered by their roots in natural order (formProl0).
MIS_SEED = 0x4D495332  # "MIS2"
_M64 = 0xFFFFFFFFFFFFFFFF


def _mix64_np(z):
    z = np.asarray(z, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def mis_keys(m, level, seed=MIS_SEED):
    """The MIS visiting order's keys: (hash >> 32) << 32 | node — unique, so
    the order is total; ascending key = visiting order."""
    i = np.arange(m, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64((seed + level * 0x632BE59BD9B4E019) & _M64) + (i + np.uint64(1)) * np.uint64(0x9E3779B97F4A7C15)
    return ((_mix64_np(z) >> np.uint64(32)) << np.uint64(32)) | i


def _graph_rows(S):
    """G1 = S + I as row lists (ascending columns)."""
    m = S.shape[0]
    G1 = (S + sp.identity(m, dtype=np.int8, format="csr")).tocsr()
    G1.sort_indices()
    return G1


def aggregate_mis(S, square, keys, return_roots=False):
    """PETSc's MIS aggregation (restated literally, sequential): returns
    (agg, na), agg[i] = -1 for removed singletons (return_roots: and the
    roots, ascending — aggregate c is rooted at roots[c])."""
    m = S.shape[0]
    G1 = _graph_rows(S)
    if square:
        G2 = (G1.astype(np.int64) @ G1.astype(np.int64)).tocsr()
        G2.sort_indices()
    else:
        G2 = G1
    NOT_DONE, DELETED, SELECTED = 0, 1, 2
    state = np.zeros(m, np.int8)
    removed = np.zeros(m, bool)
    parent = np.full(m, -1, np.int64)
    for lid in np.argsort(keys, kind="stable"):
        if removed[lid] or state[lid] != NOT_DONE:
            continue
        nb = G2.indices[G2.indptr[lid]:G2.indptr[lid + 1]]
        if len(nb) < 2:
            removed[lid] = True
            continue
        state[lid] = SELECTED
        parent[lid] = lid
        for j in nb:
            if state[j] == NOT_DONE:
                state[j] = DELETED
                parent[j] = lid
    if square:  # smoothAggs: roots in natural order take their G1 neighbours
        for lid in np.flatnonzero(state == SELECTED):
            for j in G1.indices[G1.indptr[lid]:G1.indptr[lid + 1]]:
                if state[j] == DELETED and parent[j] != lid:
                    parent[j] = lid
    roots = np.flatnonzero(state == SELECTED)
    cidx = np.full(m, -1, np.int64)
    cidx[roots] = np.arange(len(roots))
    agg = np.where(parent >= 0, cidx[np.maximum(parent, 0)], -1)
    if return_roots:
        return agg, len(roots), roots
    return agg, len(roots)


def _tridiag_count_below(d, e, x):
    """Sturm count: eigenvalues of the symmetric tridiagonal (d, e) below x."""
    c, q = 0, 1.0
    for k in range(len(d)):
        q = (d[k] - x) - ((e[k - 1] * e[k - 1]) / q if k > 0 else 0.0)
        if q == 0.0:
            q = -1e-300
        if q < 0.0:
            c += 1
    return c


def tridiag_max_eig(d, e):
    """Largest eigenvalue of the symmetric tridiagonal (d, e) by bisection
    from the Gershgorin bounds (the C++ set-up's same steps, same bits)."""
    n = len(d)
    lo, hi = d[0], d[0]
    for k in range(n):
        r = (abs(e[k - 1]) if k > 0 else 0.0) + (abs(e[k]) if k < n - 1 else 0.0)
        lo = min(lo, d[k] - r)
        hi = max(hi, d[k] + r)
    for _ in range(200):
        mid = 0.5 * (lo + hi)
        if not (lo < mid < hi):
            break
        if _tridiag_count_below(d, e, mid) >= n:
            hi = mid
        else:
            lo = mid
    return hi


def _start_vector(m):
    return np.array([2.0 * ((_mix64((0x5EED + (i + 1) * 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF) >> 11)
                            * (1.0 / 9007199254740992.0)) - 1.0 for i in range(m)])


def estimate_emax_cg(A, dinv, its):
    """PETSc 3.7's emax for the smoother (PCGAMGOptProlongator_AGG: KSPCG
    with PC Jacobi, norm none, `its` iterations from x = 0 on a random b,
    KSPComputeExtremeSingularValues): the largest eigenvalue of CG's Lanczos
    tridiagonal, T_kk = 1/alpha_k + beta_(k-1)/alpha_(k-1), T_(k+1)k =
    sqrt(beta_k)/alpha_k. Dots in the set-up's blocked order."""
    m = A.shape[0]
    r = _start_vector(m)
    z = dinv * r
    p = z.copy()
    rz = _blockdot(z, r)
    alphas, betas = [], []
    for _ in range(its):
        w = A @ p
        pw = _blockdot(p, w)
        if not (pw != 0.0 and rz != 0.0):
            break
        a = rz / pw
        alphas.append(a)
        r = r - a * w
        z = dinv * r
        rz_new = _blockdot(z, r)
        b = rz_new / rz
        betas.append(b)
        p = z + b * p
        rz = rz_new
    n = len(alphas)
    if n == 0:
        return 1.0
    d = [1.0 / alphas[0]] + [1.0 / alphas[k] + betas[k - 1] / alphas[k - 1] for k in range(1, n)]
    e = [math.sqrt(abs(betas[k])) / alphas[k] for k in range(n - 1)]
    return tridiag_max_eig(d, e)


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


def build(A, threshold=0.0, coarse_eq_limit=50, max_levels=10, nsmooths=1, smooth_scale=1.4, eig_its=10,
          coarsen=1, square_graph=1, eig_ksp=1):
    """Returns a list of levels: dict(A, P, agg, emax) (P/agg absent on the
    coarsest). coarsen 1 (default): PETSc's MIS (squared graph on the first
    square_graph levels); 0: greedy aggregation in natural order. eig_ksp 1
    (default): CG Lanczos (PETSc's estimate); 0: power iteration."""
    A = sp.csr_matrix(A)
    levels = []
    B = np.ones(A.shape[0])
    while len(levels) + 1 < max_levels and A.shape[0] > coarse_eq_limit:
        d = first_diagonal(A)
        dinv = 1.0 / np.where(d == 0.0, 1.0, d)
        S = strength_graph(A, d, threshold)
        if coarsen == 1:
            agg, na = aggregate_mis(S, len(levels) < square_graph, mis_keys(A.shape[0], len(levels)))
        else:
            agg, na = aggregate(A, S)
        if na >= A.shape[0] or na == 0:
            break
        if nsmooths > 0:
            emax = estimate_emax_cg(A, dinv, eig_its) if eig_ksp == 1 else estimate_emax(A, dinv, eig_its)
        else:
            emax = 1.0
        member = agg >= 0
        Bc = np.sqrt(np.bincount(agg[member], weights=(B * B)[member], minlength=na))
        ga = np.where(member, agg, 0)
        p0 = np.where(member & (Bc[ga] > 0), B / np.where(Bc[ga] > 0, Bc[ga], 1.0), 0.0)
        rows = np.arange(A.shape[0])
        P0 = sp.csr_matrix((p0[member], (rows[member], agg[member])), shape=(A.shape[0], na))
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
