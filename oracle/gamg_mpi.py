"""ORACLE — TEST INFRASTRUCTURE ONLY.

numpy/scipy restatement of the distributed smoothed-aggregation hierarchy of
petsc-openacc_amd/csrc/gamg_mpi.hip (PCGAMG across ranks, the agg GAMG the
reference runs on 1-16 MPI ranks: /root/reference/runs/single-node-scaling.pbs
:56-67 with /root/reference/configs/PETSc_SolverOptions_GAMG.info:6-21),
computed globally:

  - rank r owns rows [starts[r], starts[r+1]) of every level;
  - aggregates: PETSc's parallel MIS (coarsen 1, the default; mis.c
    maxIndSetAgg exchanges ghost states every round, so roots on either side
    of a rank boundary are independent and a node deleted by a root on
    another rank joins that root's aggregate) restated as the
    lexicographically-first MIS of the GLOBAL strength graph (squared on the
    first square_graph levels) by keys at GLOBAL indices: oracle/gamg.py's
    aggregate_mis on the whole operator, so the aggregates do not depend on
    the partition; rank r owns the aggregates rooted in its rows (coarse rows
    of rank r = [cstarts[r], cstarts[r+1]), the roots in natural order). The
    source (PETSc 3.7.6 src/mat/coarsen/impls/mis/mis.c) is absent from
    /root/reference (fetched by scripts/petsc.sh:37-41): parity unpinned.
    The greedy pass (coarsen 0) stays on each rank's diagonal block;
  - emax by CG's Lanczos estimate (eig_ksp 1, the default) or the power
    iteration (0) on the global D^-1 A from oracle/gamg.py's start vector at
    global indices (the device sums its dots rank by rank: equal to
    rounding);
  - P0, P = P0 - 1.4/emax D^-1 A P0 and A_c = P^T A P over the whole operator;
  - the hierarchy stops where the single-GPU one does, with global counts.

The V-cycle is oracle/gamg.py's (global operators; the distributed one is the
same arithmetic up to summation order). Parity unpinned w.r.t. PETSc, as for
oracle/gamg.py.
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp

from oracle import gamg as og


def build(A, starts, threshold=0.0, coarse_eq_limit=50, max_levels=10, nsmooths=1, smooth_scale=1.4, eig_its=10,
          B=None, coarsen=1, square_graph=1, eig_ksp=1, level0=0):
    """A: global operator; starts: row ownership (len = ranks + 1); B: the
    near-null space (ones). Returns a list of levels dict(A, P, starts, emax,
    agg, Bc) in oracle/gamg.py's format (vcycle-compatible). level0: the
    level index of A (the MIS keys' level)."""
    A = sp.csr_matrix(A)
    starts = np.asarray(starts, dtype=np.int64)
    levels = []
    B = np.ones(A.shape[0]) if B is None else np.asarray(B, dtype=np.float64)
    while len(levels) + 1 < max_levels and A.shape[0] > coarse_eq_limit:
        d = og.first_diagonal(A)
        dinv = 1.0 / np.where(d == 0.0, 1.0, d)
        lvl = level0 + len(levels)
        if coarsen == 1:  # the global MIS (partition-independent)
            As = sp.csr_matrix(A)
            As.sort_indices()
            S = og.strength_graph(As, d, threshold)
            agg, NA, roots = og.aggregate_mis(S, lvl < square_graph, og.mis_keys(A.shape[0], lvl), return_roots=True)
            cstarts = np.searchsorted(roots, starts, side="left").astype(np.int64)
        else:
            aggs, nas = [], []
            for r in range(len(starts) - 1):
                lo, hi = starts[r], starts[r + 1]
                Ad = sp.csr_matrix(A[lo:hi, lo:hi])
                Ad.sort_indices()
                S = og.strength_graph(Ad, d[lo:hi], threshold)
                agg, na = og.aggregate(Ad, S)
                aggs.append(agg)
                nas.append(na)
            cstarts = np.concatenate([[0], np.cumsum(nas)]).astype(np.int64)
            agg = np.concatenate([np.where(a >= 0, a + cstarts[r], -1) for r, a in enumerate(aggs)])
        NA = int(cstarts[-1])
        if NA == 0 or NA >= A.shape[0]:
            break
        if nsmooths > 0:
            emax = og.estimate_emax_cg(A, dinv, eig_its) if eig_ksp == 1 else og.estimate_emax(A, dinv, eig_its)
        else:
            emax = 1.0
        kept = agg >= 0  # MIS removes singletons: no aggregate, an empty row of P0
        Bc = np.sqrt(np.bincount(agg[kept], weights=(B * B)[kept], minlength=NA))
        aggk = np.where(kept, agg, 0)
        p0 = np.where(kept & (Bc[aggk] > 0), B / np.where(Bc[aggk] > 0, Bc[aggk], 1.0), 0.0)
        P0 = sp.csr_matrix((p0[kept], (np.arange(A.shape[0])[kept], agg[kept])), shape=(A.shape[0], NA))
        P = P0
        if nsmooths > 0:
            P = (-smooth_scale / emax) * (sp.diags(dinv) @ (A @ P0)) + P0
        P = sp.csr_matrix(P)
        P.sort_indices()
        Ac = sp.csr_matrix(P.T @ (A @ P))
        Ac.sort_indices()
        levels.append(dict(A=A, P=P, starts=starts, emax=emax, agg=agg, Bc=Bc))
        A, B, starts = Ac, Bc, cstarts
    levels.append(dict(A=A, starts=starts))
    return levels


def vcycle(levels, b):
    return og.vcycle(levels, b)
