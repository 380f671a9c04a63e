#!/usr/bin/env python3
"""Study (not product code): parallel MIS-2 aggregation against the greedy
natural-order aggregation the GAMG set-up uses (oracle/gamg.py aggregate),
CG + V-cycle iterations on the reference operand at N^3 (oracle CG +
oracle V-cycle, rtol 1e-12).

    python tools/agg_mis2_study.py N [thresholds, e.g. 2,3,4]

Variants: MIS-2 roots (Luby rounds on hashed priorities, distance-2 key
maxima) + their strong neighbours, left-overs joined to the strongest
aggregated neighbour; and the same plus a second MIS-2 round on the
still-free nodes that have >= t free strong neighbours. Results in
profiles/r02/agg_mis2_study.txt.
"""
import sys, time
sys.path.insert(0, '.')
import numpy as np, scipy.sparse as sp
from oracle import gamg as og, ksp_cg, seqaij

M64 = np.uint64(0xFFFFFFFFFFFFFFFF)
def mix64v(z):
    with np.errstate(over='ignore'):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))

def rowmax(S, v):
    out = v.copy()
    nz = np.diff(S.indptr) > 0
    if S.nnz:
        red = np.maximum.reduceat(v[S.indices], S.indptr[:-1][nz])
        out[nz] = np.maximum(out[nz], red)
    return out

def mis2(S, cand, seed=0x6A09E667F3BCC908):
    """MIS-2 restricted to cand nodes (others treated as absent). returns root mask"""
    m = S.shape[0]
    idx = np.arange(m, dtype=np.uint64)
    with np.errstate(over='ignore'):
        h = mix64v(np.uint64(seed) + idx) >> np.uint64(35)
    base = (h << np.uint64(32)) | idx
    state = np.where(cand, 1, 0).astype(np.uint64)
    while True:
        und = state == 1
        if not und.any(): break
        key = np.where(cand, (state << np.uint64(61)) | base, np.uint64(0))
        k2 = rowmax(S, rowmax(S, key))
        win = und & ((k2 & np.uint64(0xFFFFFFFF)) == idx)
        lose = und & ~win & ((k2 >> np.uint64(61)) == 2)
        state[win] = 2; state[lose] = 0
    return state == 2

def join_roots(S, roots, agg, na):
    m = S.shape[0]
    ids = np.full(m, -1, np.int64); ids[roots] = na + np.arange(roots.sum())
    agg[roots] = ids[roots]
    r = np.where(roots[S.indices], ids[S.indices], -1)
    nz = np.diff(S.indptr) > 0
    best = np.full(m, -1, np.int64)
    if S.nnz: best[nz] = np.maximum.reduceat(r, S.indptr[:-1][nz])
    sel = (agg == -1) & (best >= 0)
    agg[sel] = best[sel]
    return na + int(roots.sum())

def phase2(A, S, agg):
    phase1 = agg.copy()
    m = A.shape[0]
    for i in np.flatnonzero(phase1 == -1):
        nbset = set(S.indices[S.indptr[i]:S.indptr[i+1]].tolist())
        best, bv = -1, -1.0
        for k in range(A.indptr[i], A.indptr[i+1]):
            j = A.indices[k]
            if j == i or phase1[j] == -1 or j not in nbset: continue
            v = abs(A.data[k])
            if v > bv or (v == bv and j < best): bv, best = v, j
        if best >= 0: agg[i] = phase1[best]

def agg_mis2(A, S):
    m = A.shape[0]; agg = -np.ones(m, np.int64)
    na = join_roots(S, mis2(S, np.ones(m, bool)), agg, 0)
    phase2(A, S, agg)
    left = agg == -1
    for i in np.flatnonzero(left):
        if agg[i] != -1: continue
        agg[i] = na
        for j in S.indices[S.indptr[i]:S.indptr[i+1]]:
            if agg[j] == -1: agg[j] = na
        na += 1
    return agg, na

def agg_mis2_rounds(A, S):
    """MIS-2 roots + neighbours; then repeatedly MIS-2 on the free nodes among
    themselves (aggregates of free nodes only, needing all neighbours... ) """
    m = A.shape[0]; agg = -np.ones(m, np.int64)
    na = join_roots(S, mis2(S, np.ones(m, bool)), agg, 0)
    # second round: free nodes whose strong neighbours are all free... rarely; use free subgraph
    free = agg == -1
    Sf = sp.csr_matrix(S.multiply(free[:, None]).multiply(free[None, :]))
    Sf.eliminate_zeros()
    cand = free & (np.diff(Sf.indptr) > 0)
    r2 = mis2(Sf, cand)
    na = join_roots(Sf, r2, agg, na)
    phase2(A, S, agg)
    for i in np.flatnonzero(agg == -1):
        if agg[i] != -1: continue
        agg[i] = na
        for j in S.indices[S.indptr[i]:S.indptr[i+1]]:
            if agg[j] == -1: agg[j] = na
        na += 1
    return agg, na

N = int(sys.argv[1]) if len(sys.argv) > 1 else 48
ai, aj, aa, rhs, ex = seqaij.create_system(N, N, N)
_greedy = og.aggregate
for name, fn in (("greedy", _greedy), ("mis2+free", agg_mis2_rounds)):
    og.aggregate = fn
    t = time.time()
    lv = og.build(sp.csr_matrix((aa, aj, ai), shape=(N**3,)*2))
    x, its, reason, hist = ksp_cg.cg(ai, aj, aa, rhs, rtol=1e-12, atol=1e-50, pc=lambda r: og.vcycle(lv, r))
    print(N, name, "levels", [L["A"].shape[0] for L in lv], "nnz", [L["A"].nnz for L in lv], "its", its, "%.1fs" % (time.time() - t), flush=True)

def make_thr(t):
    def f(A, S):
        m = A.shape[0]; agg = -np.ones(m, np.int64)
        na = join_roots(S, mis2(S, np.ones(m, bool)), agg, 0)
        free = agg == -1
        Sf = sp.csr_matrix(S.multiply(free[:, None]).multiply(free[None, :]))
        Sf.eliminate_zeros()
        cand = free & (np.diff(Sf.indptr) >= t)
        r2 = mis2(Sf, cand)
        na = join_roots(Sf, r2, agg, na)
        phase2(A, S, agg)
        for i in np.flatnonzero(agg == -1):
            if agg[i] != -1: continue
            agg[i] = na
            for j in S.indices[S.indptr[i]:S.indptr[i+1]]:
                if agg[j] == -1: agg[j] = na
            na += 1
        return agg, na
    return f

if len(sys.argv) > 2:
    for t in [int(v) for v in sys.argv[2].split(",")]:
        og.aggregate = make_thr(t)
        lv = og.build(sp.csr_matrix((aa, aj, ai), shape=(N**3,)*2))
        x, its, reason, hist = ksp_cg.cg(ai, aj, aa, rhs, rtol=1e-12, atol=1e-50, pc=lambda r: og.vcycle(lv, r))
        nnz = [L["A"].nnz for L in lv]
        print(N, "thr", t, "levels", [L["A"].shape[0] for L in lv], "nnz", nnz, "its", its, flush=True)
