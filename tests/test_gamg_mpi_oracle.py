"""oracle/gamg_mpi.py (the distributed smoothed-aggregation hierarchy,
restated globally) on the CPU: at one rank it is oracle/gamg.py's hierarchy;
PETSc's parallel MIS (ghost states exchanged, restated as the global MIS by
global keys) makes the aggregates independent of the partition, so over k
z-slabs the hierarchy and the CG iterations are one rank's, where block
Jacobi with a hierarchy per slab grows (the reference's multi-rank solver is
PETSc's parallel agg GAMG: /root/reference/runs/single-node-scaling.pbs:56-67)."""
import numpy as np
import scipy.sparse as sp

from oracle import gamg as og
from oracle import gamg_mpi as ogm
from oracle import ksp_cg, seqaij

TOL = dict(rtol=1e-14, atol=1e-12, max_it=1000)


def _system(N):
    ai, aj, aa, rhs, _ = seqaij.create_system(N, N, N)
    return ai, aj, aa, rhs, sp.csr_matrix((aa, aj, ai), shape=(N ** 3,) * 2)


def test_one_rank_is_the_single_hierarchy():
    ai, aj, aa, rhs, A = _system(14)
    single = og.build(A)
    dist = ogm.build(A, [0, A.shape[0]])
    assert [L["A"].shape for L in single] == [L["A"].shape for L in dist]
    for s, d in zip(single, dist):
        assert (s["A"] != d["A"]).nnz == 0
        if "P" in s:
            assert np.array_equal(s["agg"], d["agg"])
            np.testing.assert_allclose(s["P"].toarray(), d["P"].toarray(), rtol=0, atol=1e-15)


def test_slabs_keep_the_iteration_count():
    N = 20
    ai, aj, aa, rhs, A = _system(N)
    its = {}
    for k in (1, 2, 4):
        starts = [(r * N // k) * N * N for r in range(k)] + [N ** 3]
        L = ogm.build(A, starts)
        its[k] = ksp_cg.cg(ai, aj, aa, rhs, pc=lambda r: ogm.vcycle(L, r), **TOL)[1]
    # block Jacobi + a hierarchy per slab (no coupling) at 4 slabs, for contrast
    starts = [(r * N // 4) * N * N for r in range(4)] + [N ** 3]
    blocks = [(lo, hi, og.build(sp.csr_matrix(A[lo:hi, lo:hi]))) for lo, hi in zip(starts[:-1], starts[1:])]

    def bjacobi(r):
        return np.concatenate([og.vcycle(lv, r[lo:hi]) for lo, hi, lv in blocks])

    bj = ksp_cg.cg(ai, aj, aa, rhs, pc=bjacobi, **TOL)[1]
    print(f"\nCG iterations: distributed GAMG {its}, bjacobi+GAMG at 4 slabs {bj}")
    assert its[2] == its[1] and its[4] == its[1]
    assert bj > 1.1 * its[1]


def test_mis_aggregates_do_not_depend_on_the_partition():
    """Roots independent across slab boundaries (no two within reach of each
    other, wherever they live), every node with a strong neighbour in an
    aggregate, and the same aggregates and coarse numbering at 1, 2, 3 and 5
    slabs; the greedy pass (coarsen 0) stays per slab and differs."""
    N = 12
    _, _, _, _, A = _system(N)
    ref = ogm.build(A, [0, N ** 3], max_levels=2)
    for k in (2, 3, 5):
        starts = [(r * N // k) * N * N for r in range(k)] + [N ** 3]
        L = ogm.build(A, starts, max_levels=2)
        assert np.array_equal(L[0]["agg"], ref[0]["agg"]), k
        assert L[0]["P"].shape == ref[0]["P"].shape
        np.testing.assert_allclose(L[0]["P"].toarray(), ref[0]["P"].toarray(), rtol=0, atol=1e-15)
        cs = L[1]["starts"]
        assert cs[0] == 0 and cs[-1] == ref[1]["A"].shape[0] and np.all(np.diff(cs) >= 0)
    # roots: distance >= 3 in S (the squared graph's independence)
    S = og.strength_graph(sp.csr_matrix(A), og.first_diagonal(A), 0.0)
    _, _, roots = og.aggregate_mis(S, True, og.mis_keys(N ** 3, 0), return_roots=True)
    G1 = (S + sp.identity(N ** 3, format="csr")).tocsr()
    G2 = (G1 @ G1).tocsr()
    assert G2[roots][:, roots].nnz == len(roots)  # only each root itself within two steps
    g = ogm.build(A, [0, N ** 3 // 2, N ** 3], coarsen=0, max_levels=2)
    assert not np.array_equal(g[0]["agg"], ogm.build(A, [0, N ** 3], coarsen=0, max_levels=2)[0]["agg"])
