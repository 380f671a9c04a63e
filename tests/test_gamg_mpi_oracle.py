"""oracle/gamg_mpi.py (the distributed smoothed-aggregation hierarchy,
restated globally) on the CPU: at one rank it is oracle/gamg.py's hierarchy;
over k z-slabs its CG iterations stay within 10 % of one rank's, where block
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
    assert all(its[k] <= 1.1 * its[1] for k in its)
    assert bj > 1.1 * its[1]
