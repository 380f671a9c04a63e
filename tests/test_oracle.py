"""Oracle pinning (CPU): the two independent restatements of MatMult_SeqAIJ
agree bit for bit, reproduce the committed fixtures, and the operand
restatement has the structure helper.cpp implies (SURVEY.md §8 preamble)."""
import numpy as np
import pytest

from conftest import GOLDEN_NAMES, golden
from oracle import seqaij


@pytest.mark.parametrize("name", GOLDEN_NAMES)
def test_c_oracle_matches_numpy_oracle_bitwise(coracle, name):
    g = golden(name)
    ai, aj, aa, n = g["ai"], g["aj"], g["aa"], int(g["ncols"])
    y_c = coracle.matmult(ai, aj, aa, g["x"])
    y_np = seqaij.matmult(ai, aj, aa, g["x"])
    assert np.array_equal(y_c.view(np.uint64), y_np.view(np.uint64))
    w_c = coracle.matmult_add(ai, aj, aa, g["x"], g["z"])
    assert np.array_equal(w_c.view(np.uint64), seqaij.matmult_add(ai, aj, aa, g["x"], g["z"]).view(np.uint64))
    yt_c = coracle.matmult_transpose(ai, aj, aa, g["xt"], n)
    assert np.array_equal(yt_c.view(np.uint64), seqaij.matmult_transpose(ai, aj, aa, g["xt"], n).view(np.uint64))


@pytest.mark.parametrize("name", GOLDEN_NAMES)
def test_oracle_reproduces_golden(coracle, name):
    g = golden(name)
    ai, aj, aa, n = g["ai"], g["aj"], g["aa"], int(g["ncols"])
    assert np.array_equal(coracle.matmult(ai, aj, aa, g["x"]).view(np.uint64), g["y"].view(np.uint64))
    assert np.array_equal(coracle.matmult_add(ai, aj, aa, g["x"], g["z"]).view(np.uint64), g["w"].view(np.uint64))
    assert np.array_equal(coracle.matmult_transpose(ai, aj, aa, g["xt"], n).view(np.uint64),
                          g["yt"].view(np.uint64))


def test_omp_variant_bitwise(coracle):
    g = golden("poisson16")
    y1 = coracle.matmult(g["ai"], g["aj"], g["aa"], g["x"])
    yp = coracle.matmult(g["ai"], g["aj"], g["aa"], g["x"], omp=True)
    assert np.array_equal(y1.view(np.uint64), yp.view(np.uint64))


@pytest.mark.parametrize("N", [2, 3, 4, 6, 8])
def test_poisson_structure(N):
    ai, aj, aa = seqaij.generate_a(N, N, N)
    m = N ** 3
    assert len(aj) == 7 * N ** 3 - 6 * N ** 2
    lens = np.bincount(np.diff(ai), minlength=8)
    assert lens[4] == 8 and lens[5] == 12 * (N - 2) and lens[6] == 6 * (N - 2) ** 2 and lens[7] == (N - 2) ** 3
    rows = np.repeat(np.arange(m), np.diff(ai))
    assert np.all(np.diff(aj)[np.diff(rows) == 0] > 0)  # ascending within a row
    import scipy.sparse as sp
    A = sp.csr_matrix((aa, aj, ai), shape=(m, m))
    assert (A - A.T).nnz == 0  # symmetric
    assert np.all(A @ np.ones(m) == 0.0)  # all-Neumann: zero row sums (exact)


def test_ref_point(N=6):
    ai, aj, aa, rhs, exact = seqaij.create_system(N, N, N)
    m = N ** 3
    ai0, aj0, aa0 = seqaij.generate_a(N, N, N)
    assert np.array_equal(ai, ai0) and np.array_equal(aj, aj0)  # structure kept (explicit zeros)
    row0 = slice(ai[0], ai[1])
    diag = aa0[(aj0 == np.repeat(np.arange(m), np.diff(ai0)))]
    assert aa[row0][aj[row0] == 0][0] == np.add.accumulate(diag)[-1] / m
    assert np.all(aa[row0][aj[row0] != 0] == 0.0)
    rows = np.repeat(np.arange(m), np.diff(ai))
    assert np.all(aa[(aj == 0) & (rows != 0)] == 0.0)
    # the discrete problem is consistent with the analytic one: A*exact ~ rhs
    y = seqaij.matmult(ai, aj, aa, exact)
    assert np.max(np.abs(y - rhs)) / np.max(np.abs(rhs)) < 0.2


def test_splitmix_known_values():
    x = seqaij.splitmix_uniform(4, seed=42)
    assert np.all((x >= -1) & (x < 1))
    assert len(set(x.tolist())) == 4


def test_host_cg_gamg_matches_numpy_restatement():
    """oracle/cg_gamg.c (the measured host CG+GAMG baseline) against
    oracle/ksp_cg.py + oracle/gamg.py's V-cycle on the same host hierarchy."""
    import importlib

    import scipy.sparse as sp

    from oracle import gamg as ogamg
    from oracle import host_cg_gamg, ksp_cg, seqaij
    G = importlib.import_module("petsc-openacc_amd.gamg")
    ai, aj, aa, rhs, exact = seqaij.create_system(14, 14, 14)
    lv = G.build_host(ai, aj, aa)
    levels = [dict(A=sp.csr_matrix((aa, aj, ai), shape=(lv[0]["m"],) * 2))]
    for l in range(1, len(lv)):
        a_i, a_j, a_a = lv[l]["A"]
        levels.append(dict(A=sp.csr_matrix((a_a, a_j, a_i), shape=(lv[l]["m"],) * 2)))
        p_i, p_j, p_a = lv[l - 1]["P"]
        levels[l - 1]["P"] = sp.csr_matrix((p_a, p_j, p_i), shape=(lv[l - 1]["m"], lv[l]["m"]))
    xo, its_o, reason_o, hist_o = ksp_cg.cg(ai, aj, aa, rhs, rtol=1e-12, atol=1e-50,
                                            pc=lambda r: ogamg.vcycle(levels, r))
    for threads in (1, 3):
        h = host_cg_gamg.solve(ai, aj, aa, rhs, rtol=1e-12, atol=1e-50, threads=threads, levels=lv)
        assert h["reason"] == reason_o and abs(h["its"] - its_o) <= 1
        # threaded dots sum in another order: the late, 1e-12-reduced norms
        # carry round-off relative to the initial one, not to themselves
        n = min(its_o, len(h["hist"]))
        np.testing.assert_allclose(h["hist"][:n], hist_o[:n], rtol=1e-8, atol=1e-14 * hist_o[0])
        assert np.linalg.norm(h["x"] - xo) <= 1e-9 * np.linalg.norm(xo)
