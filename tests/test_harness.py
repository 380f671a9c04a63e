"""Host-side operand producers (CPU): the C++ restatement of helper.cpp used
by the benchmark must equal the numpy oracle bit for bit."""
import ctypes

import numpy as np
import pytest

from oracle import seqaij


@pytest.mark.parametrize("dims", [(4, 4, 4), (8, 8, 8), (16, 16, 16), (5, 3, 7), (1, 4, 3), (30, 30, 30)])
def test_poisson_csr_matches_oracle(pkg, dims):
    nx, ny, nz = dims
    ai, aj, aa = pkg.poisson_csr(nx, ny, nz)
    oai, oaj, oaa, orhs, oexact = seqaij.create_system(nx, ny, nz)
    assert np.array_equal(ai, oai) and np.array_equal(aj, oaj)
    assert np.array_equal(aa.view(np.uint64), oaa.view(np.uint64))
    rhs, exact = pkg.poisson_vectors(nx, ny, nz)
    assert np.array_equal(exact.view(np.uint64), oexact.view(np.uint64))
    np.testing.assert_allclose(rhs, orhs, rtol=1e-15, atol=1e-12)


def test_poisson_slabs_concatenate(pkg):
    N = 10
    ai, aj, aa = pkg.poisson_csr(N)
    parts = [pkg.poisson_csr(N, z0=z0, z1=z1) for z0, z1 in [(0, 3), (3, 4), (4, 10)]]
    cat_aj = np.concatenate([p[1] for p in parts])
    cat_aa = np.concatenate([p[2] for p in parts])
    assert np.array_equal(cat_aj, aj) and np.array_equal(cat_aa.view(np.uint64), aa.view(np.uint64))
    off = 0
    for p in parts:
        assert np.array_equal(p[0] + off, ai[off_rows(ai, p, parts)])
        off += len(p[1])


def off_rows(ai, p, parts):
    # row range of part p in the global ai
    start = 0
    for q in parts:
        if q is p:
            break
        start += len(q[0]) - 1
    return slice(start, start + len(p[0]))


def test_poisson_nnz_formula(pkg):
    import ctypes
    for N in (2, 3, 7, 300):
        n = ctypes.c_int64()
        assert pkg.lib().aijhip_poisson_nnz(N, N, N, 0, N, ctypes.byref(n)) == 0
        assert n.value == 7 * N ** 3 - 6 * N ** 2


def test_splitmix_matches_oracle(pkg):
    assert np.array_equal(pkg.splitmix_uniform(1000, 42, 17), seqaij.splitmix_uniform(1000, 42, 17))


def test_skewed_csr_shape(pkg):
    ai, aj, aa = pkg.skewed_csr(200000, seed=1565)
    m = len(ai) - 1
    lens = np.diff(ai)
    assert ai[0] == 0 and np.all(lens >= 0)
    assert aj.min() >= 0 and aj.max() < m
    rows = np.repeat(np.arange(m), lens)
    assert np.all(np.diff(aj)[np.diff(rows) == 0] > 0)  # sorted, unique
    assert lens.max() > 2048  # heavy tail beyond one STREAM block
    assert 60 < lens.mean() < 90
    ai2, aj2, aa2 = pkg.skewed_csr(200000, seed=1565)
    assert np.array_equal(aj, aj2) and np.array_equal(aa, aa2)  # deterministic


def test_split_rows_is_mpiaij_split(pkg):
    N = 6
    ai, aj, aa = pkg.poisson_csr(N, z0=2, z1=4)
    lo, hi = 2 * N * N, 4 * N * N
    (dai, daj, daa), (oai, oaj, oaa), garray = pkg.split_rows(ai, aj, aa, lo, hi)
    assert np.all(np.diff(garray) > 0)
    assert np.array_equal(garray, np.concatenate([np.arange(N * N) + N * N, np.arange(N * N) + 4 * N * N]))
    x = seqaij.splitmix_uniform(N ** 3, 3)
    y_ref = seqaij.matmult(ai, aj, aa, x)
    y_d = seqaij.matmult(dai, daj, daa, x[lo:hi])
    y = seqaij.matmult_add(oai, oaj, oaa, x[garray], y_d)
    np.testing.assert_allclose(y, y_ref, rtol=1e-14, atol=1e-10)


def _fem_hex_reference(nx, ny, nz, dofs, seed):
    """Loop restatement of aijhip_fem_hex_csr (include/aijhip_harness.h)."""
    ai, aj = [0], []
    for k in range(nz):
        for j in range(ny):
            for i in range(nx):
                for _ in range(dofs):
                    for dk in (-1, 0, 1):
                        for dj in (-1, 0, 1):
                            for di in (-1, 0, 1):
                                a, b, c = i + di, j + dj, k + dk
                                if 0 <= a < nx and 0 <= b < ny and 0 <= c < nz:
                                    node = a + nx * (b + ny * c)
                                    aj.extend(node * dofs + e for e in range(dofs))
                    ai.append(len(aj))
    # entry p's value is rnd(seed, 5, p) = splitmix(seed + 5 * 0xD1B54A32D192ED03, p)
    aa = seqaij.splitmix_uniform(len(aj), (seed + 5 * 0xD1B54A32D192ED03) % (1 << 64), 0)
    return np.array(ai, np.int32), np.array(aj, np.int32), aa


@pytest.mark.parametrize("dims", [(4, 3, 5, 3), (1, 2, 3, 2), (3, 3, 3, 1)])
def test_fem_hex_csr_matches_loop_restatement(pkg, dims):
    ai, aj, aa = pkg.fem_hex_csr(*dims, seed=1565)
    ri, rj, ra = _fem_hex_reference(*dims, seed=1565)
    assert np.array_equal(ai, ri) and np.array_equal(aj, rj)
    assert np.array_equal(aa.view(np.uint64), ra.view(np.uint64))


def test_fem_hex_csr_flan_shape(pkg):
    nx, ny, nz = pkg.FLAN_HEX_GRID
    L = pkg.lib()
    nnz = ctypes.c_int64()
    assert L.aijhip_fem_hex_csr(nx, ny, nz, 3, 1565, ctypes.byref(nnz), None, None, None) == 0
    m = nx * ny * nz * 3
    assert abs(m - pkg.FLAN_1565_ROWS) / pkg.FLAN_1565_ROWS < 0.01
    assert nnz.value == 9 * (3 * nx - 2) * (3 * ny - 2) * (3 * nz - 2)
    assert 70 < nnz.value / m <= 81  # Flan_1565: 114.2 M / 1.565 M = 73 per row
