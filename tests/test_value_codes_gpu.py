"""Value codes (AIJHIP_OPT_VALUE_CODES): for operators whose entries take at
most 512 distinct values (GAMG's finest prolongator P and its transpose have
~370), the STREAM blocks read a 16-bit index per entry into a dictionary of
the values (staged in LDS) in aa's place — with aj (the branch-free plain
blocks) or with the packed gather-ordered columns. The products are the same
bits and the rows are summed in the same order, so every result must be
BIT-IDENTICAL to the aa layout and to the oracle (the PETSc row loop,
/root/reference/src/openacc-step1/MatMult_SeqAIJ.patch:22-31)."""
import importlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev(pkg):
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    return torch.device("cuda:0")


def to_dev(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64)).to(dev)


def assert_bits(a, b):
    a, b = np.ascontiguousarray(a), np.ascontiguousarray(b)
    bad = np.nonzero(a.view(np.uint64) != b.view(np.uint64))[0]
    assert bad.size == 0, f"{bad.size}/{a.size} entries differ bitwise; first {bad[:4]}: {a[bad[:4]]} vs {b[bad[:4]]}"


def few_valued(m, n, per_row, nvals, seed, band=None):
    """m x n, per_row entries a row (columns random, or within +-band of the
    row's diagonal position), values drawn from nvals distinct ones
    (including -0.0 and a subnormal: the dictionary keys on bits)."""
    rng = np.random.default_rng(seed)
    vals = np.concatenate([rng.uniform(-2, 2, max(nvals - 2, 1)), [-0.0, 5e-310]])[:nvals]
    rows = []
    for i in range(m):
        k = int(rng.integers(1, per_row + 1))
        if band is None:
            c = rng.choice(n, size=min(k, n), replace=False)
        else:
            mid = i * n // m
            c = np.unique(np.clip(mid + rng.integers(-band, band + 1, k), 0, n - 1))
        rows.append(np.sort(c))
    ai = np.concatenate([[0], np.cumsum([len(c) for c in rows])]).astype(np.int32)
    aj = np.concatenate(rows).astype(np.int32)
    aa = vals[rng.integers(0, len(vals), len(aj))]
    return ai, aj, aa


def products(A, x, z, dev):
    xd, zd = to_dev(x, dev), to_dev(z, dev)
    y = torch.full((A.m,), np.nan, dtype=torch.float64, device=dev)
    w = torch.full((A.m,), np.nan, dtype=torch.float64, device=dev)
    wi = zd.clone()
    A.mult(xd, y)
    A.mult_add(xd, zd, w)
    A.mult_add(xd, wi, wi)  # in place (PCMG's x = x + P x_c)
    torch.cuda.synchronize()
    return y.cpu().numpy(), w.cpu().numpy(), wi.cpu().numpy()


@pytest.mark.parametrize("m,n,per_row,nvals,band", [(200_000, 20_000, 4, 370, 2000), (5000, 900, 7, 512, None),
                                                     (70_001, 70_001, 5, 3, 40)])
def test_value_codes_plain_blocks_bitwise(pkg, dev, coracle, m, n, per_row, nvals, band):
    """Short rows (a prolongator's shape and a banded one), up to the 512-value
    cap: the plain blocks read aj and the codes; y, z + A x and the in-place
    add equal the oracle and the aa layout bit for bit."""
    ai, aj, aa = few_valued(m, n, per_row, nvals, m, band)
    x, z = pkg.splitmix_uniform(n, 5), pkg.splitmix_uniform(m, 6)
    out = {}
    for vc in (0, 1):
        with pkg.SeqAIJHIP(ai, aj, aa, ncols=n, row_patterns=0, column_codes=0, gather_sort=0, value_codes=vc) as A:
            info = A.info()
            assert info["value_codes"] == (len(np.unique(aa.view(np.uint64))) if vc else 0)
            if vc:
                assert info["mult_layout_bytes"] == 6 * len(aj) + 4 * (m + 1) + 8 * n + 8 * m + 8 * info["value_codes"]
            out[vc] = products(A, x, z, dev)
    assert_bits(out[1][0], coracle.matmult(ai, aj, aa, x, omp=True))
    ref_add = coracle.matmult_add(ai, aj, aa, x, z)
    assert_bits(out[1][1], ref_add)
    assert_bits(out[1][2], ref_add)
    for a, b in zip(out[0], out[1]):
        assert_bits(a, b)


def test_value_codes_packed_gather_order_bitwise(pkg, dev, coracle):
    """Long rows with scattered columns (a restriction Pᵀ's shape): the packed
    gather-ordered blocks read their 20-bit columns and slots with the codes
    of the sorted copy; bit-identical to the oracle and to the sorted values."""
    m, n = 60_000, 700_000
    ai, aj, aa = few_valued(m, n, 40, 200, 11)
    x, z = pkg.splitmix_uniform(n, 5), pkg.splitmix_uniform(m, 6)
    out = {}
    for vc in (0, 1):
        with pkg.SeqAIJHIP(ai, aj, aa, ncols=n, row_patterns=0, column_codes=0, gather_sort=1, exact=1,
                           value_codes=vc) as A:
            info = A.info()
            assert info["gather_sorted"] == 2
            assert (info["value_codes"] > 0) == bool(vc)
            out[vc] = products(A, x, z, dev)
    assert_bits(out[1][0], coracle.matmult(ai, aj, aa, x, omp=True))
    assert_bits(out[1][1], coracle.matmult_add(ai, aj, aa, x, z))
    for a, b in zip(out[0], out[1]):
        assert_bits(a, b)


def test_value_codes_fall_back_and_update_values(pkg, dev, coracle):
    """More than 512 distinct values: no codes (the aa layout); new values
    through update_values re-plan (few again: codes; the products follow)."""
    m = n = 20_000
    ai, aj, aa = few_valued(m, n, 6, 512, 3, band=100)
    aa_many = np.random.default_rng(4).uniform(-1, 1, len(aj))
    x = pkg.splitmix_uniform(n, 5)
    with pkg.SeqAIJHIP(ai, aj, aa_many, ncols=n, row_patterns=0, column_codes=0, value_codes=1) as A:
        assert A.info()["value_codes"] == 0
        A.update_values(aa)
        assert A.info()["value_codes"] > 0
        y, _, _ = products(A, x, np.zeros(m), dev)
        assert_bits(y, coracle.matmult(ai, aj, aa, x, omp=True))
        A.update_values(aa_many)
        assert A.info()["value_codes"] == 0
        y, _, _ = products(A, x, np.zeros(m), dev)
        assert_bits(y, coracle.matmult(ai, aj, aa_many, x, omp=True))


def test_cg_gamg_value_codes_bitwise(pkg, dev, monkeypatch):
    """CG + GAMG with the set-up's operators on value codes (the default: the
    finest P and Pᵀ fit the dictionary) against AIJHIP_SETUP_VCODES=0: the
    same iterations, residual history and solution bits, and fewer bytes per
    iteration (aijhip_ksp_get_iteration_bytes)."""
    K = importlib.import_module("petsc-openacc_amd.ksp")
    N = 40
    ai, aj, aa = pkg.poisson_csr(N)
    rhs, _ = pkg.poisson_vectors(N, N, N)
    b = torch.from_numpy(rhs).to(dev)
    out = {}
    for vc in ("0", None):
        if vc is None:
            monkeypatch.delenv("AIJHIP_SETUP_VCODES", raising=False)
        else:
            monkeypatch.setenv("AIJHIP_SETUP_VCODES", vc)
        with pkg.SeqAIJHIP(ai, aj, aa) as A:
            x = torch.zeros_like(b)
            with K.KSPCG(A, pc="gamg", rtol=1e-14, atol=1e-12) as ksp:
                ksp.set_up()
                ksp.solve(b, x)
                torch.cuda.synchronize()
                out[vc] = (ksp.its, ksp.history(), x.cpu().numpy(), ksp.iteration_bytes()[0])
    assert out["0"][0] == out[None][0]
    assert_bits(out["0"][1], out[None][1])
    assert_bits(out["0"][2], out[None][2])
    assert out[None][3] < out["0"][3]
