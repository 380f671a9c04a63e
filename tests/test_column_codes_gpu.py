"""Column codes (AIJHIP_OPT_COLUMN_CODES): the STREAM kernel reading one
16-bit code per entry, (row - row0) << b | index into the row block's
dictionary of column - row offsets, instead of aj. aa, the products, their
LDS slots and the row sums are the plain kernel's, so every result must be
BIT-IDENTICAL to the uncoded kernel and, in exact mode, to the oracle
(the PETSc row loop, step1 MatMult_SeqAIJ.patch:22-31)."""
import importlib

import numpy as np
import pytest

from conftest import GOLDEN_NAMES, golden

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev(pkg):
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    return torch.device("cuda:0")


def to_dev(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64)).to(dev)


def assert_bits(a, b, mask=None):
    a, b = np.ascontiguousarray(a), np.ascontiguousarray(b)
    if mask is not None:
        a, b = a[mask], b[mask]
    bad = np.nonzero(a.view(np.uint64) != b.view(np.uint64))[0]
    assert bad.size == 0, f"{bad.size}/{a.size} entries differ bitwise; first {bad[:4]}: {a[bad[:4]]} vs {b[bad[:4]]}"


def products(A, x, z, dev):
    """y = A x and w = z + A x on the device (NaN-filled outputs)."""
    xd, zd = to_dev(x, dev), to_dev(z, dev)
    y = torch.full((A.m,), np.nan, dtype=torch.float64, device=dev)
    w = torch.full((A.m,), np.nan, dtype=torch.float64, device=dev)
    A.mult(xd, y)
    A.mult_add(xd, zd, w)
    torch.cuda.synchronize()
    return y.cpu().numpy(), w.cpu().numpy()


def test_poisson_codes_bitwise(pkg, dev, coracle):
    """7-point Poisson with the reference point (helper.cpp:161-279): 7
    offsets per 512-row block, every block coded; MatMult / MatMultAdd equal
    the oracle and the uncoded kernel bit for bit, also after new values."""
    ai, aj, aa = pkg.poisson_csr(37)
    m = len(ai) - 1
    x, z = pkg.splitmix_uniform(m, 42), pkg.splitmix_uniform(m, 7)
    with pkg.SeqAIJHIP(ai, aj, aa, row_patterns=0, column_codes=1) as A:
        info = A.info()
        assert info["column_codes"] == 1 and info["stream_geometry"] == 6
        y1, w1 = products(A, x, z, dev)
        assert_bits(y1, coracle.matmult(ai, aj, aa, x, omp=True))
        A.set_option("column_codes", 0)
        assert A.info()["column_codes"] == 0
        y0, w0 = products(A, x, z, dev)
        assert_bits(y1, y0)
        assert_bits(w1, w0)
        A.set_option("column_codes", 1)
        aa2 = np.random.default_rng(5).uniform(-1, 1, len(aa))
        A.update_values(aa2)  # the codes do not depend on the values
        y2, _ = products(A, x, z, dev)
        assert_bits(y2, coracle.matmult(ai, aj, aa2, x, omp=True))


@pytest.mark.parametrize("name", GOLDEN_NAMES)
def test_golden_codes(pkg, dev, name):
    """Every golden fixture with codes requested: ragged rows, empty rows,
    rows longer than a block (split into segments), >60 % empty rows
    (compressed-row form: no codes). Rows within the block cap stay
    bit-identical to the fixture (exact mode)."""
    g = golden(name)
    ai, aj, aa, n = g["ai"], g["aj"], g["aa"], int(g["ncols"])
    with pkg.SeqAIJHIP(ai, aj, aa, ncols=n, row_patterns=0, column_codes=1, exact=1) as A:
        xd = to_dev(g["x"], dev)
        y = torch.full((A.m,), np.nan, dtype=torch.float64, device=dev)
        A.mult(xd, y)
        torch.cuda.synchronize()
        short = np.diff(ai) <= A.info()["stream_nnz_cap"]
        assert_bits(y.cpu().numpy(), g["y"], short)


def test_split_coded_and_uncoded_blocks(pkg, dev, coracle):
    """A Poisson operand with a row of 300 scattered extra columns every
    25,000 rows: those blocks (2 % of the entries) exceed their 128-offset dictionary and run
    from aj in a second launch, the rest coded. Results equal the oracle
    (exact mode) and the uncoded kernel bit for bit; the CG's fused dot
    takes aj in one launch then."""
    ai0, aj0, aa0 = pkg.poisson_csr(50)
    m = len(ai0) - 1
    rng = np.random.default_rng(3)
    rows = []
    for i in range(m):
        c, v = aj0[ai0[i]:ai0[i + 1]], aa0[ai0[i]:ai0[i + 1]]
        if i % 25000 == 17:
            extra = np.setdiff1d(rng.choice(m, 300, replace=False), c)
            c = np.concatenate([c, extra])
            v = np.concatenate([v, rng.uniform(-1, 1, len(extra))])
            o = np.argsort(c, kind="stable")
            c, v = c[o], v[o]
        rows.append((c, v))
    ai = np.concatenate([[0], np.cumsum([len(c) for c, _ in rows])]).astype(np.int32)
    aj = np.concatenate([c for c, _ in rows]).astype(np.int32)
    aa = np.concatenate([v for _, v in rows])
    x, z = pkg.splitmix_uniform(m, 1), pkg.splitmix_uniform(m, 2)
    with pkg.SeqAIJHIP(ai, aj, aa, row_patterns=0, column_codes=1, exact=1) as A:
        assert A.info()["column_codes"] == 1
        y1, w1 = products(A, x, z, dev)
        assert_bits(y1, coracle.matmult(ai, aj, aa, x, omp=True))
        A.set_option("column_codes", 0)
        y0, w0 = products(A, x, z, dev)
        assert_bits(y1, y0)
        assert_bits(w1, w0)


def test_fem_rows_codes(pkg, dev, coracle):
    """FEM-structured rows (hexahedral mesh, 3 dofs per node, 81-entry
    interior rows): ~50 rows per block, so 9 index bits and up to 512
    offsets (a block has ~135). Coded (the automatic layout; gather order
    off): equal to the oracle and the uncoded kernel bit for bit."""
    ai, aj, aa = pkg.fem_hex_csr(21, 20, 19)
    m = len(ai) - 1
    x, z = pkg.splitmix_uniform(m, 11), pkg.splitmix_uniform(m, 12)
    with pkg.SeqAIJHIP(ai, aj, aa) as A:
        assert A.info()["column_codes"] == 1 and A.info()["gather_sorted"] == 0
        y1, w1 = products(A, x, z, dev)
        assert_bits(y1, coracle.matmult(ai, aj, aa, x, omp=True))
        A.set_option("gather_sort", 0)
        A.set_option("column_codes", 0)
        y0, w0 = products(A, x, z, dev)
        assert_bits(y1, y0)
        assert_bits(w1, w0)


def test_scattered_rows_fall_back(pkg, dev):
    """Random columns within +-3000 of the diagonal: most blocks hold more
    distinct offsets than their dictionary, so the plan keeps aj (asked
    for) or, automatically, takes the gather-ordered copy."""
    ai, aj, aa = pkg.skewed_csr(100000, seed=1565)
    with pkg.SeqAIJHIP(ai, aj, aa, gather_sort=0, column_codes=1, geometry=6) as A:
        assert A.info()["column_codes"] == 0
    with pkg.SeqAIJHIP(ai, aj, aa) as A:
        assert (A.info()["column_codes"], A.info()["gather_sorted"]) == (0, 2)


def test_cg_and_gamg_with_codes_bitwise(pkg, dev):
    """The solver path on a coded operator: CG + Jacobi (the fused SpMV + p.w
    epilogue) and CG + GAMG (the fused V-cycle smoothers on the fine level)
    give the uncoded run's residual history and solution bit for bit."""
    K = importlib.import_module("petsc-openacc_amd.ksp")
    ai, aj, aa = pkg.poisson_csr(40)
    rhs, _ = pkg.poisson_vectors(40, 40, 40)
    b = torch.from_numpy(rhs).to(dev)
    for pc, kw in (("jacobi", dict(rtol=1e-10, max_it=500)), ("gamg", dict(rtol=1e-14, atol=1e-12))):
        out = {}
        for codes in (0, 1):
            with pkg.SeqAIJHIP(ai, aj, aa, row_patterns=0, column_codes=codes) as A:
                assert A.info()["column_codes"] == codes
                x = torch.zeros_like(b)
                with K.KSPCG(A, pc=pc, **kw) as ksp:
                    ksp.set_up()
                    ksp.solve(b, x)
                    torch.cuda.synchronize()
                    assert ksp.fused
                    out[codes] = (ksp.its, ksp.history(), x.cpu().numpy())
        assert out[0][0] == out[1][0]
        assert_bits(out[0][1], out[1][1])
        assert_bits(out[0][2], out[1][2])
