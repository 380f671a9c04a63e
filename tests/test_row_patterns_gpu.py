"""Row patterns (AIJHIP_OPT_ROW_PATTERNS) and row templates
(AIJHIP_OPT_ROW_TEMPLATES: the patterns with their values, for a constant-
coefficient stencil; neither aj nor aa read): for short-row operands whose rows
follow at most 256 distinct column - row offset lists (a stencil), the STREAM
row blocks read no column per entry — a pattern id per row, the lists staged
in LDS, x gathered by one lane per row. aa and the summation (s = seed, then
s += aa[k] * x[col] in storage order) are the plain kernel's, so every result
must be BIT-IDENTICAL to the aj layout and to the oracle (the PETSc row loop,
/root/reference/src/openacc-step1/MatMult_SeqAIJ.patch:22-31)."""
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
    xd, zd = to_dev(x, dev), to_dev(z, dev)
    y = torch.full((A.m,), np.nan, dtype=torch.float64, device=dev)
    w = torch.full((A.m,), np.nan, dtype=torch.float64, device=dev)
    A.mult(xd, y)
    A.mult_add(xd, zd, w)
    torch.cuda.synchronize()
    return y.cpu().numpy(), w.cpu().numpy()


@pytest.mark.parametrize("dims", [(37, 37, 37), (20, 17, 13), (1, 9, 40), (300, 2, 3)])
def test_poisson_patterns_bitwise(pkg, dev, coracle, dims):
    """7-point Poisson with the reference point (helper.cpp:161-279), cubes,
    boxes and thin grids: the automatic layout takes row templates (the
    distinct rows, offsets and values: interior, faces, edges, corners, the
    reference rows; AIJHIP_OPT_ROW_TEMPLATES), or with templates off row
    patterns (the distinct offset lists). MatMult and MatMultAdd equal the
    oracle and the aj layout bit for bit in all three, also after new values:
    values that no longer fit the templates re-plan to the patterns, values
    that do keep them."""
    ai, aj, aa = pkg.poisson_csr(*dims)
    m = len(ai) - 1
    x, z = pkg.splitmix_uniform(m, 42), pkg.splitmix_uniform(m, 7)
    rows = np.repeat(np.arange(m), np.diff(ai))
    lists = {tuple(aj[ai[i]:ai[i + 1]] - rows[ai[i]:ai[i + 1]]) for i in range(m)}  # the distinct offset lists
    temps = {tuple(aj[ai[i]:ai[i + 1]] - rows[ai[i]:ai[i + 1]]) + tuple(aa[ai[i]:ai[i + 1]].view(np.uint64))
             for i in range(m)}  # the distinct rows
    with pkg.SeqAIJHIP(ai, aj, aa) as A:
        info = A.info()
        assert (info["row_templates"], info["row_patterns"], info["column_codes"]) == (1, len(temps), 0)
        assert info["mult_layout_bytes"] == m + 12 * (len(temps) + sum(len(t) // 2 for t in temps)) + 16 * m
        yt, wt = products(A, x, z, dev)
        assert_bits(yt, coracle.matmult(ai, aj, aa, x, omp=True))
        A.set_option("row_templates", 0)
        assert (A.info()["row_templates"], A.info()["row_patterns"]) == (0, len(lists))
        y1, w1 = products(A, x, z, dev)
        assert_bits(yt, y1)
        assert_bits(wt, w1)
        A.set_option("row_patterns", 0)
        A.set_option("column_codes", 0)
        assert A.info()["row_patterns"] == 0
        y0, w0 = products(A, x, z, dev)
        assert_bits(y1, y0)
        assert_bits(w1, w0)
        A.set_option("row_patterns", -1)
        A.set_option("row_templates", -1)
        assert A.info()["row_templates"] == 1
        A.update_values(2.0 * aa)  # still one template per distinct row
        assert A.info()["row_templates"] == 1
        y3, _ = products(A, x, z, dev)
        assert_bits(y3, coracle.matmult(ai, aj, 2.0 * aa, x, omp=True))
        aa2 = np.random.default_rng(5).uniform(-1, 1, len(aa))
        A.update_values(aa2)  # the patterns do not depend on the values; the templates do
        assert (A.info()["row_templates"], A.info()["row_patterns"]) == (0, len(lists))
        y2, _ = products(A, x, z, dev)
        assert_bits(y2, coracle.matmult(ai, aj, aa2, x, omp=True))


def box_stencil_csr(nz, ny, nx):
    """Constant-coefficient box stencil (27 points in 3-D, 9 with nz = 1) on
    an nz x ny x nx grid: the point count less one on the diagonal, -1 off
    it; rows of up to 27 (9) entries."""
    idx = np.arange(nz * ny * nx).reshape(nz, ny, nx)
    rows, cols, vals = [], [], []
    dzs = (-1, 0, 1) if nz > 1 else (0,)
    npts = 9 * len(dzs)
    for dz in dzs:
        for dy in (-1, 0, 1):
            for dx in (-1, 0, 1):
                def sl(d, n):
                    return slice(max(0, -d), n - max(0, d)), slice(max(0, d), n - max(0, -d))
                (sz, tz), (sy, ty), (sx, tx) = sl(dz, nz), sl(dy, ny), sl(dx, nx)
                src, dst = idx[sz, sy, sx], idx[tz, ty, tx]
                rows.append(src.ravel())
                cols.append(dst.ravel())
                vals.append(np.full(src.size, npts - 1.0 if (dz, dy, dx) == (0, 0, 0) else -1.0))
    r, c, v = np.concatenate(rows), np.concatenate(cols), np.concatenate(vals)
    o = np.lexsort((c, r))
    r, c, v = r[o], c[o], v[o]
    ai = np.concatenate([[0], np.cumsum(np.bincount(r, minlength=nz * ny * nx))]).astype(np.int32)
    return ai, c.astype(np.int32), v


@pytest.mark.parametrize("dims", [(1, 40, 37), (1, 700, 650)])
def test_templates_longer_than_the_fast_slots(pkg, dev, coracle, dims):
    """Row templates of 9 entries (a 2-D 9-point stencil; mean row <= 16, so
    templates apply): more than the pipelined kernel's 8 fast slots, so the
    launch takes the 2-rows-per-lane template kernel; MatMult / MatMultAdd
    bitwise the oracle's and the row patterns' (templates off)."""
    ai, aj, aa = box_stencil_csr(*dims)
    m = len(ai) - 1
    assert np.diff(ai).max() == 9
    x, z = pkg.splitmix_uniform(m, 3), pkg.splitmix_uniform(m, 4)
    with pkg.SeqAIJHIP(ai, aj, aa) as A:
        assert A.info()["row_templates"] == 1
        yt, wt = products(A, x, z, dev)
        assert_bits(yt, coracle.matmult(ai, aj, aa, x, omp=True))
        A.set_option("row_templates", 0)
        assert A.info()["row_patterns"] > 0
        y1, w1 = products(A, x, z, dev)
        assert_bits(yt, y1)
        assert_bits(wt, w1)


@pytest.mark.parametrize("m,n", [(119, 4), (250, 17), (1537, None), (70001, None)])
def test_templates_inplace_mult_add(pkg, dev, coracle, m, n):
    """In-place MatMultAdd (w = z, PCMG's x = x + P x_c) on row templates: a
    coarse prolongator's shape (m x n, n < m, every row its own template) and
    banded operators of one to 137 row blocks (a few value patterns). A lane
    past a block's rows and the re-summed last block of a workgroup must not
    store — another wave may already have updated that row, which an
    in-place add reads as its seed. w equals z + A x bit for bit."""
    rng = np.random.default_rng(m)
    if n is not None:
        rows = [np.unique(rng.integers(0, n, rng.integers(1, 4))) for _ in range(m)]
        vals = [rng.uniform(-1, 1, len(c)) for c in rows]
    else:
        n = m
        rows = [np.arange(max(0, i - 1), min(m, i + 2)) for i in range(m)]
        pick = rng.integers(0, 3, m)
        vals = [np.array([0.5, -1.0, 2.0, 0.25])[(pick[i] + np.arange(len(c))) % 4] for i, c in enumerate(rows)]
    ai = np.concatenate([[0], np.cumsum([len(c) for c in rows])]).astype(np.int32)
    aj = np.concatenate(rows).astype(np.int32)
    aa = np.concatenate(vals)
    x, z = rng.uniform(-1, 1, n), rng.uniform(-1, 1, m)
    ref = coracle.matmult_add(ai, aj, aa, x, z)
    with pkg.SeqAIJHIP(ai, aj, aa, ncols=n, row_patterns=1) as A:
        assert A.info()["row_templates"] == 1
        xd, zd = to_dev(x, dev), to_dev(z, dev)
        w = zd.clone()
        A.mult_add(xd, w, w)
        w2 = torch.full_like(zd, np.nan)
        A.mult_add(xd, zd, w2)
        torch.cuda.synchronize()
        assert_bits(w.cpu().numpy(), ref)
        assert_bits(w2.cpu().numpy(), ref)


def test_templates_cg_dots_match_csr_on_odd_block_counts(pkg, dev):
    """CG + Jacobi on operands whose persistent template grid leaves some
    workgroups an odd number of row blocks (the last one summed twice) and
    blocks shorter than 512 rows: the residual history and solution equal
    the CSR layout's bit for bit (the fused SpMV + p.w partials per block)."""
    K = importlib.import_module("petsc-openacc_amd.ksp")
    for dims in ((23, 19, 17), (64, 64, 61)):
        ai, aj, aa = pkg.poisson_csr(*dims)
        rhs, _ = pkg.poisson_vectors(*dims)
        b = torch.from_numpy(rhs).to(dev)
        out = {}
        for temps in (0, 1):
            with pkg.SeqAIJHIP(ai, aj, aa, row_patterns=temps, row_templates=temps, column_codes=0) as A:
                assert A.info()["row_templates"] == temps
                x = torch.zeros_like(b)
                with K.KSPCG(A, pc="jacobi", rtol=1e-10, max_it=300) as ksp:
                    ksp.set_up()
                    ksp.solve(b, x)
                    torch.cuda.synchronize()
                    out[temps] = (ksp.its, ksp.history(), x.cpu().numpy())
        assert out[0][0] == out[1][0]
        assert_bits(out[0][1], out[1][1])
        assert_bits(out[0][2], out[1][2])


@pytest.mark.parametrize("name", GOLDEN_NAMES)
def test_golden_patterns(pkg, dev, name):
    """Every golden fixture with patterns requested (taken where they fit):
    rows within the block cap stay bit-identical to the fixture."""
    g = golden(name)
    ai, aj, aa, n = g["ai"], g["aj"], g["aa"], int(g["ncols"])
    with pkg.SeqAIJHIP(ai, aj, aa, ncols=n, row_patterns=1, exact=1) as A:
        xd = to_dev(g["x"], dev)
        y = torch.full((A.m,), np.nan, dtype=torch.float64, device=dev)
        A.mult(xd, y)
        torch.cuda.synchronize()
        short = np.diff(ai) <= A.info()["stream_nnz_cap"]
        assert_bits(y.cpu().numpy(), g["y"], short)


def test_many_patterns_fall_back(pkg, dev, coracle):
    """Short random rows (>256 distinct offset lists): no patterns; the plan
    keeps another layout and the product stays the oracle's."""
    rng = np.random.default_rng(9)
    m = 50000
    lens = rng.integers(3, 9, m)
    cols = [np.unique(np.clip(i + rng.integers(-40, 41, l), 0, m - 1)) for i, l in enumerate(lens)]
    ai = np.concatenate([[0], np.cumsum([len(c) for c in cols])]).astype(np.int32)
    aj = np.concatenate(cols).astype(np.int32)
    aa = rng.uniform(-1, 1, len(aj))
    x = rng.uniform(-1, 1, m)
    with pkg.SeqAIJHIP(ai, aj, aa, row_patterns=1) as A:
        assert A.info()["row_patterns"] == 0
        xd = to_dev(x, dev)
        y = torch.empty(m, dtype=torch.float64, device=dev)
        A.mult(xd, y)
        torch.cuda.synchronize()
        assert_bits(y.cpu().numpy(), coracle.matmult(ai, aj, aa, x, omp=True))


def test_many_patterns_plan_time_large(pkg, dev, coracle):
    """a ~10^6-row random short-row operand (far more than 256
    distinct offset lists) must leave the row-pattern attempt early (the
    insert stops once the table has overflowed) instead of probing all 4096
    slots for every row: the plan stays within seconds, the product the
    oracle's."""
    import time
    rng = np.random.default_rng(21)
    m, L = 1_000_000, 6
    offs = -40 + rng.integers(0, 10, (m, 1)) + np.cumsum(rng.integers(1, 14, (m, L)), axis=1)
    cols = np.arange(m)[:, None] + offs
    keep = (cols >= 0) & (cols < m)
    ai = np.concatenate([[0], np.cumsum(keep.sum(axis=1))]).astype(np.int32)
    aj = cols[keep].astype(np.int32)
    aa = rng.uniform(-1, 1, len(aj))
    x = rng.uniform(-1, 1, m)
    t0 = time.perf_counter()
    with pkg.SeqAIJHIP(ai, aj, aa, row_patterns=1) as A:
        torch.cuda.synchronize()
        t_plan = time.perf_counter() - t0
        assert A.info()["row_patterns"] == 0
        assert t_plan < 10.0, f"plan took {t_plan:.2f} s"
        xd = to_dev(x, dev)
        y = torch.empty(m, dtype=torch.float64, device=dev)
        A.mult(xd, y)
        torch.cuda.synchronize()
        assert_bits(y.cpu().numpy(), coracle.matmult(ai, aj, aa, x, omp=True))


def test_cg_and_gamg_with_patterns_bitwise(pkg, dev):
    """The solver path on a patterned operator: CG + Jacobi (the fused
    SpMV + p.w epilogue) and CG + GAMG (the fused V-cycle smoothers and the
    set-up's power iteration on the fine level) give the aj run's residual
    history and solution bit for bit, with row patterns and with row
    templates."""
    K = importlib.import_module("petsc-openacc_amd.ksp")
    ai, aj, aa = pkg.poisson_csr(40)
    rhs, _ = pkg.poisson_vectors(40, 40, 40)
    b = torch.from_numpy(rhs).to(dev)
    for pc, kw in (("jacobi", dict(rtol=1e-10, max_it=500)), ("gamg", dict(rtol=1e-14, atol=1e-12))):
        out = {}
        for pats, temps in ((0, 0), (1, 0), (1, 1)):
            with pkg.SeqAIJHIP(ai, aj, aa, row_patterns=pats, row_templates=temps, column_codes=0) as A:
                assert (A.info()["row_patterns"] > 0) == bool(pats)
                assert A.info()["row_templates"] == temps
                x = torch.zeros_like(b)
                with K.KSPCG(A, pc=pc, **kw) as ksp:
                    ksp.set_up()
                    ksp.solve(b, x)
                    torch.cuda.synchronize()
                    assert ksp.fused
                    out[pats, temps] = (ksp.its, ksp.history(), x.cpu().numpy())
        for key in ((1, 0), (1, 1)):
            assert out[0, 0][0] == out[key][0]
            assert_bits(out[0, 0][1], out[key][1])
            assert_bits(out[0, 0][2], out[key][2])
