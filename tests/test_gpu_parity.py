"""GPU parity of the HIP SpMV (through the C ABI) against the oracle.

Bar: the STREAM and SCALAR kernels sum each row in PETSc's
order without FMA, so they must be BIT-IDENTICAL to the CPU restatement.
VECTOR and the long-row windows / segments reorder the row sum and must meet the
componentwise fp64 bound |dy_i| <= 2 gamma(n_i) (|A||x|)_i (+ the |z| term),
gamma(n) = n u / (1 - n u), u = 2^-53, plus ||dy||_inf / |||A||x|||_inf <= 1e-14.
"""
import numpy as np
import pytest

from conftest import GOLDEN_NAMES, golden, spmv_tolerance
from oracle import seqaij

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

BITEXACT = ("stream", "scalar")
ALL_KERNELS = ("stream", "scalar", "vector")


@pytest.fixture(scope="module")
def dev(pkg):
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    assert pkg.device_count() > 0
    return torch.device("cuda:0")


def to_dev(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64)).to(dev)


def bits(a):
    return np.ascontiguousarray(a).view(np.uint64)


def assert_bits(a, b, mask=None):
    a, b = np.ascontiguousarray(a), np.ascontiguousarray(b)
    if mask is not None:
        a, b = a[mask], b[mask]
    bad = np.nonzero(bits(a) != bits(b))[0]
    assert bad.size == 0, f"{bad.size}/{a.size} entries differ bitwise; first {bad[:4]}: {a[bad[:4]]} vs {b[bad[:4]]}"


def check(y_gpu, y_ref, ai, aj, aa, x, exact, z=None):
    if exact:
        bad = np.nonzero(bits(y_gpu) != bits(y_ref))[0]
        assert bad.size == 0, f"{bad.size} rows differ bitwise, first {bad[:5]}: {y_gpu[bad[:5]]} vs {y_ref[bad[:5]]}"
        return
    tol, absax = spmv_tolerance(ai, aj, aa, x)
    if z is not None:
        tol = tol + 2 * 2.0 ** -53 * (np.abs(z) + absax)
    err = np.abs(y_gpu - y_ref)
    assert np.all(err <= tol), f"max excess {np.max(err - tol)}"
    scale = max(np.max(absax), 1e-300)
    assert np.max(err) / scale <= 1e-14


def mult(pkg, dev, ai, aj, aa, n, x, kernel, lanes=0, **opts):
    if kernel == "stream" and not opts:
        opts = {"exact": 1}  # bit-exact mode; default mode is checked separately
    with pkg.SeqAIJHIP(ai, aj, aa, ncols=n, kernel=kernel, lanes=lanes, **opts) as A:
        xd = to_dev(x, dev)
        yd = torch.full((len(ai) - 1,), np.nan, dtype=torch.float64, device=dev)
        A.mult(xd, yd)
        torch.cuda.synchronize()
        return yd.cpu().numpy(), A.info()


@pytest.mark.parametrize("name", GOLDEN_NAMES)
@pytest.mark.parametrize("kernel", ALL_KERNELS)
def test_mult_golden(pkg, dev, name, kernel):
    g = golden(name)
    ai, aj, aa, n = g["ai"], g["aj"], g["aa"], int(g["ncols"])
    y, info = mult(pkg, dev, ai, aj, aa, n, g["x"], kernel)
    long_rows = info["n_long_rows"] > 0
    check(y, g["y"], ai, aj, aa, g["x"], exact=kernel in BITEXACT and not long_rows)
    if long_rows:  # rows <= 2048 entries stay bit-exact even when long rows exist
        short = np.diff(ai) <= 2048
        if kernel in BITEXACT:
            assert_bits(y, g["y"], short)


@pytest.mark.parametrize("name", GOLDEN_NAMES)
def test_stream_default_mode(pkg, dev, name):
    """Default STREAM (long-row blocks reduced by several lanes per row):
    within the fp64 bound everywhere, bit-exact on short-row blocks."""
    g = golden(name)
    ai, aj, aa, n = g["ai"], g["aj"], g["aa"], int(g["ncols"])
    y, info = mult(pkg, dev, ai, aj, aa, n, g["x"], "stream", exact=0)
    assert info["exact"] == 0
    check(y, g["y"], ai, aj, aa, g["x"], exact=False)
    if name.startswith("poisson"):
        assert_bits(y, g["y"])


@pytest.mark.parametrize("row_len", [150, 300, 1000])
def test_stream_multilane_long_rows(pkg, dev, row_len):
    """Blocks of rows longer than kSplitMinMean (128) are summed by several
    lanes per row by default (fp64 bound), sequentially with exact=1
    (bit-exact); a ragged tail of short rows stays exact either way."""
    rng = np.random.default_rng(row_len)
    m = 3000
    lens = np.where(np.arange(m) < 2500, row_len, rng.integers(1, 9, m))
    ai = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    aj = np.concatenate([np.sort(rng.choice(m, size=l, replace=False)) for l in lens]).astype(np.int32)
    aa = rng.uniform(-1, 1, ai[-1])
    x = rng.uniform(-1, 1, m)
    y_ref = seqaij.matmult(ai, aj, aa, x)
    y, info = mult(pkg, dev, ai, aj, aa, m, x, "stream", exact=0)
    check(y, y_ref, ai, aj, aa, x, exact=False)
    assert_bits(y[2600:], y_ref[2600:])  # blocks of short rows only
    y1, _ = mult(pkg, dev, ai, aj, aa, m, x, "stream", exact=1)
    assert_bits(y1, y_ref)


@pytest.mark.parametrize("geometry", list(range(10)))
def test_stream_banded_geometries(pkg, dev, geometry):
    """A banded matrix of 10-40 entries per row (a row every 997 reaching
    five far places of x) at every block geometry, PETSc's order: bit-exact.
    (Round 5 removed the two geometries cut for the withdrawn LDS x tiles;
    the ten left are all selectable, speed-only, and 10 is refused.)"""
    rng = np.random.default_rng(11)
    m = 20000
    lens = rng.integers(10, 40, m)
    cols = []
    for i, l in enumerate(lens):
        lo, hi = max(0, i - 300), min(m, i + 300)
        c = np.sort(rng.choice(np.arange(lo, hi), size=min(l, hi - lo), replace=False))
        if i % 997 == 0:
            c = np.unique(np.concatenate([c, [0, m // 4, m // 2, 3 * m // 4, m - 1]]))
        cols.append(c)
    ai = np.concatenate([[0], np.cumsum([len(c) for c in cols])]).astype(np.int32)
    aj = np.concatenate(cols).astype(np.int32)
    aa = rng.uniform(-1, 1, len(aj))
    x = rng.uniform(-1, 1, m)
    y, info = mult(pkg, dev, ai, aj, aa, m, x, "stream", exact=1, geometry=geometry, gather_sort=0)
    assert info["stream_geometry"] == geometry
    assert_bits(y, seqaij.matmult(ai, aj, aa, x))
    if geometry == 9:
        with pkg.SeqAIJHIP(ai, aj, aa) as A:
            with pytest.raises(pkg.AIJHIPError):
                A.set_option("geometry", 10)


@pytest.mark.parametrize("grid", [(16, 16, 16), (40, 40, 40), (300, 7, 5), (3, 200, 60)])
def test_stream_csr_poisson(pkg, dev, coracle, grid):
    """The CSR kernel (aj read, as the bench's headline) on boxes and thin
    grids of the 7-point operand: PETSc's loop bit for bit."""
    ai, aj, aa = pkg.poisson_csr(*grid)
    m = len(ai) - 1
    x = pkg.splitmix_uniform(m, 17)
    ref = coracle.matmult(ai, aj, aa, x, omp=True)
    y, info = mult(pkg, dev, ai, aj, aa, m, x, "stream", row_patterns=0, column_codes=0)
    assert info["row_patterns"] == 0 and info["column_codes"] == 0 and info["gather_sorted"] == 0
    assert info["mult_layout_bytes"] == info["mult_bytes"]
    assert_bits(y, ref)


@pytest.mark.parametrize("name", GOLDEN_NAMES)
@pytest.mark.parametrize("kernel", ALL_KERNELS)
def test_mult_add_golden(pkg, dev, name, kernel):
    g = golden(name)
    ai, aj, aa, n = g["ai"], g["aj"], g["aa"], int(g["ncols"])
    with pkg.SeqAIJHIP(ai, aj, aa, ncols=n, kernel=kernel, **({"exact": 1} if kernel == "stream" else {})) as A:
        xd, zd = to_dev(g["x"], dev), to_dev(g["z"], dev)
        wd = torch.empty_like(zd)
        A.mult_add(xd, zd, wd)
        A.mult_add(xd, zd, zd)  # z aliases w (PETSc yy == zz)
        torch.cuda.synchronize()
        exact = kernel in BITEXACT and A.info()["n_long_rows"] == 0
        check(wd.cpu().numpy(), g["w"], ai, aj, aa, g["x"], exact, z=g["z"])
        check(zd.cpu().numpy(), g["w"], ai, aj, aa, g["x"], exact, z=g["z"])


@pytest.mark.parametrize("name", GOLDEN_NAMES)
def test_mult_transpose_golden(pkg, dev, name):
    g = golden(name)
    ai, aj, aa, n = g["ai"], g["aj"], g["aa"], int(g["ncols"])
    with pkg.SeqAIJHIP(ai, aj, aa, ncols=n, exact=1) as A:
        yd = torch.empty(n, dtype=torch.float64, device=dev)
        A.mult_transpose(to_dev(g["xt"], dev), yd)
        torch.cuda.synchronize()
        At = (np.argsort(aj, kind="stable"))
        # A^T row lengths = column counts; bit-exact unless a column exceeds 2048 entries
        colcount = np.bincount(aj, minlength=n)
        yt = yd.cpu().numpy()
        ok = colcount <= 2048
        assert_bits(yt, g["yt"], ok)
        np.testing.assert_allclose(yt, g["yt"], rtol=1e-13, atol=1e-13)


@pytest.mark.parametrize("lanes", [2, 4, 8, 16, 32, 64])
def test_vector_all_lane_widths(pkg, dev, lanes):
    g = golden("skewed_small")
    ai, aj, aa, n = g["ai"], g["aj"], g["aa"], int(g["ncols"])
    y, info = mult(pkg, dev, ai, aj, aa, n, g["x"], "vector", lanes)
    assert info["vector_lanes"] == lanes
    check(y, g["y"], ai, aj, aa, g["x"], exact=False)


def test_edge_cases(pkg, dev, coracle):
    # empty matrix (m = 0), all-empty rows, 1x1, a single very long row
    A = pkg.SeqAIJHIP(np.zeros(1, np.int32), np.zeros(0, np.int32), np.zeros(0), ncols=0)
    A.mult(torch.empty(0, dtype=torch.float64, device=dev), torch.empty(0, dtype=torch.float64, device=dev))
    A.destroy()
    for kernel in ALL_KERNELS:
        y, _ = mult(pkg, dev, np.zeros(11, np.int32), np.zeros(0, np.int32), np.zeros(0), 4, np.ones(4), kernel)
        assert np.all(y == 0.0)
        y, _ = mult(pkg, dev, np.array([0, 1], np.int32), np.array([0], np.int32), np.array([3.0]), 1,
                    np.array([-2.0]), kernel)
        assert y[0] == -6.0
    rng = np.random.default_rng(5)
    n = 300000
    aj = np.sort(rng.choice(n, size=200000, replace=False)).astype(np.int32)
    aa = rng.standard_normal(len(aj))
    ai = np.array([0, 0, len(aj), len(aj)], np.int32)
    x = rng.standard_normal(n)
    ref = coracle.matmult(ai, aj, aa, x)
    for kernel in ALL_KERNELS:
        y, _ = mult(pkg, dev, ai, aj, aa, n, x, kernel)
        check(y, ref, ai, aj, aa, x, exact=(kernel == "scalar"))


def test_update_values_and_assembly_end(pkg, dev, coracle):
    g = golden("poisson8")
    ai, aj, aa = g["ai"], g["aj"], g["aa"]
    x = g["x"]
    A = pkg.SeqAIJHIP(ai, aj, aa, exact=1)
    xd = to_dev(x, dev)
    yd = torch.empty_like(xd)
    aa2 = aa * 3.0 - 1.0
    A.update_values(aa2)
    A.mult(xd, yd)
    torch.cuda.synchronize()
    assert_bits(yd.cpu().numpy(), coracle.matmult(ai, aj, aa2, x))
    g2 = golden("skewed_small")
    ai3 = g2["ai"][: len(ai)].copy()  # same row count as poisson8 (513 offsets)
    nz3 = int(ai3[-1])
    aj3 = np.minimum(g2["aj"][:nz3], 511).astype(np.int32)
    aa3 = g2["aa"][:nz3]
    A.assembly_end(ai3, aj3, aa3)
    A.mult(xd, yd)
    torch.cuda.synchronize()
    ref = coracle.matmult(ai3, aj3, aa3, x)
    y = yd.cpu().numpy()
    cap = A.info()["stream_nnz_cap"]
    short = np.diff(ai3) <= cap  # longer rows take the segmented sum
    assert A.info()["n_long_rows"] == int((~short).sum())
    check(y[short], ref[short], None, None, None, None, exact=True)
    check(y, ref, ai3, aj3, aa3, x, exact=False)
    A.destroy()


def test_mult_host_step2_semantics(pkg, dev):
    g = golden("poisson16")
    with pkg.SeqAIJHIP(g["ai"], g["aj"], g["aa"]) as A:
        y = A.mult_host(g["x"])
        assert_bits(y, g["y"])


@pytest.mark.parametrize("operand,chunk", [("poisson", 5000), ("poisson", -1), ("poisson", 0), ("random", 3000)])
def test_mult_host_pipeline_bitwise(pkg, dev, operand, chunk):
    """The host-vector MatMult (step-3/4 analogue, host_pipe.cpp) with many
    chunks, the default chunking and the serial form, on a banded operand
    and a scattered one (every row chunk waits for all of x): bit-identical
    to the device-vector product, with pageable and with pinned host arrays."""
    if operand == "poisson":
        ai, aj, aa = pkg.poisson_csr(40, 40, 40)
    else:
        rng = np.random.default_rng(7)  # columns anywhere: every row chunk needs all of x
        m, k = 60000, 9
        ai = np.arange(m + 1, dtype=np.int32) * k
        aj = np.sort(rng.integers(0, m, size=(m, k)), axis=1).astype(np.int32).ravel()
        aa = rng.standard_normal(m * k)
    n = len(ai) - 1
    x = seqaij.splitmix_uniform(n, 42)
    with pkg.SeqAIJHIP(ai, aj, aa) as A:
        if A.info()["n_long_rows"]:
            pytest.skip("long rows take the serial form")
        A.set_option("host_pipeline", chunk)
        y_dev = torch.empty(n, dtype=torch.float64, device=dev)
        A.mult(to_dev(x, dev), y_dev)
        ref = y_dev.cpu().numpy()
        assert_bits(A.mult_host(x), ref)
        assert_bits(A.mult_host(x), ref)  # staging reused
        xp = torch.from_numpy(x).pin_memory()
        yp = torch.full((n,), float("nan"), dtype=torch.float64).pin_memory()
        A.mult_host(xp.numpy(), out=yp.numpy())
        assert_bits(yp.numpy(), ref)


@pytest.mark.parametrize("name", GOLDEN_NAMES)
def test_mult_add_and_transpose_host_match_device_forms(pkg, dev, name):
    """MatMultAdd / MatMultTranspose with host vectors (the PETSc adapter's
    multadd / multtranspose): bit-identical to the device-vector entry points
    (same kernels, same order), z aliasing w accepted, against the goldens."""
    g = golden(name)
    ai, aj, aa, n = g["ai"], g["aj"], g["aa"], int(g["ncols"])
    m = len(ai) - 1
    with pkg.SeqAIJHIP(ai, aj, aa, ncols=n, exact=1) as A:
        xd, zd = to_dev(g["x"], dev), to_dev(g["z"], dev)
        wd = torch.empty_like(zd)
        A.mult_add(xd, zd, wd)
        ytd = torch.empty(n, dtype=torch.float64, device=dev)
        A.mult_transpose(to_dev(g["xt"], dev), ytd)
        torch.cuda.synchronize()
        w_ref, yt_ref = wd.cpu().numpy(), ytd.cpu().numpy()
        w = A.mult_add_host(g["x"], g["z"])
        assert_bits(w, w_ref)
        z = np.array(g["z"], dtype=np.float64)
        A.mult_add_host(g["x"], z, out=z)  # PETSc's yy == zz
        assert_bits(z, w_ref)
        assert_bits(A.mult_transpose_host(g["xt"]), yt_ref)
        assert_bits(A.mult_transpose_host(g["xt"]), yt_ref)  # A^T and its staging reused
        exact = A.info()["n_long_rows"] == 0
        check(w, g["w"], ai, aj, aa, g["x"], exact, z=g["z"])
        np.testing.assert_allclose(A.mult_transpose_host(g["xt"]), g["yt"], rtol=1e-13, atol=1e-13)
        assert m == len(w)


def test_alias_rejected(pkg, dev):
    g = golden("poisson4")
    with pkg.SeqAIJHIP(g["ai"], g["aj"], g["aa"]) as A:
        xd = to_dev(g["x"], dev)
        with pytest.raises(pkg.AIJHIPError):
            A.mult(xd, xd)


def test_stream_ordering_on_side_stream(pkg, dev):
    g = golden("poisson16")
    s = torch.cuda.Stream()
    with pkg.SeqAIJHIP(g["ai"], g["aj"], g["aa"]) as A:
        with torch.cuda.stream(s):
            xd = to_dev(g["x"], dev)
            yd = torch.empty_like(xd)
            for _ in range(3):
                A.mult(xd, yd, stream=s)
        s.synchronize()
        assert_bits(yd.cpu().numpy(), g["y"])


def _csr_layout(A):
    """The headline's layout: PETSc's aj / aa as stored (bench.py --layout
    csr): no row patterns, no column codes."""
    A.set_option("row_patterns", 0)
    A.set_option("column_codes", 0)
    info = A.info()
    assert not info["row_patterns"] and not info["column_codes"] and not info.get("gather_sorted")
    return info


@pytest.mark.parametrize("layout", ["auto", "csr"])
@pytest.mark.parametrize("N", [100, 300])
def test_full_size_poisson_bitexact(pkg, dev, coracle, N, layout):
    """BASELINE configs[0]/[1] operand at full size: STREAM vs the C oracle,
    bit for bit, plus the size-independent property A*1 = row sums — in the
    library's automatic layout (row patterns) and in the CSR layout the
    headline `value` times (the timed kernel pinned at the
    size it is timed)."""
    ai, aj, aa = pkg.poisson_csr(N)
    m = N ** 3
    x = pkg.splitmix_uniform(m, 42)
    ref = coracle.matmult(ai, aj, aa, x, omp=True)
    with pkg.SeqAIJHIP(ai, aj, aa) as A:
        info = _csr_layout(A) if layout == "csr" else A.info()
        assert info["kernel"] == "stream" and info["n_long_rows"] == 0
        assert info["nz"] == 7 * N ** 3 - 6 * N ** 2
        if layout == "csr":  # the bytes the headline's roofline divides by
            assert info["mult_layout_bytes"] == pkg.algorithmic_bytes(m, m, info["nz"])
        xd = to_dev(x, dev)
        yd = torch.empty_like(xd)
        A.mult(xd, yd)
        torch.cuda.synchronize()
        assert_bits(yd.cpu().numpy(), ref)
        ones = torch.ones(m, dtype=torch.float64, device=dev)
        A.mult(ones, yd)
        rs = coracle.matmult(ai, aj, aa, np.ones(m), omp=True)
        assert_bits(yd.cpu().numpy(), rs)
        del xd, yd, ones
        torch.cuda.empty_cache()


def test_max_size_600_device_assembly_bitexact(pkg, dev, coracle):
    """The largest operand of BASELINE (configs[3]'s 600^3 global grid: 216 M
    rows, 1.51 G entries — 70 % of the int32 entry range, 18 GB of CSR) on one
    GPU: assembled on the device, multiplied by STREAM, and compared bit for
    bit with the C oracle on the host-assembled operand (which also checks the
    device assembly at maximum size)."""
    N = 600
    m = N ** 3
    A, _ = pkg.poisson_device(N)
    try:
        info = A.info()
        assert info["nz"] == 7 * N ** 3 - 6 * N ** 2 and info["n_long_rows"] == 0
        x = pkg.splitmix_uniform(m, 42)
        xd = to_dev(x, dev)
        yd = torch.empty_like(xd)
        A.mult(xd, yd)
        torch.cuda.synchronize()
        y = yd.cpu().numpy()
        _csr_layout(A)  # and the headline's CSR kernel on the same operand
        A.mult(xd, yd)
        torch.cuda.synchronize()
        y_csr = yd.cpu().numpy()
        del xd, yd
    finally:
        A.destroy()
        torch.cuda.empty_cache()
    ai, aj, aa = pkg.poisson_csr(N)
    ref = coracle.matmult(ai, aj, aa, x, omp=True)
    del ai, aj, aa
    assert_bits(y, ref)
    assert_bits(y_csr, ref)


def test_skewed_flan_standin_all_kernels(pkg, dev, coracle):
    """Flan_1565 stand-in (BASELINE configs[4]) at a reduced row count."""
    ai, aj, aa = pkg.skewed_csr(300000, seed=1565)
    x = pkg.splitmix_uniform(len(ai) - 1, 9)
    ref = coracle.matmult(ai, aj, aa, x, omp=True)
    for kernel in ALL_KERNELS:
        y, info = mult(pkg, dev, ai, aj, aa, len(ai) - 1, x, kernel)
        check(y, ref, ai, aj, aa, x, exact=False)
        if kernel in BITEXACT:
            short = np.diff(ai) <= 2048
            assert_bits(y, ref, short)
    y, info = mult(pkg, dev, ai, aj, aa, len(ai) - 1, x, "stream", exact=0)  # default mode
    check(y, ref, ai, aj, aa, x, exact=False)


def test_long_row_xcd_placement_is_speed_only(pkg, dev, coracle):
    """Long-row segments dealt to XCDs by column range (AIJHIP_OPT_LONG_XCD)
    give the same bits as segment order: the same partials, summed in the
    same order; only the workgroup that computes each one moves."""
    ai, aj, aa = pkg.skewed_csr(300000, seed=1565)
    x = pkg.splitmix_uniform(len(ai) - 1, 5)
    ref = coracle.matmult(ai, aj, aa, x, omp=True)
    with pkg.SeqAIJHIP(ai, aj, aa) as A:
        assert A.info()["n_long_rows"] > 0
        xd = to_dev(x, dev)
        yd = torch.empty(len(ai) - 1, dtype=torch.float64, device=dev)
        ys = []
        for lx in (1, 0, 1):
            A.set_option("long_xcd", lx)
            yd.fill_(float("nan"))
            A.mult(xd, yd)
            torch.cuda.synchronize()
            ys.append(yd.cpu().numpy())
        for y in ys[1:]:
            assert_bits(y, ys[0])
        check(ys[0], ref, ai, aj, aa, x, exact=False)
        # MatMultAdd: w = z + A x, both placements
        zd = to_dev(pkg.splitmix_uniform(len(ai) - 1, 6), dev)
        A.mult_add(xd, zd, yd)
        torch.cuda.synchronize()
        A.set_option("long_xcd", 0)
        wd = torch.empty_like(yd)
        A.mult_add(xd, zd, wd)
        torch.cuda.synchronize()
        assert_bits(yd.cpu().numpy(), wd.cpu().numpy())


def test_long_row_segments_skewed(pkg, dev, coracle):
    """Hub rows of the skewed stand-in as 4096-entry segments summed in
    segment order: MatMult and MatMultAdd within the fp64 bound, the same bits
    launch after launch, the short rows bit-exact; an MPIAIJ-style unaligned
    x (offset by one entry) gives the same bits."""
    ai, aj, aa = pkg.skewed_csr(300000, seed=1565)
    m = len(ai) - 1
    x = pkg.splitmix_uniform(m + 1, 7)
    z = pkg.splitmix_uniform(m, 8)
    ref = coracle.matmult(ai, aj, aa, x[:m], omp=True)
    short = np.diff(ai) <= 2048
    with pkg.SeqAIJHIP(ai, aj, aa, exact=1) as A:
        info = A.info()
        assert info["n_long_rows"] > 0
        xd = to_dev(x, dev)
        zd = to_dev(z, dev)
        y1 = torch.full((m,), np.nan, dtype=torch.float64, device=dev)
        y2 = torch.empty_like(y1)
        w = torch.empty_like(y1)
        A.mult(xd, y1)
        A.mult(xd, y2)
        A.mult_add(xd, zd, w)
        torch.cuda.synchronize()
        y = y1.cpu().numpy()
        assert torch.equal(y1, y2)
        check(y, ref, ai, aj, aa, x[:m], exact=False)
        assert_bits(y, ref, short)
        check(w.cpu().numpy(), coracle.matmult_add(ai, aj, aa, x[:m], z), ai, aj, aa, x[:m], exact=False, z=z)
        # x at an 8-byte offset (a ghost buffer inside a larger tensor)
        xo = torch.zeros(m + 2, dtype=torch.float64, device=dev)
        xo[1:m + 1] = xd[:m]
        A.mult(xo[1:m + 1], y2)
        torch.cuda.synchronize()
        assert torch.equal(y1, y2)


def test_rows_over_1024_get_their_own_block(pkg, dev, coracle, monkeypatch):
    """kIsolateRowNnz: a row of 1025..cap entries among short rows gets a row
    block of its own (one block more than the plain greedy cut, which
    AIJHIP_ISOLATE_ROW_NNZ=0 restores), summed by several lanes by default
    (within the fp64 bound) and in PETSc's order with exact = 1 (bit-exact);
    the short rows keep PETSc's order."""
    rng = np.random.default_rng(1024)
    m = 4000
    lens = rng.integers(20, 60, m)
    lens[[500, 501, 2600]] = (1500, 3000, 1025)  # inside the 4094-entry cap
    ai = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    aj = np.concatenate([np.sort(rng.choice(m, size=l, replace=False)) for l in lens]).astype(np.int32)
    aa = rng.uniform(-1, 1, ai[-1])
    x = rng.uniform(-1, 1, m)
    ref = coracle.matmult(ai, aj, aa, x)
    short = lens <= 1024
    blocks = {}
    for iso in ("0", None):
        if iso is None:
            monkeypatch.delenv("AIJHIP_ISOLATE_ROW_NNZ", raising=False)
        else:
            monkeypatch.setenv("AIJHIP_ISOLATE_ROW_NNZ", iso)
        for exact in (0, 1):
            y, info = mult(pkg, dev, ai, aj, aa, m, x, "stream", exact=exact, gather_sort=0, geometry=6)
            check(y, ref, ai, aj, aa, x, exact=False)
            if exact:
                assert_bits(y, ref)
            elif iso is None:  # (without isolation a long row can lift its block's mean past 128)
                assert_bits(y, ref, short)
            blocks[(iso, exact)] = info["n_blocks"]
    # isolating rows 500, 501 and 2600 adds blocks (a cut before and after each)
    assert blocks[(None, 0)] > blocks[("0", 0)] and blocks[(None, 0)] == blocks[(None, 1)]


def test_long_overlap_auto(pkg, dev):
    """AIJHIP_OPT_LONG_OVERLAP -1 (default): the long rows after the row
    blocks (no side stream), except in exact mode, whose 1-4 K-entry rows keep
    one lane's sequential sum on the side stream."""
    ai, aj, aa = pkg.skewed_csr(300000, seed=1565)
    for exact, want in ((0, 0), (1, 1)):
        with pkg.SeqAIJHIP(ai, aj, aa, exact=exact) as A:
            inf = A.info()
            assert inf["n_long_rows"] > 0 and inf["long_overlap"] == want, (exact, inf["long_overlap"])


@pytest.mark.parametrize("gather_sort,geometry,nt", [(-1, -1, -1), (0, -1, -1), (0, 1, 1), (0, 6, 0), (1, 6, -1)])
def test_long_overlap_is_speed_only(pkg, dev, gather_sort, geometry, nt):
    """AIJHIP_OPT_LONG_OVERLAP: the hub segments and the wide blocks on a
    side stream (1), concurrent with the row blocks: the same launches, so
    the same bits as one stream, for MatMult and MatMultAdd, back to back."""
    ai, aj, aa = pkg.skewed_csr(300000, seed=1565)
    m = len(ai) - 1
    x = to_dev(pkg.splitmix_uniform(m, 7), dev)
    z = to_dev(pkg.splitmix_uniform(m, 8), dev)
    out = []
    for ov in (0, 1):
        with pkg.SeqAIJHIP(ai, aj, aa, gather_sort=gather_sort, long_overlap=ov, geometry=geometry,
                           nt_loads=nt) as A:
            inf = A.info()
            assert inf["n_long_rows"] > 0
            assert inf["long_overlap"] == ov
            y = torch.empty(m, dtype=torch.float64, device=dev)
            w = torch.empty_like(y)
            for _ in range(3):
                A.mult(x, y)
                A.mult_add(x, z, w)
            torch.cuda.synchronize()
            out.append((y.cpu().numpy(), w.cpu().numpy()))
    assert_bits(out[0][0], out[1][0])
    assert_bits(out[0][1], out[1][1])


def test_long_rows_unsorted_columns(pkg, dev, coracle):
    """Long rows whose columns are not ascending (one descending): the
    segments take them in storage order, within the fp64 bound."""
    rng = np.random.default_rng(3)
    m = 50000
    lens = np.full(m, 5)
    lens[[100, 20000]] = 30000
    ai = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    rows = [np.sort(rng.choice(m, size=l, replace=False)) for l in lens]
    rows[20000] = rows[20000][::-1].copy()  # descending
    aj = np.concatenate(rows).astype(np.int32)
    aa = rng.uniform(-1, 1, ai[-1])
    x = rng.uniform(-1, 1, m)
    with pkg.SeqAIJHIP(ai, aj, aa) as A:
        assert A.info()["n_long_rows"] == 2
        xd = to_dev(x, dev)
        yd = torch.empty(m, dtype=torch.float64, device=dev)
        A.mult(xd, yd)
        torch.cuda.synchronize()
        check(yd.cpu().numpy(), coracle.matmult(ai, aj, aa, x, omp=True), ai, aj, aa, x, exact=False)


def test_merge_kernel_withdrawn(pkg, dev):
    """ABI 2 withdrew the explicit merge-path kernel (STREAM's planner is the
    merge-path decomposition): set_kernel("merge") is refused and the handle
    keeps its plan."""
    g = golden("skewed_small")
    with pkg.SeqAIJHIP(g["ai"], g["aj"], g["aa"], ncols=int(g["ncols"])) as A:
        with pytest.raises(pkg.AIJHIPError, match="withdrawn"):
            A.set_kernel("merge")
        assert A.info()["kernel"] == "stream"


@pytest.mark.parametrize("name", ["poisson16", "skewed_small", "compressed_small"])
def test_stream_options_do_not_change_results(pkg, dev, name):
    """Every STREAM geometry / non-temporal setting is speed-only; the
    options withdrawn in ABI 2 are refused."""
    g = golden(name)
    ai, aj, aa, n = g["ai"], g["aj"], g["aa"], int(g["ncols"])
    with pkg.SeqAIJHIP(ai, aj, aa, ncols=n) as A:
        xd = to_dev(g["x"], dev)
        yd = torch.empty(len(ai) - 1, dtype=torch.float64, device=dev)
        for opt in pkg.WITHDRAWN_OPTIONS:
            with pytest.raises(pkg.AIJHIPError, match="withdrawn"):
                A.set_option(opt, 1)
        first = None
        for geom in range(10):
            for nt in (0, 1):
                A.set_option("geometry", geom)
                A.set_option("nt_loads", nt)
                A.set_option("exact", 1)
                A.mult(xd, yd)
                torch.cuda.synchronize()
                y = yd.cpu().numpy()
                if first is None:
                    first = y
                short = np.diff(ai) <= 1024  # below every geometry's block cap
                assert_bits(y, first, short)
                assert_bits(y, g["y"], short)
                check(y, g["y"], ai, aj, aa, g["x"], exact=False)
        # the gather-ordered copy at every geometry (block caps 1024..8190),
        # exact and default modes
        A.set_option("nt_loads", -1)
        short = np.diff(ai) <= 1024
        for geom in range(10):
            ys = {}
            for gs, ex in ((1, 1), (1, 0), (0, 0)):
                A.set_option("geometry", geom)
                A.set_option("gather_sort", gs)
                A.set_option("exact", ex)
                assert (A.info()["gather_sorted"] > 0) == bool(gs and A.info()["n_blocks"] > 0)
                A.mult(xd, yd)
                torch.cuda.synchronize()
                ys[gs, ex] = y = yd.cpu().numpy()
                check(y, g["y"], ai, aj, aa, g["x"], exact=False)
            assert_bits(ys[1, 1], g["y"], short)
            assert_bits(ys[1, 0], ys[0, 0])  # same row sums, sorted gathers or not


def test_fem_hex_flan_standin_all_kernels(pkg, dev, coracle):
    """Flan_1565's mesh structure (BASELINE configs[4]; hexahedral, 3 dofs per
    node, 81-entry interior rows) at a reduced grid: STREAM and SCALAR keep
    PETSc's order (rows fit one block), the others meet the fp64 bound."""
    ai, aj, aa = pkg.fem_hex_csr(21, 20, 19)
    assert np.diff(ai).max() == 81
    x = pkg.splitmix_uniform(len(ai) - 1, 11)
    ref = coracle.matmult(ai, aj, aa, x, omp=True)
    for kernel in ALL_KERNELS:
        y, _ = mult(pkg, dev, ai, aj, aa, len(ai) - 1, x, kernel)
        check(y, ref, ai, aj, aa, x, exact=kernel in BITEXACT)


def test_auto_geometry_follows_gather_locality(pkg, dev, coracle):
    """Automatic STREAM layout (aijhip_api.cpp plan_build): row patterns at
    geometry 6 for short rows that follow few offset lists (the 7-point
    stencil); column codes wherever the row blocks' offset dictionaries fit
    (the FEM rows); otherwise long rows -> the gather-ordered copy in its
    packed form at geometry 6, and without it (gather_sort 0) long scattered
    rows -> geometry 1. The gather-ordered product equals the unsorted one
    and the oracle bit for bit (rows within the block cap)."""
    cases = [(pkg.poisson_csr(12), 6, 0, 0, True, 6), (pkg.fem_hex_csr(21, 20, 19), 6, 0, 1, False, 6),
             (pkg.skewed_csr(300000, seed=1565), 6, 2, 0, False, 1)]  # 2: packed block-relative columns
    for (ai, aj, aa), geom, sorted_, codes, pats, geom_unsorted in cases:
        with pkg.SeqAIJHIP(ai, aj, aa) as A:
            info = A.info()
            assert (info["stream_geometry"], info["gather_sorted"], info["column_codes"],
                    info["row_patterns"] > 0) == (geom, sorted_, codes, pats)
            if not sorted_:
                continue
            x = torch.from_numpy(pkg.splitmix_uniform(A.n, 42)).to(dev)
            y1 = torch.empty(A.m, dtype=torch.float64, device=dev)
            A.mult(x, y1)
            A.set_option("gather_sort", 0)
            assert A.info()["gather_sorted"] == 0 and A.info()["stream_geometry"] == geom_unsorted
            y0 = torch.empty_like(y1)
            A.mult(x, y0)
            torch.cuda.synchronize()
            assert torch.equal(y0, y1)
            A.set_option("gather_sort", -1)
            A.set_option("exact", 1)  # every row within the block cap in PETSc's order
            assert A.info()["gather_sorted"] == 2
            A.mult(x, y1)
            torch.cuda.synchronize()
            ref = coracle.matmult(ai, aj, aa, x.cpu().numpy(), omp=True)
            short = np.diff(ai) <= info["stream_nnz_cap"]
            assert np.array_equal(y1.cpu().numpy()[short].view(np.uint64), ref[short].view(np.uint64))


@pytest.mark.parametrize("wide,form", [(0, 2), (40, 1), (4999, 2)])
def test_gather_sort_32_bit_and_packed_columns(pkg, dev, coracle, wide, form):
    """The gather-ordered copy in its packed form (a word per entry: the
    column relative to the block's first in 20 bits, the product slot in 12;
    every block's columns within 2^20), with 32-bit columns (a row every 40
    reaching both ends of a 2^21-column x: every block wide), and split (a
    wide row every 4999: those blocks from the original arrays, the rest
    packed): MatMult and MatMultAdd equal the unsorted kernel and the oracle
    bit for bit (exact mode), and new values (aijhip_mat_update_values) reach
    the sorted copy."""
    rng = np.random.default_rng(21)
    m, n = 90000, 1 << 21
    lens = rng.integers(40, 100, m)
    cols = []
    for i, l in enumerate(lens):
        lo, hi = max(0, i - 3000), min(m, i + 3000)
        c = np.sort(rng.choice(np.arange(lo, hi), size=l, replace=False))
        if wide and i % wide == 0:
            c = np.unique(np.concatenate([c, [0, n - 1]]))
        cols.append(c)
    ai = np.concatenate([[0], np.cumsum([len(c) for c in cols])]).astype(np.int32)
    aj = np.concatenate(cols).astype(np.int32)
    aa = rng.uniform(-1, 1, len(aj))
    x = rng.uniform(-1, 1, n)
    z = rng.uniform(-1, 1, m)
    with pkg.SeqAIJHIP(ai, aj, aa, ncols=n, exact=1, gather_sort=1) as A:
        assert A.info()["gather_sorted"] == form
        xd, zd = to_dev(x, dev), to_dev(z, dev)
        y = torch.empty(m, dtype=torch.float64, device=dev)
        w = torch.empty_like(y)
        A.mult(xd, y)
        A.mult_add(xd, zd, w)
        torch.cuda.synchronize()
        assert_bits(y.cpu().numpy(), coracle.matmult(ai, aj, aa, x, omp=True))
        A.set_option("gather_sort", 0)
        w0 = torch.empty_like(y)
        A.mult_add(xd, zd, w0)
        torch.cuda.synchronize()
        assert torch.equal(w, w0)
        A.set_option("gather_sort", 1)
        aa2 = rng.uniform(-1, 1, len(aj))
        A.update_values(aa2)
        A.mult(xd, y)
        torch.cuda.synchronize()
        assert_bits(y.cpu().numpy(), coracle.matmult(ai, aj, aa2, x, omp=True))
