"""GAMG hierarchy: the C++ host set-up vs the scipy restatement
(oracle/gamg.py), CPU only; the device V-cycle and CG+GAMG are in the GPU
section."""
import importlib

import numpy as np
import pytest
import scipy.sparse as sp

from oracle import gamg as ogamg
from oracle import ksp_cg, seqaij


def _csr(t, shape):
    ai, aj, aa = t
    M = sp.csr_matrix((aa, aj, ai), shape=shape)
    M.eliminate_zeros()
    M.sort_indices()
    return M


def _cmp(A, B, rtol=1e-12):
    A = sp.csr_matrix(A); A.eliminate_zeros(); A.sort_indices()
    B = sp.csr_matrix(B); B.eliminate_zeros(); B.sort_indices()
    assert A.shape == B.shape
    # structure equal up to entries that cancel to ~0 in one but not the other
    D = (A - B).tocoo()
    scale = max(abs(A).max(), 1e-300)
    assert np.all(np.abs(D.data) <= rtol * scale), np.max(np.abs(D.data)) / scale


@pytest.mark.parametrize("dims", [(8, 8, 8), (12, 12, 12), (6, 7, 5), (20, 20, 20), (24, 24, 24)])
def test_host_hierarchy_matches_oracle_bitwise(pkg, dims):
    """Aggregation at level l+1 depends on the last bit of A_{l+1} (zero
    threshold, ties), so the two set-ups must agree exactly."""
    G = importlib.import_module("petsc-openacc_amd.gamg")
    ai, aj, aa = pkg.poisson_csr(*dims)
    m = len(ai) - 1
    A = sp.csr_matrix((aa, aj, ai), shape=(m, m))
    lv = G.build_host(ai, aj, aa, coarse_eq_limit=20, coarsen=0, eig_ksp=0)  # greedy + power iteration
    ol = ogamg.build(A, coarse_eq_limit=20, coarsen=0, eig_ksp=0)
    assert len(lv) == len(ol) >= 2
    for l in range(len(lv) - 1):
        assert np.array_equal(lv[l]["agg"], ol[l]["agg"])
        assert lv[l]["emax"] == ol[l]["emax"]
        mc = lv[l + 1]["m"]
        for mine, theirs in ((_csr(lv[l]["P"], (lv[l]["m"], mc)), ol[l]["P"]),
                             (_csr(lv[l + 1]["A"], (mc, mc)), ol[l + 1]["A"])):
            theirs = theirs.copy()
            theirs.eliminate_zeros()
            theirs.sort_indices()
            assert np.array_equal(mine.indptr, theirs.indptr) and np.array_equal(mine.indices, theirs.indices)
            assert np.array_equal(mine.data, theirs.data)


@pytest.mark.parametrize("dims", [(8, 8, 8), (12, 12, 12), (6, 7, 5), (16, 16, 16)])
@pytest.mark.parametrize("eig_ksp", [0, 1])
def test_host_mis_hierarchy_matches_oracle_bitwise(pkg, dims, eig_ksp):
    """PETSc 3.7 agg's coarsening (coarsen 1: MIS on the squared graph at the
    finest level, smoothAggs, then MIS on the graph; the reference point row
    0 a removed singleton) and its CG emax estimate (eig_ksp 1): the C++ host
    set-up equals the literal sequential restatement (oracle/gamg.py
    aggregate_mis, estimate_emax_cg) bit for bit."""
    G = importlib.import_module("petsc-openacc_amd.gamg")
    ai, aj, aa = pkg.poisson_csr(*dims)
    m = len(ai) - 1
    A = sp.csr_matrix((aa, aj, ai), shape=(m, m))
    lv = G.build_host(ai, aj, aa, coarse_eq_limit=20, coarsen=1, eig_ksp=eig_ksp)
    ol = ogamg.build(A, coarse_eq_limit=20, coarsen=1, eig_ksp=eig_ksp)
    assert len(lv) == len(ol) >= 2
    assert lv[0]["agg"][0] == -1 and ol[0]["agg"][0] == -1  # row 0: only explicit zeros off the diagonal
    for l in range(len(lv) - 1):
        assert np.array_equal(lv[l]["agg"], ol[l]["agg"])
        assert lv[l]["emax"] == ol[l]["emax"]
        mc = lv[l + 1]["m"]
        for mine, theirs in ((_csr(lv[l]["P"], (lv[l]["m"], mc)), ol[l]["P"]),
                             (_csr(lv[l + 1]["A"], (mc, mc)), ol[l + 1]["A"])):
            theirs = theirs.copy()
            theirs.eliminate_zeros()
            theirs.sort_indices()
            assert np.array_equal(mine.indptr, theirs.indptr) and np.array_equal(mine.indices, theirs.indices)
            assert np.array_equal(mine.data, theirs.data)


def test_mis_aggregates_are_petsc_shaped():
    """The restated MIS on the squared graph: roots pairwise more than two
    steps apart in S, every other node (but the removed singletons) in the
    aggregate of a root within two steps (one, after smoothAggs, when a root
    is adjacent), aggregates numbered by their roots' order."""
    ai, aj, aa, _, _ = seqaij.create_system(10, 10, 10)
    m = len(ai) - 1
    A = sp.csr_matrix((aa, aj, ai), shape=(m, m))
    d = ogamg.first_diagonal(A)
    S = ogamg.strength_graph(A, d, 0.0)
    agg, na = ogamg.aggregate_mis(S, True, ogamg.mis_keys(m, 0))
    G1 = (S + sp.identity(m, format="csr")).astype(bool).tocsr()
    G2 = (G1.astype(np.int32) @ G1.astype(np.int32)).astype(bool).tocsr()
    # the roots, by PETSc's rule (an undone node at its turn in key order)
    isroot = np.zeros(m, bool)
    keys = ogamg.mis_keys(m, 0)
    order = np.argsort(keys, kind="stable")
    taken = np.zeros(m, bool)
    for v in order:
        if taken[v] or S.indptr[v] == S.indptr[v + 1]:
            continue
        isroot[v] = True
        taken[G2.indices[G2.indptr[v]:G2.indptr[v + 1]]] = True
    r = np.flatnonzero(isroot)
    assert len(r) == na and np.array_equal(agg[r], np.arange(na))
    for v in r:  # independent in G2
        nb = G2.indices[G2.indptr[v]:G2.indptr[v + 1]]
        assert isroot[nb].sum() == 1
    for v in np.flatnonzero(agg >= 0):
        if isroot[v]:
            continue
        root = r[agg[v]]
        assert G2[v, root]
    assert np.all((agg == -1) == (np.diff(S.indptr) == 0))


def test_host_hierarchy_thread_invariant(pkg):
    G = importlib.import_module("petsc-openacc_amd.gamg")
    ai, aj, aa = pkg.poisson_csr(16)
    a = G.build_host(ai, aj, aa, threads=1)
    b = G.build_host(ai, aj, aa, threads=4)
    for la, lb in zip(a, b):
        for key in ("A", "P"):
            if key in la:
                for x, y in zip(la[key], lb[key]):
                    assert np.array_equal(np.asarray(x).view(np.uint8), np.asarray(y).view(np.uint8))


def test_hierarchy_galerkin_and_coarsening(pkg):
    G = importlib.import_module("petsc-openacc_amd.gamg")
    ai, aj, aa = pkg.poisson_csr(16)
    lv = G.build_host(ai, aj, aa)
    sizes = [L["m"] for L in lv]
    assert all(b < a for a, b in zip(sizes, sizes[1:])) and sizes[-1] <= 50 or len(lv) == 10
    # the coarse operators stay symmetric; P's columns reproduce the near-null
    # space on the aggregates before smoothing (unit norm columns)
    for l in range(1, len(lv)):
        Ac = _csr(lv[l]["A"], (lv[l]["m"],) * 2)
        assert abs(Ac - Ac.T).max() <= 1e-10 * abs(Ac).max()


@pytest.mark.gpu
@pytest.mark.parametrize("N,norm", [(12, "preconditioned"), (20, "preconditioned"), (16, "unpreconditioned")])
def test_gpu_cg_gamg_matches_oracle(pkg, N, norm):
    torch = pytest.importorskip("torch")
    assert torch.cuda.is_available()
    K = importlib.import_module("petsc-openacc_amd.ksp")
    ai, aj, aa = pkg.poisson_csr(N)
    rhs, exact = pkg.poisson_vectors(N)
    m = len(ai) - 1
    levels = ogamg.build(sp.csr_matrix((aa, aj, ai), shape=(m, m)), coarse_eq_limit=50)
    tol = dict(rtol=1e-14, atol=1e-12, max_it=10000)
    xo, its_o, reason_o, hist_o = ksp_cg.cg(ai, aj, aa, rhs, pc=lambda r: ogamg.vcycle(levels, r), norm=norm, **tol)
    A = pkg.SeqAIJHIP(ai, aj, aa)
    b = torch.from_numpy(rhs).cuda()
    x = torch.empty_like(b)
    with K.KSPCG(A, pc="gamg", norm=norm, **tol) as ksp:
        ksp.solve(b, x)
        rows, nnz, secs = ksp.pc_levels()
        assert rows == [L["A"].shape[0] for L in levels]
        assert ksp.reason == reason_o and abs(ksp.its - its_o) <= 1, (ksp.its, its_o, ksp.reason, reason_o)
        h = ksp.history()
        k = min(10, len(h), len(hist_o))
        np.testing.assert_allclose(h[:k], hist_o[:k], rtol=1e-7)
        xg = x.cpu().numpy()
        assert np.linalg.norm(xg - xo) <= 1e-8 * np.linalg.norm(xo)
        # fewer iterations than CG + Jacobi on the same problem
        _, its_j, _, _ = ksp_cg.cg(ai, aj, aa, rhs, **tol)
        assert ksp.its < its_j
    A.destroy()


@pytest.mark.gpu
def test_gpu_vcycle_fused_smoothers_bitwise(pkg, monkeypatch):
    """The fused V-cycle smoothers (residual and Richardson+Jacobi step in the
    SpMV epilogue, default) and the unfused kernels (PCMG's separate
    smoother, MatResidual and vector passes; AIJHIP_MG_UNFUSED=1) round every
    entry the same way on one GPU; only CG's z.z / z.r are summed in another
    block order (the fused finest post-smoothing's STREAM blocks against the
    vector grid), so the iterations are the same and the histories and
    solutions agree to 1e-12 relative."""
    torch = pytest.importorskip("torch")
    assert torch.cuda.is_available()
    K = importlib.import_module("petsc-openacc_amd.ksp")
    N = 24
    ai, aj, aa = pkg.poisson_csr(N)
    rhs, _ = pkg.poisson_vectors(N)
    b = torch.from_numpy(rhs).cuda()
    out = []
    for unfused in (None, "1"):
        if unfused is None:
            monkeypatch.delenv("AIJHIP_MG_UNFUSED", raising=False)
        else:
            monkeypatch.setenv("AIJHIP_MG_UNFUSED", unfused)
        with pkg.SeqAIJHIP(ai, aj, aa) as A:
            x = torch.empty_like(b)
            with K.KSPCG(A, pc="gamg", rtol=1e-14, atol=1e-12) as ksp:
                ksp.solve(b, x)
                out.append((ksp.its, np.array(ksp.history()), x.cpu().numpy()))
    for its, h, xv in out[1:]:
        assert its == out[0][0]
        np.testing.assert_allclose(h, out[0][1], rtol=1e-12, atol=1e-15 * out[0][1][0])
        np.testing.assert_allclose(xv, out[0][2], rtol=1e-10, atol=1e-12 * np.abs(out[0][2]).max())


@pytest.mark.gpu
def test_gpu_cg_gamg_fused_default_deterministic_and_values_update(pkg):
    """The default (fused) CG + GAMG pinned bit for bit: two
    solves on fresh handles give the same history and solution bits; and a
    set-up KSP whose operator got new values (aijhip_mat_update_values, the
    MatAssemblyEnd re-upload) redoes its PC set-up — its next solve equals, bit
    for bit, a fresh KSP's on the new values (PETSc's PCSetUp on a changed
    operator state), not the stale hierarchy's."""
    torch = pytest.importorskip("torch")
    assert torch.cuda.is_available()
    K = importlib.import_module("petsc-openacc_amd.ksp")
    N = 24
    ai, aj, aa = pkg.poisson_csr(N)
    rhs, _ = pkg.poisson_vectors(N)
    b = torch.from_numpy(rhs).cuda()
    aa2 = aa * 2.0 + np.where(aj == np.repeat(np.arange(len(ai) - 1), np.diff(ai)), -1.0, 0.0)

    def solve(vals, A=None, ksp=None):
        own = A is None
        A = A or pkg.SeqAIJHIP(ai, aj, vals)
        ksp = ksp or K.KSPCG(A, pc="gamg", rtol=1e-14, atol=1e-12)
        x = torch.empty_like(b)
        ksp.solve(b, x)
        r = (ksp.its, np.array(ksp.history()), x.cpu().numpy())
        if own:
            ksp.destroy()
            A.destroy()
        return r

    def same(r, q):
        assert r[0] == q[0]
        assert np.array_equal(r[1].view(np.uint64), q[1].view(np.uint64))
        assert np.array_equal(r[2].view(np.uint64), q[2].view(np.uint64))

    first, again = solve(aa), solve(aa)
    same(first, again)
    fresh2 = solve(aa2)
    with pkg.SeqAIJHIP(ai, aj, aa) as A:
        with K.KSPCG(A, pc="gamg", rtol=1e-14, atol=1e-12) as ksp:
            same(solve(aa, A, ksp), first)
            A.update_values(aa2)
            same(solve(aa2, A, ksp), fresh2)
    assert fresh2[0] != first[0] or not np.array_equal(fresh2[2], first[2])


@pytest.mark.gpu
@pytest.mark.parametrize("N", [24, 48])
def test_gpu_cg_gamg_gather_ordered_levels_bitwise(pkg, N, monkeypatch):
    """The set-up's operators (levels, P, Pᵀ) with the gather-ordered copy
    (each block's entries sorted by column, products stored at their CSR
    slots; the fused V-cycle launches take the sorted arrays too) — on long
    rows (the default), on none (AIJHIP_SETUP_GSORT=0) or on every operator
    (1) — solve bit for bit the same."""
    torch = pytest.importorskip("torch")
    assert torch.cuda.is_available()
    K = importlib.import_module("petsc-openacc_amd.ksp")
    ai, aj, aa = pkg.poisson_csr(N)
    rhs, _ = pkg.poisson_vectors(N)
    b = torch.from_numpy(rhs).cuda()
    out = []
    for gs in ("0", None, "1"):
        if gs is None:
            monkeypatch.delenv("AIJHIP_SETUP_GSORT", raising=False)
        else:
            monkeypatch.setenv("AIJHIP_SETUP_GSORT", gs)
        with pkg.SeqAIJHIP(ai, aj, aa) as A:
            x = torch.empty_like(b)
            with K.KSPCG(A, pc="gamg", rtol=1e-14, atol=1e-12) as ksp:
                ksp.solve(b, x)
                out.append((ksp.its, np.array(ksp.history()), x.cpu().numpy()))
    for its, h, xv in out[1:]:
        assert its == out[0][0]
        assert np.array_equal(h.view(np.uint64), out[0][1].view(np.uint64))
        assert np.array_equal(xv.view(np.uint64), out[0][2].view(np.uint64))


def test_oracle_vcycle_preconditions_cg():
    ai, aj, aa, rhs, exact = seqaij.create_system(10, 10, 10)
    m = len(ai) - 1
    A = sp.csr_matrix((aa, aj, ai), shape=(m, m))
    levels = ogamg.build(A, coarse_eq_limit=20)
    _, its_j, _, _ = ksp_cg.cg(ai, aj, aa, rhs, rtol=1e-10, max_it=1000)
    # CG with the V-cycle as preconditioner (oracle only)
    x = np.zeros(m)
    r = rhs.copy()
    z = ogamg.vcycle(levels, r)
    p = z.copy()
    beta = r @ z
    its = 0
    r0 = np.linalg.norm(z)
    while its < 200:
        w = A @ p
        a = beta / (p @ w)
        x += a * p
        r -= a * w
        z = ogamg.vcycle(levels, r)
        its += 1
        if np.linalg.norm(z) <= 1e-10 * r0:
            break
        bn = r @ z
        p = z + (bn / beta) * p
        beta = bn
    # the reference's options (undamped Richardson+Jacobi smoothing, one
    # Jacobi sweep as the coarse solve) make a modest V-cycle, still < half
    # of Jacobi-CG's iterations at 10^3
    assert its < its_j / 2, (its, its_j)


def _bits(x):
    return np.ascontiguousarray(x).view(np.uint64)


@pytest.mark.gpu
@pytest.mark.parametrize("dims,params", [
    ((8, 8, 8), dict(coarse_eq_limit=20)),
    ((12, 12, 12), dict(coarse_eq_limit=20)),
    ((6, 7, 5), dict(coarse_eq_limit=20)),
    ((20, 20, 20), {}),
    ((24, 24, 24), dict(coarse_eq_limit=20)),
    ((16, 16, 16), dict(threshold=0.05)),
    ((16, 16, 16), dict(nsmooths=0)),
    ((32, 32, 32), dict(device_min_rows=20000)),  # device level 0, host below
])
@pytest.mark.parametrize("agg", ["auto", "device"])
def test_gpu_device_setup_matches_host_bitwise(pkg, dims, params, agg, monkeypatch):
    """The KSP's device-built hierarchy (aijhip_gamg::build_device, host
    continuation below device_min_rows) equals the host builder's — itself
    bit-identical to oracle/gamg.py — entry for entry. agg = device: the
    aggregation's phase 1 as the device sweep on every level (automatic only
    from 2^20 rows), phase 3 over the gathered left-over rows."""
    if agg == "device":
        monkeypatch.setenv("AIJHIP_GAMG_AGG", "device")
    ai, aj, aa = pkg.poisson_csr(*dims)
    _check_device_setup(pkg, ai, aj, aa, params)


@pytest.mark.gpu
@pytest.mark.parametrize("dims,params", [
    ((8, 8, 8), dict(coarse_eq_limit=20)),
    ((12, 12, 12), dict(coarse_eq_limit=20, eig_ksp=1)),
    ((6, 7, 5), dict(coarse_eq_limit=20)),
    ((24, 24, 24), dict(eig_ksp=1)),
    ((16, 16, 16), dict(square_graph=2, eig_ksp=1)),
    ((40, 40, 40), dict(device_min_rows=20000, eig_ksp=1)),  # device level 0, host below
])
def test_gpu_device_mis_setup_matches_host_bitwise(pkg, dims, params):
    """coarsen 1 (PETSc 3.7 agg's MIS, squared graph on the first
    square_graph levels, smoothAggs; singletons removed) on the device — the
    parallel rounds of gamg_aggregate.hip aggregate_mis_device — equals the
    host builder's sequential pass (itself the oracle's, bit for bit), with
    the CG emax estimate (eig_ksp 1) on the device too."""
    ai, aj, aa = pkg.poisson_csr(*dims)
    prm = dict(coarsen=1)
    prm.update(params)
    _check_device_setup(pkg, ai, aj, aa, prm)


def _check_device_setup(pkg, ai, aj, aa, params):
    torch = pytest.importorskip("torch")
    assert torch.cuda.is_available()
    K = importlib.import_module("petsc-openacc_amd.ksp")
    G = importlib.import_module("petsc-openacc_amd.gamg")
    prm = dict(device_min_rows=0)
    prm.update(params)
    lv = G.build_host(ai, aj, aa, **prm)
    A = pkg.SeqAIJHIP(ai, aj, aa)
    with K.KSPCG(A, pc="gamg", gamg=prm) as ksp:
        ksp.set_up()
        rows, nnz, _ = ksp.pc_levels()
        assert rows == [L["m"] for L in lv]
        for l in range(1, len(lv)):
            dai, daj, daa, _ = ksp.pc_level(l, "A")
            hai, haj, haa = lv[l]["A"]
            assert np.array_equal(dai, hai) and np.array_equal(daj, haj), l
            assert np.array_equal(_bits(daa), _bits(haa)), l
        for l in range(len(lv) - 1):
            pai, paj, paa, pn = ksp.pc_level(l, "P")
            hai, haj, haa = lv[l]["P"]
            assert pn == lv[l + 1]["m"]
            assert np.array_equal(pai, hai) and np.array_equal(paj, haj), l
            assert np.array_equal(_bits(paa), _bits(haa)), l
        path, _ = ksp.setup_path()
    A.destroy()
    return path


def _hub_operator(n_side, hubs, seed, unsorted):
    """A 3-D Poisson operator plus `hubs` rows coupled (symmetrically, weakly)
    to many others — strength lists of 65..1024 and of more than 1024 entries
    — with the diagonal raised to keep it diagonally dominant."""
    import scipy.sparse as sp
    rng = np.random.default_rng(seed)
    import importlib as _il
    pkg = _il.import_module("petsc-openacc_amd")
    ai, aj, aa = pkg.poisson_csr(n_side)
    m = len(ai) - 1
    A = sp.csr_matrix((aa, aj, ai), shape=(m, m)).tocoo()
    r, c, v = [A.row], [A.col], [A.data]
    for h, deg in hubs:
        nb = rng.choice(np.setdiff1d(np.arange(m), [h]), size=deg, replace=False)
        w = rng.uniform(1.0, 50.0, size=deg)
        r += [np.full(deg, h), nb]
        c += [nb, np.full(deg, h)]
        v += [w, w]
    B = sp.coo_matrix((np.concatenate(v), (np.concatenate(r), np.concatenate(c))), shape=(m, m)).tocsr()
    B.sum_duplicates()
    off = np.asarray(abs(B).sum(axis=1)).ravel() - abs(B.diagonal())
    B.setdiag(-(off + 1.0))  # the Poisson rows' sign: negative diagonal
    B.sort_indices()
    ai, aj, aa = B.indptr.astype(np.int32), B.indices.astype(np.int32), B.data.astype(np.float64)
    if unsorted:  # reverse every row's storage order
        aj, aa = aj.copy(), aa.copy()
        for i in range(m):
            aj[ai[i]:ai[i + 1]] = aj[ai[i]:ai[i + 1]][::-1]
            aa[ai[i]:ai[i + 1]] = aa[ai[i]:ai[i + 1]][::-1]
    return ai, aj, aa


@pytest.mark.gpu
@pytest.mark.parametrize("unsorted", [False, True])
@pytest.mark.parametrize("agg", ["auto", "device"])
def test_gpu_device_setup_long_strength_lists(pkg, unsorted, agg, monkeypatch):
    """Strength lists past one wavefront (a workgroup per row) and past the
    LDS list (a lane per row), on sorted and on unsorted rows: the device
    hierarchy still equals the host builder's bit for bit (with the phase-1
    sweep too: hub rows make long walks and irregular root chains)."""
    if agg == "device":
        monkeypatch.setenv("AIJHIP_GAMG_AGG", "device")
    ai, aj, aa = _hub_operator(14, [(5, 40), (100, 300), (2000, 700), (7, 1500)], 7, unsorted)
    _check_device_setup(pkg, ai, aj, aa, dict(coarse_eq_limit=20))


def _spd_from_pattern(m, rows, cols, seed):
    """Symmetric, diagonally dominant (negative diagonal, as the Poisson
    rows) from an off-diagonal pattern; rows sorted."""
    import scipy.sparse as sp
    rng = np.random.default_rng(seed)
    w = rng.uniform(0.5, 2.0, size=len(rows))
    B = sp.coo_matrix((np.concatenate([w, w]), (np.concatenate([rows, cols]), np.concatenate([cols, rows]))),
                      shape=(m, m)).tocsr()
    B.sum_duplicates()
    off = np.asarray(abs(B).sum(axis=1)).ravel()
    B = B + sp.diags(-(off + 1.0))
    B = sp.csr_matrix(B)
    B.sort_indices()
    return B.indptr.astype(np.int32), B.indices.astype(np.int32), B.data.astype(np.float64)


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["path", "random", "isolated"])
def test_gpu_device_aggregation_sweep_on_irregular_graphs(pkg, case, monkeypatch):
    """The phase-1 device sweep (gamg_aggregate.hip, forced on every level)
    on graphs unlike the 7-point lattice: a path (a chain of ~m/3 roots, one
    per round), a random symmetric graph, and a lattice with isolated rows
    (no strong neighbour: never a root, phase 3 singletons). The hierarchy
    must equal the host builder's bit for bit."""
    monkeypatch.setenv("AIJHIP_GAMG_AGG", "device")
    if case == "path":
        m = 6000
        r = np.arange(m - 1)
        ai, aj, aa = _spd_from_pattern(m, r, r + 1, 1)
    elif case == "random":
        m = 30000
        rng = np.random.default_rng(3)
        r = rng.integers(0, m, size=m)  # mean degree 2 (wider Galerkin rows outgrow the device classes)
        c = rng.integers(0, m, size=m)
        keep = r != c
        ai, aj, aa = _spd_from_pattern(m, r[keep], c[keep], 2)
    else:
        import scipy.sparse as sp
        pai, paj, paa = pkg.poisson_csr(12)
        P = sp.csr_matrix((paa, paj, pai), shape=(1728, 1728))
        iso = sp.diags(np.full(200, -3.0))
        B = sp.csr_matrix(sp.block_diag([P, iso]))
        perm = np.random.default_rng(5).permutation(B.shape[0])  # isolated rows spread through the order
        B = sp.csr_matrix(B[perm][:, perm])
        B.sort_indices()
        ai, aj, aa = B.indptr.astype(np.int32), B.indices.astype(np.int32), B.data.astype(np.float64)
    path = _check_device_setup(pkg, ai, aj, aa, dict(coarse_eq_limit=20))
    assert path[0][0] == "device", path  # the finest coarsening was built on the device: the sweep ran
