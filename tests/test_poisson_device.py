"""Device-side Poisson assembly (csrc/poisson.hip) against
the host producer (harness.cpp, itself pinned to oracle/seqaij.py's
helper.cpp restatement): bit-identical CSR, vectors and SpMV results, over
whole grids, z-slabs, degenerate (1-wide) grids, with and without the
reference point."""
import ctypes

import numpy as np
import pytest

GRIDS = [(8, 8, 8, 0, 8), (6, 7, 5, 0, 5), (9, 4, 7, 2, 6), (5, 5, 6, 0, 1), (5, 5, 6, 5, 6),
         (1, 1, 5, 0, 5), (1, 6, 3, 0, 3), (7, 1, 1, 0, 1), (16, 16, 16, 3, 11), (33, 17, 9, 0, 9)]


@pytest.mark.gpu
@pytest.mark.parametrize("ref", [True, False])
@pytest.mark.parametrize("g", GRIDS)
def test_fill_device_matches_host(pkg, g, ref):
    import torch
    nx, ny, nz, z0, z1 = g
    ai, aj, aa = pkg.poisson_csr(nx, ny, nz, z0, z1, ref_point=ref)
    dai = torch.full((len(ai),), -7, dtype=torch.int32, device="cuda")
    daj = torch.full((max(len(aj), 1),), -7, dtype=torch.int32, device="cuda")
    daa = torch.full((max(len(aa), 1),), np.nan, dtype=torch.float64, device="cuda")
    sc = ctypes.c_double()
    pkg._check(pkg.lib().aijhip_poisson_fill_device(nx, ny, nz, z0, z1, int(ref), dai.data_ptr(), daj.data_ptr(),
                                                    daa.data_ptr(), ctypes.byref(sc), None))
    torch.cuda.synchronize()
    assert np.array_equal(dai.cpu().numpy(), ai)
    assert np.array_equal(daj.cpu().numpy()[: len(aj)], aj)
    assert np.array_equal(daa.cpu().numpy()[: len(aa)].view(np.uint64), aa.view(np.uint64))


@pytest.mark.gpu
@pytest.mark.parametrize("ref", [True, False])
@pytest.mark.parametrize("g", GRIDS)
def test_vectors_device_match_host(pkg, g, ref):
    import torch
    nx, ny, nz, z0, z1 = g
    rhs, exact = pkg.poisson_vectors(nx, ny, nz, z0, z1, ref_point=ref)
    r = torch.empty(len(rhs), dtype=torch.float64, device="cuda")
    e = torch.empty_like(r)
    pkg.poisson_vectors_device(nx, ny, nz, z0, z1, ref_point=ref, rhs=r, exact=e)
    assert np.array_equal(r.cpu().numpy().view(np.uint64), rhs.view(np.uint64))
    assert np.array_equal(e.cpu().numpy().view(np.uint64), exact.view(np.uint64))


@pytest.mark.gpu
@pytest.mark.parametrize("N", [24, 100])
def test_mat_create_poisson_mult_bitwise(pkg, N):
    import torch
    A, sc = pkg.poisson_device(N)
    ai, aj, aa = pkg.poisson_csr(N)
    B = pkg.SeqAIJHIP(ai, aj, aa)
    inf = A.info()
    assert (inf["m"], inf["n"], inf["nz"]) == (N ** 3, N ** 3, len(aj))
    x = torch.from_numpy(pkg.splitmix_uniform(N ** 3, 42)).cuda()
    ya, yb = torch.empty_like(x), torch.empty_like(x)
    A.mult(x, ya)
    B.mult(x, yb)
    assert torch.equal(ya, yb)
    row0 = slice(ai[0], ai[1])
    assert sc == aa[row0][aj[row0] == 0][0]  # setRefPoint's a_00 = scale
    A.destroy()
    B.destroy()


@pytest.mark.gpu
def test_create_from_device_rejects_bad_columns(pkg):
    import torch
    ai = torch.tensor([0, 2, 3], dtype=torch.int32, device="cuda")
    aj = torch.tensor([0, 5, 1], dtype=torch.int32, device="cuda")
    aa = torch.ones(3, dtype=torch.float64, device="cuda")
    h = ctypes.c_void_p()
    rc = pkg.lib().aijhip_mat_create_from_device(0, 2, 2, 3, ai.data_ptr(), aj.data_ptr(), aa.data_ptr(),
                                                  ctypes.byref(h))
    assert rc == pkg.AIJHIP_ERR_ARG and b"out of range" in pkg.lib().aijhip_last_error()


def test_device_producers_are_exported(pkg):
    L = pkg.lib()
    for n in ("aijhip_poisson_fill_device", "aijhip_poisson_vectors_device", "aijhip_mat_create_poisson"):
        assert hasattr(L, n)
