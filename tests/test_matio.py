"""Matrix / vector files (petsc-openacc_amd/matio.py): PETSc binary and
MatrixMarket into the CSR arrays of the SeqAIJ path.

CPU: byte layout of the PETSc binary format, round trips against the golden
fixtures, MatrixMarket symmetric expansion / duplicate summation / explicit
zeros, and the error paths. GPU: a file-loaded operand through the HIP SpMV is
bit-identical to the fixture's y (the loaded CSR is the same matrix).
"""
from __future__ import annotations

import importlib

import numpy as np
import pytest

from conftest import golden

matio = importlib.import_module("petsc-openacc_amd.matio")


@pytest.mark.parametrize("name", ["poisson8", "skewed_small", "compressed_small"])
def test_petsc_binary_roundtrip(tmp_path, name):
    g = golden(name)
    p = tmp_path / f"{name}.petsc"
    matio.save_petsc_binary(p, g["ai"], g["aj"], g["aa"], int(g["ncols"]))
    ai, aj, aa, n = matio.load_petsc_binary(p)
    assert n == int(g["ncols"])
    np.testing.assert_array_equal(ai, g["ai"])
    np.testing.assert_array_equal(aj, g["aj"])
    assert np.array_equal(aa.view(np.uint64), np.ascontiguousarray(g["aa"]).view(np.uint64))
    assert ai.dtype == np.int32 and aj.dtype == np.int32 and aa.dtype == np.float64


def test_petsc_binary_byte_layout(tmp_path):
    """Header {1211216, M, N, nz}, row lengths, columns, values; big-endian."""
    ai = np.array([0, 2, 2, 3], dtype=np.int32)
    aj = np.array([0, 2, 1], dtype=np.int32)
    aa = np.array([1.5, -2.0, 0.0])
    p = tmp_path / "a.petsc"
    matio.save_petsc_binary(p, ai, aj, aa, 3)
    raw = p.read_bytes()
    ints = np.frombuffer(raw[: 4 * (4 + 3 + 3)], dtype=">i4")
    np.testing.assert_array_equal(ints, [1211216, 3, 3, 3, 2, 0, 1, 0, 2, 1])
    np.testing.assert_array_equal(np.frombuffer(raw[40:], dtype=">f8"), aa)
    assert len(raw) == 40 + 24


def test_petsc_vec_roundtrip(tmp_path):
    v = np.linspace(-1, 1, 17)
    p = tmp_path / "v.petsc"
    matio.save_petsc_vec(p, v)
    assert np.frombuffer(p.read_bytes()[:8], dtype=">i4").tolist() == [1211214, 17]
    np.testing.assert_array_equal(matio.load_petsc_vec(p), v)


def test_petsc_binary_errors(tmp_path):
    bad = tmp_path / "bad"
    bad.write_bytes(np.array([1211214, 3], dtype=">i4").tobytes())  # a Vec, not a Mat
    with pytest.raises(ValueError, match="not a PETSc binary Mat"):
        matio.load_petsc_binary(bad)
    p = tmp_path / "t.petsc"
    matio.save_petsc_binary(p, [0, 1, 2], [0, 1], [1.0, 2.0], 2)
    p.write_bytes(p.read_bytes()[:-8])
    with pytest.raises(ValueError, match="truncated"):
        matio.load_petsc_binary(p)
    with pytest.raises(ValueError, match="out of range"):
        matio.save_petsc_binary(tmp_path / "o", [0, 1], [5], [1.0], 2)


MTX_SYM = """%%MatrixMarket matrix coordinate real symmetric
% lower triangle, a duplicate (3,1) and an explicit zero (4,4)
4 4 6
1 1 4.0
3 1 -1.0
3 1 -0.5
2 2 5.0
4 3 2.0
4 4 0.0
"""


def test_mtx_symmetric_duplicates_zeros(tmp_path):
    p = tmp_path / "s.mtx"
    p.write_text(MTX_SYM)
    ai, aj, aa, n = matio.load_mtx(p)
    assert n == 4
    np.testing.assert_array_equal(ai, [0, 2, 3, 5, 7])
    np.testing.assert_array_equal(aj, [0, 2, 1, 0, 3, 2, 3])   # ascending within rows
    np.testing.assert_array_equal(aa, [4.0, -1.5, 5.0, -1.5, 2.0, 2.0, 0.0])  # zero kept


def test_mtx_general_pattern(tmp_path):
    p = tmp_path / "g.mtx"
    p.write_text("%%MatrixMarket matrix coordinate pattern general\n3 5 3\n3 5\n1 2\n3 1\n")
    ai, aj, aa, n = matio.load_mtx(p)
    assert n == 5
    np.testing.assert_array_equal(ai, [0, 1, 1, 3])
    np.testing.assert_array_equal(aj, [1, 0, 4])
    np.testing.assert_array_equal(aa, [1.0, 1.0, 1.0])


def test_mtx_matches_fixture(tmp_path):
    import scipy.io
    import scipy.sparse as sp

    g = golden("skewed_small")
    m = len(g["ai"]) - 1
    A = sp.csr_matrix((g["aa"], g["aj"], g["ai"]), shape=(m, int(g["ncols"])))
    p = tmp_path / "k.mtx"
    scipy.io.mmwrite(str(p), A, precision=17)
    ai, aj, aa, n = matio.load_mtx(p)
    np.testing.assert_array_equal(ai, g["ai"])
    np.testing.assert_array_equal(aj, g["aj"])
    np.testing.assert_array_equal(aa, g["aa"])


@pytest.mark.gpu
def test_gpu_mult_of_loaded_operand(tmp_path, pkg):
    torch = pytest.importorskip("torch")
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    g = golden("poisson16")
    p = tmp_path / "p16.petsc"
    matio.save_petsc_binary(p, g["ai"], g["aj"], g["aa"], int(g["ncols"]))
    ai, aj, aa, n = matio.load_petsc_binary(p)
    dev = torch.device("cuda:0")
    with pkg.SeqAIJHIP(ai, aj, aa, ncols=n) as A:
        x = torch.from_numpy(np.ascontiguousarray(g["x"])).to(dev)
        y = torch.empty(len(ai) - 1, dtype=torch.float64, device=dev)
        A.mult(x, y)
        torch.cuda.synchronize()
        assert np.array_equal(y.cpu().numpy().view(np.uint64), np.ascontiguousarray(g["y"]).view(np.uint64))
