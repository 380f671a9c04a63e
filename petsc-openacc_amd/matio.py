"""Matrix and vector files for the SeqAIJ path: PETSc binary and MatrixMarket.

A PETSc user brings an operator as a PETSc binary file (what `MatView` with
a binary viewer writes and `MatLoad` reads — PETSc 3.7.6 MatView_SeqAIJ_Binary /
MatLoad_SeqAIJ_Binary [ext]) or as a MatrixMarket file (SuiteSparse's
Flan_1565, BASELINE configs[4], ships as `Flan_1565.mtx`). Both are read here
into the CSR arrays `SeqAIJHIP` takes: int32 `ai[m+1]`, `aj[nz]` (ascending
within a row), fp64 `aa[nz]`, i.e. PETSc's `Mat_SeqAIJ` `a->i / a->j / a->a`
with 32-bit PetscInt (no `--with-64-bit-indices` in
`/root/reference/scripts/petsc-release.sh:3-67`).

PETSc binary layout (big-endian throughout, 32-bit PetscInt, real double):
    Mat: int32 {MAT_FILE_CLASSID = 1211216, M, N, nz}, int32 row lengths[M],
         int32 columns[nz], float64 values[nz]
    Vec: int32 {VEC_FILE_CLASSID = 1211214, n}, float64 values[n]
Host-side file handling only; nothing here computes on the device.
"""
from __future__ import annotations

import numpy as np

MAT_FILE_CLASSID = 1211216
VEC_FILE_CLASSID = 1211214


def _csr_checked(ai, aj, aa, m, n):
    ai = np.ascontiguousarray(ai, dtype=np.int32)
    aj = np.ascontiguousarray(aj, dtype=np.int32)
    aa = np.ascontiguousarray(aa, dtype=np.float64)
    if len(ai) != m + 1 or ai[0] != 0 or ai[-1] != len(aj) or len(aj) != len(aa):
        raise ValueError("inconsistent CSR arrays")
    if m and np.any(np.diff(ai) < 0):
        raise ValueError("row offsets are not monotone")
    if len(aj) and (aj.min() < 0 or aj.max() >= n):
        raise ValueError("column index out of range")
    return ai, aj, aa


def save_petsc_binary(path, ai, aj, aa, ncols: int | None = None):
    """MatView(A, binary viewer) for a SeqAIJ matrix."""
    m = len(ai) - 1
    n = int(ncols) if ncols is not None else (int(np.max(aj)) + 1 if len(aj) else m)
    ai, aj, aa = _csr_checked(ai, aj, aa, m, n)
    with open(path, "wb") as f:
        np.array([MAT_FILE_CLASSID, m, n, len(aj)], dtype=">i4").tofile(f)
        np.diff(ai).astype(">i4").tofile(f)
        aj.astype(">i4").tofile(f)
        aa.astype(">f8").tofile(f)


def load_petsc_binary(path):
    """MatLoad(A, binary viewer) into CSR: returns (ai, aj, aa, ncols)."""
    with open(path, "rb") as f:
        head = np.fromfile(f, dtype=">i4", count=4)
        if len(head) != 4 or head[0] != MAT_FILE_CLASSID:
            raise ValueError(f"{path}: not a PETSc binary Mat (classid {head[0] if len(head) else None})")
        m, n, nz = (int(v) for v in head[1:])
        if m < 0 or n < 0 or nz < 0:
            raise ValueError(f"{path}: negative sizes in the header (64-bit PetscInt files are not supported)")
        rlen = np.fromfile(f, dtype=">i4", count=m)
        aj = np.fromfile(f, dtype=">i4", count=nz)
        aa = np.fromfile(f, dtype=">f8", count=nz)
    if len(rlen) != m or len(aj) != nz or len(aa) != nz:
        raise ValueError(f"{path}: truncated file")
    if int(rlen.sum(dtype=np.int64)) != nz:
        raise ValueError(f"{path}: row lengths do not add up to nz")
    ai = np.zeros(m + 1, dtype=np.int32)
    np.cumsum(rlen, out=ai[1:])
    ai, aj, aa = _csr_checked(ai, aj.astype(np.int32), aa.astype(np.float64), m, n)
    return ai, aj, aa, n


def save_petsc_vec(path, v):
    v = np.ascontiguousarray(v, dtype=np.float64)
    with open(path, "wb") as f:
        np.array([VEC_FILE_CLASSID, len(v)], dtype=">i4").tofile(f)
        v.astype(">f8").tofile(f)


def load_petsc_vec(path):
    with open(path, "rb") as f:
        head = np.fromfile(f, dtype=">i4", count=2)
        if len(head) != 2 or head[0] != VEC_FILE_CLASSID:
            raise ValueError(f"{path}: not a PETSc binary Vec")
        v = np.fromfile(f, dtype=">f8", count=int(head[1]))
    if len(v) != int(head[1]):
        raise ValueError(f"{path}: truncated file")
    return v.astype(np.float64)


def load_mtx(path):
    """MatrixMarket coordinate file (real / integer / pattern; general /
    symmetric / skew-symmetric, as SuiteSparse ships them) into CSR with the
    symmetric half expanded, columns ascending within each row and duplicate
    entries summed — the matrix PETSc holds after MatSetValues(ADD_VALUES)
    of every file entry and MatAssemblyEnd. Returns (ai, aj, aa, ncols)."""
    import scipy.io
    import scipy.sparse as sp

    A = scipy.io.mmread(str(path))
    if not sp.issparse(A):
        raise ValueError(f"{path}: array (dense) MatrixMarket files are not sparse operands")
    A = sp.csr_matrix(A, dtype=np.float64)
    A.sum_duplicates()  # canonical: sorted columns, one entry per (i, j)
    m, n = A.shape
    if A.nnz > np.iinfo(np.int32).max:
        raise ValueError(f"{path}: nnz exceeds the 32-bit PetscInt range")
    return _csr_checked(A.indptr, A.indices, A.data, m, n) + (n,)
