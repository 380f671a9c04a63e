"""Generate the committed SpMV fixtures in tests/golden/ from the oracle.

    python tests/golden/make_golden.py

The reference ships no golden vectors for MatMult_SeqAIJ
and PETSc is not in the image, so these fixtures come from the numpy
restatement oracle/seqaij.py (cross-checked bit for bit against the C
restatement oracle/matmult_seqaij.c by tests/test_oracle.py). They pin the
oracle and the GPU path against regressions; they are NOT outputs of a
reference run ("parity unpinned").

Each .npz holds: ai, aj, aa, ncols, x, y = A x, z, w = z + A x, xt, yt = A^T xt.
"""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent.parent))

from oracle import seqaij  # noqa: E402


def _save(name, ai, aj, aa, ncols, x, z, xt, **extra):
    y = seqaij.matmult(ai, aj, aa, x)
    w = seqaij.matmult_add(ai, aj, aa, x, z)
    yt = seqaij.matmult_transpose(ai, aj, aa, xt, ncols)
    np.savez_compressed(HERE / f"{name}.npz", ai=ai.astype(np.int32), aj=aj.astype(np.int32),
                        aa=aa.astype(np.float64), ncols=np.int64(ncols), x=x, y=y, z=z, w=w,
                        xt=xt, yt=yt, **extra)
    print(f"{name}: m={len(ai) - 1} n={ncols} nnz={len(aj)}")


def skewed_small(m=2000, n=2500, seed=11):
    """Ragged CSR: empty rows, 1-entry rows, typical rows and three rows
    longer than the 2048-entry STREAM block (one > 16384, split into segments)."""
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, 40, size=m)
    lens[rng.random(m) < 0.1] = 0
    lens[5] = 1
    lens[100] = 3000
    lens[1000] = 2049
    lens[1999] = 17000
    lens = np.minimum(lens, n)
    ai = np.zeros(m + 1, np.int64)
    np.cumsum(lens, out=ai[1:])
    aj = np.concatenate([np.sort(rng.choice(n, size=L, replace=False)) for L in lens]).astype(np.int32)
    aa = rng.standard_normal(len(aj))
    return ai.astype(np.int32), aj, aa, n


def compressed_small(m=3000, n=3000, seed=12):
    """>60% empty rows: exercises PETSc's compressed-row form."""
    rng = np.random.default_rng(seed)
    lens = np.where(rng.random(m) < 0.75, 0, rng.integers(1, 12, size=m))
    ai = np.zeros(m + 1, np.int64)
    np.cumsum(lens, out=ai[1:])
    aj = np.concatenate([np.sort(rng.choice(n, size=L, replace=False)) for L in lens]).astype(np.int32)
    aa = rng.standard_normal(len(aj))
    return ai.astype(np.int32), aj, aa, n


def main():
    for N in (4, 8, 16):
        ai, aj, aa, rhs, exact = seqaij.create_system(N, N, N)
        m = N ** 3
        z = seqaij.splitmix_uniform(m, seed=7)
        _save(f"poisson{N}", ai, aj, aa, m, exact, z, seqaij.splitmix_uniform(m, seed=42),
              rhs=rhs, exact=exact, x_uniform=seqaij.splitmix_uniform(m, seed=42))
    ai, aj, aa, n = skewed_small()
    _save("skewed_small", ai, aj, aa, n, seqaij.splitmix_uniform(n, seed=1), seqaij.splitmix_uniform(len(ai) - 1, seed=2),
          seqaij.splitmix_uniform(len(ai) - 1, seed=3))
    ai, aj, aa, n = compressed_small()
    _save("compressed_small", ai, aj, aa, n, seqaij.splitmix_uniform(n, seed=4),
          seqaij.splitmix_uniform(len(ai) - 1, seed=5), seqaij.splitmix_uniform(len(ai) - 1, seed=6))


if __name__ == "__main__":
    main()
