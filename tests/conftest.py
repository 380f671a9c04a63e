"""Shared test plumbing.

`-m "not gpu"`: oracle vs golden fixtures, host logic, C-ABI load/export
checks and gloo multi-process tests — run here, no GPU.
`-m gpu`: parity of the HIP path (through the C ABI) against the oracle on a
real MI355X. There is no CPU fallback: GPU tests fail if the device or the
extension is missing.
"""
from __future__ import annotations

import ctypes
import importlib
import os
import sys
from pathlib import Path

# the library's side / exchange streams each need a hardware queue of their
# own (bench.py, profiles/r05/e/): set before HIP initialises
if int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0) < 8:
    os.environ["GPU_MAX_HW_QUEUES"] = "8"

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent
GOLDEN = ROOT / "tests" / "golden"
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run on the GPU box)")


def load_pkg():
    """The product package (its directory name has a hyphen)."""
    return importlib.import_module("petsc-openacc_amd")


@pytest.fixture(scope="session")
def pkg():
    build = importlib.import_module("petsc-openacc_amd.build")
    build.build_all()
    return load_pkg()


@pytest.fixture(scope="session")
def coracle():
    """The C restatement (oracle/liboracle.so) — checker only."""
    build = importlib.import_module("petsc-openacc_amd.build")
    path = build.build_oracle()
    L = ctypes.CDLL(str(path))
    P = ctypes.c_void_p
    L.oracle_matmult_seqaij.argtypes = [ctypes.c_int32, P, P, P, P, P]
    L.oracle_matmult_seqaij_omp.argtypes = [ctypes.c_int32, P, P, P, P, P]
    L.oracle_matmultadd_seqaij.argtypes = [ctypes.c_int32, P, P, P, P, P, P]
    L.oracle_matmulttranspose_seqaij.argtypes = [ctypes.c_int32, ctypes.c_int32, P, P, P, P, P]
    L.oracle_matmult_seqaij.restype = None
    L.oracle_matmult_seqaij_omp.restype = None
    L.oracle_matmultadd_seqaij.restype = None
    L.oracle_matmulttranspose_seqaij.restype = None
    return COracle(L)


class COracle:
    def __init__(self, L):
        self.L = L

    @staticmethod
    def _c(a, dt):
        a = np.ascontiguousarray(a, dtype=dt)
        return a, a.ctypes.data

    def matmult(self, ai, aj, aa, x, omp=False):
        ai, pai = self._c(ai, np.int32); aj, paj = self._c(aj, np.int32)
        aa, paa = self._c(aa, np.float64); x, px = self._c(x, np.float64)
        y = np.empty(len(ai) - 1)
        f = self.L.oracle_matmult_seqaij_omp if omp else self.L.oracle_matmult_seqaij
        f(len(ai) - 1, pai, paj, paa, px, y.ctypes.data)
        return y

    def matmult_add(self, ai, aj, aa, x, z):
        ai, pai = self._c(ai, np.int32); aj, paj = self._c(aj, np.int32)
        aa, paa = self._c(aa, np.float64); x, px = self._c(x, np.float64); z, pz = self._c(z, np.float64)
        w = np.empty(len(ai) - 1)
        self.L.oracle_matmultadd_seqaij(len(ai) - 1, pai, paj, paa, px, pz, w.ctypes.data)
        return w

    def matmult_transpose(self, ai, aj, aa, x, ncols):
        ai, pai = self._c(ai, np.int32); aj, paj = self._c(aj, np.int32)
        aa, paa = self._c(aa, np.float64); x, px = self._c(x, np.float64)
        y = np.empty(ncols)
        self.L.oracle_matmulttranspose_seqaij(len(ai) - 1, ncols, pai, paj, paa, px, y.ctypes.data)
        return y


GOLDEN_NAMES = ("poisson4", "poisson8", "poisson16", "skewed_small", "compressed_small")


def golden(name):
    d = np.load(GOLDEN / f"{name}.npz", allow_pickle=False)
    return {k: d[k] for k in d.files}


def spmv_tolerance(ai, aj, aa, x, seed=None):
    """Componentwise bound of SURVEY.md §8d for a reordered fp64 row sum:
    |dy_i| <= 2 * gamma(n_i) * (|A||x|)_i (+ |z_i| term for mult_add),
    gamma(n) = n u / (1 - n u), u = 2^-53. Plus a tiny absolute floor for
    rows whose |A||x| underflows."""
    u = 2.0 ** -53
    ai = np.asarray(ai, dtype=np.int64)
    lens = np.diff(ai).astype(np.float64) + 1.0
    rows = np.repeat(np.arange(len(ai) - 1), np.diff(ai))
    absax = np.zeros(len(ai) - 1)
    np.add.at(absax, rows, np.abs(aa) * np.abs(np.asarray(x)[aj]))
    gamma = lens * u / (1 - lens * u)
    return 2.0 * gamma * absax + 1e-300, absax
