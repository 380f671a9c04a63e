"""ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes binding of oracle/cg_gamg.c (the host CG + GAMG solve on all host
cores) for bench.py's cpu_baseline leg and tests/. The hierarchy comes from
the library's host builder (petsc-openacc_amd/gamg.py build_host), so the
host and device solves precondition with the same levels.
"""
from __future__ import annotations

import ctypes
import importlib
import time

import numpy as np

_P = ctypes.c_void_p


class Level(ctypes.Structure):
    _fields_ = [("m", ctypes.c_int32), ("ai", _P), ("aj", _P), ("aa", _P), ("pi", _P), ("pj", _P), ("pa", _P)]


def _lib():
    build = importlib.import_module("petsc-openacc_amd.build")
    L = ctypes.CDLL(str(build.build_oracle()))
    L.oracle_cg_gamg.restype = ctypes.c_int
    L.oracle_cg_gamg.argtypes = [ctypes.c_int, _P, _P, _P, ctypes.c_double, ctypes.c_double, ctypes.c_int32,
                                 ctypes.c_int, ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_double), _P,
                                 ctypes.POINTER(ctypes.c_double)]
    L.oracle_omp_threads.restype = ctypes.c_int
    return L


def solve(ai, aj, aa, b, rtol=1e-14, atol=1e-12, max_it=10000, threads=0, levels=None, build_threads=None):
    """Host CG + GAMG from x = 0. Returns dict(x, its, reason, rnorm, hist,
    setup_s (hierarchy + P^T/Jacobi), solve_s, threads)."""
    G = importlib.import_module("petsc-openacc_amd.gamg")
    L = _lib()
    ai = np.ascontiguousarray(ai, np.int32)
    aj = np.ascontiguousarray(aj, np.int32)
    aa = np.ascontiguousarray(aa, np.float64)
    t0 = time.perf_counter()
    if levels is None:
        bt = threads if build_threads is None else build_threads
        levels = G.build_host(ai, aj, aa, **({"threads": bt} if bt else {}))
    t_build = time.perf_counter() - t0
    keep = []
    arr = (Level * len(levels))()
    for l, d in enumerate(levels):
        a = (ai, aj, aa) if l == 0 else d["A"]
        arr[l].m = d["m"]
        arr[l].ai, arr[l].aj, arr[l].aa = (x.ctypes.data for x in a)
        keep.append(a)
        if "P" in d:
            arr[l].pi, arr[l].pj, arr[l].pa = (x.ctypes.data for x in d["P"])
            keep.append(d["P"])
    b = np.ascontiguousarray(b, np.float64)
    x = np.empty_like(b)
    hist = np.empty(max_it + 2)
    its, rnorm, su = ctypes.c_int32(), ctypes.c_double(), ctypes.c_double()
    t0 = time.perf_counter()
    reason = L.oracle_cg_gamg(len(levels), ctypes.addressof(arr), b.ctypes.data, x.ctypes.data, rtol, atol,
                              int(max_it), int(threads), ctypes.byref(its), ctypes.byref(rnorm), hist.ctypes.data,
                              ctypes.byref(su))
    t_all = time.perf_counter() - t0
    used = threads if threads > 0 else L.oracle_omp_threads()
    return {"x": x, "its": its.value, "reason": reason, "rnorm": rnorm.value, "hist": hist[: its.value + 1],
            "setup_s": t_build + su.value, "solve_s": t_all - su.value, "threads": used,
            "levels": [d["m"] for d in levels]}
