"""Host-side smoothed-aggregation hierarchy (include/aijhip_gamg.h), exposed
for inspection and testing; the KSP builds it itself for AIJHIP_PC_GAMG."""
from __future__ import annotations

import ctypes
import importlib

import numpy as np

_pkg = importlib.import_module("petsc-openacc_amd")

GAMG_SYMBOLS = (
    "aijhip_gamg_params_default", "aijhip_gamg_build_host", "aijhip_gamg_host_num_levels",
    "aijhip_gamg_host_level_info", "aijhip_gamg_host_get_A", "aijhip_gamg_host_get_P",
    "aijhip_gamg_host_get_aggregates", "aijhip_gamg_host_view", "aijhip_gamg_host_destroy",
)


class GamgParams(ctypes.Structure):
    _fields_ = [("threshold", ctypes.c_double), ("coarse_eq_limit", ctypes.c_int32),
                ("max_levels", ctypes.c_int32), ("nsmooths", ctypes.c_int32),
                ("smooth_scale", ctypes.c_double), ("eig_its", ctypes.c_int32), ("threads", ctypes.c_int32),
                ("device_min_rows", ctypes.c_int32), ("coarsen", ctypes.c_int32), ("square_graph", ctypes.c_int32),
                ("eig_ksp", ctypes.c_int32), ("pad0", ctypes.c_int32)]


_P = ctypes.c_void_p
_bound = False


def _lib():
    global _bound
    L = _pkg.lib()
    if not _bound:
        for n in GAMG_SYMBOLS:
            getattr(L, n).restype = ctypes.c_int
        L.aijhip_gamg_params_default.argtypes = [ctypes.POINTER(GamgParams)]
        L.aijhip_gamg_build_host.argtypes = [ctypes.c_int32, _P, _P, _P, ctypes.POINTER(GamgParams), ctypes.POINTER(_P)]
        L.aijhip_gamg_host_num_levels.argtypes = [_P, ctypes.POINTER(ctypes.c_int32)]
        L.aijhip_gamg_host_level_info.argtypes = [_P, ctypes.c_int32, ctypes.POINTER(ctypes.c_int32),
                                                  ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64),
                                                  ctypes.POINTER(ctypes.c_double)]
        L.aijhip_gamg_host_get_A.argtypes = [_P, ctypes.c_int32, _P, _P, _P]
        L.aijhip_gamg_host_get_P.argtypes = [_P, ctypes.c_int32, _P, _P, _P]
        L.aijhip_gamg_host_get_aggregates.argtypes = [_P, ctypes.c_int32, _P]
        L.aijhip_gamg_host_destroy.argtypes = [_P]
        _bound = True
    return L


def default_params(**over) -> GamgParams:
    p = GamgParams()
    _lib().aijhip_gamg_params_default(ctypes.byref(p))
    for k, v in over.items():
        setattr(p, k, v)
    return p


def build_host(ai, aj, aa, **params):
    """Returns [dict(m, A=(ai,aj,aa) for l>=1, P=(ai,aj,aa), agg, emax)] per level."""
    L = _lib()
    ai = np.ascontiguousarray(ai, dtype=np.int32)
    aj = np.ascontiguousarray(aj, dtype=np.int32)
    aa = np.ascontiguousarray(aa, dtype=np.float64)
    h = _P()
    p = default_params(**params)
    rc = L.aijhip_gamg_build_host(len(ai) - 1, ai.ctypes.data, aj.ctypes.data, aa.ctypes.data, ctypes.byref(p),
                                  ctypes.byref(h))
    if rc:
        raise _pkg.AIJHIPError(rc, "aijhip_gamg_build_host failed")
    try:
        n = ctypes.c_int32()
        L.aijhip_gamg_host_num_levels(h, ctypes.byref(n))
        out = []
        for lvl in range(n.value):
            m, na, npp, em = ctypes.c_int32(), ctypes.c_int64(), ctypes.c_int64(), ctypes.c_double()
            L.aijhip_gamg_host_level_info(h, lvl, ctypes.byref(m), ctypes.byref(na), ctypes.byref(npp), ctypes.byref(em))
            d = {"m": m.value, "nnz_a": na.value, "emax": em.value}
            if lvl >= 1:
                a = (np.empty(m.value + 1, np.int32), np.empty(na.value, np.int32), np.empty(na.value))
                L.aijhip_gamg_host_get_A(h, lvl, *[x.ctypes.data for x in a])
                d["A"] = a
            if lvl < n.value - 1:
                pr = (np.empty(m.value + 1, np.int32), np.empty(npp.value, np.int32), np.empty(npp.value))
                L.aijhip_gamg_host_get_P(h, lvl, *[x.ctypes.data for x in pr])
                d["P"] = pr
                agg = np.empty(m.value, np.int32)
                L.aijhip_gamg_host_get_aggregates(h, lvl, agg.ctypes.data)
                d["agg"] = agg
            out.append(d)
        return out
    finally:
        L.aijhip_gamg_host_destroy(h)
