"""Device-resident CG (include/aijhip_ksp.h) — the KSP side of the path.

Mirrors the reference's solver set-up (/root/reference/src/main_ksp.cpp:92-103:
KSPCreate, KSPSetOperators, KSPSetType(KSPCG), KSPSetFromOptions, KSPSetUp,
KSPSolve, KSPGetConvergedReason / IterationNumber / ResidualNorm) over the
C ABI. Options follow /root/reference/configs/PETSc_SolverOptions_GAMG.info
(-ksp_atol 1e-12 -ksp_rtol 1e-14 -ksp_max_it 10000); the preconditioner is
Jacobi (the reference's smoother / coarse PC) until the GAMG hierarchy lands.
"""
from __future__ import annotations

import ctypes
import math
import importlib
import time

import numpy as np

_pkg = importlib.import_module("petsc-openacc_amd")

PC_TYPES = {"none": 0, "jacobi": 1, "gamg": 2, "bjacobi_gamg": 3}
NORM_TYPES = {"none": 0, "preconditioned": 1, "unpreconditioned": 2, "natural": 3}
REASONS = {2: "CONVERGED_RTOL", 3: "CONVERGED_ATOL", -3: "DIVERGED_ITS", -4: "DIVERGED_DTOL",
           -8: "DIVERGED_INDEFINITE_PC", -9: "DIVERGED_NANORINF", -10: "DIVERGED_INDEFINITE_MAT"}
KSP_SYMBOLS = (
    "aijhip_ksp_create", "aijhip_ksp_set_tolerances", "aijhip_ksp_set_pc_type", "aijhip_ksp_set_norm_type",
    "aijhip_ksp_set_initial_guess_nonzero", "aijhip_ksp_set_up", "aijhip_ksp_solve",
    "aijhip_ksp_get_iteration_number", "aijhip_ksp_get_residual_norm", "aijhip_ksp_get_converged_reason",
    "aijhip_ksp_get_residual_history", "aijhip_ksp_get_fused", "aijhip_ksp_destroy",
    "aijhip_ksp_set_gamg_params", "aijhip_ksp_get_pc_levels", "aijhip_ksp_get_pc_level",
    "aijhip_ksp_get_gamg_setup_path", "aijhip_ksp_get_host_syncs", "aijhip_ksp_get_iteration_bytes",
    "aijhip_ksp_solve_host",
)
_P = ctypes.c_void_p
_bound = False


def _lib():
    global _bound
    L = _pkg.lib()
    if not _bound:
        for n in KSP_SYMBOLS:
            getattr(L, n).restype = ctypes.c_int
        L.aijhip_ksp_create.argtypes = [_P, ctypes.POINTER(_P)]
        L.aijhip_ksp_set_tolerances.argtypes = [_P, ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_int32]
        L.aijhip_ksp_set_pc_type.argtypes = [_P, ctypes.c_int]
        L.aijhip_ksp_set_norm_type.argtypes = [_P, ctypes.c_int]
        L.aijhip_ksp_set_initial_guess_nonzero.argtypes = [_P, ctypes.c_int]
        L.aijhip_ksp_set_up.argtypes = [_P]
        L.aijhip_ksp_solve.argtypes = [_P, _P, _P, _P]
        L.aijhip_ksp_solve_host.argtypes = [_P, _P, _P]
        L.aijhip_ksp_get_iteration_number.argtypes = [_P, ctypes.POINTER(ctypes.c_int32)]
        L.aijhip_ksp_get_residual_norm.argtypes = [_P, ctypes.POINTER(ctypes.c_double)]
        L.aijhip_ksp_get_converged_reason.argtypes = [_P, ctypes.POINTER(ctypes.c_int)]
        L.aijhip_ksp_get_residual_history.argtypes = [_P, _P, ctypes.c_int32, ctypes.POINTER(ctypes.c_int32)]
        L.aijhip_ksp_get_fused.argtypes = [_P, ctypes.POINTER(ctypes.c_int)]
        L.aijhip_ksp_get_host_syncs.argtypes = [_P, ctypes.POINTER(ctypes.c_int32)]
        L.aijhip_ksp_get_iteration_bytes.argtypes = [_P, ctypes.POINTER(ctypes.c_int64),
                                                     ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)]
        L.aijhip_ksp_destroy.argtypes = [_P]
        L.aijhip_ksp_set_gamg_params.argtypes = [_P, _P]
        L.aijhip_ksp_get_pc_level.argtypes = [_P, ctypes.c_int32, ctypes.c_char, ctypes.POINTER(ctypes.c_int32),
                                              ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int64), _P, _P, _P]
        L.aijhip_ksp_get_pc_levels.argtypes = [_P, ctypes.POINTER(ctypes.c_int32), _P, _P, ctypes.c_int32,
                                               ctypes.POINTER(ctypes.c_double)]
        L.aijhip_ksp_get_gamg_setup_path.argtypes = [_P, ctypes.c_int32, _P, _P, ctypes.POINTER(ctypes.c_int32)]
        _bound = True
    return L


class KSPCG:
    """KSPCG on a SeqAIJHIP operator (device vectors)."""

    def __init__(self, A, rtol=1e-5, atol=1e-50, dtol=1e5, max_it=10000, pc="jacobi",
                 norm="preconditioned", guess_nonzero=False, gamg=None):
        L = _lib()
        self.A = A
        self._h = _P()
        _pkg._check(L.aijhip_ksp_create(A._h, ctypes.byref(self._h)))
        self.set_tolerances(rtol, atol, dtol, max_it)
        _pkg._check(L.aijhip_ksp_set_pc_type(self._h, PC_TYPES[pc]))
        if gamg:
            G = importlib.import_module("petsc-openacc_amd.gamg")
            self._gp = G.default_params(**gamg)
            _pkg._check(L.aijhip_ksp_set_gamg_params(self._h, ctypes.byref(self._gp)))
        _pkg._check(L.aijhip_ksp_set_norm_type(self._h, NORM_TYPES[norm]))
        _pkg._check(L.aijhip_ksp_set_initial_guess_nonzero(self._h, int(guess_nonzero)))

    def set_tolerances(self, rtol, atol, dtol, max_it):
        _pkg._check(_lib().aijhip_ksp_set_tolerances(self._h, rtol, atol, dtol, int(max_it)))

    def set_up(self):
        _pkg._check(_lib().aijhip_ksp_set_up(self._h))

    def solve(self, b, x, stream=None):
        _pkg._check(_lib().aijhip_ksp_solve(self._h, _pkg._dev_ptr(b, self.A.m, "b"),
                                            _pkg._dev_ptr(x, self.A.m, "x"), _pkg._stream_handle(stream)))

    def solve_host(self, b: np.ndarray, x: np.ndarray):
        """KSPSolve with host arrays (aijhip_ksp_solve_host): b up and x down
        once per solve, the solve itself on the device."""
        b = np.ascontiguousarray(b, dtype=np.float64)
        if x.dtype != np.float64 or not x.flags["C_CONTIGUOUS"] or len(x) < self.A.m or len(b) < self.A.m:
            raise TypeError("solve_host: contiguous float64 arrays of the operator's size")
        _pkg._check(_lib().aijhip_ksp_solve_host(self._h, b.ctypes.data, x.ctypes.data))

    @property
    def its(self) -> int:
        v = ctypes.c_int32()
        _pkg._check(_lib().aijhip_ksp_get_iteration_number(self._h, ctypes.byref(v)))
        return v.value

    @property
    def reason(self) -> int:
        v = ctypes.c_int()
        _pkg._check(_lib().aijhip_ksp_get_converged_reason(self._h, ctypes.byref(v)))
        return v.value

    @property
    def rnorm(self) -> float:
        v = ctypes.c_double()
        _pkg._check(_lib().aijhip_ksp_get_residual_norm(self._h, ctypes.byref(v)))
        return v.value

    @property
    def host_syncs(self) -> int:
        """Host synchronisations of the last solve (polls + the final read)."""
        v = ctypes.c_int32()
        _pkg._check(_lib().aijhip_ksp_get_host_syncs(self._h, ctypes.byref(v)))
        return v.value

    def iteration_bytes(self):
        """(total, SpMV part, finest-level part): compulsory HBM bytes of one
        CG iteration of the set-up solver (aijhip_ksp_get_iteration_bytes)."""
        t, sp, l0 = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        _pkg._check(_lib().aijhip_ksp_get_iteration_bytes(self._h, ctypes.byref(t), ctypes.byref(sp),
                                                          ctypes.byref(l0)))
        return t.value, sp.value, l0.value

    @property
    def fused(self) -> bool:
        v = ctypes.c_int()
        _pkg._check(_lib().aijhip_ksp_get_fused(self._h, ctypes.byref(v)))
        return bool(v.value)

    def pc_levels(self):
        """(rows per level, nnz per level, host set-up seconds) of the PC."""
        n = ctypes.c_int32()
        rows = np.zeros(32, np.int32)
        nnz = np.zeros(32, np.int64)
        secs = ctypes.c_double()
        _pkg._check(_lib().aijhip_ksp_get_pc_levels(self._h, ctypes.byref(n), rows.ctypes.data, nnz.ctypes.data,
                                                     32, ctypes.byref(secs)))
        return rows[: n.value].tolist(), nnz[: n.value].tolist(), secs.value

    def setup_path(self):
        """Per coarsening l -> l+1: ("device"|"host", widest product
        accumulator: 0 = wavefront form, 32/64/128/256 LDS columns, -1 host), and
        whether a device level overflowed to the host builder."""
        path = np.zeros(32, np.int32)
        cols = np.zeros(32, np.int32)
        fb = ctypes.c_int32()
        _pkg._check(_lib().aijhip_ksp_get_gamg_setup_path(self._h, 32, path.ctypes.data, cols.ctypes.data,
                                                           ctypes.byref(fb)))
        n = len(self.pc_levels()[0]) - 1
        return [("device" if path[l] else "host", int(cols[l])) for l in range(n)], bool(fb.value)

    def pc_level(self, l: int, which: str = "A"):
        """(ai, aj, aa, ncols) of GAMG level l's operator ('A') or
        interpolation to level l+1 ('P'), copied from the device."""
        m, n, nz = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int64()
        L = _lib()
        _pkg._check(L.aijhip_ksp_get_pc_level(self._h, l, which.encode(), ctypes.byref(m), ctypes.byref(n),
                                              ctypes.byref(nz), None, None, None))
        ai = np.empty(m.value + 1, np.int32)
        aj = np.empty(max(nz.value, 1), np.int32)
        aa = np.empty(max(nz.value, 1), np.float64)
        _pkg._check(L.aijhip_ksp_get_pc_level(self._h, l, which.encode(), None, None, None, ai.ctypes.data,
                                              aj.ctypes.data, aa.ctypes.data))
        return ai, aj[: nz.value], aa[: nz.value], n.value

    def history(self) -> np.ndarray:
        buf = np.empty(self.its + 1)
        n = ctypes.c_int32()
        _pkg._check(_lib().aijhip_ksp_get_residual_history(self._h, buf.ctypes.data, len(buf), ctypes.byref(n)))
        return buf[: n.value]

    def destroy(self):
        if getattr(self, "_h", None) and self._h.value:
            _lib().aijhip_ksp_destroy(self._h)
            self._h = _P()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.destroy()

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass


def bench_cg(pkg, A, nx, ny, nz, dev, iters=200):
    """CG iterations/s on the device at the benchmark operand: a fixed count
    of iterations (rtol = atol = 0, so every iteration runs), timed whole."""
    import torch
    rhs, _ = pkg.poisson_vectors(nx, ny, nz)
    b = torch.from_numpy(rhs).to(dev)
    x = torch.empty_like(b)
    with KSPCG(A, rtol=0.0, atol=0.0, max_it=iters) as ksp:
        ksp.set_up()
        ksp.solve(b, x)  # warm-up
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ksp.solve(b, x)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        its, fused = ksp.its, ksp.fused
        nb, nb_spmv, _ = ksp.iteration_bytes()
    return {"iters": its, "seconds": round(dt, 4), "iters_per_s": round(its / dt, 2),
            "ms_per_iter": round(dt / its * 1e3, 4), "pc": "jacobi", "fused_spmv_dot": fused,
            "bytes_per_iter": nb, "GBs": round(nb * its / dt / 1e9, 1),
            "roofline": {"bound": "hbm", "bytes_per_iter": nb, "spmv_bytes_per_iter": nb_spmv,
                         "achieved": round(nb * its / dt / 1e9, 1), "peak": 8000.0, "unit": "GB/s",
                         "frac": round(nb * its / dt / 1e9 / 8000.0, 4),
                         "note": "aijhip_ksp_get_iteration_bytes: the SpMV at its layout's bytes + the vector "
                                 "passes, per iteration, over the measured wall time of the iterations"}}


def bench_cg_gamg(pkg, A, nx, ny, nz, dev, rtol=1e-14, atol=1e-12, max_it=10000, gamg=None, light=False):
    """The reference's solver configuration (CG + GAMG to atol 1e-12 / rtol
    1e-14, configs/cg_gamg.info) solved to convergence on the benchmark
    operand from x = 0: KSPSetUp (host hierarchy + uploads) and KSPSolve
    timed separately, the solve once warm (a second solve on the same
    hierarchy, as a time-stepping caller would). gamg: the hierarchy's
    parameters (aijhip_gamg_params_t fields); light: skip the host-vector
    solve and the second set-up."""
    import torch
    rhs, exact = pkg.poisson_vectors(nx, ny, nz)
    b = torch.from_numpy(rhs).to(dev)
    x = torch.zeros_like(b)
    with KSPCG(A, rtol=rtol, atol=atol, max_it=max_it, pc="gamg", gamg=gamg) as ksp:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ksp.set_up()
        torch.cuda.synchronize()
        t_setup = time.perf_counter() - t0
        rows, nnz, t_host = ksp.pc_levels()
        t0 = time.perf_counter()
        ksp.solve(b, x)
        torch.cuda.synchronize()
        t_first = time.perf_counter() - t0
        x.zero_()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ksp.solve(b, x)
        torch.cuda.synchronize()
        t_solve = time.perf_counter() - t0
        its, reason, rnorm, syncs = ksp.its, ksp.reason, ksp.rnorm, ksp.host_syncs
        nb, nb_spmv, nb_l0 = ksp.iteration_bytes()
        # the same solve from HOST b / x (aijhip_ksp_solve_host: the PETSc KSP
        # type "cghip" for an unchanged caller with host Vecs)
        t_host_solve, host_same = None, None
        if not light:
            xh = np.zeros(A.m)
            t0 = time.perf_counter()
            ksp.solve_host(rhs, xh)
            t_host_solve = time.perf_counter() - t0
            host_same = bool(np.array_equal(xh.view(np.uint64), x.cpu().numpy().view(np.uint64)))
    err = float((x.cpu() - torch.from_numpy(exact)).abs().max())
    roof = {"bound": "hbm", "bytes_per_iter": nb, "spmv_bytes_per_iter": nb_spmv,
            "finest_level_bytes_per_iter": nb_l0,
            "achieved": round(nb * its / t_solve / 1e9, 1), "peak": 8000.0, "unit": "GB/s",
            "frac": round(nb * its / t_solve / 1e9 / 8000.0, 4),
            "note": "aijhip_ksp_get_iteration_bytes (every SpMV of the hierarchy at its layout's "
                    "bytes — A_l twice, P, P^T per level — plus CG's and the V-cycle's vector passes) "
                    "x iterations / the solve's wall time (polls and launch gaps included)"}
    # the same set-up again in this process (a caller that rebuilds the
    # hierarchy after new values): the first one above also pays one-time
    # costs (the set-up kernels' first launch, pinned staging)
    with KSPCG(A, rtol=rtol, atol=atol, max_it=max_it, pc="gamg", gamg=gamg) as ksp2:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ksp2.set_up()
        torch.cuda.synchronize()
        t_again = time.perf_counter() - t0
    if light:
        return {"its": its, "reason": reason, "max_err": err, "setup_s": round(t_setup, 3),
                "setup_again_s": round(t_again, 3), "solve_s": round(t_solve, 4),
                "time_to_solution_s": round(t_setup + t_solve, 3),
                "ms_per_iter": round(t_solve / max(its, 1) * 1e3, 4),
                "levels": [{"rows": r, "nnz": z} for r, z in zip(rows, nnz)], "roofline": roof}
    return {"its": its, "reason": reason, "rnorm": rnorm, "max_err": err,
            "setup_s": round(t_setup, 3), "setup_again_s": round(t_again, 3), "setup_pc_s": round(t_host, 3),
            "solve_s": round(t_solve, 4), "first_solve_s": round(t_first, 4),
            "solve_host_vectors": {"s": round(t_host_solve, 4), "bitwise_equal_device_solve": host_same,
                                   "note": "aijhip_ksp_solve_host: b up and x down once per solve (the KSP type "
                                           "cghip of the PETSc adapter for host Vecs), PCIe included"},
            "ms_per_iter": round(t_solve / max(its, 1) * 1e3, 4), "host_syncs": syncs,
            "time_to_solution_s": round(t_setup + t_solve, 3),
            "levels": [{"rows": r, "nnz": z} for r, z in zip(rows, nnz)],
            "roofline": roof,
            "options": "cg, gamg agg nsmooths 1 threshold 0, mg levels richardson(1)+jacobi, "
                       "coarse preonly+jacobi, rtol 1e-14 atol 1e-12"}


# ----------------------------------------------------------------------------
# Row-partitioned CG: one process per GPU, the operator an
# MPIAIJ row block (petsc-openacc_amd/mpiaij.py), every dot product a local
# fixed-order reduction on the device (include/aijhip_vec.h) combined across
# ranks by one all-reduce (RCCL over xGMI with the nccl backend) — PETSc's
# VecDot/VecNorm -> MPI_Allreduce. The iteration is KSPSolve_CG [ext] as in
# aijhip_ksp (and oracle/ksp_cg.py): the scalar decisions run on the host
# from the reduced values, which every rank holds identically, so all ranks
# take the same branch. PC: Jacobi (PETSc's bjacobi + jacobi sub-PC per rank)
# or none.

VEC_SYMBOLS = ("aijhip_vec_aypx", "aijhip_vec_dot", "aijhip_vec_cg_update", "aijhip_vec_jacobi",
               "aijhip_mat_jacobi_inverse", "aijhip_read_probe", "aijhip_delay_probe")

_vec_bound = False


def _veclib():
    global _vec_bound
    L = _pkg.lib()
    if not _vec_bound:
        for n in VEC_SYMBOLS:
            getattr(L, n).restype = ctypes.c_int
        i64, d = ctypes.c_int64, ctypes.c_double
        L.aijhip_vec_aypx.argtypes = [i64, d, _P, _P, _P]
        L.aijhip_vec_dot.argtypes = [i64, _P, _P, _P, _P]
        L.aijhip_vec_cg_update.argtypes = [i64, d, _P, _P, _P, _P, _P, _P, _P, _P]
        L.aijhip_vec_jacobi.argtypes = [i64, _P, _P, _P, _P, _P]
        L.aijhip_mat_jacobi_inverse.argtypes = [_P, _P, _P]
        L.aijhip_read_probe.argtypes = [_P, i64, ctypes.c_int, _P]
        L.aijhip_delay_probe.argtypes = [d, _P]
        _vec_bound = True
    return L


class DeviceVecOps:
    """The HIP vector kernels (aijhip_vec.h) on float64 GPU tensors; each
    reduction lands in a small device tensor ready for the all-reduce."""

    def __init__(self, device):
        import torch
        self.red = torch.zeros(3, dtype=torch.float64, device=device)

    @staticmethod
    def _s():
        import torch
        return torch.cuda.current_stream().cuda_stream

    def aypx(self, beta, x, y):
        _pkg._check(_veclib().aijhip_vec_aypx(x.numel(), beta, x.data_ptr(), y.data_ptr(), self._s()))

    def dot(self, x, y):
        _pkg._check(_veclib().aijhip_vec_dot(x.numel(), x.data_ptr(), y.data_ptr(), self.red.data_ptr(), self._s()))
        return self.red[:1]

    def cg_update(self, a, x, p, r, w, z, dinv):
        _pkg._check(_veclib().aijhip_vec_cg_update(x.numel(), a, x.data_ptr(), p.data_ptr(), r.data_ptr(),
                                                   w.data_ptr(), z.data_ptr(),
                                                   dinv.data_ptr() if dinv is not None else None,
                                                   self.red.data_ptr(), self._s()))
        return self.red

    def jacobi(self, r, dinv, z):
        _pkg._check(_veclib().aijhip_vec_jacobi(r.numel(), r.data_ptr(), dinv.data_ptr() if dinv is not None else None,
                                                z.data_ptr(), self.red.data_ptr(), self._s()))
        return self.red

    @staticmethod
    def jacobi_inverse(A_diag, dinv):
        _pkg._check(_veclib().aijhip_mat_jacobi_inverse(A_diag._h, dinv.data_ptr(), DeviceVecOps._s()))


class KSPCGMPI:
    """KSPSolve_CG over a row-partitioned operator. op: object with
    mult(x, y) on this rank's rows (MPIAIJ); dinv: this rank's Jacobi inverse
    (None = PCNONE); ops: vector backend (DeviceVecOps on the GPU)."""

    CONVERGED_RTOL, CONVERGED_ATOL = 2, 3
    DIVERGED_ITS, DIVERGED_DTOL, DIVERGED_INDEFINITE_PC, DIVERGED_NANORINF, DIVERGED_INDEFINITE_MAT = \
        -3, -4, -8, -9, -10

    def __init__(self, op, mloc, dinv=None, ops=None, rtol=1e-5, atol=1e-50, dtol=1e5, max_it=10000,
                 norm="preconditioned", group=None, device=None):
        import torch
        self.op, self.m, self.dinv = op, mloc, dinv
        self.ops = ops if ops is not None else DeviceVecOps(device)
        self.rtol, self.atol, self.dtol, self.max_it, self.norm = rtol, atol, dtol, max_it, norm
        self.group = group
        dev = device if device is not None else (dinv.device if dinv is not None else None)
        mk = lambda: torch.zeros(mloc, dtype=torch.float64, device=dev)  # noqa: E731
        self.r, self.z, self.p = mk(), mk(), mk()
        self.its, self.reason, self.rnorm, self.hist = 0, 0, 0.0, []

    def _allreduce(self, t):
        """Sum over ranks (in place) and return the values on the host."""
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized() and dist.get_world_size(self.group) > 1:
            dist.all_reduce(t, group=self.group)
        return [float(v) for v in t.tolist()]

    def _norm(self, zz, zr, rr):
        if self.norm == "preconditioned":
            return math.sqrt(zz)
        if self.norm == "unpreconditioned":
            return math.sqrt(rr)
        return math.sqrt(abs(zr))

    def _test(self, rn):
        if math.isnan(rn) or math.isinf(rn):
            return self.DIVERGED_NANORINF
        if rn <= self.ttol:
            return self.CONVERGED_ATOL if rn < self.atol else self.CONVERGED_RTOL
        if rn >= self.dtol * self.rnorm0:
            return self.DIVERGED_DTOL
        return 0

    def solve(self, b, x):
        """Zero initial guess (main_ksp.cpp: VecSet(lhs, 0))."""
        ops, r, z, p = self.ops, self.r, self.z, self.p
        x.zero_()
        r.copy_(b)
        zz, zr, rr = self._allreduce(ops.jacobi(r, self.dinv, z))
        dp = self._norm(zz, zr, rr)
        self.hist = [dp]
        self.rnorm0 = dp
        self.ttol = max(self.rtol * dp, self.atol)
        self.reason = self._test(dp)
        self.its, self.rnorm = 0, dp
        if self.reason:
            return self.reason
        beta, betaold, dpi = zr, 0.0, 0.0
        i = 0
        while i < self.max_it:
            self.its = i + 1
            if beta == 0.0:
                self.reason = self.CONVERGED_ATOL
                return self.reason
            if i > 0 and beta * betaold < 0.0:
                self.reason = self.DIVERGED_INDEFINITE_PC
                return self.reason
            if i == 0:
                p.copy_(z)
            else:
                ops.aypx(beta / betaold, z, p)
            self.op.mult(p, z)  # W = A P (W shares Z's storage)
            dpiold, dpi = dpi, self._allreduce(ops.dot(p, z))[0]
            betaold = beta
            if dpi == 0.0 or (i > 0 and dpi * dpiold <= 0.0):
                self.reason = self.DIVERGED_INDEFINITE_MAT
                return self.reason
            a = beta / dpi
            zz, zr, rr = self._allreduce(ops.cg_update(a, x, p, r, z, z, self.dinv))
            dp = self._norm(zz, zr, rr)
            self.hist.append(dp)
            self.rnorm = dp
            self.reason = self._test(dp)
            if self.reason:
                return self.reason
            beta = zr
            i += 1
        self.reason = self.DIVERGED_ITS
        return self.reason
