"""Communicators, MatMult_MPIAIJ and the distributed KSPCG over the C ABI
(include/aijhip_mpi.h) — one process per GPU.

The reference runs PETSc's MPIAIJ + KSPSolve_CG on 1-16 MPI ranks
(/root/reference/runs/single-node-scaling.pbs:56-67): MatMult_MPIAIJ [ext]
overlaps the VecScatter of ghost x entries with the diagonal-block
MatMult_SeqAIJ, and every dot is an MPI_Allreduce. Here both live in the
library: the ghost exchange is RCCL send/recv (or all-gather) on a second HIP
stream and the dots are RCCL all-reduces of device doubles, so a CG iteration
makes no host round trip (aijhip_kspmpi_get_host_syncs counts the polls).

Two transports:
  Comm.rccl(group)  RCCL over xGMI; the ncclUniqueId travels over the
                    torch.distributed group (one broadcast at creation).
  Comm.host(group)  the caller's host transport — here torch.distributed
                    over gloo on CPU tensors, used where RCCL cannot run
                    (several ranks sharing one GPU in the tests: RCCL refuses
                    duplicate devices).
"""
from __future__ import annotations

import ctypes
import importlib

import numpy as np

_pkg = importlib.import_module("petsc-openacc_amd")
_P = ctypes.c_void_p
_i32, _i64, _d = ctypes.c_int32, ctypes.c_int64, ctypes.c_double
_DP = ctypes.POINTER(ctypes.c_double)

COMM_RCCL, COMM_HOST = 1, 2
HALO = {"p2p": 0, "allgather": 1}
AIJHIP_ERR_COMM = 6

ALLREDUCE_FN = ctypes.CFUNCTYPE(ctypes.c_int, _P, _DP, _i32)
EXCHANGE_FN = ctypes.CFUNCTYPE(ctypes.c_int, _P, _P, _DP, _i64, _DP, _i64)
_I32P, _I64P = ctypes.POINTER(_i32), ctypes.POINTER(_i64)
SENDRECV_FN = ctypes.CFUNCTYPE(ctypes.c_int, _P, _i32, _I32P, _I64P, _DP, _i32, _I32P, _I64P, _DP)

MPI_SYMBOLS = (
    "aijhip_comm_rccl_unique_id", "aijhip_comm_create_rccl", "aijhip_comm_create_host", "aijhip_comm_info",
    "aijhip_comm_allreduce_sum", "aijhip_comm_set_timeout", "aijhip_comm_destroy",
    "aijhip_mpiaij_create", "aijhip_mpiaij_mult", "aijhip_mpiaij_get_ghost", "aijhip_mpiaij_destroy",
    "aijhip_kspmpi_create", "aijhip_kspmpi_set_tolerances", "aijhip_kspmpi_set_pc_type",
    "aijhip_kspmpi_set_gamg_params",
    "aijhip_kspmpi_set_norm_type", "aijhip_kspmpi_set_poll_interval", "aijhip_kspmpi_solve",
    "aijhip_kspmpi_get_iteration_number", "aijhip_kspmpi_get_residual_norm", "aijhip_kspmpi_get_converged_reason",
    "aijhip_kspmpi_get_residual_history", "aijhip_kspmpi_get_host_syncs", "aijhip_kspmpi_destroy",
    "aijhip_comm_set_host_sendrecv", "aijhip_kspmpi_get_pc_levels", "aijhip_kspmpi_get_setup_seconds",
    "aijhip_kspmpi_get_pc_level", "aijhip_mpiaij_set_overlap", "aijhip_mpiaij_get_overlap",
    "aijhip_kspmpi_set_graph", "aijhip_kspmpi_get_graph_batches",
)
_bound = False


def _lib():
    global _bound
    L = _pkg.lib()
    if not _bound:
        for n in MPI_SYMBOLS:
            getattr(L, n).restype = ctypes.c_int
        L.aijhip_comm_rccl_unique_id.argtypes = [_P]
        L.aijhip_comm_create_rccl.argtypes = [_P, _i32, _i32, _i32, ctypes.POINTER(_P)]
        L.aijhip_comm_create_host.argtypes = [_i32, _i32, _i32, ALLREDUCE_FN, EXCHANGE_FN, _P, ctypes.POINTER(_P)]
        L.aijhip_comm_info.argtypes = [_P] + [ctypes.POINTER(_i32)] * 4
        L.aijhip_comm_allreduce_sum.argtypes = [_P, _P, _i32, _P]
        L.aijhip_comm_set_timeout.argtypes = [_P, _d]
        L.aijhip_comm_destroy.argtypes = [_P]
        L.aijhip_mpiaij_create.argtypes = [_P, _P, _P, _i32, _i32, _P, _P, _P, _i32, _P, _P, _i32, ctypes.POINTER(_P)]
        L.aijhip_mpiaij_mult.argtypes = [_P, _P, _P, _P]
        L.aijhip_mpiaij_set_overlap.argtypes = [_P, ctypes.c_int]
        L.aijhip_mpiaij_get_overlap.argtypes = [_P, ctypes.POINTER(_i32), ctypes.POINTER(_i32)]
        L.aijhip_mpiaij_get_ghost.argtypes = [_P, ctypes.POINTER(_P), ctypes.POINTER(_i64)]
        L.aijhip_mpiaij_destroy.argtypes = [_P]
        L.aijhip_kspmpi_create.argtypes = [_P, ctypes.POINTER(_P)]
        L.aijhip_kspmpi_set_tolerances.argtypes = [_P, _d, _d, _d, _i32]
        L.aijhip_kspmpi_set_pc_type.argtypes = [_P, ctypes.c_int]
        L.aijhip_kspmpi_set_gamg_params.argtypes = [_P, _P]
        L.aijhip_kspmpi_set_norm_type.argtypes = [_P, ctypes.c_int]
        L.aijhip_kspmpi_set_poll_interval.argtypes = [_P, _i32]
        L.aijhip_kspmpi_set_graph.argtypes = [_P, ctypes.c_int]
        L.aijhip_kspmpi_get_graph_batches.argtypes = [_P, ctypes.POINTER(_i32)]
        L.aijhip_kspmpi_solve.argtypes = [_P, _P, _P, _P]
        L.aijhip_kspmpi_get_iteration_number.argtypes = [_P, ctypes.POINTER(_i32)]
        L.aijhip_kspmpi_get_residual_norm.argtypes = [_P, ctypes.POINTER(_d)]
        L.aijhip_kspmpi_get_converged_reason.argtypes = [_P, ctypes.POINTER(ctypes.c_int)]
        L.aijhip_kspmpi_get_residual_history.argtypes = [_P, _P, _i32, ctypes.POINTER(_i32)]
        L.aijhip_kspmpi_get_host_syncs.argtypes = [_P, ctypes.POINTER(_i32)]
        L.aijhip_kspmpi_destroy.argtypes = [_P]
        L.aijhip_comm_set_host_sendrecv.argtypes = [_P, SENDRECV_FN]
        L.aijhip_kspmpi_get_pc_levels.argtypes = [_P, ctypes.POINTER(_i32), _P, _P, _i32]
        L.aijhip_kspmpi_get_setup_seconds.argtypes = [_P, ctypes.POINTER(_d)]
        L.aijhip_kspmpi_get_pc_level.argtypes = [_P, _i32, ctypes.c_char, ctypes.POINTER(_i64), ctypes.POINTER(_i32),
                                                 ctypes.POINTER(_i64), _P, _P, _P]
        _bound = True
    return L


class Comm:
    """An aijhip_comm_t bound to one device (this rank's GPU)."""

    def __init__(self, handle, kind, rank, world, device, keep=()):
        self._h, self.kind, self.rank, self.world, self.device = handle, kind, rank, world, device
        self._keep = keep  # ctypes callbacks and the plan they read

    @classmethod
    def rccl(cls, group=None, device: int | None = None, timeout_s: float = 300.0):
        import torch
        import torch.distributed as dist
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        device = torch.cuda.current_device() if device is None else device
        L = _lib()
        box = [None]
        if rank == 0:
            uid = ctypes.create_string_buffer(128)
            _pkg._check(L.aijhip_comm_rccl_unique_id(uid))
            box[0] = bytes(uid.raw)
        dist.broadcast_object_list(box, src=dist.get_global_rank(group, 0) if group is not None else 0,
                                   group=group)
        uid = ctypes.create_string_buffer(box[0], 128)
        h = _P()
        _pkg._check(L.aijhip_comm_create_rccl(uid, world, rank, device, ctypes.byref(h)))
        c = cls(h, COMM_RCCL, rank, world, device)
        c.set_timeout(timeout_s)
        return c

    @classmethod
    def host(cls, group=None, device: int = 0, timeout_s: float = 300.0):
        """torch.distributed (gloo) on host buffers. Each operator registers
        its exchange pattern (NativeMPIAIJ), looked up by its handle."""
        import torch
        import torch.distributed as dist
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        state = {"plans": {}}

        def allreduce(_ctx, buf, n):
            try:
                t = torch.from_numpy(np.ctypeslib.as_array(buf, shape=(n,)))
                dist.all_reduce(t, group=group)
                return 0
            except Exception:  # noqa: BLE001 — reported to the library as a failed collective
                return 1

        def exchange(_ctx, op, send, nsend, recv, nrecv):
            try:
                s = np.ctypeslib.as_array(send, shape=(nsend,)) if nsend > 0 else np.zeros(0)
                r = np.ctypeslib.as_array(recv, shape=(nrecv,)) if nrecv > 0 else np.zeros(0)
                plan = state["plans"][op]
                if plan["halo"] == "allgather":
                    g = plan["gather_len"]
                    outs = [torch.from_numpy(r[q * g:(q + 1) * g]) for q in range(world)]
                    dist.all_gather(outs, torch.from_numpy(s[:g].copy()), group=group)
                    return 0
                works, bufs, own = [], [], None
                for q, a, b in plan["send"]:
                    if q == rank:  # a segment for this rank itself: a local copy
                        own = s[a:b].copy()
                        continue
                    bufs.append(torch.from_numpy(s[a:b].copy()))
                    works.append(dist.isend(bufs[-1], q, group=group))
                for p, a, b in plan["recv"]:
                    if p == rank:
                        r[a:b] = own
                        continue
                    works.append(dist.irecv(torch.from_numpy(r[a:b]), p, group=group))
                for w in works:
                    w.wait()
                return 0
            except Exception:  # noqa: BLE001
                return 1

        def sendrecv(_ctx, ns, speer, soff, send, nr, rpeer, roff, recv):
            """The library's own point-to-point plans (the distributed GAMG's
            set-up messages and the halos of the operators it makes)."""
            try:
                works, outs = [], []
                sall = np.ctypeslib.as_array(send, shape=(max(int(soff[ns]), 1),)) if ns else None
                for i in range(ns):
                    buf = torch.from_numpy(sall[int(soff[i]):int(soff[i + 1])].copy())
                    outs.append(buf)
                    works.append(dist.isend(buf, int(speer[i]), group=group))
                rall = np.ctypeslib.as_array(recv, shape=(max(int(roff[nr]), 1),)) if nr else None
                ins = []
                for i in range(nr):
                    buf = torch.empty(int(roff[i + 1]) - int(roff[i]), dtype=torch.float64)
                    ins.append((int(roff[i]), buf))
                    works.append(dist.irecv(buf, int(rpeer[i]), group=group))
                for w in works:
                    w.wait()
                for a, buf in ins:
                    rall[a:a + buf.numel()] = buf.numpy()
                return 0
            except Exception:  # noqa: BLE001
                return 1

        cb = (ALLREDUCE_FN(allreduce), EXCHANGE_FN(exchange), SENDRECV_FN(sendrecv))
        h = _P()
        _pkg._check(_lib().aijhip_comm_create_host(world, rank, device, cb[0], cb[1], None, ctypes.byref(h)))
        _pkg._check(_lib().aijhip_comm_set_host_sendrecv(h, cb[2]))
        c = cls(h, COMM_HOST, rank, world, device, keep=(cb, state))
        c.set_timeout(timeout_s)
        return c

    def set_timeout(self, seconds: float):
        _pkg._check(_lib().aijhip_comm_set_timeout(self._h, float(seconds)))

    def info(self) -> dict:
        v = [_i32() for _ in range(4)]
        _pkg._check(_lib().aijhip_comm_info(self._h, *[ctypes.byref(x) for x in v]))
        return {"nranks": v[0].value, "rank": v[1].value,
                "kind": {COMM_RCCL: "rccl", COMM_HOST: "host"}.get(v[2].value, v[2].value),
                "version": v[3].value}

    def allreduce_sum(self, t, stream=None):
        """In-place sum of a float64 GPU tensor over all ranks (stream-ordered)."""
        _pkg._check(_lib().aijhip_comm_allreduce_sum(self._h, _pkg._dev_ptr(t, t.numel(), "buf"), t.numel(),
                                                     _pkg._stream_handle(stream)))

    def destroy(self):
        if getattr(self, "_h", None) and self._h.value:
            _lib().aijhip_comm_destroy(self._h)
            self._h = _P()

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass


class NativeMPIAIJ:
    """aijhip_mpiaij_t over this rank's SeqAIJHIP blocks and exchange plan."""

    def __init__(self, comm: Comm, A_d, A_o, halo: str, send, recv, gather_len: int = 0):
        """send: [(peer, rows)] in peer order (all-gather: [(-1, rows)]);
        recv: [(peer, start, stop)] covering the ghost vector in order."""
        self.comm, self.A_d, self.A_o, self.halo = comm, A_d, A_o, halo
        send_peer = np.array([q for q, _ in send], np.int32)
        send_off = np.zeros(len(send) + 1, np.int64)
        for i, (_, rows) in enumerate(send):
            send_off[i + 1] = send_off[i] + len(rows)
        send_rows = (np.concatenate([np.asarray(r, np.int32) for _, r in send]) if send
                     else np.zeros(1, np.int32)).astype(np.int32)
        recv_peer = np.array([p for p, _, _ in recv], np.int32)
        recv_off = np.array([0] + [b for _, _, b in recv], np.int64)
        if len(recv) and any(recv[i][1] != recv_off[i] for i in range(len(recv))):
            raise ValueError("receive segments must tile the ghost vector in order")
        self._arrays = (send_peer, send_off, send_rows, recv_peer, recv_off)
        if comm.kind == COMM_HOST:  # the host callback reads the plan
            plan = {
                "halo": halo, "gather_len": gather_len,
                "send": [(int(q), int(send_off[i]), int(send_off[i + 1])) for i, (q, _) in enumerate(send)],
                "recv": [(int(p), int(a), int(b)) for p, a, b in recv]}
        self._h = _P()
        self._plans = comm._keep[1]["plans"] if comm.kind == COMM_HOST else None
        ptr = lambda a: a.ctypes.data if len(a) else None  # noqa: E731
        _pkg._check(_lib().aijhip_mpiaij_create(
            comm._h, A_d._h, A_o._h if A_o is not None else None, HALO[halo], len(send), ptr(send_peer),
            send_off.ctypes.data, send_rows.ctypes.data, len(recv), ptr(recv_peer), recv_off.ctypes.data,
            int(gather_len), ctypes.byref(self._h)))
        if self._plans is not None:
            self._plans[self._h.value] = plan
        self.mloc = A_d.m

    def mult(self, x, y, stream=None):
        _pkg._check(_lib().aijhip_mpiaij_mult(self._h, _pkg._dev_ptr(x, self.mloc, "x"),
                                              _pkg._dev_ptr(y, self.mloc, "y"), _pkg._stream_handle(stream)))

    def set_overlap(self, overlap):
        """RCCL exchange on the exchange stream beside A_d (True) or in order
        on the caller's stream (False: no fork / join events); None: the
        library's automatic choice (by the hardware-queue count, the default)."""
        _pkg._check(_lib().aijhip_mpiaij_set_overlap(self._h, -1 if overlap is None else (1 if overlap else 0)))

    def overlap(self):
        """(placement in effect 0 / 1, the process's hardware queues)."""
        o, q = _i32(), _i32()
        _pkg._check(_lib().aijhip_mpiaij_get_overlap(self._h, ctypes.byref(o), ctypes.byref(q)))
        return o.value, q.value

    def ghost(self):
        """(device pointer, length) of the ghost vector."""
        p, n = _P(), _i64()
        _pkg._check(_lib().aijhip_mpiaij_get_ghost(self._h, ctypes.byref(p), ctypes.byref(n)))
        return p.value, n.value

    def destroy(self):
        if getattr(self, "_h", None) and self._h.value:
            if self._plans is not None:
                self._plans.pop(self._h.value, None)
            _lib().aijhip_mpiaij_destroy(self._h)
            self._h = _P()

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass


class KSPCGMPINative:
    """KSPSolve_CG over a NativeMPIAIJ (aijhip_kspmpi_t): PC none / Jacobi
    (bjacobi + jacobi per rank), every scalar decision on the device."""

    def __init__(self, op: NativeMPIAIJ, rtol=1e-5, atol=1e-50, dtol=1e5, max_it=10000, pc="jacobi",
                 norm="preconditioned", poll: int = 8, gamg=None, graph=None):
        """pc: "none", "jacobi" (bjacobi + jacobi), "gamg" (PCGAMG across the
        ranks: one distributed hierarchy) or "bjacobi_gamg" (a GAMG hierarchy
        per rank's diagonal block); gamg = the GAMG parameters; graph: the
        poll batch replayed as a captured HIP graph (None: the library's
        default, on over RCCL; False / True)."""
        K = importlib.import_module("petsc-openacc_amd.ksp")
        L = _lib()
        self.op = op
        self._h = _P()
        _pkg._check(L.aijhip_kspmpi_create(op._h, ctypes.byref(self._h)))
        self.set_tolerances(rtol, atol, dtol, max_it)
        _pkg._check(L.aijhip_kspmpi_set_pc_type(self._h, K.PC_TYPES[pc]))
        if gamg:
            G = importlib.import_module("petsc-openacc_amd.gamg")
            self._gp = G.default_params(**gamg)
            _pkg._check(L.aijhip_kspmpi_set_gamg_params(self._h, ctypes.byref(self._gp)))
        _pkg._check(L.aijhip_kspmpi_set_norm_type(self._h, K.NORM_TYPES[norm]))
        _pkg._check(L.aijhip_kspmpi_set_poll_interval(self._h, int(poll)))
        if graph is not None:
            _pkg._check(L.aijhip_kspmpi_set_graph(self._h, 1 if graph else 0))

    @property
    def graph_batches(self) -> int:
        """Poll batches the last solve replayed from its captured graph."""
        v = _i32()
        _pkg._check(_lib().aijhip_kspmpi_get_graph_batches(self._h, ctypes.byref(v)))
        return v.value

    def set_tolerances(self, rtol, atol, dtol, max_it):
        self.max_it = int(max_it)
        _pkg._check(_lib().aijhip_kspmpi_set_tolerances(self._h, rtol, atol, dtol, int(max_it)))

    def solve(self, b, x, stream=None):
        _pkg._check(_lib().aijhip_kspmpi_solve(self._h, _pkg._dev_ptr(b, self.op.mloc, "b"),
                                               _pkg._dev_ptr(x, self.op.mloc, "x"), _pkg._stream_handle(stream)))
        return self.reason

    def _get(self, fn, ctype):
        v = ctype()
        _pkg._check(fn(self._h, ctypes.byref(v)))
        return v.value

    @property
    def its(self) -> int:
        return self._get(_lib().aijhip_kspmpi_get_iteration_number, _i32)

    @property
    def reason(self) -> int:
        return self._get(_lib().aijhip_kspmpi_get_converged_reason, ctypes.c_int)

    @property
    def rnorm(self) -> float:
        return self._get(_lib().aijhip_kspmpi_get_residual_norm, _d)

    @property
    def host_syncs(self) -> int:
        return self._get(_lib().aijhip_kspmpi_get_host_syncs, _i32)

    @property
    def setup_seconds(self) -> float:
        return self._get(_lib().aijhip_kspmpi_get_setup_seconds, _d)

    def pc_level(self, l: int, which: str = "A"):
        """This rank's rows of level l's operator ('A') or interpolation ('P')
        of the distributed GAMG hierarchy: (rstart, ai, aj, aa) with global
        columns."""
        L = _lib()
        r0, m, nnz = _i64(), _i32(), _i64()
        _pkg._check(L.aijhip_kspmpi_get_pc_level(self._h, l, which.encode(), ctypes.byref(r0), ctypes.byref(m),
                                                 ctypes.byref(nnz), None, None, None))
        ai = np.zeros(m.value + 1, np.int64)
        aj = np.zeros(max(nnz.value, 1), np.int64)
        aa = np.zeros(max(nnz.value, 1))
        _pkg._check(L.aijhip_kspmpi_get_pc_level(self._h, l, which.encode(), ctypes.byref(r0), ctypes.byref(m),
                                                 ctypes.byref(nnz), ai.ctypes.data, aj.ctypes.data, aa.ctypes.data))
        return r0.value, ai, aj[: nnz.value], aa[: nnz.value]

    def pc_levels(self):
        """(global rows, global entries) per level of the set-up PC
        (collective for GAMG across ranks)."""
        n = _i32()
        rows = np.zeros(32, np.int64)
        nnz = np.zeros(32, np.int64)
        _pkg._check(_lib().aijhip_kspmpi_get_pc_levels(self._h, ctypes.byref(n), rows.ctypes.data, nnz.ctypes.data,
                                                        32))
        return rows[: n.value].tolist(), nnz[: n.value].tolist()

    @property
    def hist(self) -> np.ndarray:
        buf = np.empty(self.its + 1)
        n = _i32()
        _pkg._check(_lib().aijhip_kspmpi_get_residual_history(self._h, buf.ctypes.data, len(buf), ctypes.byref(n)))
        return buf[: n.value]

    def destroy(self):
        if getattr(self, "_h", None) and self._h.value:
            _lib().aijhip_kspmpi_destroy(self._h)
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
