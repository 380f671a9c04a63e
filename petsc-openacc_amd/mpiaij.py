"""Row-block distributed SpMV across GPUs — the MatMult_MPIAIJ analogue.

PETSc's MatMult_MPIAIJ [ext] computes y = A_d x_local
(diagonal block, the patched MatMult_SeqAIJ) while a VecScatter brings in the
ghost entries of x, then y += A_o x_ghost (MatMultAdd_SeqAIJ on the
compressed-row off-diagonal block). Here the ranks are one process per GPU,
the scatter is RCCL over xGMI through torch.distributed (backend "nccl" is
RCCL on ROCm), issued on RCCL's own stream so it overlaps the diagonal-block
SpMV running on the compute stream:

    compute stream:  A_d.mult(x, y) ........ wait(halo) -> A_o.mult_add(g, y, y)
    RCCL stream:     send/recv boundary planes -> g

The partition is the DMDA z-slab one (helper.cpp:31-36 with a 1x1xP process
grid), under which PETSc's global numbering equals natural ordering and each
rank owns a contiguous block of rows. Ghost columns are PETSc's `garray`:
the sorted, unique off-block global columns (MatSetUpMultiply_MPIAIJ [ext]).

Two halo forms:
  "p2p"       grouped send/recv with the owners of the ghosts (for a 7-point
              slab: the two neighbouring ranks, one plane each) — minimal bytes;
  "allgather" every rank all-gathers the rows other ranks need from it (the
              north-star wording) and A_o indexes the gathered buffer directly.

The local operators are pluggable so the same exchange logic runs on CPU
tensors over gloo in the tests (tests/test_mpiaij.py).
"""
from __future__ import annotations

import importlib

import numpy as np
import torch
import torch.distributed as dist


def slab_bounds(nz: int, world: int, rank: int):
    """Whole z-planes per rank, balanced (DMDA PETSC_DECIDE over z)."""
    base, rem = divmod(nz, world)
    z0 = rank * base + min(rank, rem)
    return z0, z0 + base + (1 if rank < rem else 0)


class HaloPlan:
    """Who sends which local rows to whom, derived from every rank's garray."""

    def __init__(self, garray: np.ndarray, row_starts: np.ndarray, rank: int, world: int, group=None):
        self.rank, self.world = rank, world
        owners = np.searchsorted(row_starts, garray, side="right") - 1
        # ghosts this rank receives, grouped by owner (garray is sorted, so each
        # owner's ghosts are one contiguous run of the ghost vector)
        self.recv = {}
        for p in np.unique(owners):
            idx = np.nonzero(owners == p)[0]
            self.recv[int(p)] = (int(idx[0]), int(idx[-1]) + 1, garray[idx] - row_starts[p])
        # tell owners what to send: every rank publishes its requests
        mine = {p: r[2].astype(np.int64) for p, r in self.recv.items()}
        allreq = [None] * world
        dist.all_gather_object(allreq, mine, group=group)
        self.send = {}
        for q in range(world):
            if q != rank and rank in allreq[q]:
                self.send[q] = np.asarray(allreq[q][rank], dtype=np.int64)
        # contiguous send runs (slab case) avoid a gather copy
        self.send_slices = {q: _as_slice(v) for q, v in self.send.items()}


def _as_slice(idx: np.ndarray):
    if len(idx) and np.all(np.diff(idx) == 1):
        return slice(int(idx[0]), int(idx[-1]) + 1)
    return None


class MPIAIJ:
    """y = A x for a row block of a distributed matrix.

    ai/aj/aa: this rank's rows with GLOBAL column indices; row_starts[p] = first
    global row of rank p (row_starts[world] = global size).
    make_local(ai, aj, aa, ncols) -> an object with mult(x, y, stream) and
    mult_add(x, z, w, stream) (SeqAIJHIP on the GPU).
    """

    def __init__(self, ai, aj, aa, row_starts, make_local, split_rows, device, halo: str = "p2p",
                 group=None, comm=None):
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.group = group
        self.device = device
        self.halo = halo
        self.row_starts = np.asarray(row_starts, dtype=np.int64)
        lo, hi = int(self.row_starts[self.rank]), int(self.row_starts[self.rank + 1])
        self.mloc = hi - lo
        (dai, daj, daa), (oai, oaj, oaa), garray = split_rows(ai, aj, aa, lo, hi)
        self.nz_d, self.nz_o, self.n_ghost = len(daj), len(oaj), len(garray)
        self.plan = HaloPlan(garray, self.row_starts, self.rank, self.world, group)
        self.A_d = make_local(dai, daj, daa, self.mloc)
        self._comm, self._make_local, self._twin = comm, make_local, None
        if halo == "allgather":
            self._o_p2p = (oai, oaj, oaa)  # ghost-numbered A_o, for p2p_native()
            oaj = self._allgather_layout(oaj, garray)
        self.A_o = make_local(oai, oaj, oaa, max(self.n_ghost_buf, 1)) if len(oaj) else None
        self.ghost = torch.zeros(max(self.n_ghost_buf, 1), dtype=torch.float64, device=device)
        # RCCL orders its transfers after the compute stream's queued kernels;
        # gloo moves device tensors with host-side copies that are not
        # stream-ordered, so on that backend (the one-GPU tests) the stream is
        # drained first: x fully written, the previous mult_add done with `ghost`.
        self.host_ordered = dist.get_backend(group) == "gloo" and torch.device(device).type == "cuda"
        # comm (petsc-openacc_amd/comm.py Comm): the exchange and both products
        # run inside the library (aijhip_mpiaij_t: RCCL send/recv on a second
        # HIP stream, or the host transport) instead of through this class.
        self.native = None
        if comm is not None:
            C = importlib.import_module("petsc-openacc_amd.comm")
            if halo == "allgather":
                send, recv = [(-1, self.gather_rows.cpu().numpy())], []
            else:
                send = [(q, idx) for q, idx in sorted(self.plan.send.items())]
                recv = [(p, a, b) for p, (a, b, _) in sorted(self.plan.recv.items(), key=lambda kv: kv[1][0])]
            self.native = C.NativeMPIAIJ(comm, self.A_d, self.A_o, halo, send, recv,
                                         getattr(self, "gather_len", 0))

    def p2p_native(self):
        """The native operator with the point-to-point halo: `native` itself,
        or (all-gather halo) a twin sharing A_d, with A_o in ghost numbering
        and the p2p plan. The distributed GAMG set-up (csrc/gamg_mpi.hip)
        builds every level's exchange from p2p plans, so PCGAMG across ranks
        runs on this; the product is the same either way."""
        if self.native is None:
            raise RuntimeError("p2p_native needs the library's communicator (comm=...)")
        if self.halo == "p2p":
            return self.native
        if self._twin is None:
            C = importlib.import_module("petsc-openacc_amd.comm")
            oai, oaj, oaa = self._o_p2p
            A_o = self._make_local(oai, oaj, oaa, max(self.n_ghost, 1)) if len(oaj) else None
            send = [(q, idx) for q, idx in sorted(self.plan.send.items())]
            recv = [(p, a, b) for p, (a, b, _) in sorted(self.plan.recv.items(), key=lambda kv: kv[1][0])]
            self._twin = (A_o, C.NativeMPIAIJ(self._comm, self.A_d, A_o, "p2p", send, recv, 0))
        return self._twin[1]

    # -------------------------------------------------------------- layouts
    @property
    def n_ghost_buf(self):
        return self.gather_len * self.world if self.halo == "allgather" else self.n_ghost

    def _allgather_layout(self, oaj, garray):
        """Each rank contributes the union of rows anyone requests from it,
        padded to a common length; A_o's columns are remapped to positions in
        the gathered [world x gather_len] buffer."""
        my_rows = np.unique(np.concatenate([v for v in self.plan.send.values()] or [np.zeros(0, np.int64)]))
        lens = [None] * self.world
        dist.all_gather_object(lens, my_rows.tolist(), group=self.group)
        self.gather_len = max(1, max(len(v) for v in lens))
        self.gather_rows = torch.as_tensor(my_rows, dtype=torch.long, device=self.device)
        self.gather_slice = _as_slice(my_rows)
        self.gbuf_send = torch.zeros(self.gather_len, dtype=torch.float64, device=self.device)
        pos = {}
        for p, rows in enumerate(lens):
            for t, r in enumerate(rows):
                pos[(p, r)] = p * self.gather_len + t
        owners = np.searchsorted(self.row_starts, garray, side="right") - 1
        remap = np.array([pos[(int(p), int(g - self.row_starts[p]))] for p, g in zip(owners, garray)],
                         dtype=np.int32)
        return remap[oaj] if len(oaj) else oaj

    # ---------------------------------------------------------------- halo
    def _post_halo(self, x):
        """Start the ghost exchange; returns a list of works to wait on."""
        if self.host_ordered:
            torch.cuda.current_stream(x.device).synchronize()
        if self.halo == "allgather":
            if self.gather_slice is not None:
                n = self.gather_slice.stop - self.gather_slice.start
                self.gbuf_send[:n].copy_(x[self.gather_slice])
            elif len(self.gather_rows):
                self.gbuf_send[: len(self.gather_rows)].copy_(x[self.gather_rows])
            w = dist.all_gather_into_tensor(self.ghost, self.gbuf_send, group=self.group, async_op=True)
            return [w]
        ops = []
        for q, idx in self.plan.send.items():
            sl = self.plan.send_slices[q]
            buf = x[sl] if sl is not None else x[torch.as_tensor(idx, device=x.device)]
            ops.append(dist.P2POp(dist.isend, buf, q, group=self.group))
        for p, (a, b, _) in self.plan.recv.items():
            ops.append(dist.P2POp(dist.irecv, self.ghost[a:b], p, group=self.group))
        return dist.batch_isend_irecv(ops) if ops else []

    def mult(self, x, y, stream=None):
        """y = A_d x_local + A_o x_ghost, the exchange overlapped with A_d."""
        if self.native is not None:
            self.native.mult(x, y, stream)
            return
        works = self._post_halo(x)
        self.A_d.mult(x, y, stream)
        for w in works:
            w.wait()
        if self.A_o is not None:
            self.A_o.mult_add(self.ghost, y, y, stream)

    def algorithmic_bytes_local(self):
        m = self.mloc
        return 12 * (self.nz_d + self.nz_o) + 4 * (m + 1) + 8 * m + 8 * m
