"""BASELINE configs[3] at full size on one GPU: the 600^3 Poisson operand
row-partitioned into 8 z-slabs of 75 planes (216 M rows, 1.51 G entries in
all), one process per slab, through the native MatMult_MPIAIJ
(include/aijhip_mpi.h) over the host transport — the 8 processes share the
one card, which RCCL refuses, so the exchange goes over gloo; the RCCL form
of the same code runs in the driver's 8-GPU bench.

Check per rank, against the same rows of the global operator multiplied on
the device with the whole x (STREAM, PETSc's row order): rows with no ghost
entry are bit-identical; rows whose ghost entries MatMult_MPIAIJ adds after
the diagonal block (PETSc's order for MPIAIJ) agree to the SURVEY §8d fp64
bound. Also the halo itself: every ghost value equals x at its global
column."""
import importlib
import os
import socket

import numpy as np
import pytest

N = 600
WORLD = 8
CG_ITS = 30


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, port, q):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        pkg = importlib.import_module("petsc-openacc_amd")
        mp_mod = importlib.import_module("petsc-openacc_amd.mpiaij")
        C = importlib.import_module("petsc-openacc_amd.comm")
        dev = torch.device("cuda:0")
        planes = N // WORLD
        z0, z1 = rank * planes, (rank + 1) * planes
        row_starts = np.array([r * planes * N * N for r in range(WORLD + 1)], dtype=np.int64)
        lo, hi = int(row_starts[rank]), int(row_starts[rank + 1])
        ai, aj, aa = pkg.poisson_csr(N, N, N, z0, z1)
        comm = C.Comm.host(device=0, timeout_s=600)

        def make_local(a_i, a_j, a_a, ncols):
            return pkg.SeqAIJHIP(a_i, a_j, a_a, ncols=ncols)

        op = mp_mod.MPIAIJ(ai, aj, aa, row_starts, make_local, pkg.split_rows, dev, comm=comm)
        xg = pkg.splitmix_uniform(N ** 3, 42)  # the whole x (1.7 GB), for the reference rows
        x = torch.from_numpy(xg[lo:hi].copy()).to(dev)
        y = torch.empty(hi - lo, dtype=torch.float64, device=dev)
        op.mult(x, y)
        torch.cuda.synchronize()
        gptr, gn = op.native.ghost()
        ghost = torch.empty(max(gn, 1), dtype=torch.float64, device=dev)
        if gn:  # the library's ghost buffer, copied device to device
            import ctypes
            hip = ctypes.CDLL("libamdhip64.so")
            hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
            assert hip.hipMemcpy(ghost.data_ptr(), gptr, 8 * gn, 3) == 0  # hipMemcpyDeviceToDevice
        # global columns of the ghosts (PETSc's garray: sorted off-slab columns)
        off = np.flatnonzero((aj < lo) | (aj >= hi))  # the off-slab entries
        garray = np.unique(aj[off])
        halo_ok = bool(np.array_equal(ghost.cpu().numpy()[:gn], xg[garray]))
        y_mpi = y.cpu().numpy()
        # the distributed CG (aijhip_kspmpi) on the same slabs: CG_ITS fixed iterations
        rhs, _ = pkg.poisson_vectors(N, N, N, z0, z1)
        b = torch.from_numpy(rhs).to(dev)
        xs = torch.zeros_like(b)
        with C.KSPCGMPINative(op.native, rtol=0.0, atol=0.0, max_it=CG_ITS) as kn:
            kn.solve(b, xs)
            cg = dict(its=kn.its, reason=kn.reason, hist=kn.hist.tolist(), syncs=kn.host_syncs)
        del b, xs
        op.native.destroy()
        op.A_d.destroy()
        if op.A_o is not None:
            op.A_o.destroy()
        del x, y, ghost
        torch.cuda.empty_cache()
        # reference rows: the same slab with GLOBAL columns, times the whole x
        with pkg.SeqAIJHIP(ai, aj, aa, ncols=N ** 3) as Ag:
            xd = torch.from_numpy(xg).to(dev)
            yr = torch.empty(hi - lo, dtype=torch.float64, device=dev)
            Ag.mult(xd, yr)
            torch.cuda.synchronize()
            y_ref = yr.cpu().numpy()
            del xd, yr
        grows = np.unique(np.searchsorted(ai, off, side="right") - 1)  # rows with a ghost entry
        ghost_row = np.zeros(hi - lo, dtype=bool)
        ghost_row[grows] = True
        inner_bitwise = bool(np.array_equal(y_mpi[~ghost_row].view(np.uint64), y_ref[~ghost_row].view(np.uint64)))
        u = 2.0 ** -53
        bound_ok, max_err = True, 0.0
        # SURVEY §8d bound on the rows MPIAIJ sums in two parts, per contiguous run of them
        cuts = np.flatnonzero(np.diff(grows) != 1) + 1
        for run in np.split(grows, cuts):
            a, b = int(run[0]), int(run[-1]) + 1
            k0, k1 = int(ai[a]), int(ai[b])
            absax = np.add.reduceat(np.abs(aa[k0:k1]) * np.abs(xg[aj[k0:k1]]), ai[a:b] - k0)
            n = np.diff(ai[a:b + 1]).astype(np.float64)
            err = np.abs(y_mpi[a:b] - y_ref[a:b])
            bound_ok &= bool(np.all(err <= 2 * (n * u / (1 - n * u)) * absax))
            max_err = max(max_err, float(err.max()))
        q.put((rank, dict(rows=hi - lo, nnz=len(aj), ghosts=int(gn), ghost_rows=int(ghost_row.sum()),
                          halo_ok=halo_ok, inner_bitwise=inner_bitwise, bound_ok=bool(bound_ok),
                          max_err=float(max_err), cg=cg)))
    except Exception as e:  # noqa: BLE001
        q.put((rank, {"error": repr(e)}))
    finally:
        dist.destroy_process_group()


def _single(q):
    """The single-GPU device KSP on the whole 600^3 operand (assembled on the
    device: 18.9 GB), CG_ITS iterations."""
    import torch
    try:
        pkg = importlib.import_module("petsc-openacc_amd")
        K = importlib.import_module("petsc-openacc_amd.ksp")
        A, _ = pkg.poisson_device(N)
        b = torch.empty(N ** 3, dtype=torch.float64, device="cuda:0")
        pkg.poisson_vectors_device(N, rhs=b)
        x = torch.zeros_like(b)
        with K.KSPCG(A, rtol=0.0, atol=0.0, max_it=CG_ITS) as ksp:
            ksp.solve(b, x)
            q.put(dict(its=ksp.its, reason=ksp.reason, hist=ksp.history().tolist()))
        A.destroy()
    except Exception as e:  # noqa: BLE001
        q.put({"error": repr(e)})


@pytest.mark.gpu
def test_gpu_configs3_600cubed_8_slabs_native_mpiaij():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(WORLD):
        r, d = q.get(timeout=900)
        got[r] = d
    for p in procs:
        p.join(timeout=120)
    errs = {r: d["error"] for r, d in got.items() if "error" in d}
    assert not errs, errs
    assert all(p.exitcode == 0 for p in procs)
    print("\n600^3 over 8 slabs:", {r: (d["ghosts"], d["ghost_rows"], d["max_err"]) for r, d in sorted(got.items())})
    assert sum(d["rows"] for d in got.values()) == N ** 3
    assert sum(d["nnz"] for d in got.values()) == 7 * N ** 3 - 6 * N ** 2  # SURVEY §8 formula
    for r, d in got.items():
        assert d["ghosts"] == (N * N if r in (0, WORLD - 1) else 2 * N * N)
        assert d["halo_ok"], f"rank {r}: ghost values differ from x at their columns"
        assert d["inner_bitwise"], f"rank {r}: interior rows not bit-identical"
        assert d["bound_ok"], f"rank {r}: boundary rows outside the fp64 bound ({d['max_err']})"
    # distributed CG over the 8 slabs vs the single-GPU KSP on the whole operand
    cgs = [got[r]["cg"] for r in range(WORLD)]
    assert len({tuple(c["hist"]) for c in cgs}) == 1  # one history on every rank
    # (host transport: every all-reduce and halo waits on the host; over RCCL only the polls do)
    p = ctx.Process(target=_single, args=(q,))
    p.start()
    single = q.get(timeout=600)
    p.join(timeout=120)
    assert "error" not in single, single
    assert cgs[0]["its"] == single["its"] == CG_ITS
    print("CG history (8 slabs vs 1 GPU):", cgs[0]["hist"][-1], single["hist"][-1])
    np.testing.assert_allclose(cgs[0]["hist"], single["hist"], rtol=1e-9)
