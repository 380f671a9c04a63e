#!/usr/bin/env python3
"""Which stream-capture shapes this HIP / RCCL stack turns into a graph
(the capture_end segfault). Each case runs in its own
child process (a segfault ends only that case) and prints one JSON line:

  fork_memset   capture stream gs: memset; event on gs, side stream xs waits,
                memset on xs, event on xs, gs waits; memset on gs
  rccl_on_gs    an RCCL all-reduce (one rank, the library's communicator)
                enqueued on the capturing stream itself
  fork_rccl     the all-reduce on the side stream xs inside the fork / join
  fork_p2p      grouped ncclSend / ncclRecv to self on xs inside the fork /
                join (the distributed MatMult's exchange; one aijhip_mpiaij
                self-halo multiply captured)
  serial_p2p    the same multiply with the exchange on the capturing stream

    python tools/capture_probe.py [case ...]
"""
import ctypes
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
CASES = ("fork_memset", "rccl_on_gs", "fork_rccl", "fork_p2p", "serial_p2p")


def hip():
    import torch
    L = ctypes.CDLL(str(Path(torch.__file__).parent / "lib" / "libamdhip64.so"), mode=ctypes.RTLD_GLOBAL)
    P = ctypes.c_void_p
    for f, a in (("hipStreamCreateWithFlags", [ctypes.POINTER(P), ctypes.c_uint]),
                 ("hipEventCreateWithFlags", [ctypes.POINTER(P), ctypes.c_uint]),
                 ("hipStreamBeginCapture", [P, ctypes.c_int]), ("hipStreamEndCapture", [P, ctypes.POINTER(P)]),
                 ("hipGraphInstantiate", [ctypes.POINTER(P), P, P, P, ctypes.c_size_t]),
                 ("hipGraphLaunch", [P, P]), ("hipEventRecord", [P, P]), ("hipStreamWaitEvent", [P, P, ctypes.c_uint]),
                 ("hipMemsetAsync", [P, ctypes.c_int, ctypes.c_size_t, P]), ("hipStreamSynchronize", [P])):
        getattr(L, f).argtypes = a
        getattr(L, f).restype = ctypes.c_int
    return L


def run_case(case):
    import numpy as np
    import torch
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=0, world_size=1)
    H = hip()
    pkg = __import__("importlib").import_module("petsc-openacc_amd")
    C = __import__("importlib").import_module("petsc-openacc_amd.comm")
    comm = C.Comm.rccl(device=0, timeout_s=60)
    P = ctypes.c_void_p
    gs, xs, e1, e2 = P(), P(), P(), P()
    assert H.hipStreamCreateWithFlags(ctypes.byref(gs), 1) == 0 and H.hipStreamCreateWithFlags(ctypes.byref(xs), 1) == 0
    assert H.hipEventCreateWithFlags(ctypes.byref(e1), 2) == 0 and H.hipEventCreateWithFlags(ctypes.byref(e2), 2) == 0
    buf = torch.ones(1024, dtype=torch.float64, device="cuda")
    p = buf.data_ptr()
    op = None
    if case in ("fork_p2p", "serial_p2p"):
        from test_rccl_selfhalo_gpu import split_self
        N = 20
        ai, aj, aa = pkg.poisson_csr(N)
        m = N ** 3
        G = np.arange(m - 2 * N * N, m)
        (dai, daj, daa), (oai, oaj, oaa) = split_self(ai, aj, aa, G)
        Ad = pkg.SeqAIJHIP(dai, daj, daa, ncols=m)
        Ao = pkg.SeqAIJHIP(oai, oaj, oaa, ncols=len(G))
        op = C.NativeMPIAIJ(comm, Ad, Ao, "p2p", [(0, G)], [(0, 0, len(G))], 0)
        op.set_overlap(case == "fork_p2p")
        x = torch.from_numpy(pkg.splitmix_uniform(m, 42)).cuda()
        y = torch.empty_like(x)
        op.mult(x, y)
        torch.cuda.synchronize()
        y_ref = y.clone()
        y.fill_(float("nan"))
        torch.cuda.synchronize()
    L = C._lib()
    rc = {}
    rc["begin"] = H.hipStreamBeginCapture(gs, 2)  # relaxed
    if case == "fork_memset":
        H.hipMemsetAsync(P(p), 0, 64, gs)
        H.hipEventRecord(e1, gs)
        H.hipStreamWaitEvent(xs, e1, 0)
        H.hipMemsetAsync(P(p + 64), 0, 64, xs)
        H.hipEventRecord(e2, xs)
        H.hipStreamWaitEvent(gs, e2, 0)
        H.hipMemsetAsync(P(p + 128), 0, 64, gs)
    elif case == "rccl_on_gs":
        rc["allreduce"] = L.aijhip_comm_allreduce_sum(comm._h, P(p), 16, gs)
    elif case == "fork_rccl":
        H.hipEventRecord(e1, gs)
        H.hipStreamWaitEvent(xs, e1, 0)
        rc["allreduce"] = L.aijhip_comm_allreduce_sum(comm._h, P(p), 16, xs)
        H.hipEventRecord(e2, xs)
        H.hipStreamWaitEvent(gs, e2, 0)
    else:
        rc["mult"] = L.aijhip_mpiaij_mult(op._h, P(x.data_ptr()), P(y.data_ptr()), gs)
    print(json.dumps({"case": case, "stage": "captured", **rc}), flush=True)
    g = P()
    rc["end"] = H.hipStreamEndCapture(gs, ctypes.byref(g))
    print(json.dumps({"case": case, "stage": "ended", **rc}), flush=True)
    ex = P()
    rc["instantiate"] = H.hipGraphInstantiate(ctypes.byref(ex), g, None, None, 0)
    rc["launch"] = H.hipGraphLaunch(ex, gs)
    rc["sync"] = H.hipStreamSynchronize(gs)
    out = {"case": case, "stage": "replayed", **rc}
    if op is not None:
        out["bitwise_equal"] = bool(torch.equal(y, y_ref))
    print(json.dumps(out), flush=True)
    dist.destroy_process_group()


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "--case":
        run_case(sys.argv[2])
        return
    for case in (sys.argv[1:] or CASES):
        r = subprocess.run([sys.executable, "-u", __file__, "--case", case], capture_output=True, text=True,
                           timeout=120)
        lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
        last = json.loads(lines[-1]) if lines else {"case": case, "stage": "none"}
        last["exit"] = r.returncode
        if r.returncode:
            last["stderr_tail"] = [x for x in r.stderr.splitlines() if x.strip()][-6:]
        print(json.dumps(last), flush=True)


if __name__ == "__main__":
    main()
