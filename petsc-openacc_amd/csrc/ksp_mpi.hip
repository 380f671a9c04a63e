// ksp_mpi.hip — the row-partitioned path (include/aijhip_mpi.h): the
// communicator, MatMult_MPIAIJ and KSPSolve_CG over it, one process per GPU.
//
// PETSc's MatMult_MPIAIJ [ext] and KSPSolve_CG [ext] with
// its MPI_Allreduce per dot (/root/reference/src/main_ksp.cpp:103 on
// /root/reference/runs/single-node-scaling.pbs:56-67's 1-16 ranks), laid out
// for MI355X:
//
//   caller stream s   : [aypx] -- A_d p (+ p.w partials) ------ wait(halo) -- A_o g (+ correction) -- ...
//   exchange stream xs:   wait(s) -- pack -- RCCL send/recv ----^
//   s (cont.)         : reduce partials -> RCCL all-reduce (1 double) -> scalar step -> update ->
//                       reduce -> RCCL all-reduce (3 doubles) -> scalar step
//
// No iteration needs the host: the reduced sums are identical on every rank
// (an all-reduce leaves one value everywhere), so the scalar steps
// (cg_device.h) take the same branch on every rank, and the host reads the
// stop flag every `poll` iterations. Kernels return at once after the flag
// is set; the halo exchange and the all-reduces keep running so that every
// rank issues the same collectives.
//
// RCCL is resolved with dlopen at communicator creation: the librccl.so.1
// the process already holds (PyTorch's) or /opt/rocm/lib's; libaijhip.so
// itself has no link-time RCCL dependency and loads on machines without it.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <functional>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <type_traits>
#include <vector>

#include "aijhip_internal.h"
#include "aijhip_mpi.h"
#include "cg_device.h"
#include "gamg_device.h"
#include "gamg_mpi.h"
#include "mpi_internal.h"

namespace aijhip_mpi {

int mfail(int code, const std::string &msg) {
    aijhip::set_error(msg);
    return code;
}

int mhip(hipError_t e, const char *what) {
    aijhip::set_error(std::string(what) + ": " + hipGetErrorString(e));
    return AIJHIP_ERR_HIP;
}

}  // namespace aijhip_mpi

using namespace aijhip_mpi;

namespace {

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        int cur = -1;
        if (hipGetDevice(&cur) == hipSuccess && cur != dev && hipSetDevice(dev) == hipSuccess) prev = cur;
    }
    ~DeviceGuard() { if (prev >= 0) (void)hipSetDevice(prev); }
};

// ------------------------------------------------------------ RCCL table
struct Rccl {
    decltype(&ncclGetVersion) GetVersion = nullptr;
    decltype(&ncclGetUniqueId) GetUniqueId = nullptr;
    decltype(&ncclCommInitRank) CommInitRank = nullptr;
    decltype(&ncclCommDestroy) CommDestroy = nullptr;
    decltype(&ncclCommAbort) CommAbort = nullptr;
    decltype(&ncclCommGetAsyncError) CommGetAsyncError = nullptr;
    decltype(&ncclAllReduce) AllReduce = nullptr;
    decltype(&ncclAllGather) AllGather = nullptr;
    decltype(&ncclSend) Send = nullptr;
    decltype(&ncclRecv) Recv = nullptr;
    decltype(&ncclGroupStart) GroupStart = nullptr;
    decltype(&ncclGroupEnd) GroupEnd = nullptr;
    decltype(&ncclGetErrorString) GetErrorString = nullptr;
    bool ok = false;
    std::string why;
};

const Rccl &rccl() {
    static Rccl R;
    static std::once_flag once;
    std::call_once(once, [] {
        void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);  // already in the process (PyTorch's)
        if (!h) h = dlopen("librccl.so.1", RTLD_NOW);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW);
        if (!h) {
            const char *d = dlerror();
            R.why = std::string("librccl.so.1 not loadable: ") + (d ? d : "?");
            return;
        }
        bool all = true;
        auto sym = [&](auto &f, const char *name) {
            f = reinterpret_cast<std::remove_reference_t<decltype(f)>>(dlsym(h, name));
            if (!f) {
                all = false;
                R.why += std::string(" missing ") + name;
            }
        };
        sym(R.GetVersion, "ncclGetVersion");
        sym(R.GetUniqueId, "ncclGetUniqueId");
        sym(R.CommInitRank, "ncclCommInitRank");
        sym(R.CommDestroy, "ncclCommDestroy");
        sym(R.CommAbort, "ncclCommAbort");
        sym(R.CommGetAsyncError, "ncclCommGetAsyncError");
        sym(R.AllReduce, "ncclAllReduce");
        sym(R.AllGather, "ncclAllGather");
        sym(R.Send, "ncclSend");
        sym(R.Recv, "ncclRecv");
        sym(R.GroupStart, "ncclGroupStart");
        sym(R.GroupEnd, "ncclGroupEnd");
        sym(R.GetErrorString, "ncclGetErrorString");
        R.ok = all;
    });
    return R;
}

int nfail(ncclResult_t r, const char *what) {
    const Rccl &R = rccl();
    aijhip::set_error(std::string(what) + ": " + (R.GetErrorString ? R.GetErrorString(r) : "RCCL error"));
    return AIJHIP_ERR_COMM;
}

}  // namespace


namespace {
constexpr int kMaxRed = 64;
}  // namespace

namespace aijhip_mpi {

void comm_abort(aijhip_comm *C) {
    if (C->aborted) return;
    C->aborted = true;
    if (C->kind == AIJHIP_COMM_RCCL && C->nc) {
        rccl().CommAbort(C->nc);
        C->nc = nullptr;
    }
}

// Block the host until `s` has drained up to now, failing (and aborting the
// communicator) if a collective reports an error or the wait exceeds the
// timeout: a stuck peer makes the solve return AIJHIP_ERR_COMM instead of
// hanging the process.
int wait_stream(aijhip_comm *C, hipStream_t s) {
    ++C->waits;
    hipError_t e = hipEventRecord(C->ev_wait, s);
    if (e != hipSuccess) return mhip(e, "comm wait");
    if (C->timeout_s <= 0.0) {
        e = hipEventSynchronize(C->ev_wait);
        return e == hipSuccess ? AIJHIP_OK : mhip(e, "comm wait");
    }
    const auto t0 = std::chrono::steady_clock::now();
    for (int spin = 0;; ++spin) {
        e = hipEventQuery(C->ev_wait);
        if (e == hipSuccess) return AIJHIP_OK;
        if (e != hipErrorNotReady) return mhip(e, "comm wait");
        if (C->kind == AIJHIP_COMM_RCCL && C->nc && (spin & 255) == 255) {
            ncclResult_t ae = ncclSuccess;
            rccl().CommGetAsyncError(C->nc, &ae);
            if (ae != ncclSuccess && ae != ncclInProgress) {
                comm_abort(C);
                return nfail(ae, "RCCL asynchronous error");
            }
        }
        const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (el > C->timeout_s) {
            comm_abort(C);
            return mfail(AIJHIP_ERR_COMM, "collective timed out after " + std::to_string(C->timeout_s) +
                                              " s (communicator aborted)");
        }
        if (el > 1e-3) std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
}

int comm_allreduce(aijhip_comm *C, double *d_buf, int32_t n, hipStream_t s) {
    if (C->aborted) return mfail(AIJHIP_ERR_COMM, "communicator aborted");
    if (n <= 0) return AIJHIP_OK;
    if (C->kind == AIJHIP_COMM_RCCL) {
        const ncclResult_t r = rccl().AllReduce(d_buf, d_buf, (size_t)n, ncclFloat64, ncclSum, C->nc, s);
        return r == ncclSuccess ? AIJHIP_OK : nfail(r, "ncclAllReduce");
    }
    if (n > kMaxRed) return mfail(AIJHIP_ERR_ARG, "host all-reduce of more than 64 values");
    hipError_t e = hipMemcpyAsync(C->h_red, d_buf, sizeof(double) * (size_t)n, hipMemcpyDeviceToHost, s);
    if (e != hipSuccess) return mhip(e, "all-reduce staging");
    int rc = wait_stream(C, s);
    if (rc) return rc;
    if (C->har(C->ctx, C->h_red, n) != 0) {
        comm_abort(C);
        return mfail(AIJHIP_ERR_COMM, "host all-reduce callback failed");
    }
    e = hipMemcpyAsync(d_buf, C->h_red, sizeof(double) * (size_t)n, hipMemcpyHostToDevice, s);
    return e == hipSuccess ? AIJHIP_OK : mhip(e, "all-reduce staging");
}

int comm_allreduce_host(aijhip_comm *C, double *v, int32_t n) {
    if (C->aborted) return mfail(AIJHIP_ERR_COMM, "communicator aborted");
    if (n <= 0 || C->nranks == 1) return AIJHIP_OK;
    if (C->kind == AIJHIP_COMM_HOST) {
        if (n > kMaxRed) return mfail(AIJHIP_ERR_ARG, "host all-reduce of more than 64 values");
        std::memcpy(C->h_red, v, sizeof(double) * (size_t)n);
        ++C->waits;
        if (C->har(C->ctx, C->h_red, n) != 0) {
            comm_abort(C);
            return mfail(AIJHIP_ERR_COMM, "host all-reduce callback failed");
        }
        std::memcpy(v, C->h_red, sizeof(double) * (size_t)n);
        return AIJHIP_OK;
    }
    double *d = nullptr;
    hipError_t e = hipMalloc(&d, sizeof(double) * (size_t)n);
    if (e != hipSuccess) return mhip(e, "all-reduce buffer");
    int rc = AIJHIP_OK;
    if (!C->xs && (e = hipStreamCreateWithFlags(&C->xs, hipStreamNonBlocking)) != hipSuccess) rc = mhip(e, "stream");
    if (!rc && (e = hipMemcpyAsync(d, v, sizeof(double) * (size_t)n, hipMemcpyHostToDevice, C->xs)) != hipSuccess)
        rc = mhip(e, "all-reduce upload");
    if (!rc) rc = comm_allreduce(C, d, n, C->xs);
    if (!rc && (e = hipMemcpyAsync(v, d, sizeof(double) * (size_t)n, hipMemcpyDeviceToHost, C->xs)) != hipSuccess)
        rc = mhip(e, "all-reduce download");
    if (!rc) rc = wait_stream(C, C->xs);
    hipFree(d);
    return rc;
}

// Counts first (one word per peer pair), then the payloads: RCCL grouped
// send/recv of device copies, or the host transport's sendrecv callback.
int comm_sendrecv(aijhip_comm *C, const std::vector<std::vector<uint64_t>> &out,
                  std::vector<std::vector<uint64_t>> &in) {
    const int P = C->nranks, me = C->rank;
    in.assign((size_t)P, {});
    if ((int)out.size() != P) return mfail(AIJHIP_ERR_ARG, "sendrecv: one list per rank");
    in[me] = out[me];
    if (P == 1) return AIJHIP_OK;
    if (C->aborted) return mfail(AIJHIP_ERR_COMM, "communicator aborted");
    // the counts: word q of my row goes to rank q
    std::vector<std::vector<uint64_t>> cnt_out((size_t)P), cnt_in;
    std::vector<int64_t> nin((size_t)P, 0);
    auto exchange = [&](const std::vector<std::vector<uint64_t>> &o, std::vector<std::vector<uint64_t>> &i,
                        const std::vector<int64_t> &isize) -> int {
        std::vector<int32_t> sp, rp;
        std::vector<int64_t> so{0}, ro{0};
        std::vector<uint64_t> sbuf;
        for (int q = 0; q < P; ++q) {
            if (q == me || o[q].empty()) continue;
            sp.push_back(q);
            sbuf.insert(sbuf.end(), o[q].begin(), o[q].end());
            so.push_back((int64_t)sbuf.size());
        }
        for (int p = 0; p < P; ++p) {
            if (p == me || isize[p] == 0) continue;
            rp.push_back(p);
            ro.push_back(ro.back() + isize[p]);
        }
        std::vector<uint64_t> rbuf((size_t)ro.back());
        if (C->kind == AIJHIP_COMM_HOST) {
            if (!C->hsr) return mfail(AIJHIP_ERR_STATE, "host transport without a sendrecv callback "
                                                        "(aijhip_comm_set_host_sendrecv)");
            ++C->waits;
            if (C->hsr(C->ctx, (int32_t)sp.size(), sp.data(), so.data(), reinterpret_cast<const double *>(sbuf.data()),
                       (int32_t)rp.size(), rp.data(), ro.data(), reinterpret_cast<double *>(rbuf.data())) != 0) {
                comm_abort(C);
                return mfail(AIJHIP_ERR_COMM, "host sendrecv callback failed");
            }
        } else {
            const Rccl &R = rccl();
            hipError_t e;
            if (!C->xs && (e = hipStreamCreateWithFlags(&C->xs, hipStreamNonBlocking)) != hipSuccess)
                return mhip(e, "stream");
            uint64_t *ds = nullptr, *dr = nullptr;
            if ((e = hipMalloc(&ds, sizeof(uint64_t) * std::max<size_t>(1, sbuf.size()))) != hipSuccess ||
                (e = hipMalloc(&dr, sizeof(uint64_t) * std::max<size_t>(1, rbuf.size()))) != hipSuccess) {
                hipFree(ds);
                return mhip(e, "sendrecv buffers");
            }
            int rc = AIJHIP_OK;
            if (!sbuf.empty() && (e = hipMemcpyAsync(ds, sbuf.data(), sizeof(uint64_t) * sbuf.size(),
                                                     hipMemcpyHostToDevice, C->xs)) != hipSuccess)
                rc = mhip(e, "sendrecv upload");
            if (!rc) {
                ncclResult_t r = R.GroupStart();
                for (size_t q = 0; r == ncclSuccess && q < sp.size(); ++q)
                    r = R.Send(ds + so[q], (size_t)(so[q + 1] - so[q]), ncclUint64, sp[q], C->nc, C->xs);
                for (size_t p = 0; r == ncclSuccess && p < rp.size(); ++p)
                    r = R.Recv(dr + ro[p], (size_t)(ro[p + 1] - ro[p]), ncclUint64, rp[p], C->nc, C->xs);
                const ncclResult_t r2 = R.GroupEnd();
                if (r != ncclSuccess) rc = nfail(r, "set-up ncclSend/ncclRecv");
                else if (r2 != ncclSuccess) rc = nfail(r2, "ncclGroupEnd");
            }
            if (!rc && !rbuf.empty() && (e = hipMemcpyAsync(rbuf.data(), dr, sizeof(uint64_t) * rbuf.size(),
                                                            hipMemcpyDeviceToHost, C->xs)) != hipSuccess)
                rc = mhip(e, "sendrecv download");
            if (!rc) rc = wait_stream(C, C->xs);
            hipFree(ds);
            hipFree(dr);
            if (rc) return rc;
        }
        for (size_t p = 0; p < rp.size(); ++p) i[rp[p]].assign(rbuf.begin() + ro[p], rbuf.begin() + ro[p + 1]);
        return AIJHIP_OK;
    };
    for (int q = 0; q < P; ++q) cnt_out[q].assign(1, (uint64_t)out[q].size());
    std::vector<int64_t> ones((size_t)P, 1);
    ones[me] = 0;
    cnt_in.assign((size_t)P, {});
    int rc = exchange(cnt_out, cnt_in, ones);
    if (rc) return rc;
    for (int p = 0; p < P; ++p) nin[p] = p == me ? 0 : (int64_t)cnt_in[p][0];
    std::vector<std::vector<uint64_t>> got((size_t)P);
    if ((rc = exchange(out, got, nin))) return rc;
    for (int p = 0; p < P; ++p)
        if (p != me) in[p] = std::move(got[p]);
    return AIJHIP_OK;
}

}  // namespace aijhip_mpi

namespace {

// ------------------------------------------------------------- kernels
// Pack the send rows: buf[i] = x[rows[i]] (zero past n up to n_pad).
// y[rows[k]] += v[k] over one peer's segment (rows distinct within it)
__global__ __launch_bounds__(256) void k_add_rows(int64_t n, const int32_t *__restrict__ rows,
                                                  const double *__restrict__ v, double *y) {
    const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (k < n) y[rows[k]] = y[rows[k]] + v[k];
}

__global__ __launch_bounds__(256) void k_pack(int64_t n, int64_t n_pad, const int32_t *__restrict__ rows,
                                              const double *__restrict__ x, double *buf) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n_pad; i += (int64_t)gridDim.x * 256)
        buf[i] = i < n ? x[rows[i]] : 0.0;
}

// w[o] += (A_o g)_o for every row o of A_o's row list (MatMultAdd_SeqAIJ
// order: the sum starts from w[o] and adds the products in storage order),
// and, in the CG, the partials of p_o w_o(new) - p_o w_o(old): the A_d
// epilogue already summed p_o w_o(old), so the two give p . w.
__global__ __launch_bounds__(kVecThreads) void k_offdiag(int32_t nr, const int32_t *__restrict__ rai,
                                                         const int32_t *__restrict__ ridx,
                                                         const int32_t *__restrict__ aj,
                                                         const double *__restrict__ aa,
                                                         const double *__restrict__ g,
                                                         const double *__restrict__ p, double *w, double *part,
                                                         const CGState *S) {
    __shared__ double scratch[kVecThreads / 64];
    if (S && S->done) return;
    double d = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * kVecThreads + threadIdx.x; i < nr; i += (int64_t)gridDim.x * kVecThreads) {
        const int32_t o = ridx ? ridx[i] : (int32_t)i;
        const double old = w[o];
        double s = old;
        for (int32_t k = rai[i]; k < rai[i + 1]; ++k) s += aa[k] * g[aj[k]];
        w[o] = s;
        if (part) {
            const double po = p[o];
            d += po * s + (-(po * old));
        }
    }
    if (!part) return;
    const double v = bsum<kVecThreads>(d, scratch);
    if (threadIdx.x == 0) part[blockIdx.x] = v;
}

// red[q] = this device's fixed-order sum of part[q*nb .. (q+1)*nb), q < nq
// (the single-GPU solver's k_reduce_* sums). step: one rank, no all-reduce
// in between — apply the scalar step here (1: init, 2: iteration) as the
// single-GPU solver's fused reduce kernels do.
__global__ __launch_bounds__(kRedThreads) void k_local_sums(const double *part, int nb, int nq, double *red,
                                                            int step, CGState *S, double *hist, CGParams p) {
    __shared__ double scratch[kRedThreads / 64];
    if (step == 2 && S->done) return;
    double v[4] = {0.0, 0.0, 0.0, 0.0};
    for (int q = 0; q < nq; ++q) v[q] = reduce_parts(part + (size_t)q * nb, nb, scratch);
    if (threadIdx.x != 0) return;
    if (step == 1) step_init(v[0], v[1], v[2], v[3], S, hist, p);
    else if (step == 2) step_iter(v[0], v[1], v[2], S, hist, p);
    else for (int q = 0; q < nq; ++q) red[q] = v[q];
}

// dpi's local sum: the A_d epilogue's partials, then the A_o corrections
// (step: apply step_dpi here, one rank).
__global__ __launch_bounds__(kRedThreads) void k_local_dpi(const double *part, int nb, const double *opart,
                                                           int nob, double *red, CGState *S, int step) {
    __shared__ double scratch[kRedThreads / 64];
    if (S->done) return;
    double v = reduce_parts(part, nb, scratch);
    if (nob > 0) {
        const double o = reduce_parts(opart, nob, scratch);
        v += o;
    }
    if (threadIdx.x != 0) return;
    if (step) step_dpi(v, S);
    else red[0] = v;
}

// GAMG sub-PC: zz, zr from pz[0, nbz) and pz[nbz, 2 nbz) (the V-cycle's fused
// finest post-smoothing, or k_dots), rr from pr[0, nbr) — ksp.hip
// k_reduce_iter's sums; step: apply step_iter here (one rank).
__global__ __launch_bounds__(kRedThreads) void k_local_iter(const double *pz, int nbz, const double *pr, int nbr,
                                                            double *red, int step, CGState *S, double *hist,
                                                            CGParams p) {
    __shared__ double scratch[kRedThreads / 64];
    if (S->done) return;
    const double zz = reduce_parts(pz, nbz, scratch);
    const double zr = reduce_parts(pz + nbz, nbz, scratch);
    const double rr = reduce_parts(pr, nbr, scratch);
    if (threadIdx.x != 0) return;
    if (step) step_iter(zz, zr, rr, S, hist, p);
    else { red[0] = zz; red[1] = zr; red[2] = rr; }
}

__global__ void k_step_init(const double *red, CGState *S, double *hist, CGParams p) {
    if (threadIdx.x == 0) step_init(red[0], red[1], red[2], red[3], S, hist, p);
}

__global__ void k_step_dpi(const double *red, CGState *S) {
    if (threadIdx.x == 0 && !S->done) step_dpi(red[0], S);
}

__global__ void k_step_iter(const double *red, CGState *S, double *hist, CGParams p) {
    if (threadIdx.x == 0 && !S->done) step_iter(red[0], red[1], red[2], S, hist, p);
}

int grid_of(int64_t n, int cap) {
    return (int)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, cap));
}

}  // namespace


namespace {

// aijhip_mpiaij_set_overlap(-1): the exchange stream only with a hardware
// queue of its own to run on (aijhip::hw_queues)
int auto_overlap() { return aijhip::hw_queues() >= aijhip::kOverlapMinQueues ? 1 : 0; }

void mpiaij_free(aijhip_mpiaij *M) {
    hipFree(M->d_send_rows); hipFree(M->d_sendbuf); hipFree(M->d_ghost);
    if (M->h_send) hipHostFree(M->h_send);
    if (M->h_ghost) hipHostFree(M->h_ghost);
    if (M->xs) hipStreamDestroy(M->xs);
    if (M->ev_x) hipEventDestroy(M->ev_x);
    if (M->ev_halo) hipEventDestroy(M->ev_halo);
}

}  // namespace

namespace aijhip_mpi {

// Start the ghost exchange on the exchange stream (ordered after everything
// already enqueued on s, i.e. after x is written and the previous A_o
// product has read the ghost vector): the fork and the pack kernels. The
// RCCL collective itself is enqueued by halo_finish — after the caller has
// launched the diagonal block — because RCCL's host-side enqueue takes tens
// of microseconds (hipExtLaunchKernel ~63 us median in profiles/r05/ of
// round 5): issued first, it held back the A_d launch and the device
// idled; issued second, A_d runs while the host is inside RCCL. The device
// order is unchanged (the collective waits only for the fork).
// Set while aijhip_kspmpi_solve captures its poll batch: the exchanges are
// captured in the serial form. Measured on this stack (tools/capture_probe.py,
// profiles/r06/i/): grouped ncclSend / ncclRecv on a stream forked inside a
// capture makes hipStreamEndCapture segfault (an all-reduce there, memsets
// there, or the exchange on the capturing stream itself do not).
thread_local bool g_capturing = false;

int halo_post(aijhip_mpiaij *M, const double *x, hipStream_t s) {
    aijhip_comm *C = M->comm;
    if (C->aborted) return mfail(AIJHIP_ERR_COMM, "communicator aborted");
    hipError_t e;
    // serial (RCCL, overlap 0, or under capture): everything on the caller's stream, in order
    const bool serial = C->kind == AIJHIP_COMM_RCCL && (!M->overlap || g_capturing);
    const hipStream_t xs = serial ? s : M->xs;
    M->post_s = xs;
    if (!serial &&
        ((e = hipEventRecord(M->ev_x, s)) != hipSuccess || (e = hipStreamWaitEvent(M->xs, M->ev_x, 0)) != hipSuccess))
        return mhip(e, "halo order");
    const int64_t npack = M->halo == AIJHIP_HALO_ALLGATHER ? M->gather_len : M->n_send;
    const int64_t nrows = M->send_off.empty() ? 0 : M->send_off.back();
    if (npack > 0 && (M->pack_all || M->halo == AIJHIP_HALO_ALLGATHER)) {
        hipLaunchKernelGGL(k_pack, dim3(grid_of(npack, 1024)), dim3(256), 0, xs, nrows, npack, M->d_send_rows,
                           x, M->d_sendbuf);
    } else if (npack > 0) {  // RCCL p2p: only the non-contiguous peers are packed
        for (size_t q = 0; q < M->send_peer.size(); ++q) {
            if (M->send_first[q] >= 0) continue;
            const int64_t a = M->send_off[q], n = M->send_off[q + 1] - a;
            hipLaunchKernelGGL(k_pack, dim3(grid_of(n, 1024)), dim3(256), 0, xs, n, n, M->d_send_rows + a, x,
                               M->d_sendbuf + a);
        }
    }
    if ((e = hipGetLastError()) != hipSuccess) return mhip(e, "halo pack");
    if (C->kind == AIJHIP_COMM_RCCL) {
        M->post_x = x;  // the collective is enqueued by halo_finish
    } else if (npack > 0) {
        if ((e = hipMemcpyAsync(M->h_send, M->d_sendbuf, sizeof(double) * (size_t)npack, hipMemcpyDeviceToHost,
                                M->xs)) != hipSuccess)
            return mhip(e, "halo staging");
    }
    M->posted = true;
    return AIJHIP_OK;
}

namespace {

// The RCCL collective of a posted exchange, on the stream halo_post chose
// (the exchange stream, or the caller's in the serial form).
int halo_send_rccl(aijhip_mpiaij *M) {
    aijhip_comm *C = M->comm;
    const double *x = M->post_x;
    const hipStream_t xs = M->post_s;
    M->post_x = nullptr;
    if (!x) return mfail(AIJHIP_ERR_STATE, "halo_finish without halo_post");
    const Rccl &R = rccl();
    ncclResult_t r;
    if (M->halo == AIJHIP_HALO_ALLGATHER) {
        r = R.AllGather(M->d_sendbuf, M->d_ghost, (size_t)M->gather_len, ncclFloat64, C->nc, xs);
        if (r != ncclSuccess) return nfail(r, "ncclAllGather");
    } else {
        if ((r = R.GroupStart()) != ncclSuccess) return nfail(r, "ncclGroupStart");
        for (size_t q = 0; q < M->send_peer.size(); ++q) {
            const int64_t a = M->send_off[q], n = M->send_off[q + 1] - a;
            const double *src = M->send_first[q] >= 0 ? x + M->send_first[q] : M->d_sendbuf + a;
            if (n > 0 && (r = R.Send(src, (size_t)n, ncclFloat64, M->send_peer[q], C->nc, xs)) != ncclSuccess)
                break;
        }
        for (size_t p = 0; r == ncclSuccess && p < M->recv_peer.size(); ++p) {
            const int64_t a = M->recv_off[p], n = M->recv_off[p + 1] - a;
            if (n > 0 && (r = R.Recv(M->d_ghost + a, (size_t)n, ncclFloat64, M->recv_peer[p], C->nc, xs)) !=
                             ncclSuccess)
                break;
        }
        const ncclResult_t r2 = R.GroupEnd();
        if (r != ncclSuccess) return nfail(r, "ncclSend/ncclRecv");
        if (r2 != ncclSuccess) return nfail(r2, "ncclGroupEnd");
    }
    return AIJHIP_OK;
}

}  // namespace

// Finish the exchange (host transport: the callback, then the ghost upload)
// and order s after it.
int halo_finish(aijhip_mpiaij *M, hipStream_t s) {
    aijhip_comm *C = M->comm;
    hipError_t e;
    if (!M->posted) return mfail(AIJHIP_ERR_STATE, "halo_finish without halo_post");
    M->posted = false;
    if (C->kind == AIJHIP_COMM_RCCL) {
        const int rc = halo_send_rccl(M);
        if (rc) return rc;
        // the serial form (the exchange enqueued on s itself): already in
        // order, no join; otherwise s waits for the stream post chose — the
        // stream recorded at post time, whatever stream finish is given
        if (M->post_s == s) return AIJHIP_OK;
        if ((e = hipEventRecord(M->ev_halo, M->post_s)) != hipSuccess) return mhip(e, "halo event");
    } else if (C->kind == AIJHIP_COMM_HOST) {
        const int64_t npack = M->halo == AIJHIP_HALO_ALLGATHER ? M->gather_len : M->n_send;
        int rc = wait_stream(C, M->xs);
        if (rc) return rc;
        int bad = 0;
        if (C->hsr && M->halo == AIJHIP_HALO_P2P) {
            // the library's own plan over the generic point-to-point callback
            // (operators the library made itself have no plan on the caller's
            // side); segments for this rank itself are local copies
            std::vector<int32_t> sp, rp;
            std::vector<int64_t> so{0}, ro{0};
            std::vector<double> sb, rb;
            for (size_t q = 0; q < M->send_peer.size(); ++q) {
                if (M->send_peer[q] == C->rank) continue;
                sp.push_back(M->send_peer[q]);
                sb.insert(sb.end(), M->h_send + M->send_off[q], M->h_send + M->send_off[q + 1]);
                so.push_back((int64_t)sb.size());
            }
            for (size_t pp = 0; pp < M->recv_peer.size(); ++pp) {
                if (M->recv_peer[pp] == C->rank) continue;
                rp.push_back(M->recv_peer[pp]);
                ro.push_back(ro.back() + (M->recv_off[pp + 1] - M->recv_off[pp]));
            }
            rb.resize((size_t)ro.back());
            bad = C->hsr(C->ctx, (int32_t)sp.size(), sp.data(), so.data(), sb.data(), (int32_t)rp.size(), rp.data(),
                         ro.data(), rb.data());
            for (size_t pp = 0, k = 0; !bad && pp < M->recv_peer.size(); ++pp) {
                const int64_t a = M->recv_off[pp], n = M->recv_off[pp + 1] - a;
                if (M->recv_peer[pp] == C->rank) {
                    for (size_t q = 0; q < M->send_peer.size(); ++q)
                        if (M->send_peer[q] == C->rank)
                            std::memcpy(M->h_ghost + a, M->h_send + M->send_off[q], sizeof(double) * (size_t)n);
                } else {
                    std::memcpy(M->h_ghost + a, rb.data() + ro[k], sizeof(double) * (size_t)n);
                    ++k;
                }
            }
        } else {
            bad = C->hex(C->ctx, M, M->h_send, npack, M->h_ghost, M->n_ghost);
        }
        if (bad != 0) {
            comm_abort(C);
            return mfail(AIJHIP_ERR_COMM, "host exchange callback failed");
        }
        if (M->n_ghost > 0 && (e = hipMemcpyAsync(M->d_ghost, M->h_ghost, sizeof(double) * (size_t)M->n_ghost,
                                                  hipMemcpyHostToDevice, M->xs)) != hipSuccess)
            return mhip(e, "ghost upload");
        if ((e = hipEventRecord(M->ev_halo, M->xs)) != hipSuccess) return mhip(e, "halo event");
    }
    if ((e = hipStreamWaitEvent(s, M->ev_halo, 0)) != hipSuccess) return mhip(e, "halo wait");
    return AIJHIP_OK;
}

// The exchange run backwards (PETSc's VecScatter SCATTER_REVERSE with
// ADD_VALUES, as MatMultTranspose_MPIAIJ uses it): each ghost slot's value
// goes to the slot's owner, which adds it to the row it sends for that slot
// — per peer in the plan's order, so the sums' order is fixed. On `s`, in
// order (no exchange stream). Collective over the operator's ranks.
int halo_reverse_add(aijhip_mpiaij *M, const double *d_gvals, double *y, hipStream_t s) {
    aijhip_comm *C = M->comm;
    if (C->aborted) return mfail(AIJHIP_ERR_COMM, "communicator aborted");
    if (M->halo != AIJHIP_HALO_P2P) return mfail(AIJHIP_ERR_ARG, "reverse exchange: p2p plans only");
    if (M->posted) return mfail(AIJHIP_ERR_STATE, "reverse exchange while an exchange is posted");
    hipError_t e;
    if (C->kind == AIJHIP_COMM_RCCL) {
        const Rccl &R = rccl();
        ncclResult_t r;
        if ((r = R.GroupStart()) != ncclSuccess) return nfail(r, "ncclGroupStart");
        for (size_t p = 0; r == ncclSuccess && p < M->recv_peer.size(); ++p) {
            const int64_t a = M->recv_off[p], n = M->recv_off[p + 1] - a;
            if (n > 0) r = R.Send(d_gvals + a, (size_t)n, ncclFloat64, M->recv_peer[p], C->nc, s);
        }
        for (size_t q = 0; r == ncclSuccess && q < M->send_peer.size(); ++q) {
            const int64_t a = M->send_off[q], n = M->send_off[q + 1] - a;
            if (n > 0) r = R.Recv(M->d_sendbuf + a, (size_t)n, ncclFloat64, M->send_peer[q], C->nc, s);
        }
        const ncclResult_t r2 = R.GroupEnd();
        if (r != ncclSuccess) return nfail(r, "ncclSend/ncclRecv (reverse)");
        if (r2 != ncclSuccess) return nfail(r2, "ncclGroupEnd (reverse)");
    } else {
        if (!C->hsr) return mfail(AIJHIP_ERR_STATE, "host transport without a sendrecv callback");
        if (M->n_ghost > 0 &&
            (e = hipMemcpyAsync(M->h_ghost, d_gvals, sizeof(double) * (size_t)M->n_ghost, hipMemcpyDeviceToHost, s)) !=
                hipSuccess)
            return mhip(e, "reverse exchange staging");
        int rc = wait_stream(C, s);
        if (rc) return rc;
        std::vector<int32_t> sp, rp;
        std::vector<int64_t> so{0}, ro{0};
        std::vector<double> sb, rb;
        const double *self = nullptr;
        for (size_t p = 0; p < M->recv_peer.size(); ++p) {
            if (M->recv_peer[p] == C->rank) {
                self = M->h_ghost + M->recv_off[p];
                continue;
            }
            sp.push_back(M->recv_peer[p]);
            sb.insert(sb.end(), M->h_ghost + M->recv_off[p], M->h_ghost + M->recv_off[p + 1]);
            so.push_back((int64_t)sb.size());
        }
        for (size_t q = 0; q < M->send_peer.size(); ++q) {
            if (M->send_peer[q] == C->rank) continue;
            rp.push_back(M->send_peer[q]);
            ro.push_back(ro.back() + (M->send_off[q + 1] - M->send_off[q]));
        }
        rb.resize((size_t)ro.back());
        if (C->hsr(C->ctx, (int32_t)sp.size(), sp.data(), so.data(), sb.data(), (int32_t)rp.size(), rp.data(),
                   ro.data(), rb.data()) != 0) {
            comm_abort(C);
            return mfail(AIJHIP_ERR_COMM, "host sendrecv callback failed (reverse exchange)");
        }
        for (size_t q = 0, k = 0; q < M->send_peer.size(); ++q) {
            const int64_t a = M->send_off[q], n = M->send_off[q + 1] - a;
            if (M->send_peer[q] == C->rank) {
                if (n > 0 && self) std::memcpy(M->h_send + a, self, sizeof(double) * (size_t)n);
            } else {
                std::memcpy(M->h_send + a, rb.data() + ro[k], sizeof(double) * (size_t)n);
                ++k;
            }
        }
        if (M->n_send > 0 && (e = hipMemcpyAsync(M->d_sendbuf, M->h_send, sizeof(double) * (size_t)M->n_send,
                                                 hipMemcpyHostToDevice, s)) != hipSuccess)
            return mhip(e, "reverse exchange upload");
    }
    for (size_t q = 0; q < M->send_peer.size(); ++q) {
        const int64_t a = M->send_off[q], n = M->send_off[q + 1] - a;
        if (n > 0)
            hipLaunchKernelGGL(k_add_rows, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, n, M->d_send_rows + a,
                               M->d_sendbuf + a, y);
    }
    e = hipGetLastError();
    return e == hipSuccess ? AIJHIP_OK : mhip(e, "reverse exchange add");
}

int halo_abort(aijhip_mpiaij *M, hipStream_t s, int rc) {
    if (M->posted) {
        const std::string why = aijhip_last_error();  // keep the first failure's message
        (void)halo_finish(M, s);
        aijhip::set_error(why);
    }
    return rc;
}

// y = A_d x + A_o g; with dot: W = y and the p.w partials (p = x) into
// part (A_d blocks, fused when A_d's plan allows) and opart (A_o rows).
int mpiaij_apply(aijhip_mpiaij *M, const double *x, double *y, hipStream_t s, double *part, double *opart,
                 const CGState *S, bool fused, const int *stop) {
    // nothing to send or receive (one rank, or a block with no coupling):
    // no exchange, no second stream
    const bool exchange = M->n_send > 0 || M->n_ghost > 0 || M->halo == AIJHIP_HALO_ALLGATHER;
    int rc = exchange ? halo_post(M, x, s) : AIJHIP_OK;
    if (rc) return rc;
    hipError_t e;
    if (M->fault_ad) e = hipErrorInvalidValue;
    else if (part && fused) e = aijhip::launch_stream_dot(*M->Ad, x, y, part, S ? &S->done : nullptr, s);
    else e = aijhip::launch_mult(*M->Ad, x, nullptr, y, false, s, stop);
    if (e != hipSuccess) return exchange ? halo_abort(M, s, mhip(e, "A_d product")) : mhip(e, "A_d product");
    if (exchange && (rc = halo_finish(M, s))) return rc;
    if (M->Ao) {
        const aijhip::RowList L = aijhip::row_list(*M->Ao);
        if (part) {
            if (L.nr > 0)
                hipLaunchKernelGGL(k_offdiag, dim3(M->o_grid), dim3(kVecThreads), 0, s, L.nr, L.rai, L.ridx,
                                   M->Ao->d_aj, M->Ao->d_aa, M->d_ghost, x, y, opart, S);
            e = hipGetLastError();
        } else {
            e = aijhip::launch_mult(*M->Ao, M->d_ghost, y, y, true, s, stop);  // MatMultAdd_SeqAIJ(A_o, g, y, y)
        }
        if (e != hipSuccess) return mhip(e, "A_o product");
    }
    return AIJHIP_OK;
}

}  // namespace aijhip_mpi

struct aijhip_kspmpi {
    aijhip_mpiaij *M = nullptr;
    double rtol = 1e-5, abstol = 1e-50, dtol = 1e5;
    int32_t max_it = 10000;
    int pc = AIJHIP_PC_JACOBI;
    int normtype = AIJHIP_KSP_NORM_PRECONDITIONED;
    int32_t poll = 8;
    bool set_up = false, fused = false;
    // the blocks' plan and values generations at set-up: new values or a
    // re-plan (on every rank: MatAssemblyEnd is collective) redo the set-up,
    // as PETSc's PCSetUp does when the operator's state changed
    uint64_t gens[4] = {0, 0, 0, 0};
    // PC GAMG = PETSc's -pc_type bjacobi -sub_pc_type gamg: a GAMG hierarchy of
    // this rank's diagonal block (a single-GPU KSP's set-up), one V-cycle per
    // application, no communication inside the preconditioner
    aijhip_ksp_t sub = nullptr;
    // PC GAMG across ranks (gamg_mpi.hip)
    aijhip_gamg_mpi::Hierarchy *dh = nullptr;
    double setup_seconds = 0.0;
    aijhip_gamg_params_t gamg{};
    bool gamg_set = false;
    int vec_grid = 1, n_dparts = 1;
    double *d_dinv = nullptr, *d_r = nullptr, *d_z = nullptr, *d_p = nullptr, *d_part = nullptr,
           *d_opart = nullptr, *d_red = nullptr, *d_hist = nullptr;
    int32_t hist_cap = 0;
    CGState *d_state = nullptr, *h_state = nullptr;
    int32_t its = 0, host_syncs = 0;
    int reason = 0;
    double rnorm = 0.0;
    std::vector<double> hist;
    // The poll batch (poll iterations) captured once into a HIP graph and
    // replayed by one hipGraphLaunch (aijhip_kspmpi_set_graph): the RCCL
    // enqueues of the halo and the all-reduces (15-25 us of host time per
    // call, profiles/r05/a/) leave the iteration. 0 off (default), 1 on
    // (RCCL only: the host transport waits on the host).
    int graph = 0;
    hipStream_t gs = nullptr;  // the capture stream (the caller's may be the legacy one)
    hipGraphExec_t gexec = nullptr;
    const double *g_x = nullptr;  // what the captured batch baked in
    int32_t g_poll = 0;
    uint64_t g_key = 0;
    int32_t graph_batches = 0;  // batches the last solve replayed
};

namespace {

void kspmpi_free(aijhip_kspmpi *K) {
    if (K->gexec) (void)hipGraphExecDestroy(K->gexec);
    K->gexec = nullptr;
    K->g_x = nullptr;
    hipFree(K->d_dinv); hipFree(K->d_r); hipFree(K->d_z); hipFree(K->d_p); hipFree(K->d_part);
    hipFree(K->d_opart); hipFree(K->d_red); hipFree(K->d_hist); hipFree(K->d_state);
    if (K->h_state) hipHostFree(K->h_state);
    if (K->sub) aijhip_ksp_destroy(K->sub);
    K->sub = nullptr;
    if (K->dh) {
        K->dh->destroy();
        delete K->dh;
        K->dh = nullptr;
    }
    K->d_dinv = K->d_r = K->d_z = K->d_p = K->d_part = K->d_opart = K->d_red = K->d_hist = nullptr;
    K->d_state = K->h_state = nullptr;
    K->set_up = false;
}

void block_gens(const aijhip_mpiaij *M, uint64_t g[4]) {
    g[0] = M->Ad->plan_gen;
    g[1] = M->Ad->values_gen;
    g[2] = M->Ao ? M->Ao->plan_gen : 0;
    g[3] = M->Ao ? M->Ao->values_gen : 0;
}

int kspmpi_set_up(aijhip_kspmpi *K) {
    uint64_t g[4];
    block_gens(K->M, g);
    if (K->set_up && std::equal(g, g + 4, K->gens)) return AIJHIP_OK;
    const auto t_setup = std::chrono::steady_clock::now();
    kspmpi_free(K);
    aijhip_mpiaij *M = K->M;
    aijhip_mat *A = M->Ad;
    const int64_t m = A->m;
    K->fused = aijhip::stream_dot_fusable(*A);
    K->vec_grid = (int)std::max<int64_t>(1, std::min<int64_t>((m + kVecThreads - 1) / kVecThreads,
                                                              (int64_t)A->n_cu * 8));
    K->n_dparts = K->fused ? std::max(1, A->plan.n_blocks) : K->vec_grid;
    const int64_t nparts = std::max<int64_t>((int64_t)kNQ * K->vec_grid, K->n_dparts);
    K->hist_cap = K->max_it + 2;
    const size_t vb = sizeof(double) * (size_t)std::max<int64_t>(m, 1);
    hipError_t e;
    if ((e = hipMalloc(&K->d_dinv, vb)) != hipSuccess || (e = hipMalloc(&K->d_r, vb)) != hipSuccess ||
        (e = hipMalloc(&K->d_z, vb)) != hipSuccess || (e = hipMalloc(&K->d_p, vb)) != hipSuccess ||
        (e = hipMalloc(&K->d_part, sizeof(double) * (size_t)nparts)) != hipSuccess ||
        (e = hipMalloc(&K->d_opart, sizeof(double) * (size_t)M->o_grid)) != hipSuccess ||
        (e = hipMalloc(&K->d_red, sizeof(double) * 8)) != hipSuccess ||
        (e = hipMalloc(&K->d_hist, sizeof(double) * (size_t)K->hist_cap)) != hipSuccess ||
        (e = hipMalloc(&K->d_state, sizeof(CGState))) != hipSuccess ||
        (e = hipHostMalloc(&K->h_state, sizeof(CGState), hipHostMallocDefault)) != hipSuccess) {
        kspmpi_free(K);
        return mhip(e, "KSPSetUp (distributed) allocation");
    }
    if (m > 0) {
        hipLaunchKernelGGL(k_diag_inv, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, nullptr, A->m, A->d_ai,
                           A->d_aj, A->d_aa, K->d_dinv);
        if ((e = hipGetLastError()) != hipSuccess || (e = hipDeviceSynchronize()) != hipSuccess) {
            kspmpi_free(K);
            return mhip(e, "PCSetUp_Jacobi (distributed)");
        }
    }
    // GAMG across ranks: more than one rank (AIJHIP_GAMG_DIST=1 forces the
    // distributed set-up at one rank too, for tests)
    const char *force = std::getenv("AIJHIP_GAMG_DIST");
    const bool dist = K->pc == AIJHIP_PC_GAMG && (M->comm->nranks > 1 || (force && std::atoi(force) != 0));
    if (dist) {
        aijhip_gamg_params_t gp;
        if (K->gamg_set) gp = K->gamg;
        else aijhip_gamg_params_default(&gp);
        K->dh = new (std::nothrow) aijhip_gamg_mpi::Hierarchy();
        int rc = K->dh ? aijhip_gamg_mpi::build(M, gp, *K->dh) : mfail(AIJHIP_ERR_ALLOC, "host allocation");
        if (rc) {
            kspmpi_free(K);
            return rc;
        }
    } else if (K->pc == AIJHIP_PC_GAMG || K->pc == AIJHIP_PC_BJACOBI_GAMG) {
        // PCSetUp_BJacobi + the sub-PC's PCSetUp_GAMG on A_d (at one rank: PCGAMG itself)
        int rc = aijhip_ksp_create(A, &K->sub);
        if (!rc) rc = aijhip_ksp_set_pc_type(K->sub, AIJHIP_PC_GAMG);
        if (!rc && K->gamg_set) rc = aijhip_ksp_set_gamg_params(K->sub, &K->gamg);
        if (!rc) rc = aijhip_ksp_set_up(K->sub);
        if (rc) {
            kspmpi_free(K);
            return rc;
        }
    }
    K->setup_seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t_setup).count();
    K->set_up = true;
    std::copy(g, g + 4, K->gens);
    return AIJHIP_OK;
}

// z = B r with the GAMG PC: the distributed hierarchy or the per-rank one.
// *dots: the fused finest post-smoothing's z.z / z.r partials, or NULL.
// stop: CG's flag, NULL for the V-cycle before the first scalar step (the
// device state is initialised by that step).
int pc_gamg_apply(aijhip_kspmpi *K, hipStream_t s, const double **dots, int *nbz, const int *stop) {
    *dots = nullptr;
    *nbz = 0;
    if (K->dh) return aijhip_gamg_mpi::vcycle(*K->dh, K->d_r, K->d_z, s, stop);
    const hipError_t e = aijhip::ksp_pc_vcycle(K->sub, K->d_r, K->d_z, s, dots, nbz, stop);
    return e == hipSuccess ? AIJHIP_OK : mhip(e, "GAMG V-cycle");
}

}  // namespace

extern "C" {

// ---------------------------------------------------------------- comm
int aijhip_comm_rccl_unique_id(unsigned char id[128]) {
    if (!id) return mfail(AIJHIP_ERR_ARG, "NULL id");
    const Rccl &R = rccl();
    if (!R.ok) return mfail(AIJHIP_ERR_COMM, "RCCL unavailable: " + R.why);
    ncclUniqueId u;
    const ncclResult_t r = R.GetUniqueId(&u);
    if (r != ncclSuccess) return nfail(r, "ncclGetUniqueId");
    std::memcpy(id, u.internal, NCCL_UNIQUE_ID_BYTES);
    return AIJHIP_OK;
}

static int comm_new(int kind, int32_t nranks, int32_t rank, int32_t device, aijhip_comm **out) {
    if (!out) return mfail(AIJHIP_ERR_ARG, "out is NULL");
    *out = nullptr;
    if (nranks < 1 || rank < 0 || rank >= nranks) return mfail(AIJHIP_ERR_ARG, "bad rank / size");
    int ndev = aijhip::visible_devices();
    if (device < 0 || device >= ndev) return mfail(AIJHIP_ERR_NODEVICE, "no such device");
    aijhip_comm *C = new (std::nothrow) aijhip_comm();
    if (!C) return mfail(AIJHIP_ERR_ALLOC, "host allocation");
    C->kind = kind; C->nranks = nranks; C->rank = rank; C->device = device;
    DeviceGuard g(device);
    hipError_t e;
    if ((e = hipEventCreateWithFlags(&C->ev_wait, hipEventDisableTiming)) != hipSuccess ||
        (e = hipHostMalloc(&C->h_red, sizeof(double) * kMaxRed, hipHostMallocDefault)) != hipSuccess) {
        if (C->ev_wait) hipEventDestroy(C->ev_wait);
        delete C;
        return mhip(e, "communicator set-up");
    }
    *out = C;
    return AIJHIP_OK;
}

int aijhip_comm_destroy(aijhip_comm_t C) {
    if (!C) return AIJHIP_OK;
    {
        DeviceGuard g(C->device);
        if (C->kind == AIJHIP_COMM_RCCL && C->nc) rccl().CommDestroy(C->nc);
        if (C->xs) hipStreamDestroy(C->xs);
        if (C->ev_wait) hipEventDestroy(C->ev_wait);
        if (C->h_red) hipHostFree(C->h_red);
    }
    delete C;
    return AIJHIP_OK;
}

int aijhip_comm_create_rccl(const unsigned char id[128], int32_t nranks, int32_t rank, int32_t device,
                            aijhip_comm_t *out) {
    if (!id) return mfail(AIJHIP_ERR_ARG, "NULL id");
    const Rccl &R = rccl();
    if (!R.ok) return mfail(AIJHIP_ERR_COMM, "RCCL unavailable: " + R.why);
    aijhip_comm *C = nullptr;
    int rc = comm_new(AIJHIP_COMM_RCCL, nranks, rank, device, &C);
    if (rc) return rc;
    DeviceGuard g(device);
    ncclUniqueId u;
    std::memcpy(u.internal, id, NCCL_UNIQUE_ID_BYTES);
    ncclResult_t r = R.CommInitRank(&C->nc, nranks, u, rank);
    if (r != ncclSuccess) {
        C->nc = nullptr;
        aijhip_comm_destroy(C);
        return nfail(r, "ncclCommInitRank");
    }
    R.GetVersion(&C->version);
    *out = C;
    return AIJHIP_OK;
}

int aijhip_comm_create_host(int32_t nranks, int32_t rank, int32_t device, aijhip_host_allreduce_fn allreduce,
                            aijhip_host_exchange_fn exchange, void *ctx, aijhip_comm_t *out) {
    if (!allreduce || !exchange) return mfail(AIJHIP_ERR_ARG, "NULL callback");
    aijhip_comm *C = nullptr;
    int rc = comm_new(AIJHIP_COMM_HOST, nranks, rank, device, &C);
    if (rc) return rc;
    C->har = allreduce;
    C->hex = exchange;
    C->ctx = ctx;
    *out = C;
    return AIJHIP_OK;
}

int aijhip_comm_set_host_sendrecv(aijhip_comm_t C, aijhip_host_sendrecv_fn fn) {
    if (!C) return mfail(AIJHIP_ERR_ARG, "NULL comm");
    if (C->kind != AIJHIP_COMM_HOST) return mfail(AIJHIP_ERR_ARG, "not a host-transport communicator");
    C->hsr = fn;
    return AIJHIP_OK;
}

int aijhip_comm_info(aijhip_comm_t C, int32_t *nranks, int32_t *rank, int32_t *kind, int32_t *version) {
    if (!C) return mfail(AIJHIP_ERR_ARG, "NULL comm");
    if (nranks) *nranks = C->nranks;
    if (rank) *rank = C->rank;
    if (kind) *kind = C->kind;
    if (version) *version = C->version;
    return AIJHIP_OK;
}

int aijhip_comm_allreduce_sum(aijhip_comm_t C, double *d_buf, int32_t n, void *stream) {
    if (!C || (n > 0 && !d_buf) || n < 0) return mfail(AIJHIP_ERR_ARG, "bad all-reduce arguments");
    DeviceGuard g(C->device);
    return comm_allreduce(C, d_buf, n, reinterpret_cast<hipStream_t>(stream));
}

int aijhip_comm_set_timeout(aijhip_comm_t C, double seconds) {
    if (!C) return mfail(AIJHIP_ERR_ARG, "NULL comm");
    C->timeout_s = seconds;
    return AIJHIP_OK;
}

// ---------------------------------------------------- MatMult_MPIAIJ
int aijhip_mpiaij_create(aijhip_comm_t comm, aijhip_mat_t A_d, aijhip_mat_t A_o, int32_t halo, int32_t n_send,
                         const int32_t *send_peer, const int64_t *send_off, const int32_t *send_rows,
                         int32_t n_recv, const int32_t *recv_peer, const int64_t *recv_off, int32_t gather_len,
                         aijhip_mpiaij_t *out) {
    if (!out) return mfail(AIJHIP_ERR_ARG, "out is NULL");
    *out = nullptr;
    if (!comm || !A_d) return mfail(AIJHIP_ERR_ARG, "NULL comm or diagonal block");
    if (A_d->m != A_d->n) return mfail(AIJHIP_ERR_ARG, "diagonal block must be square");
    if (A_d->device != comm->device || (A_o && A_o->device != comm->device))
        return mfail(AIJHIP_ERR_ARG, "blocks and communicator on different devices");
    if (A_o && A_o->m != A_d->m) return mfail(AIJHIP_ERR_ARG, "off-diagonal block row count");
    if (halo != AIJHIP_HALO_P2P && halo != AIJHIP_HALO_ALLGATHER) return mfail(AIJHIP_ERR_ARG, "bad halo kind");
    if (n_send < 0 || n_recv < 0 || (n_send > 0 && (!send_peer || !send_off)) ||
        (halo == AIJHIP_HALO_P2P && n_recv > 0 && (!recv_peer || !recv_off)))
        return mfail(AIJHIP_ERR_ARG, "bad exchange plan");
    aijhip_mpiaij *M = new (std::nothrow) aijhip_mpiaij();
    if (!M) return mfail(AIJHIP_ERR_ALLOC, "host allocation");
    M->comm = comm; M->Ad = A_d; M->Ao = A_o; M->halo = halo; M->mloc = A_d->m;
    M->overlap = auto_overlap();
    if (const char *f = std::getenv("AIJHIP_FAULT_AD_RANK")) M->fault_ad = std::atoi(f) == comm->rank;
    auto bad = [&](const std::string &msg) {
        mpiaij_free(M);
        delete M;
        return mfail(AIJHIP_ERR_ARG, msg);
    };
    M->send_off.assign(1, 0);
    std::vector<int32_t> rows;
    if (n_send > 0) {
        if (send_off[0] != 0) return bad("send_off[0] must be 0");
        for (int32_t q = 0; q < n_send; ++q) {
            const int64_t a = send_off[q], b = send_off[q + 1];
            if (b < a || (b > a && !send_rows)) return bad("bad send_off");
            if (halo == AIJHIP_HALO_P2P && (send_peer[q] < 0 || send_peer[q] >= comm->nranks))
                return bad("bad send peer");
            bool contig = b > a;
            for (int64_t i = a; i < b; ++i) {
                if (send_rows[i] < 0 || send_rows[i] >= A_d->m) return bad("send row out of range");
                if (i > a && send_rows[i] != send_rows[i - 1] + 1) contig = false;
            }
            M->send_peer.push_back(send_peer[q]);
            M->send_off.push_back(b);
            M->send_first.push_back(contig ? send_rows[a] : -1);
        }
        rows.assign(send_rows, send_rows + send_off[n_send]);
        M->h_send_rows = rows;
    }
    M->n_send = M->send_off.back();
    if (halo == AIJHIP_HALO_ALLGATHER) {
        if (n_send > 1 || gather_len < std::max<int64_t>(M->n_send, 1)) return bad("all-gather plan");
        M->gather_len = gather_len;
        M->n_ghost = (int64_t)gather_len * comm->nranks;
    } else {
        M->recv_off.assign(1, 0);
        if (n_recv > 0 && recv_off[0] != 0) return bad("recv_off[0] must be 0");
        for (int32_t p = 0; p < n_recv; ++p) {
            if (recv_off[p + 1] < recv_off[p]) return bad("bad recv_off");
            if (recv_peer[p] < 0 || recv_peer[p] >= comm->nranks)
                return bad("bad recv peer");
            M->recv_peer.push_back(recv_peer[p]);
            M->recv_off.push_back(recv_off[p + 1]);
        }
        M->n_ghost = M->recv_off.back();
    }
    if (A_o && A_o->n != std::max<int64_t>(M->n_ghost, 1) && A_o->n != M->n_ghost)
        return bad("off-diagonal block columns != ghost length");
    M->pack_all = comm->kind == AIJHIP_COMM_HOST;
    DeviceGuard g(comm->device);
    hipError_t e = hipSuccess;
    const int64_t nbuf = std::max<int64_t>(1, halo == AIJHIP_HALO_ALLGATHER ? M->gather_len : M->n_send);
    const int64_t ng = std::max<int64_t>(1, M->n_ghost);
    if ((e = hipMalloc(&M->d_send_rows, sizeof(int32_t) * (size_t)std::max<int64_t>(1, M->n_send))) != hipSuccess ||
        (e = hipMalloc(&M->d_sendbuf, sizeof(double) * (size_t)nbuf)) != hipSuccess ||
        (e = hipMalloc(&M->d_ghost, sizeof(double) * (size_t)ng)) != hipSuccess ||
        (e = hipMemset(M->d_ghost, 0, sizeof(double) * (size_t)ng)) != hipSuccess ||
        (e = hipMemset(M->d_sendbuf, 0, sizeof(double) * (size_t)nbuf)) != hipSuccess ||
        (M->n_send > 0 && (e = hipMemcpy(M->d_send_rows, rows.data(), sizeof(int32_t) * (size_t)M->n_send,
                                         hipMemcpyHostToDevice)) != hipSuccess) ||
        (e = hipStreamCreateWithFlags(&M->xs, hipStreamNonBlocking)) != hipSuccess ||
        (e = hipEventCreateWithFlags(&M->ev_x, aijhip::sync_event_flags())) != hipSuccess ||
        (e = hipEventCreateWithFlags(&M->ev_halo, aijhip::sync_event_flags())) != hipSuccess ||
        (M->pack_all && ((e = hipHostMalloc(&M->h_send, sizeof(double) * (size_t)nbuf, hipHostMallocDefault)) !=
                             hipSuccess ||
                         (e = hipHostMalloc(&M->h_ghost, sizeof(double) * (size_t)ng, hipHostMallocDefault)) !=
                             hipSuccess))) {
        mpiaij_free(M);
        delete M;
        return mhip(e, "MPIAIJ set-up");
    }
    if (A_o) {
        const aijhip::RowList L = aijhip::row_list(*A_o);
        M->o_grid = grid_of(L.nr, A_o->n_cu * 4);
    }
    *out = M;
    return AIJHIP_OK;
}

int aijhip_mpiaij_mult(aijhip_mpiaij_t M, const double *x, double *y, void *stream) {
    if (!M) return mfail(AIJHIP_ERR_ARG, "NULL matrix");
    if (M->mloc > 0 && (!x || !y)) return mfail(AIJHIP_ERR_ARG, "NULL vector");
    if (x == y) return mfail(AIJHIP_ERR_ARG, "x and y alias");
    DeviceGuard g(M->comm->device);
    return mpiaij_apply(M, x, y, reinterpret_cast<hipStream_t>(stream), nullptr, nullptr, nullptr, false);
}

int aijhip_mpiaij_set_overlap(aijhip_mpiaij_t M, int overlap) {
    if (!M) return mfail(AIJHIP_ERR_ARG, "NULL matrix");
    if (overlap < -1 || overlap > 1)
        return mfail(AIJHIP_ERR_ARG, "overlap: -1 (automatic), 0 (one stream) or 1 (exchange stream)");
    if (M->posted) return mfail(AIJHIP_ERR_STATE, "an exchange is posted");
    M->overlap = overlap >= 0 ? overlap : auto_overlap();
    return AIJHIP_OK;
}

int aijhip_mpiaij_get_overlap(aijhip_mpiaij_t M, int32_t *overlap, int32_t *hw_queues) {
    if (!M) return mfail(AIJHIP_ERR_ARG, "NULL matrix");
    if (overlap) *overlap = M->overlap;
    if (hw_queues) *hw_queues = aijhip::hw_queues();
    return AIJHIP_OK;
}

int aijhip_mpiaij_get_ghost(aijhip_mpiaij_t M, const double **ghost, int64_t *n) {
    if (!M) return mfail(AIJHIP_ERR_ARG, "NULL matrix");
    if (ghost) *ghost = M->d_ghost;
    if (n) *n = M->n_ghost;
    return AIJHIP_OK;
}

int aijhip_mpiaij_destroy(aijhip_mpiaij_t M) {
    if (!M) return AIJHIP_OK;
    {
        DeviceGuard g(M->comm->device);
        (void)hipStreamSynchronize(M->xs);
        mpiaij_free(M);
    }
    delete M;
    return AIJHIP_OK;
}

// ------------------------------------------------- KSPSolve_CG over it
int aijhip_kspmpi_create(aijhip_mpiaij_t M, aijhip_kspmpi_t *out) {
    if (!out) return mfail(AIJHIP_ERR_ARG, "out is NULL");
    *out = nullptr;
    if (!M) return mfail(AIJHIP_ERR_ARG, "NULL operator");
    if (M->Ad->compressed) return mfail(AIJHIP_ERR_ARG, "diagonal block in compressed-row form");
    aijhip_kspmpi *K = new (std::nothrow) aijhip_kspmpi();
    if (!K) return mfail(AIJHIP_ERR_ALLOC, "host allocation");
    K->M = M;
    *out = K;
    return AIJHIP_OK;
}

int aijhip_kspmpi_set_tolerances(aijhip_kspmpi_t K, double rtol, double abstol, double dtol, int32_t max_it) {
    if (!K) return mfail(AIJHIP_ERR_ARG, "NULL ksp");
    if (rtol < 0 || abstol < 0 || dtol <= 0 || max_it < 0) return mfail(AIJHIP_ERR_ARG, "bad tolerance");
    K->rtol = rtol; K->abstol = abstol; K->dtol = dtol;
    K->max_it = max_it;
    if (K->set_up && max_it + 2 > K->hist_cap) {  // regrow the history only (keeps dinv and the sub-PC)
        DeviceGuard g(K->M->comm->device);
        hipFree(K->d_hist);
        K->d_hist = nullptr;
        K->hist_cap = max_it + 2;
        if (hipMalloc(&K->d_hist, sizeof(double) * (size_t)K->hist_cap) != hipSuccess) {
            K->set_up = false;
            return mfail(AIJHIP_ERR_ALLOC, "residual history");
        }
    }
    return AIJHIP_OK;
}

int aijhip_kspmpi_set_pc_type(aijhip_kspmpi_t K, int pc) {
    if (!K) return mfail(AIJHIP_ERR_ARG, "NULL ksp");
    if (pc != AIJHIP_PC_NONE && pc != AIJHIP_PC_JACOBI && pc != AIJHIP_PC_GAMG && pc != AIJHIP_PC_BJACOBI_GAMG)
        return mfail(AIJHIP_ERR_ARG, "distributed CG: PC none, jacobi, gamg or bjacobi_gamg");
    // PCGAMG across ranks builds every level's exchange from the operator's
    // p2p plan: refuse an all-gather-halo operator here, with the way out,
    // rather than at KSPSetUp
    if (pc == AIJHIP_PC_GAMG && K->M->comm->nranks > 1 && K->M->halo != AIJHIP_HALO_P2P)
        return mfail(AIJHIP_ERR_ARG,
                     "PC gamg across ranks needs the operator's p2p halo: create a p2p twin of this all-gather "
                     "operator sharing A_d (aijhip_mpiaij_create with AIJHIP_HALO_P2P; mpiaij.MPIAIJ.p2p_native()), "
                     "or use AIJHIP_PC_BJACOBI_GAMG");
    if (pc != K->pc) K->set_up = false;
    K->pc = pc;
    if (pc == AIJHIP_PC_GAMG || pc == AIJHIP_PC_BJACOBI_GAMG)  // the set-up's streams, made once per process
        for (int slot = 0; slot < 2; ++slot) (void)aijhip_gamg::setup_stream(K->M->comm->device, slot);
    return AIJHIP_OK;
}

int aijhip_kspmpi_set_gamg_params(aijhip_kspmpi_t K, const aijhip_gamg_params_t *p) {
    if (!K) return mfail(AIJHIP_ERR_ARG, "NULL ksp");
    K->gamg_set = p != nullptr;
    if (p) K->gamg = *p;
    if (K->pc == AIJHIP_PC_GAMG) K->set_up = false;
    return AIJHIP_OK;
}

int aijhip_kspmpi_set_norm_type(aijhip_kspmpi_t K, int nt) {
    if (!K) return mfail(AIJHIP_ERR_ARG, "NULL ksp");
    if (nt < AIJHIP_KSP_NORM_NONE || nt > AIJHIP_KSP_NORM_NATURAL) return mfail(AIJHIP_ERR_ARG, "bad norm type");
    K->normtype = nt;
    return AIJHIP_OK;
}

int aijhip_kspmpi_set_poll_interval(aijhip_kspmpi_t K, int32_t iters) {
    if (!K || iters < 1) return mfail(AIJHIP_ERR_ARG, "bad poll interval");
    K->poll = iters;
    return AIJHIP_OK;
}

int aijhip_kspmpi_set_graph(aijhip_kspmpi_t K, int mode) {
    if (!K || mode < -1 || mode > 1) return mfail(AIJHIP_ERR_ARG, "graph: -1 auto, 0 off, 1 on");
    K->graph = mode;
    return AIJHIP_OK;
}

int aijhip_kspmpi_get_graph_batches(aijhip_kspmpi_t K, int32_t *batches) {
    if (!K || !batches) return mfail(AIJHIP_ERR_ARG, "NULL argument");
    *batches = K->graph_batches;
    return AIJHIP_OK;
}

int aijhip_kspmpi_solve(aijhip_kspmpi_t K, const double *b, double *x, void *stream) {
    aijhip::Range range("KSPSolve (MPIAIJ)");
    if (!K) return mfail(AIJHIP_ERR_ARG, "NULL ksp");
    aijhip_mpiaij *M = K->M;
    aijhip_comm *C = M->comm;
    DeviceGuard g(C->device);
    int rc = kspmpi_set_up(K);
    if (rc) return rc;
    const int64_t m = M->mloc;
    if (m > 0 && (!b || !x)) return mfail(AIJHIP_ERR_ARG, "NULL vector");
    if (b == x) return mfail(AIJHIP_ERR_ARG, "b and x alias");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const bool multi = C->nranks > 1;
    CGParams p{K->rtol, K->abstol, K->dtol, K->max_it, K->normtype, 1, K->pc};
    const dim3 vg(K->vec_grid), vt(kVecThreads), rt(kRedThreads);
    const int nb = K->vec_grid;
    const double *dinv = K->pc == AIJHIP_PC_JACOBI ? K->d_dinv : nullptr;
    const int64_t waits0 = C->waits;
    hipError_t e = hipSuccess;
    if (m > 0 && (e = hipMemsetAsync(x, 0, sizeof(double) * (size_t)m, s)) != hipSuccess) return mhip(e, "x = 0");
    // r = b, z = B r, then ||z|| etc. summed over all ranks
    const bool gamg = K->pc == AIJHIP_PC_GAMG || K->pc == AIJHIP_PC_BJACOBI_GAMG;
    hipLaunchKernelGGL(k_init, vg, vt, 0, s, m, b, K->d_r, K->d_z, dinv, K->d_part, p);
    if (gamg) {  // z = B r, then its z.z, z.r partials (as ksp.hip with a zero guess)
        const double *dots = nullptr;
        int nbz = 0;
        if ((rc = pc_gamg_apply(K, s, &dots, &nbz, nullptr))) return rc;
        hipLaunchKernelGGL(k_dots, vg, vt, 0, s, m, K->d_z, K->d_r, K->d_part, 0, 1, nullptr);
    }
    hipLaunchKernelGGL(k_local_sums, dim3(1), rt, 0, s, K->d_part, nb, 4, K->d_red, multi ? 0 : 1, K->d_state,
                       K->d_hist, p);
    if (multi) {
        if ((rc = comm_allreduce(C, K->d_red, 4, s))) return rc;
        hipLaunchKernelGGL(k_step_init, dim3(1), dim3(64), 0, s, K->d_red, K->d_state, K->d_hist, p);
    }
    if ((e = hipGetLastError()) != hipSuccess) return mhip(e, "KSPSolve init");
    const bool have_o = M->Ao && aijhip::row_list(*M->Ao).nr > 0;
    // The A_o correction partials (p_o w_o(new) - p_o w_o(old)) complete p.w
    // only when the A_d epilogue summed p_o w_o(old), i.e. in the fused path;
    // otherwise k_dot sums p.w over the final w and the A_o rows are already
    // in it (counting them twice broke conjugacy).
    double *opart = (have_o && K->fused) ? K->d_opart : nullptr;
    const int nob = opart ? M->o_grid : 0;
    // one CG iteration on stream st (every kernel returns at once past the
    // device stop flag; every collective is issued on every rank regardless)
    auto iteration = [&](hipStream_t st) -> int {
        int r;
        hipLaunchKernelGGL(k_aypx<true>, vg, vt, 0, st, m, K->d_z, K->d_p, x, K->d_state);
        // W = A P with the p.w partials (W shares Z's storage)
        if ((r = mpiaij_apply(M, K->d_p, K->d_z, st, K->d_part, opart, K->d_state, K->fused))) return r;
        if (!K->fused) hipLaunchKernelGGL(k_dot, vg, vt, 0, st, m, K->d_p, K->d_z, K->d_part, K->d_state);
        hipLaunchKernelGGL(k_local_dpi, dim3(1), rt, 0, st, K->d_part, K->n_dparts, opart, nob, K->d_red,
                           K->d_state, multi ? 0 : 1);
        if (multi) {
            if ((r = comm_allreduce(C, K->d_red, 1, st))) return r;
            hipLaunchKernelGGL(k_step_dpi, dim3(1), dim3(64), 0, st, K->d_red, K->d_state);
        }
        hipLaunchKernelGGL(k_update<true>, vg, vt, 0, st, m, K->d_r, K->d_z, dinv, K->d_part, K->d_state, K->pc,
                           K->d_p, nullptr);
        if (gamg) {  // z = B r; z.z and z.r from the fused finest post-smoothing, else k_dots
            const double *dots = nullptr;
            int nbz = 0;
            if ((r = pc_gamg_apply(K, st, &dots, &nbz, &K->d_state->done))) return r;
            if (!dots) {
                hipLaunchKernelGGL(k_dots, vg, vt, 0, st, m, K->d_z, K->d_r, K->d_part, 0, 1, K->d_state);
                dots = K->d_part;
                nbz = nb;
            }
            hipLaunchKernelGGL(k_local_iter, dim3(1), rt, 0, st, dots, nbz, K->d_part + 2 * nb, nb, K->d_red,
                               multi ? 0 : 1, K->d_state, K->d_hist, p);
        } else {
            hipLaunchKernelGGL(k_local_sums, dim3(1), rt, 0, st, K->d_part, nb, 3, K->d_red, multi ? 0 : 2,
                               K->d_state, K->d_hist, p);
        }
        if (multi) {
            if ((r = comm_allreduce(C, K->d_red, 3, st))) return r;
            hipLaunchKernelGGL(k_step_iter, dim3(1), dim3(64), 0, st, K->d_red, K->d_state, K->d_hist, p);
        }
        const hipError_t le = hipGetLastError();
        return le == hipSuccess ? AIJHIP_OK : mhip(le, "KSPSolve iteration");
    };
    // the poll batch as a HIP graph: RCCL only (the host transport waits on
    // the host inside the exchanges); captured on the handle's own stream
    // and re-captured when what it baked in changes (x, the batch length,
    // the tolerances and norm, the set-up)
    const bool use_graph = C->kind == AIJHIP_COMM_RCCL && K->graph == 1;  // (-1: the default, off)
    static const bool gdbg = std::getenv("AIJHIP_GRAPH_DEBUG") != nullptr;
    auto dbg = [&](const char *what) {
        if (gdbg) std::fprintf(stderr, "[kspmpi graph, rank %d] %s\n", C->rank, what);
    };
    uint64_t key = 1469598103934665603ULL;
    for (double v : {p.rtol, p.abstol, p.dtol})
        key = (key ^ std::hash<double>{}(v)) * 1099511628211ULL;
    key = (key ^ (uint64_t)(uint32_t)p.max_it ^ ((uint64_t)(uint32_t)p.normtype << 32) ^
           ((uint64_t)(uint32_t)p.pc << 40)) * 1099511628211ULL;
    key = (key ^ K->gens[0] ^ (K->gens[1] << 1) ^ (K->gens[2] << 2) ^ (K->gens[3] << 3) ^
           (uint64_t)(uintptr_t)K->d_state) * 1099511628211ULL;
    K->graph_batches = 0;
    int32_t launched = 0;
    for (;;) {
        if ((e = hipMemcpyAsync(K->h_state, K->d_state, sizeof(CGState), hipMemcpyDeviceToHost, s)) != hipSuccess)
            return mhip(e, "KSPSolve poll");
        if ((rc = wait_stream(C, s))) return rc;
        if (use_graph) dbg("polled");
        if (K->h_state->done || launched >= K->max_it) break;
        const int32_t poll = K->poll;  // every CG and V-cycle kernel returns at once past the flag
        if (use_graph && K->max_it - launched >= poll) {
            if (!K->gexec || K->g_x != x || K->g_poll != poll || K->g_key != key) {
                if (K->gexec) (void)hipGraphExecDestroy(K->gexec);
                K->gexec = nullptr;
                if (!K->gs && (e = hipStreamCreateWithFlags(&K->gs, hipStreamNonBlocking)) != hipSuccess)
                    return mhip(e, "KSPSolve capture stream");
                dbg("begin capture");
                if ((e = hipStreamBeginCapture(K->gs, hipStreamCaptureModeRelaxed)) != hipSuccess)
                    return mhip(e, "KSPSolve capture");
                int crc = AIJHIP_OK;
                aijhip_mpi::g_capturing = true;
                for (int j = 0; j < poll && !crc; ++j) {
                    crc = iteration(K->gs);
                    dbg("iteration captured");
                }
                aijhip_mpi::g_capturing = false;
                hipGraph_t graph = nullptr;
                e = hipStreamEndCapture(K->gs, &graph);
                dbg(e == hipSuccess ? "end capture" : "end capture failed");
                if (!crc && e == hipSuccess) e = hipGraphInstantiate(&K->gexec, graph, nullptr, nullptr, 0);
                dbg(e == hipSuccess ? "instantiated" : "instantiate failed");
                if (graph) (void)hipGraphDestroy(graph);
                if (crc) return crc;
                if (e != hipSuccess) {
                    K->gexec = nullptr;
                    return mhip(e, "KSPSolve capture (end / instantiate)");
                }
                K->g_x = x;
                K->g_poll = poll;
                K->g_key = key;
            }
            if ((e = hipGraphLaunch(K->gexec, s)) != hipSuccess) return mhip(e, "KSPSolve graph launch");
            dbg("batch launched");
            launched += poll;
            ++K->graph_batches;
            continue;
        }
        for (int j = 0; j < poll && launched < K->max_it; ++j, ++launched)
            if ((rc = iteration(s))) return rc;
    }
    hipLaunchKernelGGL(k_final_x, vg, vt, 0, s, m, K->d_p, x, K->d_state);
    if ((e = hipGetLastError()) != hipSuccess ||
        (e = hipMemcpyAsync(K->h_state, K->d_state, sizeof(CGState), hipMemcpyDeviceToHost, s)) != hipSuccess)
        return mhip(e, "KSPSolve final update");
    if ((rc = wait_stream(C, s))) return rc;
    K->host_syncs = (int32_t)(C->waits - waits0);
    const CGState &st = *K->h_state;
    K->its = st.its;
    K->reason = st.reason ? st.reason : AIJHIP_KSP_DIVERGED_ITS;
    K->rnorm = st.dp;
    const int32_t nh = std::min<int32_t>(K->hist_cap, st.its + 1);
    K->hist.resize((size_t)std::max(nh, 0));
    if (nh > 0 &&
        (e = hipMemcpy(K->hist.data(), K->d_hist, sizeof(double) * (size_t)nh, hipMemcpyDeviceToHost)) != hipSuccess)
        return mhip(e, "residual history");
    return AIJHIP_OK;
}

int aijhip_kspmpi_get_iteration_number(aijhip_kspmpi_t K, int32_t *its) {
    if (!K || !its) return mfail(AIJHIP_ERR_ARG, "NULL argument");
    *its = K->its;
    return AIJHIP_OK;
}

int aijhip_kspmpi_get_residual_norm(aijhip_kspmpi_t K, double *rnorm) {
    if (!K || !rnorm) return mfail(AIJHIP_ERR_ARG, "NULL argument");
    *rnorm = K->rnorm;
    return AIJHIP_OK;
}

int aijhip_kspmpi_get_converged_reason(aijhip_kspmpi_t K, int *reason) {
    if (!K || !reason) return mfail(AIJHIP_ERR_ARG, "NULL argument");
    *reason = K->reason;
    return AIJHIP_OK;
}

int aijhip_kspmpi_get_residual_history(aijhip_kspmpi_t K, double *hist, int32_t na, int32_t *n) {
    if (!K || !n || (na > 0 && !hist)) return mfail(AIJHIP_ERR_ARG, "NULL argument");
    const int32_t c = std::min<int32_t>(na, (int32_t)K->hist.size());
    std::copy(K->hist.begin(), K->hist.begin() + c, hist);
    *n = c;
    return AIJHIP_OK;
}

int aijhip_kspmpi_get_host_syncs(aijhip_kspmpi_t K, int32_t *n) {
    if (!K || !n) return mfail(AIJHIP_ERR_ARG, "NULL argument");
    *n = K->host_syncs;
    return AIJHIP_OK;
}

int aijhip_kspmpi_get_pc_levels(aijhip_kspmpi_t K, int32_t *nlevels, int64_t *rows, int64_t *nnz, int32_t cap) {
    if (!K || !nlevels) return mfail(AIJHIP_ERR_ARG, "NULL argument");
    if (!K->set_up) return mfail(AIJHIP_ERR_STATE, "KSP not set up");
    if (K->dh) {
        const auto &lv = K->dh->lv;
        *nlevels = (int32_t)lv.size();
        const int32_t n = std::min<int32_t>(cap, *nlevels);
        std::vector<double> z((size_t)std::max(n, 1), 0.0);
        for (int32_t l = 0; l < n; ++l) {
            if (rows) rows[l] = lv[l].starts.back();
            z[l] = (double)lv[l].Ad->nz + (lv[l].Ao ? (double)lv[l].Ao->nz : 0.0);
        }
        DeviceGuard g(K->M->comm->device);
        for (int32_t l0 = 0; l0 < n; l0 += 64) {  // the host transport reduces 64 values at a time
            const int32_t c = std::min<int32_t>(64, n - l0);
            int rc = aijhip_mpi::comm_allreduce_host(K->M->comm, z.data() + l0, c);
            if (rc) return rc;
        }
        for (int32_t l = 0; l < n; ++l)
            if (nnz) nnz[l] = (int64_t)z[l];
        return AIJHIP_OK;
    }
    if (K->sub) {
        std::vector<int32_t> r((size_t)std::max(cap, 1));
        std::vector<int64_t> z((size_t)std::max(cap, 1));
        int rc = aijhip_ksp_get_pc_levels(K->sub, nlevels, r.data(), z.data(), cap, nullptr);
        if (rc) return rc;
        for (int32_t l = 0; l < std::min(cap, *nlevels); ++l) {
            if (rows) rows[l] = r[l];
            if (nnz) nnz[l] = z[l];
        }
        return AIJHIP_OK;
    }
    *nlevels = 1;
    if (cap > 0 && rows) rows[0] = K->M->mloc;
    if (cap > 0 && nnz) nnz[0] = K->M->Ad->nz + (K->M->Ao ? K->M->Ao->nz : 0);
    return AIJHIP_OK;
}

int aijhip_kspmpi_get_pc_level(aijhip_kspmpi_t K, int32_t l, char which, int64_t *rstart, int32_t *m, int64_t *nnz,
                               int64_t *ai, int64_t *aj, double *aa) {
    if (!K || !rstart || !m || !nnz) return mfail(AIJHIP_ERR_ARG, "NULL argument");
    if (!K->set_up || !K->dh) return mfail(AIJHIP_ERR_STATE, "no distributed GAMG hierarchy (set up a GAMG solve)");
    DeviceGuard g(K->M->comm->device);
    std::vector<int64_t> vi, vj;
    std::vector<double> va;
    const int rc = aijhip_gamg_mpi::get_level(*K->dh, l, which, rstart, m, vi, vj, va);
    if (rc) return rc;
    *nnz = (int64_t)vj.size();
    if (ai) std::copy(vi.begin(), vi.end(), ai);
    if (aj) std::copy(vj.begin(), vj.end(), aj);
    if (aa) std::copy(va.begin(), va.end(), aa);
    return AIJHIP_OK;
}

int aijhip_kspmpi_get_setup_seconds(aijhip_kspmpi_t K, double *seconds) {
    if (!K || !seconds) return mfail(AIJHIP_ERR_ARG, "NULL argument");
    *seconds = K->setup_seconds;
    return AIJHIP_OK;
}

int aijhip_kspmpi_destroy(aijhip_kspmpi_t K) {
    if (!K) return AIJHIP_OK;
    {
        DeviceGuard g(K->M->comm->device);
        (void)hipDeviceSynchronize();
        kspmpi_free(K);
        if (K->gs) (void)hipStreamDestroy(K->gs);
    }
    delete K;
    return AIJHIP_OK;
}

}  // extern "C"
