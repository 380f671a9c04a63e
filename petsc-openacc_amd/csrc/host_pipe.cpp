// host_pipe.cpp — MatMult with host vectors (aijhip_mat_mult_host), the
// drop-in path an unchanged PETSc caller takes: x and y are
// the Vec arrays in host memory, the matrix is resident in HBM.
//
// The reference's answer to the PCIe cost is steps 3 and 4
// (/root/reference/src/openacc-step3/MatMult_SeqAIJ.patch:30-48: the CPU
// computes leading rows while x uploads asynchronously;
// /root/reference/src/openacc-step4/MatMult_SeqAIJ.patch:51-91: GPU rows in
// 983,040-row blocks on async queues so each block's y download overlaps the
// next block's compute). Here the whole product stays on the GPU and three
// HIP streams keep both PCIe directions and the CUs busy at once:
//
//   calling thread, h2d : upload x chunk i --> event x_i, then launch every
//   comp                :   row chunk c whose columns have arrived (wait
//                           x_need(c)) --> event c
//   y thread, d2h       : wait c -- download y chunk c
//
// Row chunk c multiplies as soon as the x chunk holding its largest column
// has arrived (banded operators: a few chunks behind the upload; a general
// matrix waits for all of x and still overlaps every y download). The y
// downloads are issued from a second host thread because a copy to pageable
// memory holds its issuing thread until the data has landed (the HIP runtime
// stages it): one thread per direction keeps both PCIe directions busy.
// Measured at 300^3 (profiles/r02/): staging through our own pinned slots
// with threaded memcpy was slower than the runtime's pageable path (15.0 vs
// 8.2 ms serial), so the chunks go straight from and to the caller's arrays.
// Results are bit-identical to aijhip_mat_mult: the same STREAM blocks run,
// only grouped into launches.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "aijhip_internal.h"

namespace aijhip {

namespace {

constexpr int32_t kDefaultChunkRows = 983040;  // step4 patch:51 block size (7.5 MiB of fp64)

struct Chunk {
    int32_t b0, nb;     // STREAM blocks
    int32_t row0, row1;  // rows (= y entries)
    int32_t need;       // last x chunk the rows read (-1: none)
};

}  // namespace

struct HostPipe {
    int32_t chunk_rows = 0;
    std::vector<Chunk> chunks;
    std::vector<int32_t> xoff;  // x chunk boundaries (size nxc + 1)
    hipStream_t h2d = nullptr, comp = nullptr, d2h = nullptr;
    std::vector<hipEvent_t> xev, cev;  // per x chunk uploaded, per row chunk computed
};

void host_pipe_free(HostPipe *p) {
    if (!p) return;
    for (hipEvent_t e : p->xev) (void)hipEventDestroy(e);
    for (hipEvent_t e : p->cev) (void)hipEventDestroy(e);
    if (p->h2d) (void)hipStreamDestroy(p->h2d);
    if (p->comp) (void)hipStreamDestroy(p->comp);
    if (p->d2h) (void)hipStreamDestroy(p->d2h);
    delete p;
}

namespace {

int pfail(int code, const std::string &msg) {
    set_error(msg);
    return code;
}

int phip(hipError_t e, const char *what) {
    set_error(std::string(what) + ": " + hipGetErrorString(e));
    return AIJHIP_ERR_HIP;
}

bool pipelinable(const aijhip_mat &A) {
    const Plan &P = A.plan;
    return P.kernel == AIJHIP_KERNEL_STREAM && !A.compressed && P.n_longs == 0 &&
           P.tune.host_chunk != 0 && P.n_blocks > 0;
}

// Chunks of whole STREAM blocks of >= chunk_rows rows; x split evenly into as
// many chunks; need(c) from the blocks' column ranges (non-decreasing).
int build(aijhip_mat *A, HostPipe **out) {
    const Plan &P = A->plan;
    std::vector<BlockDesc> blk((size_t)P.n_blocks);
    std::vector<int2> xr((size_t)P.n_blocks);
    int2 *d_xr = nullptr;
    hipError_t e = hipMalloc(&d_xr, sizeof(int2) * xr.size());
    if (e == hipSuccess) e = block_column_ranges(*A, P.d_blocks, P.n_blocks, d_xr);
    if (e == hipSuccess) e = hipMemcpy(xr.data(), d_xr, sizeof(int2) * xr.size(), hipMemcpyDeviceToHost);
    if (e == hipSuccess)
        e = hipMemcpy(blk.data(), P.d_blocks, sizeof(BlockDesc) * blk.size(), hipMemcpyDeviceToHost);
    hipFree(d_xr);
    if (e != hipSuccess) return phip(e, "host pipeline plan");
    HostPipe *p = new (std::nothrow) HostPipe();
    if (!p) return pfail(AIJHIP_ERR_ALLOC, "host allocation");
    p->chunk_rows = P.tune.host_chunk > 0 ? P.tune.host_chunk : kDefaultChunkRows;
    // row chunks
    std::vector<int32_t> col_hi;
    for (int32_t b = 0; b < P.n_blocks;) {
        Chunk c{b, 0, blk[(size_t)b].row0, blk[(size_t)b].row0, -1};
        int32_t hi = -1;
        while (b < P.n_blocks && (c.row1 - c.row0 < p->chunk_rows || c.nb == 0)) {
            const BlockDesc &d = blk[(size_t)b];
            c.row1 = d.row0 + d.nrows;
            if (xr[(size_t)b].y > 0) hi = std::max(hi, xr[(size_t)b].x + xr[(size_t)b].y - 1);
            ++c.nb;
            ++b;
        }
        p->chunks.push_back(c);
        col_hi.push_back(hi);
    }
    const int32_t nxc = std::max<int32_t>(1, (int32_t)((A->n + (int64_t)p->chunk_rows - 1) / p->chunk_rows));
    p->xoff.resize((size_t)nxc + 1);
    for (int32_t i = 0; i <= nxc; ++i) p->xoff[(size_t)i] = (int32_t)((int64_t)A->n * i / nxc);
    int32_t need = -1;
    for (size_t c = 0; c < p->chunks.size(); ++c) {
        if (col_hi[c] >= 0) {
            const int32_t i = (int32_t)(std::upper_bound(p->xoff.begin(), p->xoff.end(), col_hi[c]) - p->xoff.begin()) - 1;
            need = std::max(need, std::min(i, nxc - 1));
        }
        p->chunks[c].need = need;
    }
    p->xev.assign((size_t)nxc, nullptr);
    p->cev.assign(p->chunks.size(), nullptr);
    for (hipEvent_t &v : p->xev)
        if (e == hipSuccess) e = hipEventCreateWithFlags(&v, hipEventDisableTiming);
    for (hipEvent_t &v : p->cev)
        if (e == hipSuccess) e = hipEventCreateWithFlags(&v, hipEventDisableTiming);
    if (e == hipSuccess && (e = hipStreamCreateWithFlags(&p->h2d, hipStreamNonBlocking)) == hipSuccess &&
        (e = hipStreamCreateWithFlags(&p->comp, hipStreamNonBlocking)) == hipSuccess)
        e = hipStreamCreateWithFlags(&p->d2h, hipStreamNonBlocking);
    if (e != hipSuccess) {
        host_pipe_free(p);
        return phip(e, "host pipeline buffers");
    }
    *out = p;
    return AIJHIP_OK;
}

// The step-2 form: whole x in, one launch, whole y out (one stream).
int serial_mult(aijhip_mat *A, const double *x, double *y) {
    hipError_t e = hipSuccess;
    if (A->n > 0 && (e = hipMemcpyAsync(A->d_xstage, x, sizeof(double) * (size_t)A->n, hipMemcpyHostToDevice,
                                        A->host_stream)) != hipSuccess)
        return phip(e, "copy x in");
    if ((e = launch_mult(*A, A->d_xstage, nullptr, A->d_ystage, false, A->host_stream)) != hipSuccess)
        return phip(e, "MatMult launch");
    if ((e = hipMemcpyAsync(y, A->d_ystage, sizeof(double) * (size_t)A->m, hipMemcpyDeviceToHost, A->host_stream)) !=
            hipSuccess ||
        (e = hipStreamSynchronize(A->host_stream)) != hipSuccess)
        return phip(e, "copy y out");
    return AIJHIP_OK;
}

}  // namespace

int host_pipe_mult(aijhip_mat *A, const double *x, double *y) {
    if (!pipelinable(*A)) return serial_mult(A, x, y);
    Plan &P = A->plan;
    int rc;
    if (!P.hpipe && (rc = build(A, &P.hpipe))) return rc;
    HostPipe &p = *P.hpipe;
    const int32_t nxc = (int32_t)p.xoff.size() - 1, nc = (int32_t)p.chunks.size();
    // y side: downloads chunk c once its launch (and event) has been issued
    std::mutex mu;
    std::condition_variable cv;
    int32_t launched = 0;
    bool abort = false;
    hipError_t ye = hipSuccess;
    int dev = A->device;
    std::thread yt([&] {
        (void)hipSetDevice(dev);
        for (int32_t c = 0; c < nc && ye == hipSuccess; ++c) {
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return launched > c || abort; });
                if (launched <= c) break;  // the upload side failed: drain what was issued
            }
            const Chunk &k = p.chunks[(size_t)c];
            if ((ye = hipStreamWaitEvent(p.d2h, p.cev[(size_t)c], 0)) == hipSuccess)
                ye = hipMemcpyAsync(y + k.row0, A->d_ystage + k.row0, sizeof(double) * (size_t)(k.row1 - k.row0),
                                    hipMemcpyDeviceToHost, p.d2h);
        }
        const hipError_t se = hipStreamSynchronize(p.d2h);
        if (ye == hipSuccess) ye = se;
    });
    hipError_t e = hipSuccess;
    const char *what = nullptr;
    int32_t ci = 0;
    for (int32_t xi = 0; xi < nxc && e == hipSuccess; ++xi) {
        const int32_t a = p.xoff[(size_t)xi], n = p.xoff[(size_t)xi + 1] - a;
        if (n > 0 && (e = hipMemcpyAsync(A->d_xstage + a, x + a, sizeof(double) * (size_t)n, hipMemcpyHostToDevice,
                                         p.h2d)) != hipSuccess) {
            what = "x upload";
            break;
        }
        if ((e = hipEventRecord(p.xev[(size_t)xi], p.h2d)) != hipSuccess) {
            what = "x event";
            break;
        }
        for (; ci < nc && p.chunks[(size_t)ci].need <= xi; ++ci) {
            const Chunk &k = p.chunks[(size_t)ci];
            if ((e = hipStreamWaitEvent(p.comp, p.xev[(size_t)xi], 0)) != hipSuccess ||
                (e = launch_stream_blocks(*A, k.b0, k.nb, A->d_xstage, A->d_ystage, p.comp)) != hipSuccess ||
                (e = hipEventRecord(p.cev[(size_t)ci], p.comp)) != hipSuccess) {
                what = "row chunk";
                break;
            }
            {
                std::lock_guard<std::mutex> lk(mu);
                launched = ci + 1;
            }
            cv.notify_one();
        }
    }
    {
        std::lock_guard<std::mutex> lk(mu);
        abort = true;
    }
    cv.notify_one();
    yt.join();
    if (e != hipSuccess) return phip(e, what);
    if (ci != nc) return pfail(AIJHIP_ERR_STATE, "host pipeline: row chunks left unlaunched");
    if (ye != hipSuccess) return phip(ye, "y download");
    if ((e = hipStreamSynchronize(p.h2d)) != hipSuccess) return phip(e, "host pipeline drain");
    return AIJHIP_OK;
}

}  // namespace aijhip
