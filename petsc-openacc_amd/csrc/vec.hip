// vec.hip — device vector operations of the Krylov path (include/aijhip_vec.h).
// The arithmetic is that of ksp.hip's fused CG kernels; the reductions write
// one partial per workgroup, summed in workgroup order by a second
// single-workgroup kernel, into device doubles.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <mutex>
#include <string>
#include <vector>

#include "aijhip_internal.h"
#include "aijhip_vec.h"

namespace {

constexpr int kThreads = 256;
constexpr int kMaxBlocks = 2048;  // partials per quantity
constexpr int kRedThreads = 1024;

template <int T>
__device__ __forceinline__ double bsum(double v, double *scratch) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
    const int t = threadIdx.x;
    __syncthreads();
    if ((t & 63) == 0) scratch[t >> 6] = v;
    __syncthreads();
    double s = 0.0;
    if (t == 0) {
#pragma unroll
        for (int w = 0; w < T / 64; ++w) s += scratch[w];
    }
    __syncthreads();
    return s;
}

#define GRID_STRIDE(i, n) \
    for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < (n); i += (int64_t)gridDim.x * kThreads)

__global__ __launch_bounds__(kThreads) void k_aypx(int64_t n, double beta, const double *__restrict__ x, double *y) {
    GRID_STRIDE(i, n) y[i] = x[i] + beta * y[i];
}

__global__ __launch_bounds__(kThreads) void k_dot(int64_t n, const double *__restrict__ x,
                                                  const double *__restrict__ y, double *part) {
    __shared__ double scratch[kThreads / 64];
    double s = 0.0;
    GRID_STRIDE(i, n) s += x[i] * y[i];
    const double v = bsum<kThreads>(s, scratch);
    if (threadIdx.x == 0) part[blockIdx.x] = v;
}

// x += a p; r += (-a) w; z = dinv r; partials z.z, z.r, r.r (ksp.hip k_update)
__global__ __launch_bounds__(kThreads) void k_cg_update(int64_t n, double a, double *x, const double *__restrict__ p,
                                                        double *r, const double *w, double *z,
                                                        const double *__restrict__ dinv, double *part) {
    __shared__ double scratch[kThreads / 64];
    const double na = -a;
    double zz = 0.0, zr = 0.0, rr = 0.0;
    GRID_STRIDE(i, n) {
        x[i] = x[i] + a * p[i];
        const double ri = r[i] + na * w[i];
        r[i] = ri;
        const double zi = dinv ? dinv[i] * ri : ri;
        z[i] = zi;
        zz += zi * zi;
        zr += zi * ri;
        rr += ri * ri;
    }
    const int nb = gridDim.x;
    double v;
    v = bsum<kThreads>(zz, scratch); if (threadIdx.x == 0) part[0 * nb + blockIdx.x] = v;
    v = bsum<kThreads>(zr, scratch); if (threadIdx.x == 0) part[1 * nb + blockIdx.x] = v;
    v = bsum<kThreads>(rr, scratch); if (threadIdx.x == 0) part[2 * nb + blockIdx.x] = v;
}

__global__ __launch_bounds__(kThreads) void k_jacobi(int64_t n, const double *__restrict__ r,
                                                     const double *__restrict__ dinv, double *z, double *part) {
    __shared__ double scratch[kThreads / 64];
    double zz = 0.0, zr = 0.0, rr = 0.0;
    GRID_STRIDE(i, n) {
        const double ri = r[i];
        const double zi = dinv ? dinv[i] * ri : ri;
        z[i] = zi;
        zz += zi * zi;
        zr += zi * ri;
        rr += ri * ri;
    }
    const int nb = gridDim.x;
    double v;
    v = bsum<kThreads>(zz, scratch); if (threadIdx.x == 0) part[0 * nb + blockIdx.x] = v;
    v = bsum<kThreads>(zr, scratch); if (threadIdx.x == 0) part[1 * nb + blockIdx.x] = v;
    v = bsum<kThreads>(rr, scratch); if (threadIdx.x == 0) part[2 * nb + blockIdx.x] = v;
}

// out[q] = sum of part[q*nb .. q*nb+nb) in a fixed order, q < nq
__global__ __launch_bounds__(kRedThreads) void k_finish(const double *part, int nb, int nq, double *out) {
    __shared__ double scratch[kRedThreads / 64];
    for (int q = 0; q < nq; ++q) {
        double s = 0.0;
        for (int j = threadIdx.x; j < nb; j += kRedThreads) s += part[q * nb + j];
        s = bsum<kRedThreads>(s, scratch);
        if (threadIdx.x == 0) out[q] = s;
    }
}

__global__ void k_diag_inv(int32_t m, const int32_t *__restrict__ ai, const int32_t *__restrict__ aj,
                           const double *__restrict__ aa, double *dinv) {
    const int32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= m) return;
    double d = 0.0;
    for (int32_t k = ai[r]; k < ai[r + 1]; ++k)
        if (aj[k] == r) { d = aa[k]; break; }
    if (d == 0.0) d = 1.0;
    dinv[r] = 1.0 / d;
}

// Partials scratch per device: kMaxBlocks x 3 doubles, allocated once.
// Calls on one device are expected from one host thread at a time (PETSc
// objects are not thread-safe either); streams order the reuse.
double *partials(hipError_t *e) {
    static std::mutex mu;
    static std::vector<double *> per_dev;
    int dev = 0;
    if ((*e = hipGetDevice(&dev)) != hipSuccess) return nullptr;
    std::lock_guard<std::mutex> lock(mu);
    if ((int)per_dev.size() <= dev) per_dev.resize(dev + 1, nullptr);
    if (!per_dev[dev]) *e = hipMalloc(&per_dev[dev], sizeof(double) * 3 * kMaxBlocks);
    return per_dev[dev];
}

// HBM read ceiling: n doubles read once by 512-lane workgroups, each a
// contiguous tile of U 16-B loads per lane issued before any use, a partial
// sum per workgroup so no load is dropped. tools/read_sweep.hip measured the
// shapes: non-temporal loads with U = 2 read fastest (7.3 TB/s at 2.8 GB);
// U = 4 plain loads is the STREAM kernel's own shape (6.1 TB/s).
constexpr int kProbeThreads = 512;
template <int U, bool NT>
__global__ __launch_bounds__(kProbeThreads) void k_read_probe(int64_t n2, const double2 *__restrict__ v,
                                                              double *part) {
    __shared__ double scratch[kProbeThreads / 64];
    const int64_t base = (int64_t)blockIdx.x * kProbeThreads * U + threadIdx.x;
    double2 r[U];
#pragma unroll
    for (int it = 0; it < U; ++it) {
        const int64_t i = base + (int64_t)it * kProbeThreads;
        if (i < n2) {
            if constexpr (NT) {
                r[it].x = __builtin_nontemporal_load(&v[i].x);
                r[it].y = __builtin_nontemporal_load(&v[i].y);
            } else {
                r[it] = v[i];
            }
        } else {
            r[it] = make_double2(0.0, 0.0);
        }
    }
    double s = 0.0;
#pragma unroll
    for (int it = 0; it < U; ++it) s += r[it].x + r[it].y;
    const double t = bsum<kProbeThreads>(s, scratch);
    if (threadIdx.x == 0) part[blockIdx.x & (kMaxBlocks - 1)] = t;
}

int grid_for(int64_t n) {
    return (int)std::max<int64_t>(1, std::min<int64_t>((n + kThreads - 1) / kThreads, kMaxBlocks));
}

int verr(int code, const std::string &msg) {
    aijhip::set_error(msg);
    return code;
}

int vhip(hipError_t e, const char *what) {
    return e == hipSuccess ? AIJHIP_OK : verr(AIJHIP_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

}  // namespace

extern "C" {

int aijhip_vec_aypx(int64_t n, double beta, const double *x, double *y, void *stream) {
    if (n < 0 || (n > 0 && (!x || !y))) return verr(AIJHIP_ERR_ARG, "vec_aypx: bad arguments");
    if (n == 0) return AIJHIP_OK;
    hipLaunchKernelGGL(k_aypx, dim3(grid_for(n)), dim3(kThreads), 0, (hipStream_t)stream, n, beta, x, y);
    return vhip(hipGetLastError(), "vec_aypx");
}

int aijhip_vec_dot(int64_t n, const double *x, const double *y, double *d_result, void *stream) {
    if (n < 0 || !d_result || (n > 0 && (!x || !y))) return verr(AIJHIP_ERR_ARG, "vec_dot: bad arguments");
    hipError_t e;
    double *part = partials(&e);
    if (!part) return vhip(e, "vec_dot scratch");
    const int nb = grid_for(n);
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(k_dot, dim3(nb), dim3(kThreads), 0, s, n, x, y, part);
    hipLaunchKernelGGL(k_finish, dim3(1), dim3(kRedThreads), 0, s, part, nb, 1, d_result);
    return vhip(hipGetLastError(), "vec_dot");
}

int aijhip_vec_cg_update(int64_t n, double alpha, double *x, const double *p, double *r, const double *w,
                         double *z, const double *dinv, double *d_result, void *stream) {
    if (n < 0 || !d_result || (n > 0 && (!x || !p || !r || !w || !z)))
        return verr(AIJHIP_ERR_ARG, "vec_cg_update: bad arguments");
    hipError_t e;
    double *part = partials(&e);
    if (!part) return vhip(e, "vec_cg_update scratch");
    const int nb = grid_for(n);
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(k_cg_update, dim3(nb), dim3(kThreads), 0, s, n, alpha, x, p, r, w, z, dinv, part);
    hipLaunchKernelGGL(k_finish, dim3(1), dim3(kRedThreads), 0, s, part, nb, 3, d_result);
    return vhip(hipGetLastError(), "vec_cg_update");
}

int aijhip_vec_jacobi(int64_t n, const double *r, const double *dinv, double *z, double *d_result, void *stream) {
    if (n < 0 || !d_result || (n > 0 && (!r || !z))) return verr(AIJHIP_ERR_ARG, "vec_jacobi: bad arguments");
    hipError_t e;
    double *part = partials(&e);
    if (!part) return vhip(e, "vec_jacobi scratch");
    const int nb = grid_for(n);
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(k_jacobi, dim3(nb), dim3(kThreads), 0, s, n, r, dinv, z, part);
    hipLaunchKernelGGL(k_finish, dim3(1), dim3(kRedThreads), 0, s, part, nb, 3, d_result);
    return vhip(hipGetLastError(), "vec_jacobi");
}

int aijhip_read_probe(const double *d_buf, int64_t n, int mode, void *stream) {
    if (n < 0 || (n > 0 && !d_buf) || ((uintptr_t)d_buf & 15) || mode < 0 || mode > 1)
        return verr(AIJHIP_ERR_ARG, "read_probe: bad arguments");
    if (n < 2) return AIJHIP_OK;
    hipError_t e;
    double *part = partials(&e);
    if (!part) return vhip(e, "read_probe scratch");
    const int64_t n2 = n / 2;
    const double2 *v = reinterpret_cast<const double2 *>(d_buf);
    hipStream_t s = (hipStream_t)stream;
    if (mode == 0) {
        const int64_t per = (int64_t)kProbeThreads * 2;
        hipLaunchKernelGGL((k_read_probe<2, true>), dim3((unsigned)((n2 + per - 1) / per)), dim3(kProbeThreads), 0, s,
                           n2, v, part);
    } else {
        const int64_t per = (int64_t)kProbeThreads * 4;
        hipLaunchKernelGGL((k_read_probe<4, false>), dim3((unsigned)((n2 + per - 1) / per)), dim3(kProbeThreads), 0,
                           s, n2, v, part);
    }
    return vhip(hipGetLastError(), "read_probe");
}

// One wave that returns after `ticks` of the constant-rate wall clock (a
// bounded loop: it exits on the clock whatever else runs).
__global__ __launch_bounds__(64) void k_delay_probe(uint64_t ticks) {
    const uint64_t t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}

int aijhip_delay_probe(double us, void *stream) {
    if (!(us >= 0.0) || us > 1e6) return verr(AIJHIP_ERR_ARG, "delay_probe: 0 <= us <= 1e6");
    static int khz = 0;  // wall-clock rate (kHz), queried once
    if (khz == 0) {
        int dev = 0, v = 0;
        hipError_t e = hipGetDevice(&dev);
        if (e == hipSuccess) e = hipDeviceGetAttribute(&v, hipDeviceAttributeWallClockRate, dev);
        if (e != hipSuccess || v <= 0) return vhip(e != hipSuccess ? e : hipErrorInvalidValue, "delay_probe clock");
        khz = v;
    }
    hipLaunchKernelGGL(k_delay_probe, dim3(1), dim3(64), 0, (hipStream_t)stream, (uint64_t)(us * khz / 1000.0));
    return vhip(hipGetLastError(), "delay_probe");
}

int aijhip_mat_jacobi_inverse(aijhip_mat_t A, double *d_dinv, void *stream) {
    if (!A || !d_dinv) return verr(AIJHIP_ERR_ARG, "mat_jacobi_inverse: NULL argument");
    if (A->m == 0) return AIJHIP_OK;
    if (A->compressed) return verr(AIJHIP_ERR_ARG, "mat_jacobi_inverse: compressed-row matrix");
    hipLaunchKernelGGL(k_diag_inv, dim3((unsigned)((A->m + 255) / 256)), dim3(256), 0, (hipStream_t)stream, A->m,
                       A->d_ai, A->d_aj, A->d_aa, d_dinv);
    return vhip(hipGetLastError(), "mat_jacobi_inverse");
}

}  // extern "C"
