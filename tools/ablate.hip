// DIAGNOSTIC ONLY (not the product): ablations of the STREAM SpMV kernel to
// find where its time goes (cdna_hip_programming.md §7 "Ablate"). Every
// variant keeps the block geometry of the product's default (1024 lanes,
// 8192-entry row blocks) and touches the same arrays; each drops one part.
//   0 full          — the product's arithmetic (same as k_spmv_stream)
//   1 no_gather     — product uses aj as a value instead of x[aj]  (no x traffic)
//   2 no_reduce     — gathers + LDS stores, but phase 2 writes prod[t] only
//   3 matrix_only   — aa/aj block loads summed per lane, one store per lane
//   4 flat_matrix   — grid-stride 16 B aa + 8 B aj loads (no blocks, no rows)
//   5 flat_read_aa  — grid-stride 16 B loads of aa only (ceiling reference)
// Build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/ablate.hip -o tools/libablate.so
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef double f64x2 __attribute__((ext_vector_type(2)));
typedef int i32x2 __attribute__((ext_vector_type(2)));

struct BlockDesc { int32_t row0, nrows, k0, nk; };

constexpr int T = 1024, CAP = 8192, ITERS = (CAP + 1 + 2 * T - 1) / (2 * T);

template <int MODE>
__global__ __launch_bounds__(T) void k_ablate(const BlockDesc *__restrict__ blk,
                                              const int32_t *__restrict__ rai,
                                              const int32_t *__restrict__ aj,
                                              const double *__restrict__ aa,
                                              const double *__restrict__ x, double *y) {
    __shared__ double prod[CAP];
    const BlockDesc d = blk[blockIdx.x];
    const int t = threadIdx.x;
    const int64_t k0 = d.k0, k1 = (int64_t)d.k0 + d.nk, kb = k0 & ~int64_t(1);
    int32_t rs = 0, re = 0;
    if (t < d.nrows) { rs = rai[d.row0 + t]; re = rai[d.row0 + t + 1]; }
    f64x2 av[ITERS];
    i32x2 cv[ITERS];
#pragma unroll
    for (int it = 0; it < ITERS; ++it) {
        const int64_t k = kb + 2 * (int64_t)(t + it * T);
        if (k < k1) {
            av[it] = *reinterpret_cast<const f64x2 *>(aa + k);
            cv[it] = *reinterpret_cast<const i32x2 *>(aj + k);
        }
    }
    if (MODE == 3) {
        double s = 0.0;
#pragma unroll
        for (int it = 0; it < ITERS; ++it) {
            const int64_t k = kb + 2 * (int64_t)(t + it * T);
            if (k < k1) s += av[it].x + av[it].y + (double)(cv[it].x + cv[it].y);
        }
        if (t < d.nrows) y[d.row0 + t] = s + rs + re;
        return;
    }
#pragma unroll
    for (int it = 0; it < ITERS; ++it) {
        const int64_t k = kb + 2 * (int64_t)(t + it * T);
        if (k < k1) {
            const double x0 = MODE == 1 ? (double)cv[it].x : x[cv[it].x];
            const double x1 = MODE == 1 ? (double)cv[it].y : x[cv[it].y];
            if (k >= k0) prod[k - k0] = av[it].x * x0;
            if (k + 1 < k1) prod[k + 1 - k0] = av[it].y * x1;
        }
    }
    __syncthreads();
    if (t < d.nrows) {
        double s = 0.0;
        if (MODE == 2) s = prod[t] + rs + re;
        else for (int32_t k = rs; k < re; ++k) s += prod[k - k0];
        y[d.row0 + t] = s;
    }
}

template <int MODE>
__global__ __launch_bounds__(256) void k_flat(int64_t nz, const int32_t *__restrict__ aj,
                                              const double *__restrict__ aa, double *y) {
    double s = 0.0;
    const int64_t n2 = nz / 2;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n2; i += (int64_t)gridDim.x * 256) {
        const f64x2 a = reinterpret_cast<const f64x2 *>(aa)[i];
        s += a.x + a.y;
        if (MODE == 4) {
            const i32x2 c = reinterpret_cast<const i32x2 *>(aj)[i];
            s += (double)(c.x + c.y);
        }
    }
    y[(int64_t)blockIdx.x * 256 + threadIdx.x] = s;
}

typedef int i32x4 __attribute__((ext_vector_type(4)));

// 6: flat, 4 entries per lane: aa as 2 x 16 B, aj as 16 B (no 8 B loads)
__global__ __launch_bounds__(256) void k_flat4(int64_t nz, const int32_t *__restrict__ aj,
                                               const double *__restrict__ aa, double *y) {
    double s = 0.0;
    const int64_t n4 = nz / 4;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
        const f64x2 a0 = reinterpret_cast<const f64x2 *>(aa)[2 * i];
        const f64x2 a1 = reinterpret_cast<const f64x2 *>(aa)[2 * i + 1];
        const i32x4 c = reinterpret_cast<const i32x4 *>(aj)[i];
        s += a0.x + a0.y + a1.x + a1.y + (double)(c.x + c.y + c.z + c.w);
    }
    y[(int64_t)blockIdx.x * 256 + threadIdx.x] = s;
}

// 7: block-structured matrix_only with 4 entries per lane (16 B loads only)
constexpr int ITERS4 = (CAP + 3 + 4 * T - 1) / (4 * T);
__global__ __launch_bounds__(T) void k_block4(const BlockDesc *__restrict__ blk,
                                              const int32_t *__restrict__ rai,
                                              const int32_t *__restrict__ aj,
                                              const double *__restrict__ aa, double *y) {
    const BlockDesc d = blk[blockIdx.x];
    const int t = threadIdx.x;
    const int64_t k0 = d.k0, k1 = (int64_t)d.k0 + d.nk, kb = k0 & ~int64_t(3);
    int32_t rs = 0, re = 0;
    if (t < d.nrows) { rs = rai[d.row0 + t]; re = rai[d.row0 + t + 1]; }
    double s = 0.0;
    f64x2 a0[ITERS4], a1[ITERS4];
    i32x4 c[ITERS4];
#pragma unroll
    for (int it = 0; it < ITERS4; ++it) {
        const int64_t k = kb + 4 * (int64_t)(t + it * T);
        if (k < k1) {
            a0[it] = *reinterpret_cast<const f64x2 *>(aa + k);
            a1[it] = *reinterpret_cast<const f64x2 *>(aa + k + 2);
            c[it] = *reinterpret_cast<const i32x4 *>(aj + k);
        }
    }
#pragma unroll
    for (int it = 0; it < ITERS4; ++it) {
        const int64_t k = kb + 4 * (int64_t)(t + it * T);
        if (k < k1) s += a0[it].x + a0[it].y + a1[it].x + a1[it].y + (double)(c[it].x + c[it].y + c[it].z + c[it].w);
    }
    if (t < d.nrows) y[d.row0 + t] = s + rs + re;
}

// Load-style study, full SpMV arithmetic, lanes TT, IT pair-iterations:
//  STYLE 0: loads under `if (k < k1)` (branchy, as k_ablate<0>)
//  STYLE 1: branch-free clamped loads + batched gathers (as the product)
//  STYLE 2: clamped loads guarded by a block-uniform iteration count
template <int TT, int IT, int STYLE>
__global__ __launch_bounds__(TT) void k_style(const BlockDesc *__restrict__ blk,
                                              const int32_t *__restrict__ rai,
                                              const int32_t *__restrict__ aj,
                                              const double *__restrict__ aa,
                                              const double *__restrict__ x, double *y) {
    __shared__ double prod[2 * TT * IT];
    const BlockDesc d = blk[blockIdx.x];
    const int t = threadIdx.x;
    const int64_t k0 = d.k0, k1 = (int64_t)d.k0 + d.nk, kb = k0 & ~int64_t(1);
    const int r = d.row0 + min(t, d.nrows - 1);
    const int32_t rs = rai[r], re = rai[r + 1];
    const int64_t klast = k1 > kb ? ((k1 - 1) & ~int64_t(1)) : kb;
    const int nit = (int)((k1 - kb + 2 * TT - 1) / (2 * TT));  // block-uniform
    f64x2 av[IT];
    i32x2 cv[IT];
    f64x2 xv[IT];
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        const int64_t k = kb + 2 * (int64_t)(t + it * TT);
        if (STYLE == 0) {
            if (k < k1) {
                av[it] = *reinterpret_cast<const f64x2 *>(aa + k);
                cv[it] = *reinterpret_cast<const i32x2 *>(aj + k);
            }
        } else if (STYLE == 1 || it < nit) {
            const int64_t kc = min(k, klast);
            av[it] = *reinterpret_cast<const f64x2 *>(aa + kc);
            cv[it] = *reinterpret_cast<const i32x2 *>(aj + kc);
        }
    }
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        const int64_t k = kb + 2 * (int64_t)(t + it * TT);
        if (STYLE == 0) {
            if (k < k1) {
                xv[it].x = x[cv[it].x];
                xv[it].y = x[cv[it].y];
            }
        } else if (STYLE == 1 || it < nit) {
            xv[it].x = x[cv[it].x];
            xv[it].y = x[cv[it].y];
        }
    }
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        const int64_t k = kb + 2 * (int64_t)(t + it * TT);
        if (k < k1) {
            if (k >= k0) prod[k - k0] = av[it].x * xv[it].x;
            if (k + 1 < k1) prod[k + 1 - k0] = av[it].y * xv[it].y;
        }
    }
    __syncthreads();
    if (t < d.nrows) {
        double s = 0.0;
        for (int32_t k = rs; k < re; ++k) s += prod[k - k0];
        y[d.row0 + t] = s;
    }
}

extern "C" int ablate_style(int tt, int it, int style, int nblk, const void *blk, const int32_t *rai,
                            const int32_t *aj, const double *aa, const double *x, double *y,
                            void *stream) {
    hipStream_t s = (hipStream_t)stream;
    const BlockDesc *b = (const BlockDesc *)blk;
#define ST(TT, IT, S)                                                                             \
    if (tt == TT && it == IT && style == S) {                                                     \
        hipLaunchKernelGGL((k_style<TT, IT, S>), dim3(nblk), dim3(TT), 0, s, b, rai, aj, aa, x, y); \
        return hipGetLastError() == hipSuccess ? 0 : 2;                                           \
    }
    ST(1024, 5, 0) ST(1024, 5, 1) ST(1024, 5, 2) ST(1024, 4, 0) ST(1024, 4, 1) ST(1024, 4, 2)
    ST(512, 4, 0) ST(512, 4, 1) ST(512, 4, 2) ST(512, 5, 1) ST(256, 4, 1) ST(256, 4, 2) ST(256, 4, 0)
#undef ST
    return 1;
}

extern "C" int ablate_launch(int mode, int nblk, const void *blk, const int32_t *rai,
                             const int32_t *aj, const double *aa, const double *x, double *y,
                             int64_t nz, void *stream) {
    hipStream_t s = (hipStream_t)stream;
    const BlockDesc *b = (const BlockDesc *)blk;
    switch (mode) {
        case 0: hipLaunchKernelGGL(k_ablate<0>, dim3(nblk), dim3(T), 0, s, b, rai, aj, aa, x, y); break;
        case 1: hipLaunchKernelGGL(k_ablate<1>, dim3(nblk), dim3(T), 0, s, b, rai, aj, aa, x, y); break;
        case 2: hipLaunchKernelGGL(k_ablate<2>, dim3(nblk), dim3(T), 0, s, b, rai, aj, aa, x, y); break;
        case 3: hipLaunchKernelGGL(k_ablate<3>, dim3(nblk), dim3(T), 0, s, b, rai, aj, aa, x, y); break;
        case 4: hipLaunchKernelGGL(k_flat<4>, dim3(256 * 8), dim3(256), 0, s, nz, aj, aa, y); break;
        case 5: hipLaunchKernelGGL(k_flat<5>, dim3(256 * 8), dim3(256), 0, s, nz, aj, aa, y); break;
        case 6: hipLaunchKernelGGL(k_flat4, dim3(256 * 8), dim3(256), 0, s, nz, aj, aa, y); break;
        case 7: hipLaunchKernelGGL(k_block4, dim3(nblk), dim3(T), 0, s, b, rai, aj, aa, y); break;
        default: return 1;
    }
    return hipGetLastError() == hipSuccess ? 0 : 2;
}
