// spmv_ladder.hip — measurement tool (not product code): where the CSR
// MatMult's time goes on the 300^3 Poisson operand, one access pattern added
// per rung, every rung moving the same compulsory bytes as the SpMV (ai, aj,
// aa, x once, y once) unless it says otherwise:
//   0  flat read of the matrix arrays + x, y written (one 16-B stream per array)
//   1  the SpMV's block shape: per 512-row block the aa / aj pairs (four 16-B /
//      8-B loads per lane), ai per row, x[row] read coalesced, y[row] written
//   2  rung 1 with x gathered by aj instead of read coalesced (products summed
//      per lane, no LDS)
//   3  rung 2 with the products staged in LDS and summed per row (the
//      product kernel's structure, PETSc's order)
// NT: non-temporal matrix loads.  Built as a shared library and driven by
// tools/spmv_ladder.py (the operand comes from the product library).
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -shared -fPIC -o tools/libspmv_ladder.so tools/spmv_ladder.hip
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {
typedef double f64x2 __attribute__((ext_vector_type(2)));
typedef int i32x2 __attribute__((ext_vector_type(2)));

template <bool NT, typename T>
__device__ __forceinline__ T ld(const T *p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}

constexpr int kT = 512;

// ROWS rows per block (512: the product's geometry 6, four pair-iterations
// per lane; 256: two pair-iterations, the flat read's best depth)
template <int RUNG, bool NT, int ROWS = 512>
__global__ __launch_bounds__(kT) void k_ladder(int32_t m, const int32_t *__restrict__ ai,
                                               const int32_t *__restrict__ aj, const double *__restrict__ aa,
                                               const double *__restrict__ x, double *__restrict__ y) {
    constexpr int kIters = ROWS == 512 ? 4 : 2;
    constexpr int kCap = 2 * kT * kIters - 2;
    __shared__ double prod[RUNG == 3 ? kCap : 1];
    const int t = threadIdx.x;
    const int32_t row0 = (int32_t)blockIdx.x * ROWS;
    const int32_t nrows = min(ROWS, m - row0);
    const int64_t k0 = ai[row0], k1 = ai[row0 + nrows];
    const int r = row0 + min(t, nrows - 1);
    const int32_t rs = ai[r], re = ai[r + 1];
    const int64_t kb = k0 & ~int64_t(1);
    f64x2 av[kIters];
    i32x2 cv[kIters];
#pragma unroll
    for (int it = 0; it < kIters; ++it) {
        const int64_t k = kb + 2 * (int64_t)(t + it * kT);
        if (k < k1) {
            av[it] = ld<NT>(reinterpret_cast<const f64x2 *>(aa + k));
            cv[it] = ld<NT>(reinterpret_cast<const i32x2 *>(aj + k));
        } else {
            av[it] = f64x2{0.0, 0.0};
            cv[it] = i32x2{r, r};
        }
    }
    double s = 0.0;
    if constexpr (RUNG == 1) {
        const double xr = x[r];
#pragma unroll
        for (int it = 0; it < kIters; ++it) s += av[it].x + av[it].y + (double)(cv[it].x ^ cv[it].y);
        s += xr + (double)(re - rs);
    } else {
        f64x2 xv[kIters];
#pragma unroll
        for (int it = 0; it < kIters; ++it) {
            const int64_t k = kb + 2 * (int64_t)(t + it * kT);
            if (k < k1) {
                xv[it].x = x[cv[it].x];
                xv[it].y = x[cv[it].y];
            } else {
                xv[it] = f64x2{0.0, 0.0};
            }
        }
        if constexpr (RUNG == 2) {
#pragma unroll
            for (int it = 0; it < kIters; ++it) s += av[it].x * xv[it].x + av[it].y * xv[it].y;
            s += (double)(re - rs);
        } else {
#pragma unroll
            for (int it = 0; it < kIters; ++it) {
                const int64_t k = kb + 2 * (int64_t)(t + it * kT);
                if (k < k1) {
                    if (k >= k0) prod[k - k0] = av[it].x * xv[it].x;
                    if (k + 1 < k1) prod[k + 1 - k0] = av[it].y * xv[it].y;
                }
            }
            __syncthreads();
            for (int32_t k = rs; k < re; ++k) s += prod[k - k0];
        }
    }
    if (t < nrows) __builtin_nontemporal_store(s, y + r);
}

// rung 0b: the SpMV's five arrays streamed in the flat read's best shape —
// per 512-lane block 2048 entries of aa (two 16-B loads per lane) and aj (one
// 16-B load per lane), its share of the rows' ai and x (16-B loads) and of y
// (16-B stores) — no CSR structure at all
template <bool NT>
__global__ __launch_bounds__(kT) void k_multi(int32_t m, int64_t nz, const int32_t *__restrict__ ai,
                                              const int32_t *__restrict__ aj, const double *__restrict__ aa,
                                              const double *__restrict__ x, double *__restrict__ y) {
    const int t = threadIdx.x;
    const int64_t nb = (nz + 2047) / 2048, b = blockIdx.x;
    const int64_t e0 = b * 2048;
    const int64_t r0 = (b * m / nb) & ~int64_t(3), r1 = b + 1 == nb ? m : (((b + 1) * m / nb) & ~int64_t(3));
    double s = 0.0;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const int64_t k = e0 + 2 * (t + u * kT);
        if (k + 1 < nz) {
            const f64x2 a = ld<NT>(reinterpret_cast<const f64x2 *>(aa + k));
            s += a.x + a.y;
        }
    }
    {
        const int64_t k = e0 + 4 * t;
        typedef int i32x4 __attribute__((ext_vector_type(4)));
        if (k + 3 < nz) {
            const i32x4 c = ld<NT>(reinterpret_cast<const i32x4 *>(aj + k));
            s += (double)(c.x ^ c.y ^ c.z ^ c.w);
        }
    }
    const int64_t r = r0 + 4 * t;
    typedef int i32x4 __attribute__((ext_vector_type(4)));
    if (r + 3 < r1) {
        const i32x4 q = ld<NT>(reinterpret_cast<const i32x4 *>(ai + r));
        s += (double)(q.x + q.w);
    }
    const int64_t rx = r0 + 2 * t;
    if (rx + 1 < r1) {
        const f64x2 xv = *reinterpret_cast<const f64x2 *>(x + rx);
        f64x2 o;
        o.x = s + xv.x;
        o.y = s + xv.y;
        __builtin_nontemporal_store(o, reinterpret_cast<f64x2 *>(y + rx));
    }
    if (rx + 1 + 2 * kT < r1) {  // blocks of more than 1024 rows (never at 7 entries per row)
        const f64x2 xv = *reinterpret_cast<const f64x2 *>(x + rx + 2 * kT);
        f64x2 o;
        o.x = s + xv.x;
        o.y = s + xv.y;
        __builtin_nontemporal_store(o, reinterpret_cast<f64x2 *>(y + rx + 2 * kT));
    }
}

// rung 0: each array read once as flat 16-B tiles (two per lane), y written
template <bool NT>
__global__ __launch_bounds__(kT) void k_flat(int64_t n2, const f64x2 *__restrict__ v, double *out, int64_t nout) {
    const int64_t base = (int64_t)blockIdx.x * kT * 2 + threadIdx.x;
    double s = 0.0;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const int64_t i = base + (int64_t)u * kT;
        if (i < n2) {
            const f64x2 q = ld<NT>(v + i);
            s += q.x + q.y;
        }
    }
    const int64_t o = (int64_t)blockIdx.x * kT + threadIdx.x;
    if (o < nout) __builtin_nontemporal_store(s, out + o);
}
}  // namespace

extern "C" {

// y = a ladder rung over the Poisson CSR (device pointers); returns hipError_t
// rows 512 (four pair-iterations per lane) or 256 (two); rung 9 = k_multi
int ladder_launch(int rung, int nt, int rows, int32_t m, int64_t nz, const int32_t *ai, const int32_t *aj,
                  const double *aa, const double *x, double *y, void *stream) {
    const hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (rung == 9) {
        const unsigned g = (unsigned)((nz + 2047) / 2048);
        if (nt) hipLaunchKernelGGL((k_multi<true>), dim3(g), dim3(kT), 0, s, m, nz, ai, aj, aa, x, y);
        else hipLaunchKernelGGL((k_multi<false>), dim3(g), dim3(kT), 0, s, m, nz, ai, aj, aa, x, y);
        return (int)hipGetLastError();
    }
    const unsigned g = (unsigned)((m + rows - 1) / rows);
#define L(R, N, W) hipLaunchKernelGGL((k_ladder<R, N, W>), dim3(g), dim3(kT), 0, s, m, ai, aj, aa, x, y)
    switch ((rows == 256 ? 8 : 0) + rung * 2 + (nt ? 1 : 0) - 2) {
        case 0: L(1, false, 512); break;
        case 1: L(1, true, 512); break;
        case 2: L(2, false, 512); break;
        case 3: L(2, true, 512); break;
        case 4: L(3, false, 512); break;
        case 5: L(3, true, 512); break;
        case 8: L(1, false, 256); break;
        case 9: L(1, true, 256); break;
        case 10: L(2, false, 256); break;
        case 11: L(2, true, 256); break;
        case 12: L(3, false, 256); break;
        case 13: L(3, true, 256); break;
        default: return (int)hipErrorInvalidValue;
    }
#undef L
    return (int)hipGetLastError();
}

// rung 0 over one array of n doubles (n even), writing nout doubles of out
int ladder_flat(int nt, int64_t n, const double *v, double *out, int64_t nout, void *stream) {
    const hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const int64_t n2 = n / 2;
    const unsigned g = (unsigned)((n2 + 2 * kT - 1) / (2 * kT));
    if (nt) hipLaunchKernelGGL((k_flat<true>), dim3(g), dim3(kT), 0, s, n2, reinterpret_cast<const f64x2 *>(v), out, nout);
    else hipLaunchKernelGGL((k_flat<false>), dim3(g), dim3(kT), 0, s, n2, reinterpret_cast<const f64x2 *>(v), out, nout);
    return (int)hipGetLastError();
}
}
