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

constexpr int kT = 512, kIters = 4, kCap = 4094;

template <int RUNG, bool NT>
__global__ __launch_bounds__(kT) void k_ladder(int32_t m, const int32_t *__restrict__ ai,
                                               const int32_t *__restrict__ aj, const double *__restrict__ aa,
                                               const double *__restrict__ x, double *__restrict__ y) {
    __shared__ double prod[RUNG == 3 ? kCap : 1];
    const int t = threadIdx.x;
    const int32_t row0 = (int32_t)blockIdx.x * kT;
    const int32_t nrows = min(kT, m - row0);
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
int ladder_launch(int rung, int nt, int32_t m, const int32_t *ai, const int32_t *aj, const double *aa,
                  const double *x, double *y, void *stream) {
    const hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const unsigned g = (unsigned)((m + kT - 1) / kT);
#define L(R, N) hipLaunchKernelGGL((k_ladder<R, N>), dim3(g), dim3(kT), 0, s, m, ai, aj, aa, x, y)
    switch (rung * 2 + (nt ? 1 : 0)) {
        case 2: L(1, false); break;
        case 3: L(1, true); break;
        case 4: L(2, false); break;
        case 5: L(2, true); break;
        case 6: L(3, false); break;
        case 7: L(3, true); break;
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
