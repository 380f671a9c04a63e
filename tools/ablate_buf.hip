// DIAGNOSTIC ONLY (not the product): STREAM SpMV block-shape and load-form
// study (cdna_hip_programming.md §7 "Ablate"). Same arithmetic as the
// product's k_spmv_stream (PETSc row order, bit-identical y), varying
//   T, IT  lanes per workgroup and pair-iterations (2*T*IT entry slots),
//   RPT    rows per lane in the row-sum phase (block rows up to RPT*T),
//   MODE   0: loads/gathers predicated on k < k1 (the product's form)
//          1: per-block buffer descriptors (SRD) — aj loads first, then aa,
//             all unconditional (the range check zeroes lanes past the block,
//             no branch, so hipcc can count vmcnt); gathers through an SRD on
//             x with an out-of-range offset for idle lanes (no request)
//          2: as 1 with aa loads first
//          3: the loads of 0, products stored as in 1/2
//   NTY    y store policy (low 3 bits): 0 plain, 1 __builtin_nontemporal_store, 2..7 buffer
//          store with cache-policy aux nt / sc0|nt / sc1|nt / sc0|sc1|nt / sc0 / sc1;
//          +8: non-temporal matrix loads as well (MODE 0/3).
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -shared -fPIC tools/ablate_buf.hip -o tools/libablate_buf.so
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef double f64x2 __attribute__((ext_vector_type(2)));
typedef int i32x2 __attribute__((ext_vector_type(2)));

struct BlockDesc { int32_t row0, nrows, k0, nk; };

template <int T, int IT, int RPT, int MODE, int NTY>
__global__ __launch_bounds__(T) void k_buf(const BlockDesc *__restrict__ blk, const int32_t *__restrict__ rai,
                                           const int32_t *__restrict__ aj, const double *__restrict__ aa,
                                           const double *__restrict__ x, int32_t n, double *y) {
    __shared__ double prod[2 * T * IT];
    const BlockDesc d = blk[blockIdx.x];
    const int t = threadIdx.x;
    const int64_t k0 = d.k0, k1 = (int64_t)d.k0 + d.nk, kb = k0 & ~int64_t(1);
    int32_t rs[RPT], re[RPT];
#pragma unroll
    for (int q = 0; q < RPT; ++q) {
        const int r = d.row0 + min(t + q * T, d.nrows - 1);
        rs[q] = rai[r];
        re[q] = rai[r + 1];
    }
    f64x2 av[IT];
    i32x2 cv[IT];
    f64x2 xv[IT];
    if constexpr (MODE == 0 || MODE == 3) {
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            const int64_t k = kb + 2 * (int64_t)(t + it * T);
            av[it] = f64x2{0.0, 0.0};
            xv[it] = f64x2{0.0, 0.0};
            if (k < k1) {
                if constexpr (NTY >= 8) {  // non-temporal matrix loads too
                    av[it] = __builtin_nontemporal_load(reinterpret_cast<const f64x2 *>(aa + k));
                    cv[it] = __builtin_nontemporal_load(reinterpret_cast<const i32x2 *>(aj + k));
                } else {
                    av[it] = *reinterpret_cast<const f64x2 *>(aa + k);
                    cv[it] = *reinterpret_cast<const i32x2 *>(aj + k);
                }
            }
        }
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            const int64_t k = kb + 2 * (int64_t)(t + it * T);
            if (k < k1) {
                xv[it].x = x[cv[it].x];
                xv[it].y = x[cv[it].y];
            }
        }
    } else {
        const int32_t span = (int32_t)(((k1 - kb) + 1) & ~int64_t(1));  // whole pairs
        const __amdgpu_buffer_rsrc_t ra =
            __builtin_amdgcn_make_buffer_rsrc((void *)(aa + kb), 0, span * 8, 0x00020000);
        const __amdgpu_buffer_rsrc_t rj =
            __builtin_amdgcn_make_buffer_rsrc((void *)(aj + kb), 0, span * 4, 0x00020000);
        const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void *)x, 0, n * 8, 0x00020000);
        if constexpr (MODE == 1) {
#pragma unroll
            for (int it = 0; it < IT; ++it)
                cv[it] = __builtin_bit_cast(i32x2, __builtin_amdgcn_raw_buffer_load_b64(rj, (t + it * T) * 8, 0, 0));
#pragma unroll
            for (int it = 0; it < IT; ++it)
                av[it] = __builtin_bit_cast(f64x2, __builtin_amdgcn_raw_buffer_load_b128(ra, (t + it * T) * 16, 0, 0));
        } else {
#pragma unroll
            for (int it = 0; it < IT; ++it) {
                av[it] = __builtin_bit_cast(f64x2, __builtin_amdgcn_raw_buffer_load_b128(ra, (t + it * T) * 16, 0, 0));
                cv[it] = __builtin_bit_cast(i32x2, __builtin_amdgcn_raw_buffer_load_b64(rj, (t + it * T) * 8, 0, 0));
            }
        }
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            const int64_t k = kb + 2 * (int64_t)(t + it * T);
            const int ox = k < k1 ? cv[it].x * 8 : -1;
            const int oy = k + 1 < k1 ? cv[it].y * 8 : -1;
            xv[it].x = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rx, ox, 0, 0));
            xv[it].y = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rx, oy, 0, 0));
        }
    }
    // MODE 0: predicated scalar LDS stores at k - k0 (the product's form).
    // MODE >= 1: one unconditional 16-B LDS store per pair at k - kb (slots
    // past the block hold 0 * 0 and are never read), so no load is sunk
    // into a store branch.
    if constexpr (MODE == 0) {
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            const int64_t k = kb + 2 * (int64_t)(t + it * T);
            if (k < k1) {
                if (k >= k0) prod[k - k0] = av[it].x * xv[it].x;
                if (k + 1 < k1) prod[k + 1 - k0] = av[it].y * xv[it].y;
            }
        }
    } else {
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            f64x2 p;
            p.x = av[it].x * xv[it].x;
            p.y = av[it].y * xv[it].y;
            reinterpret_cast<f64x2 *>(prod)[t + it * T] = p;
        }
    }
    const int64_t kp = MODE == 0 ? k0 : kb;
    __syncthreads();
#pragma unroll
    for (int q = 0; q < RPT; ++q) {
        if (t + q * T < d.nrows) {
            double s = 0.0;
            for (int32_t k = rs[q]; k < re[q]; ++k) s += prod[k - kp];
            const int row = d.row0 + t + q * T;
            constexpr int st = NTY & 7;
            if constexpr (st == 0) y[row] = s;
            else if constexpr (st == 1) __builtin_nontemporal_store(s, y + row);
            else {  // buffer store with explicit cache-policy bits (gfx940+: sc0 = 1, nt = 2, sc1 = 16)
                constexpr int aux = st == 2 ? 2 : st == 3 ? 3 : st == 4 ? 18 : st == 5 ? 19 : st == 6 ? 1 : 16;
                const __amdgpu_buffer_rsrc_t ry =
                    __builtin_amdgcn_make_buffer_rsrc((void *)(y + d.row0), 0, d.nrows * 8, 0x00020000);
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned int, s), ry,
                                                      (t + q * T) * 8, 0, aux);
            }
        }
    }
}

#define BUF_CONFIGS(X)                                                                               \
    X(512, 4, 1, 0, 0) X(512, 4, 1, 0, 1) X(512, 4, 1, 0, 2) X(512, 4, 1, 0, 3) X(512, 4, 1, 0, 4)  \
    X(512, 4, 1, 0, 5) X(512, 4, 1, 0, 6) X(512, 4, 1, 0, 7) X(512, 4, 1, 0, 9) X(512, 4, 1, 3, 1)  \
    X(512, 4, 2, 0, 1) X(512, 4, 2, 1, 1) X(512, 4, 1, 1, 1) X(256, 8, 1, 0, 1) X(1024, 4, 1, 0, 1) \
    X(512, 4, 2, 3, 1)

extern "C" int ablate_buf(int tt, int it, int rpt, int mode, int nty, int nblk, const void *blk,
                          const int32_t *rai, const int32_t *aj, const double *aa, const double *x, int32_t n,
                          double *y, void *stream) {
    hipStream_t s = (hipStream_t)stream;
    const BlockDesc *b = (const BlockDesc *)blk;
#define X(TT, IT, RPT, MODE, NTY)                                                                       \
    if (tt == TT && it == IT && rpt == RPT && mode == MODE && nty == NTY) {                        \
        hipLaunchKernelGGL((k_buf<TT, IT, RPT, MODE, NTY>), dim3(nblk), dim3(TT), 0, s, b, rai, aj, aa, x, n, y); \
        return hipGetLastError() == hipSuccess ? 0 : 2;                                                 \
    }
    BUF_CONFIGS(X)
#undef X
    return 1;
}

extern "C" int ablate_buf_configs(int *out, int cap) {
    int i = 0;
#define X(TT, IT, RPT, MODE, NTY)                                       \
    if (i + 5 <= cap) {                                                 \
        out[i] = TT; out[i + 1] = IT; out[i + 2] = RPT; out[i + 3] = MODE; out[i + 4] = NTY; \
    }                                                                   \
    i += 5;
    BUF_CONFIGS(X)
#undef X
    return i / 5;
}
