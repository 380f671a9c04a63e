// cg_device.h — KSPSolve_CG's device-side scalar state and reductions,
// shared by the single-GPU solver (ksp.hip) and the row-partitioned one
// (ksp_mpi.hip). Not part of the ABI.
//
// The scalar steps restate PETSc 3.7.6 KSPSolve_CG [ext]
// (src/ksp/ksp/impls/cg/cg.c) and KSPConvergedDefault [ext]: each takes the
// already-reduced dot products (one rank: this device's fixed-order sum; many
// ranks: that sum all-reduced, identical on every rank), so every rank runs
// the same branch without the host.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "aijhip_ksp.h"

// The device scalar state (external linkage: the distributed GAMG's
// translation unit passes it to MatMult_MPIAIJ, mpi_internal.h).
struct CGState {
    double beta, betaold, dpi, dpiold, a, b, dp, rnorm0, ttol;
    int32_t its, reason, done, i;
    int32_t xpend;  // X += a P of the last completed iteration not applied yet
};

struct CGParams {
    double rtol, abstol, dtol;
    int32_t max_it, normtype, guess_zero, pc;
};

namespace {

constexpr int kVecThreads = 256;
constexpr int kRedThreads = 1024;
constexpr int kNQ = 4;  // partial quantities per vector block: zz, zr, rr, ss

// Block sum in a fixed order (as block_sum in aijhip_kernels.hip).
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

// Sum of part[0..n) in a fixed order by one 1024-lane block (valid in lane 0).
// Each lane adds part[j], part[j + 1024], ... in that order; the loads of 8
// strides are issued together (a long partial list, e.g. one per STREAM
// block, is otherwise latency-bound), the adds keep the order.
__device__ double reduce_parts(const double *part, int n, double *scratch) {
    constexpr int U = 8;
    double s = 0.0;
    for (int j0 = threadIdx.x; j0 < n; j0 += U * kRedThreads) {
        double v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int j = j0 + u * kRedThreads;
            v[u] = j < n ? part[j] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (j0 + u * kRedThreads < n) s += v[u];
    }
    return bsum<kRedThreads>(s, scratch);
}

// KSPConvergedDefault [ext]: the n = 0 call fixes rnorm0 and
// ttol = max(rtol * rnorm0, abstol).
__device__ int32_t converged(int n, double rnorm, double snorm, CGState *S, const CGParams &p) {
    if (n == 0) {
        S->rnorm0 = snorm;
        S->ttol = fmax(p.rtol * snorm, p.abstol);
    }
    if (isnan(rnorm) || isinf(rnorm)) return AIJHIP_KSP_DIVERGED_NANORINF;
    if (rnorm <= S->ttol) return rnorm < p.abstol ? AIJHIP_KSP_CONVERGED_ATOL : AIJHIP_KSP_CONVERGED_RTOL;
    if (rnorm >= p.dtol * S->rnorm0) return AIJHIP_KSP_DIVERGED_DTOL;
    return 0;
}

__device__ double norm_of(const CGParams &p, double zz, double rr, double zr) {
    switch (p.normtype) {
        case AIJHIP_KSP_NORM_PRECONDITIONED: return sqrt(zz);
        case AIJHIP_KSP_NORM_UNPRECONDITIONED: return sqrt(rr);
        case AIJHIP_KSP_NORM_NATURAL: return sqrt(fabs(zr));
        default: return 0.0;
    }
}

// Initial residual norm, the n = 0 convergence test and the top-of-loop
// checks of iteration 0. ss: |D^-1 b|^2 or |b|^2 (nonzero initial guess).
__device__ void step_init(double zz, double zr, double rr, double ss, CGState *S, double *hist,
                          const CGParams &p) {
    CGState s{};
    s.dp = norm_of(p, zz, rr, zr);
    hist[0] = s.dp;
    s.its = 0;
    s.reason = converged(0, s.dp, p.guess_zero ? s.dp : sqrt(ss), &s, p);
    s.beta = zr;
    s.i = 0;
    if (!s.reason) {  // top of iteration 0
        s.its = 1;
        if (p.max_it <= 0) { s.reason = AIJHIP_KSP_DIVERGED_ITS; s.its = 0; }
        else if (s.beta == 0.0) s.reason = AIJHIP_KSP_CONVERGED_ATOL;
    }
    s.b = 0.0;
    s.done = s.reason != 0;
    *S = s;
}

// dpi = P.W, DIVERGED_INDEFINITE_MAT check, a = beta / dpi (S not done).
__device__ void step_dpi(double dpi, CGState *S) {
    S->dpiold = S->dpi;
    S->dpi = dpi;
    S->betaold = S->beta;
    if (dpi == 0.0 || (S->i > 0 && dpi * S->dpiold <= 0.0)) {
        S->reason = AIJHIP_KSP_DIVERGED_INDEFINITE_MAT;
        S->done = 1;
        S->xpend = 0;  // this iteration's X update never happens (PETSc returns first)
        return;
    }
    S->a = S->beta / dpi;
}

// dp, convergence test at n = i + 1, beta, top-of-loop checks of i + 1
// (S not done).
__device__ void step_iter(double zz, double zr, double rr, CGState *S, double *hist, const CGParams &p) {
    CGState s = *S;
    s.dp = norm_of(p, zz, rr, zr);
    hist[s.i + 1] = s.dp;
    s.reason = converged(s.i + 1, s.dp, 0.0, &s, p);
    if (!s.reason) {
        s.beta = zr;
        s.i += 1;
        if (s.i >= p.max_it) {
            s.reason = AIJHIP_KSP_DIVERGED_ITS;
        } else {
            s.its = s.i + 1;
            if (s.beta == 0.0) s.reason = AIJHIP_KSP_CONVERGED_ATOL;
            else if (s.beta * s.betaold < 0.0) s.reason = AIJHIP_KSP_DIVERGED_INDEFINITE_PC;
            else s.b = s.beta / s.betaold;
        }
    }
    s.done = s.reason != 0;
    s.xpend = s.done;  // stopped after this iteration's update: its X += a P is due
    *S = s;
}

// PCSetUp_Jacobi [ext]: diag = MatGetDiagonal (first stored diagonal entry,
// 0 if none), zero entries replaced by 1, then reciprocal.
__global__ void k_diag_inv(int m, const int32_t *__restrict__ ai, const int32_t *__restrict__ aj,
                           const double *__restrict__ aa, double *dinv) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= m) return;
    double d = 0.0;
    for (int32_t k = ai[r]; k < ai[r + 1]; ++k)
        if (aj[k] == r) { d = aa[k]; break; }
    if (d == 0.0) d = 1.0;
    dinv[r] = 1.0 / d;
}

// PCSetUp_Jacobi on row templates: the diagonal of each template (its
// first offset-0 entry, as k_diag_inv takes a row's), so that D^-1 of row i
// is tdinv[pid[i]] — the same bits as k_diag_inv's dinv[i] (every row equals
// its template bit for bit, verified at plan time).
__global__ void k_tmpl_dinv(int npat, const int32_t *__restrict__ ptab, const double *__restrict__ pval,
                            double *tdinv) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= npat) return;
    const int32_t pm = ptab[p], st = pm & 0xffff, n = pm >> 16;
    double d = 0.0;
    for (int32_t j = 0; j < n; ++j)
        if (ptab[st + j] == 0) { d = pval[st + j]; break; }
    if (d == 0.0) d = 1.0;
    tdinv[p] = 1.0 / d;
}

#define GRID_STRIDE(i, n) \
    for (int64_t i = (int64_t)blockIdx.x * kVecThreads + threadIdx.x; i < (n); i += (int64_t)gridDim.x * kVecThreads)

template <bool NT>
__device__ __forceinline__ void vst(double *p, double v) {
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// Initial residual: r = b (zero guess) or r = b - A x (r holds A x on entry);
// Jacobi / none: z = D^-1 r; partials Z.Z, Z.R, R.R and (nonzero guess) the
// norm of D^-1 b (or b). GAMG: z comes from the V-cycle afterwards.
__global__ __launch_bounds__(kVecThreads) void k_init(int64_t n, const double *__restrict__ b,
                                                      double *r, double *z,
                                                      const double *__restrict__ dinv,
                                                      double *part, CGParams p) {
    __shared__ double scratch[kVecThreads / 64];
    const bool jac = p.pc == AIJHIP_PC_JACOBI, gamg = p.pc == AIJHIP_PC_GAMG;
    double zz = 0.0, zr = 0.0, rr = 0.0, ss = 0.0;
    GRID_STRIDE(i, n) {
        const double bi = b[i];
        const double ri = p.guess_zero ? bi : bi + (-1.0) * r[i];  // VecAYPX(R,-1,B)
        r[i] = ri;
        rr += ri * ri;
        if (!gamg) {
            const double zi = jac ? dinv[i] * ri : ri;
            z[i] = zi;
            zz += zi * zi;
            zr += zi * ri;
            const double sb = (jac && p.normtype != AIJHIP_KSP_NORM_UNPRECONDITIONED) ? dinv[i] * bi : bi;
            ss += sb * sb;
        } else {
            ss += bi * bi;  // GAMG preconditioned snorm: overwritten from V-cycle(b)
        }
    }
    const int nb = gridDim.x;
    double v;
    v = bsum<kVecThreads>(zz, scratch); if (threadIdx.x == 0) part[0 * nb + blockIdx.x] = v;
    v = bsum<kVecThreads>(zr, scratch); if (threadIdx.x == 0) part[1 * nb + blockIdx.x] = v;
    v = bsum<kVecThreads>(rr, scratch); if (threadIdx.x == 0) part[2 * nb + blockIdx.x] = v;
    v = bsum<kVecThreads>(ss, scratch); if (threadIdx.x == 0) part[3 * nb + blockIdx.x] = v;
}

// K1: P = Z (i = 0) or P = Z + b P (VecAYPX: y = x + alpha y, product first).
// The previous iteration's VecAXPY(X, a, P) is applied here, where P is read
// anyway, before P is overwritten (same operation on every element, one
// iteration later: X and P make one pass fewer per iteration).
// x == nullptr: X += a P is applied in k_update instead (x_in_update).
// IZ (Jacobi on row templates): Z is not stored — z_i = D^-1_i r_i is formed
// here from R and the template's D^-1 (tdinv[pid[i]]), the product k_update
// formed for its dots: the same bits, one vector pass fewer per iteration.
template <bool NT, bool IZ = false>
__global__ __launch_bounds__(kVecThreads) void k_aypx(int64_t n, const double *__restrict__ z, double *p,
                                                      double *x, const CGState *S,
                                                      const double *__restrict__ r = nullptr,
                                                      const uint8_t *__restrict__ pid = nullptr,
                                                      const double *__restrict__ tdinv = nullptr) {
    if (S->done) return;
    const bool first = S->i == 0 || x == nullptr;
    const double bb = S->b, a = S->a;
    const bool p_first = S->i == 0;
    GRID_STRIDE(i, n) {
        const double pi = p[i];
        const double zi = IZ ? tdinv[pid[i]] * r[i] : z[i];
        if (!first) vst<NT>(x + i, x[i] + a * pi);
        vst<NT>(p + i, p_first ? zi : zi + bb * pi);
    }
}

// After the loop: the last iteration's X += a P when the solve stopped after
// that iteration's update (converged / diverged-its / top-of-loop checks),
// not when it stopped inside it (indefinite matrix) or before it.
__global__ __launch_bounds__(kVecThreads) void k_final_x(int64_t n, const double *__restrict__ p, double *x,
                                                         const CGState *S) {
    if (!S->xpend) return;
    const double a = S->a;
    GRID_STRIDE(i, n) x[i] = x[i] + a * p[i];
}

// Unfused dot partials of p . w (when the SpMV cannot carry the epilogue).
__global__ __launch_bounds__(kVecThreads) void k_dot(int64_t n, const double *__restrict__ p,
                                                     const double *__restrict__ w, double *part,
                                                     const CGState *S) {
    __shared__ double scratch[kVecThreads / 64];
    if (S->done) return;
    double s = 0.0;
    GRID_STRIDE(i, n) s += p[i] * w[i];
    const double v = bsum<kVecThreads>(s, scratch);
    if (threadIdx.x == 0) part[blockIdx.x] = v;
}

// partials of a.a into slot sa and a.c into slot sc (sc < 0: skip)
__global__ __launch_bounds__(kVecThreads) void k_dots(int64_t n, const double *__restrict__ a,
                                                      const double *__restrict__ c, double *part, int sa,
                                                      int sc, const CGState *S) {
    __shared__ double scratch[kVecThreads / 64];
    if (S && S->done) return;
    double aa = 0.0, ac = 0.0;
    GRID_STRIDE(i, n) {
        const double ai = a[i];
        aa += ai * ai;
        if (sc >= 0) ac += ai * c[i];
    }
    const int nb = gridDim.x;
    double v = bsum<kVecThreads>(aa, scratch);
    if (threadIdx.x == 0) part[sa * nb + blockIdx.x] = v;
    if (sc >= 0) {
        v = bsum<kVecThreads>(ac, scratch);
        if (threadIdx.x == 0) part[sc * nb + blockIdx.x] = v;
    }
}

// K4: R -= a W; Jacobi / none: Z = D^-1 R (W and Z share storage: w[i] is
// read before z[i] is written by the same lane); partials Z.Z, Z.R, R.R
// (GAMG: R.R only, Z follows from the V-cycle). VecAXPY(X, a, P) is deferred
// to the next K1 (or k_final_x).
// IZ (Jacobi on row templates): D^-1_i = tdinv[pid[i]] and Z is not
// stored (k_aypx forms it again from R).
template <bool NT, bool IZ = false>
__global__ __launch_bounds__(kVecThreads) void k_update(int64_t n, double *r, double *wz,
                                                        const double *__restrict__ dinv, double *part,
                                                        const CGState *S, int pc,
                                                        const double *__restrict__ p, double *x,
                                                        const uint8_t *__restrict__ pid = nullptr,
                                                        const double *__restrict__ tdinv = nullptr) {
    __shared__ double scratch[kVecThreads / 64];
    if (S->done) return;
    const double a = S->a, na = -S->a;
    double zz = 0.0, zr = 0.0, rr = 0.0;
    GRID_STRIDE(i, n) {
        if (x) vst<NT>(x + i, x[i] + a * p[i]);  // VecAXPY(X, a, P) (x_in_update)
        const double ri = r[i] + na * wz[i];  // VecAXPY(R, -a, W)
        vst<NT>(r + i, ri);
        rr += ri * ri;
        if (IZ) {  // Jacobi on row templates
            const double zi = tdinv[pid[i]] * ri;
            zz += zi * zi;
            zr += zi * ri;
        } else if (pc != AIJHIP_PC_GAMG) {
            const double zi = pc == AIJHIP_PC_JACOBI ? dinv[i] * ri : ri;  // PCApply_Jacobi
            vst<NT>(wz + i, zi);
            zz += zi * zi;
            zr += zi * ri;
        }
    }
    const int nb = gridDim.x;
    double v;
    if (IZ || pc != AIJHIP_PC_GAMG) {
        v = bsum<kVecThreads>(zz, scratch); if (threadIdx.x == 0) part[0 * nb + blockIdx.x] = v;
        v = bsum<kVecThreads>(zr, scratch); if (threadIdx.x == 0) part[1 * nb + blockIdx.x] = v;
    }
    v = bsum<kVecThreads>(rr, scratch); if (threadIdx.x == 0) part[2 * nb + blockIdx.x] = v;
}

}  // namespace
