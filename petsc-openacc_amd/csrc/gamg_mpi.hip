// gamg_mpi.hip — PCGAMG across ranks: the smoothed-aggregation hierarchy of
// a row-distributed operator and its V-cycle (aijhip_kspmpi with
// AIJHIP_PC_GAMG at more than one rank).
//
// The reference runs CG + PETSc's agg GAMG on 1-16 MPI ranks
// (/root/reference/runs/single-node-scaling.pbs:56-67 with
// /root/reference/configs/PETSc_SolverOptions_GAMG.info:6-21): its
// aggregation, prolongator smoothing and Galerkin products span the MPIAIJ
// operator [ext]. The same structure here, MI355X-first:
//
//   aggregates   PETSc's parallel MIS (coarsen 1, the default; dist_mis):
//                ghost states exchanged every round over the level's halo,
//                restated as the global MIS by global keys — roots on either
//                side of a rank boundary are independent, a node taken by a
//                root on another rank joins that aggregate (as mis.c's
//                lid_parent_gid), and the aggregates are the single-GPU ones
//                whatever the partition; or the greedy pass on each rank's
//                diagonal block A_d (coarsen 0, aggregates local);
//   emax         CG's Lanczos estimate (eig_ksp 1, the default) or a power
//                iteration on the distributed D^-1 A (MatMult_MPIAIJ +
//                all-reduced dots), from the single-GPU start vector taken
//                at global indices;
//   P            = P0 + alpha D^-1 (A P0) over the whole operator: A_ext = [A_d |
//                A_o] times P0 extended by its ghost rows (aggregate id and
//                value of each ghost fine node, exchanged through the halo);
//   A_c          = P^T (A P): P's rows of the ghost fine nodes are exchanged
//                (variable length), A P = A_ext P_ext and P^T (A P) are the
//                device row-wise products over an extended coarse numbering
//                (own coarse rows first, then the off-rank ones); the rows
//                that belong to other ranks' coarse nodes are sent to their
//                owners and added there;
//   level l+1    C_d (own columns) and C_o (ghost columns) with a p2p halo
//                plan; P = [P_d | P_o]; R = P^T as MatMultTranspose_MPIAIJ
//                (P_d^T r, and P_o^T r's ghost-slot sums added on their
//                owners through level l+1's plan run backwards).
// Bulk work (the large products, the transposes, the V-cycle) is on the
// device; the host handles boundary-sized data (ghost rows, contributions).
// The V-cycle is PETSc's multiplicative PCMG with the reference's options
// (Richardson(1)+Jacobi down and up, P^T restriction, coarse Jacobi), every
// SpMV a MatMult_MPIAIJ-shaped product with its halo on the operator's
// exchange stream.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "dscan.h"
#include "gamg_device.h"
#include "gamg_internal.h"
#include "gamg_mpi.h"
#include "mpi_internal.h"

namespace {

using aijhip_gamg::DCsr;
using aijhip_gamg::dalloc;
using aijhip_mpi::mfail;
using aijhip_mpi::mhip;

inline unsigned nblk(int64_t n, int t = 256) { return (unsigned)std::max<int64_t>(1, (n + t - 1) / t); }

// ---------------------------------------------------------------- kernels
__device__ __forceinline__ uint64_t mix64d(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

// the single-GPU power iteration's start vector at global indices off + i
__global__ void k_power_start_off(int32_t m, int64_t off, double *v) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    v[i] = 2.0 * ((double)(mix64d(0x5EEDULL + (uint64_t)(off + i + 1) * 0x9E3779B97F4A7C15ULL) >> 11) *
                  (1.0 / 9007199254740992.0)) - 1.0;
}

constexpr int64_t kDotBlock = 256;

__global__ void k_sumsq_blocks(int64_t n, const double *__restrict__ a, double *part) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t i0 = q * kDotBlock;
    if (i0 >= n) return;
    const int64_t e = min(n, i0 + kDotBlock);
    double s = 0.0;
    for (int64_t i = i0; i < e; ++i) s += a[i] * a[i];
    part[q] = s;
}

__global__ void k_dot_blocks(int64_t n, const double *__restrict__ a, const double *__restrict__ b, double *part) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t i0 = q * kDotBlock;
    if (i0 >= n) return;
    const int64_t e = min(n, i0 + kDotBlock);
    double s = 0.0;
    for (int64_t i = i0; i < e; ++i) s += a[i] * b[i];
    part[q] = s;
}

// CG's emax estimate (gamg_setup.cpp estimate_emax_cg) on the distributed
// operator: the start b at global indices (the power iteration's), r = b,
// z = D^-1 r, p = z; r -= a w, z = D^-1 r; p = z + b p
__global__ void k_cgest_start_off(int32_t m, int64_t off, const double *__restrict__ dinv, double *r, double *z,
                                  double *p) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const double v = 2.0 * ((double)(mix64d(0x5EEDULL + (uint64_t)(off + i + 1) * 0x9E3779B97F4A7C15ULL) >> 11) *
                            (1.0 / 9007199254740992.0)) - 1.0;
    r[i] = v;
    z[i] = dinv[i] * v;
    p[i] = z[i];
}

__global__ void k_cgest_update(int32_t m, double a, const double *__restrict__ w, const double *__restrict__ dinv,
                               double *r, double *z) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const double ri = r[i] - a * w[i];
    r[i] = ri;
    z[i] = dinv[i] * ri;
}

__global__ void k_cgest_dir(int32_t m, double b, const double *__restrict__ z, double *p) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < m) p[i] = z[i] + b * p[i];
}

__global__ void k_scale_by(int32_t m, const double *__restrict__ d, double *w) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < m) w[i] = d[i] * w[i];
}

__global__ void k_divide(int32_t m, const double *w, double nw, double *v) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < m) v[i] = w[i] / nw;
}

// global coarse id of each node's aggregate; -1 for a node MIS removed
__global__ void k_coarse_gid(int32_t m, int64_t off, const int32_t *__restrict__ agg, double *out) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < m) out[i] = agg[i] < 0 ? -1.0 : (double)(off + agg[i]);
}

__global__ void k_count_negative(int32_t m, const int32_t *__restrict__ agg, unsigned long long *n) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const unsigned long long c = __popcll(__ballot(i < m && agg[i] < 0));
    if ((threadIdx.x & 63) == 0 && c) atomicAdd(n, c);
}

__global__ void k_iota32(int32_t n, int32_t *v) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i <= n) v[i] = i;
}

// rows of [A | B] (B's columns shifted by boff; B given by a full row pointer)
__global__ void k_hcat_len(int32_t m, const int32_t *__restrict__ ai, const int32_t *__restrict__ bi, int32_t *len) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < m) len[i] = (ai[i + 1] - ai[i]) + (bi ? bi[i + 1] - bi[i] : 0);
}

__global__ void k_hcat_fill(int32_t m, const int32_t *__restrict__ ai, const int32_t *__restrict__ aj,
                            const double *__restrict__ aa, const int32_t *__restrict__ bi,
                            const int32_t *__restrict__ bj, const double *__restrict__ ba, int32_t boff,
                            const int32_t *__restrict__ ci, int32_t *cj, double *ca) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    int32_t p = ci[i];
    for (int32_t k = ai[i]; k < ai[i + 1]; ++k, ++p) {
        cj[p] = aj[k];
        ca[p] = aa[k];
    }
    if (bi)
        for (int32_t k = bi[i]; k < bi[i + 1]; ++k, ++p) {
            cj[p] = bj[k] + boff;
            ca[p] = ba[k];
        }
}

__global__ void k_add_offset(int32_t n, int32_t off, const int32_t *__restrict__ src, int32_t *dst) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dst[i] = src[i] + off;
}

__global__ void k_remap(int64_t n, const int32_t *__restrict__ table, int32_t *cols) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < n) cols[k] = table[cols[k]];
}

// rows [r0, r0 + n) of a CSR: lengths, then a compact copy
__global__ void k_rows_len(int32_t n, const int32_t *__restrict__ rows, const int32_t *__restrict__ ai, int32_t *len) {
    const int32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q < n) len[q] = ai[rows[q] + 1] - ai[rows[q]];
}

__global__ void k_rows_copy(int32_t n, const int32_t *__restrict__ rows, const int32_t *__restrict__ ai,
                            const int32_t *__restrict__ aj, const double *__restrict__ aa,
                            const int32_t *__restrict__ off, int32_t *oj, double *oa) {
    const int32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= n) return;
    int32_t p = off[q];
    for (int32_t k = ai[rows[q]]; k < ai[rows[q] + 1]; ++k, ++p) {
        oj[p] = aj[k];
        oa[p] = aa[k];
    }
}

// C = A + B (rows sorted by column; a column in both: a + b). Every
// structural entry is kept, zero sums included, as the single-GPU row
// products keep them (so one rank reproduces the single-GPU hierarchy).
template <bool FILL>
__device__ __forceinline__ int32_t add_row(int32_t i, const int32_t *__restrict__ ai, const int32_t *__restrict__ aj,
                                           const double *__restrict__ aa, const int32_t *__restrict__ bi,
                                           const int32_t *__restrict__ bj, const double *__restrict__ ba, int32_t o,
                                           int32_t *cj, double *ca) {
    int32_t p = ai[i], q = bi[i], n = 0;
    const int32_t pe = ai[i + 1], qe = bi[i + 1];
    while (p < pe || q < qe) {
        int32_t c;
        double v;
        if (q >= qe || (p < pe && aj[p] < bj[q])) { c = aj[p]; v = aa[p]; ++p; }
        else if (p >= pe || bj[q] < aj[p]) { c = bj[q]; v = ba[q]; ++q; }
        else { c = aj[p]; v = aa[p] + ba[q]; ++p; ++q; }
        if (FILL) { cj[o + n] = c; ca[o + n] = v; }
        ++n;
    }
    return n;
}

__global__ void k_add_len(int32_t m, const int32_t *__restrict__ ai, const int32_t *__restrict__ aj,
                          const double *__restrict__ aa, const int32_t *__restrict__ bi,
                          const int32_t *__restrict__ bj, const double *__restrict__ ba, int32_t *len) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < m) len[i] = add_row<false>(i, ai, aj, aa, bi, bj, ba, 0, nullptr, nullptr);
}

__global__ void k_add_fill(int32_t m, const int32_t *__restrict__ ai, const int32_t *__restrict__ aj,
                           const double *__restrict__ aa, const int32_t *__restrict__ bi,
                           const int32_t *__restrict__ bj, const double *__restrict__ ba,
                           const int32_t *__restrict__ ci, int32_t *cj, double *ca) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < m) add_row<true>(i, ai, aj, aa, bi, bj, ba, ci[i], cj, ca);
}

// split columns: < nloc -> D (same ids), >= nloc -> O (id - nloc)
__global__ void k_split_len(int32_t m, const int32_t *__restrict__ ci, const int32_t *__restrict__ cj, int32_t nloc,
                            int32_t *ld, int32_t *lo) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    int32_t d = 0;
    for (int32_t k = ci[i]; k < ci[i + 1]; ++k) d += cj[k] < nloc;
    ld[i] = d;
    lo[i] = ci[i + 1] - ci[i] - d;
}

__global__ void k_split_fill(int32_t m, const int32_t *__restrict__ ci, const int32_t *__restrict__ cj,
                             const double *__restrict__ ca, int32_t nloc, const int32_t *__restrict__ di,
                             int32_t *dj, double *da, const int32_t *__restrict__ oi, int32_t *oj, double *oa) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    int32_t pd = di[i], po = oi[i];
    for (int32_t k = ci[i]; k < ci[i + 1]; ++k) {
        if (cj[k] < nloc) { dj[pd] = cj[k]; da[pd] = ca[k]; ++pd; }
        else { oj[po] = cj[k] - nloc; oa[po] = ca[k]; ++po; }
    }
}

// V-cycle vector passes (ksp.hip's, with CG's stop flag)
__global__ __launch_bounds__(256) void k_mg_jacobi(int64_t n, const double *__restrict__ dinv,
                                                   const double *__restrict__ b, double *x, const int *stop) {
    if (stop && *stop) return;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
        x[i] = dinv[i] * b[i];
}

__global__ __launch_bounds__(256) void k_mg_resid(int64_t n, const double *__restrict__ b, double *r,
                                                  const int *stop) {
    if (stop && *stop) return;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
        r[i] = b[i] + (-1.0) * r[i];
}

__global__ __launch_bounds__(256) void k_mg_richardson(int64_t n, const double *__restrict__ dinv,
                                                       const double *__restrict__ b, const double *__restrict__ ax,
                                                       double *x, const int *stop) {
    if (stop && *stop) return;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
        x[i] = x[i] + 1.0 * (dinv[i] * (b[i] + (-1.0) * ax[i]));
}

// y[o] = y[o] + scale[o] * (-(A_o g)_o) over A_o's rows (scale NULL: 1): the
// off-diagonal block's share of a fused residual (r = b - A_d x - A_o g) or
// post-smoothing (x = t + D^-1 (b - A_d t - A_o g)) on the boundary rows
__global__ __launch_bounds__(256) void k_offdiag_axpy(int32_t nr, const int32_t *__restrict__ rai,
                                                      const int32_t *__restrict__ ridx, const int32_t *__restrict__ aj,
                                                      const double *__restrict__ aa, const double *__restrict__ g,
                                                      const double *__restrict__ scale, double *y, const int *stop) {
    if (stop && *stop) return;
    for (int32_t q = blockIdx.x * 256 + threadIdx.x; q < nr; q += gridDim.x * 256) {
        const int32_t o = ridx ? ridx[q] : q;
        double sum = 0.0;
        for (int32_t k = rai[q]; k < rai[q + 1]; ++k) sum += aa[k] * g[aj[k]];
        y[o] = y[o] + (scale ? scale[o] : 1.0) * (-sum);
    }
}


// ---- PETSc's parallel MIS (mis.c maxIndSetAgg over an MPIAIJ graph: ghost
// states exchanged every round), restated as the lexicographically-first
// maximal independent set of the GLOBAL graph by a global key — the
// single-GPU rule of gamg_aggregate.hip (aggregate_mis_device) with every
// node's key taken at its global index, the graph G1 = S_d + S_o + I (the
// strength graph of the diagonal block and of the off-diagonal block's ghost
// columns) and each round's two one-hop passes reading the neighbours on
// other ranks through the level's halo. Keys are unique, so the set, the
// parents and the aggregates do not depend on the partition: at every rank
// count the hierarchy is the single-GPU one (to the rounding of its sums).
// Values travel through the fp64 halo as raw 64-bit patterns (copies only).
typedef uint8_t dmis_t;
constexpr dmis_t kDmUndecided = 0, kDmRoot = 1, kDmOut = 2, kDmSingle = 3;

__device__ __forceinline__ uint64_t dm_key(uint32_t h, int64_t gid) { return (uint64_t)h << 32 | (uint32_t)gid; }
// roots = false: a round's decision value (0 root, key + 1 undecided, all
// ones otherwise); true: a root's key, else all ones (the parents' pass)
__device__ __forceinline__ uint64_t dm_value(dmis_t st, uint32_t h, int64_t gid, bool roots) {
    if (roots) return st == kDmRoot ? dm_key(h, gid) : ~0ull;
    return st == kDmRoot ? 0ull : st == kDmUndecided ? dm_key(h, gid) + 1 : ~0ull;
}
__device__ __forceinline__ uint64_t dm_bits(double v) { return (uint64_t)__double_as_longlong(v); }
__device__ __forceinline__ double dm_double(uint64_t v) { return __longlong_as_double((long long)v); }

__global__ void k_dm_diag(int32_t m, const int32_t *__restrict__ ai, const int32_t *__restrict__ aj,
                          const double *__restrict__ aa, double *d) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    double v = 0.0;
    for (int32_t k = ai[i]; k < ai[i + 1]; ++k)
        if (aj[k] == i) { v = aa[k]; break; }
    d[i] = v;
}

// S_o: the off-diagonal block's strong entries (|a| > theta sqrt|d_i d_g|,
// the single-GPU filter with the ghost's diagonal), full rows [0, m)
__global__ void k_dm_so_count(int32_t nr, const int32_t *__restrict__ rai, const int32_t *__restrict__ ridx,
                              const double *__restrict__ aa, const double *__restrict__ d,
                              const double *__restrict__ gd, const int32_t *__restrict__ aj, double theta,
                              int32_t *cnt) {
    const int32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nr) return;
    const int32_t i = ridx ? ridx[q] : q;
    int32_t c = 0;
    for (int32_t k = rai[q]; k < rai[q + 1]; ++k) c += fabs(aa[k]) > theta * sqrt(fabs(d[i] * gd[aj[k]]));
    cnt[i] = c;
}

__global__ void k_dm_so_fill(int32_t nr, const int32_t *__restrict__ rai, const int32_t *__restrict__ ridx,
                             const double *__restrict__ aa, const double *__restrict__ d,
                             const double *__restrict__ gd, const int32_t *__restrict__ aj, double theta,
                             const int32_t *__restrict__ soi, int32_t *soj) {
    const int32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nr) return;
    const int32_t i = ridx ? ridx[q] : q;
    int32_t o = soi[i];
    for (int32_t k = rai[q]; k < rai[q + 1]; ++k)
        if (fabs(aa[k]) > theta * sqrt(fabs(d[i] * gd[aj[k]]))) soj[o++] = aj[k];
}

__global__ void k_dm_init(int32_t m, int64_t rstart, int32_t level, const int32_t *__restrict__ sdi,
                          const int32_t *__restrict__ soi, dmis_t *state, uint32_t *hk) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    state[i] = (sdi[i] == sdi[i + 1] && soi[i] == soi[i + 1]) ? kDmSingle : kDmUndecided;
    hk[i] = (uint32_t)(aijhip_gamg::mis_key((int32_t)(rstart + i), level) >> 32);
}

__global__ void k_dm_value(int32_t m, int64_t rstart, const dmis_t *__restrict__ state,
                           const uint32_t *__restrict__ hk, bool roots, double *val) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < m) val[i] = dm_double(dm_value(state[i], hk[i], rstart + i, roots));
}

// pass A: amin[u] = min over u, its S_d neighbours and its S_o ghosts (their
// values from the halo, gval) of the value
__global__ __launch_bounds__(256) void k_dm_closed_min(int32_t m, int64_t rstart, const int32_t *__restrict__ sdi,
                                                       const int32_t *__restrict__ sdj,
                                                       const int32_t *__restrict__ soi,
                                                       const int32_t *__restrict__ soj,
                                                       const dmis_t *__restrict__ state,
                                                       const uint32_t *__restrict__ hk,
                                                       const double *__restrict__ gval, bool roots, double *amin) {
    const int32_t u = blockIdx.x * blockDim.x + threadIdx.x;
    if (u >= m) return;
    uint64_t best = dm_value(state[u], hk[u], rstart + u, roots);
    for (int32_t a = sdi[u]; a < sdi[u + 1]; ++a) {
        const int32_t j = sdj[a];
        best = min(best, dm_value(state[j], hk[j], rstart + j, roots));
    }
    for (int32_t a = soi[u]; a < soi[u + 1]; ++a) best = min(best, dm_bits(gval[soj[a]]));
    amin[u] = dm_double(best);
}

// min over i's neighbours (both blocks) of pass A's values (squared reach),
// or i's own
__device__ __forceinline__ uint64_t dm_reach(int32_t i, bool square, const int32_t *__restrict__ sdi,
                                             const int32_t *__restrict__ sdj, const int32_t *__restrict__ soi,
                                             const int32_t *__restrict__ soj, const double *__restrict__ amin,
                                             const double *__restrict__ gamin) {
    if (!square) return dm_bits(amin[i]);
    uint64_t b = ~0ull;
    for (int32_t a = sdi[i]; a < sdi[i + 1]; ++a) b = min(b, dm_bits(amin[sdj[a]]));
    for (int32_t a = soi[i]; a < soi[i + 1]; ++a) b = min(b, dm_bits(gamin[soj[a]]));
    return b;
}

// pass B: the decisions, and the workgroup's count of nodes still waiting
__global__ __launch_bounds__(256) void k_dm_decide(int32_t m, int64_t rstart, const int32_t *__restrict__ sdi,
                                                   const int32_t *__restrict__ sdj, const int32_t *__restrict__ soi,
                                                   const int32_t *__restrict__ soj, bool square,
                                                   const uint32_t *__restrict__ hk, const double *__restrict__ amin,
                                                   const double *__restrict__ gamin, dmis_t *state,
                                                   unsigned *wcount) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    bool waits = false;
    if (i < m && state[i] == kDmUndecided) {
        const uint64_t b = dm_reach(i, square, sdi, sdj, soi, soj, amin, gamin);
        if (b == 0) state[i] = kDmOut;
        else if (b == dm_key(hk[i], rstart + i) + 1) state[i] = kDmRoot;
        else waits = true;
    }
    __shared__ unsigned wc[4];
    const unsigned nw = (unsigned)__popcll(__ballot(waits));
    if ((threadIdx.x & 63) == 0) wc[threadIdx.x >> 6] = nw;
    __syncthreads();
    if (threadIdx.x == 0) wcount[blockIdx.x] = wc[0] + wc[1] + wc[2] + wc[3];
}

__global__ __launch_bounds__(1024) void k_dm_total(const unsigned *__restrict__ wcount, int32_t n,
                                                   unsigned long long *total) {
    __shared__ unsigned long long part[16];
    unsigned long long s = 0;
    for (int32_t q = threadIdx.x; q < n; q += 1024) s += wcount[q];
    for (int off = 32; off > 0; off >>= 1) s += __shfl_down(s, off, 64);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long t = 0;
        for (int w = 0; w < 16; ++w) t += part[w];
        *total = t;
    }
}

// smoothAggs' candidate: the highest global id among i's G1 neighbours that
// are roots (S_d: the state; S_o: the ghost's root key from the halo), -1
__global__ void k_dm_hiroot(int32_t m, int64_t rstart, const int32_t *__restrict__ sdi, const int32_t *__restrict__ sdj,
                            const int32_t *__restrict__ soi, const int32_t *__restrict__ soj,
                            const dmis_t *__restrict__ state, const double *__restrict__ grv,
                            const int64_t *__restrict__ ggid, int64_t *hi) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    int64_t h = -1;
    for (int32_t a = sdi[i]; a < sdi[i + 1]; ++a)
        if (state[sdj[a]] == kDmRoot) h = max(h, rstart + sdj[a]);
    for (int32_t a = soi[i]; a < soi[i + 1]; ++a)
        if (dm_bits(grv[soj[a]]) != ~0ull) h = max(h, ggid[soj[a]]);
    hi[i] = h;
}

// parent (global id): a root itself; an OUT node the lowest-key root within
// reach (its key's low word), then (squared: smoothAggs) the highest-id root
// among its G1 neighbours when it has one; otherwise -1. flag: the roots.
__global__ void k_dm_parent(int32_t m, int64_t rstart, const int32_t *__restrict__ sdi,
                            const int32_t *__restrict__ sdj, const int32_t *__restrict__ soi,
                            const int32_t *__restrict__ soj, bool square, const double *__restrict__ amin,
                            const double *__restrict__ gamin, const dmis_t *__restrict__ state,
                            const int64_t *__restrict__ hi, int64_t *parent, int32_t *flag) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const dmis_t st = state[i];
    flag[i] = st == kDmRoot;
    if (st == kDmRoot) { parent[i] = rstart + i; return; }
    if (st != kDmOut) { parent[i] = -1; return; }
    int64_t p = (int64_t)(uint32_t)dm_reach(i, square, sdi, sdj, soi, soj, amin, gamin);
    if (square && hi[i] >= 0) p = hi[i];
    parent[i] = p;
}

// coarse ids: cg[i] = the coarse global id of i's aggregate (-1: removed);
// agg[i] = its local aggregate (own roots), -1 otherwise; nodes whose root is
// on another rank go to the list (node, parent gid) and get cg -2 for now
__global__ void k_dm_coarse(int32_t m, int64_t rstart, int64_t cstart, const int64_t *__restrict__ parent,
                            const int32_t *__restrict__ idx, double *cg, int32_t *agg, int32_t *rnode,
                            int64_t *rpar, unsigned *rcount) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const int64_t p = parent[i];
    if (p < 0) {
        cg[i] = -1.0;
        agg[i] = -1;
    } else if (p >= rstart && p < rstart + m) {
        const int32_t c = idx[p - rstart];
        cg[i] = (double)(cstart + c);
        agg[i] = c;
    } else {
        const unsigned k = atomicAdd(rcount, 1u);
        rnode[k] = i;
        rpar[k] = p;
        cg[i] = -2.0;
        agg[i] = -1;
    }
}

__global__ void k_dm_gather_i32(int32_t n, const int32_t *__restrict__ at, const int32_t *__restrict__ v,
                                int32_t *out) {
    const int32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q < n) out[q] = v[at[q]];
}

__global__ void k_dm_gather_f64(int32_t n, const int32_t *__restrict__ at, const double *__restrict__ v, double *out) {
    const int32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q < n) out[q] = v ? v[at[q]] : 1.0;
}

// s2[a[q]] += add[q] (distinct a per launch)
__global__ void k_dm_add_at(int32_t n, const int32_t *__restrict__ a, const double *__restrict__ add, double *s2) {
    const int32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q < n) s2[a[q]] = s2[a[q]] + add[q];
}

__global__ void k_dm_sqrt(int32_t n, double *v) {
    const int32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q < n) v[q] = sqrt(v[q]);
}

// p0 of the nodes in own aggregates (k_tentative's formula), 0 elsewhere
__global__ void k_dm_p0(int32_t m, const int32_t *__restrict__ agg, const double *__restrict__ B,
                        const double *__restrict__ Bc, double *p0) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const double c = agg[i] >= 0 ? Bc[agg[i]] : 0.0;
    p0[i] = c > 0.0 ? (B ? B[i] : 1.0) / c : 0.0;
}

// the nodes in other ranks' aggregates: their coarse id and p0 (host-made)
__global__ void k_dm_set_remote(int32_t n, const int32_t *__restrict__ node, const double *__restrict__ cgv,
                                const double *__restrict__ p0v, double *cg, double *p0) {
    const int32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= n) return;
    cg[node[q]] = cgv[q];
    p0[node[q]] = p0v[q];
}

__global__ void k_dm_set_i32(int32_t n, const int32_t *__restrict__ node, const int32_t *__restrict__ v, int32_t *x) {
    const int32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q < n) x[node[q]] = v[q];
}

// ---------------------------------------------------------------- host side
int gerr(hipError_t e, const char *what) { return mhip(e, (std::string("distributed GAMG: ") + what).c_str()); }

// Host CSR with 64-bit column ids (global or extended numbering).
struct HCsr {
    std::vector<int64_t> ai{0};
    std::vector<int64_t> aj;
    std::vector<double> aa;
    int64_t rows() const { return (int64_t)ai.size() - 1; }
};

// exclusive prefix over ranks of one value per rank (every rank learns all)
int all_values(aijhip_comm *C, int64_t v, std::vector<int64_t> &all) {
    std::vector<std::vector<uint64_t>> out((size_t)C->nranks), in;
    for (auto &o : out) o.assign(1, (uint64_t)v);
    int rc = aijhip_mpi::comm_sendrecv(C, out, in);
    if (rc) return rc;
    all.assign((size_t)C->nranks, 0);
    for (int p = 0; p < C->nranks; ++p) all[p] = in[p].empty() ? 0 : (int64_t)in[p][0];
    return AIJHIP_OK;
}

int owner_of(const std::vector<int64_t> &starts, int64_t gid) {
    return (int)(std::upper_bound(starts.begin(), starts.end(), gid) - starts.begin()) - 1;
}

// Rows `rows` of a device CSR down to the host (columns as stored).
int download_rows(const int32_t *d_ai, const int32_t *d_aj, const double *d_aa, const std::vector<int32_t> &rows,
                  std::vector<int32_t> &off, std::vector<int32_t> &cols, std::vector<double> &vals) {
    const int32_t n = (int32_t)rows.size();
    off.assign((size_t)n + 1, 0);
    cols.clear();
    vals.clear();
    if (n == 0) return AIJHIP_OK;
    int32_t *d_rows = nullptr, *d_len = nullptr, *d_off = nullptr, *d_oj = nullptr;
    double *d_oa = nullptr;
    hipError_t e;
    int rc = AIJHIP_OK;
    std::vector<int32_t> len((size_t)n);
    if ((e = dalloc(&d_rows, n)) != hipSuccess || (e = dalloc(&d_len, n)) != hipSuccess ||
        (e = hipMemcpy(d_rows, rows.data(), sizeof(int32_t) * n, hipMemcpyHostToDevice)) != hipSuccess) {
        rc = gerr(e, "row gather");
        goto done;
    }
    hipLaunchKernelGGL(k_rows_len, dim3(nblk(n)), dim3(256), 0, nullptr, n, d_rows, d_ai, d_len);
    if ((e = hipMemcpy(len.data(), d_len, sizeof(int32_t) * n, hipMemcpyDeviceToHost)) != hipSuccess) {
        rc = gerr(e, "row gather");
        goto done;
    }
    for (int32_t q = 0; q < n; ++q) off[q + 1] = off[q] + len[q];
    cols.resize((size_t)off[n]);
    vals.resize((size_t)off[n]);
    if ((e = dalloc(&d_off, (int64_t)n + 1)) != hipSuccess || (e = dalloc(&d_oj, off[n])) != hipSuccess ||
        (e = dalloc(&d_oa, off[n])) != hipSuccess ||
        (e = hipMemcpy(d_off, off.data(), sizeof(int32_t) * ((size_t)n + 1), hipMemcpyHostToDevice)) != hipSuccess) {
        rc = gerr(e, "row gather");
        goto done;
    }
    hipLaunchKernelGGL(k_rows_copy, dim3(nblk(n)), dim3(256), 0, nullptr, n, d_rows, d_ai, d_aj, d_aa, d_off, d_oj,
                       d_oa);
    if (off[n] > 0 &&
        ((e = hipMemcpy(cols.data(), d_oj, sizeof(int32_t) * (size_t)off[n], hipMemcpyDeviceToHost)) != hipSuccess ||
         (e = hipMemcpy(vals.data(), d_oa, sizeof(double) * (size_t)off[n], hipMemcpyDeviceToHost)) != hipSuccess))
        rc = gerr(e, "row gather");
done:
    hipFree(d_rows); hipFree(d_len); hipFree(d_off); hipFree(d_oj); hipFree(d_oa);
    return rc;
}

// Host CSR (int32 columns) -> device DCsr with the +2 tail pad.
int upload_csr(int32_t m, int32_t n, const std::vector<int32_t> &ai, const std::vector<int32_t> &aj,
               const std::vector<double> &aa, DCsr &D) {
    D = DCsr();
    D.m = m;
    D.n = n;
    D.nz = ai.empty() ? 0 : ai.back();
    hipError_t e;
    if ((e = dalloc(&D.ai, (int64_t)m + 1)) != hipSuccess || (e = dalloc(&D.aj, D.nz + 2)) != hipSuccess ||
        (e = dalloc(&D.aa, D.nz + 2)) != hipSuccess ||
        (e = hipMemcpy(D.ai, ai.data(), sizeof(int32_t) * ((size_t)m + 1), hipMemcpyHostToDevice)) != hipSuccess ||
        (e = hipMemset(D.aj, 0, sizeof(int32_t) * (size_t)(D.nz + 2))) != hipSuccess ||
        (e = hipMemset(D.aa, 0, sizeof(double) * (size_t)(D.nz + 2))) != hipSuccess ||
        (D.nz > 0 &&
         ((e = hipMemcpy(D.aj, aj.data(), sizeof(int32_t) * (size_t)D.nz, hipMemcpyHostToDevice)) != hipSuccess ||
          (e = hipMemcpy(D.aa, aa.data(), sizeof(double) * (size_t)D.nz, hipMemcpyHostToDevice)) != hipSuccess))) {
        D.release();
        return gerr(e, "upload");
    }
    return AIJHIP_OK;
}

__global__ void k_fill_value(int32_t m, double v, double *x) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < m) x[i] = v;
}

__global__ void k_len_total(int32_t m, const int32_t *__restrict__ len, unsigned long long *off) {
    if (threadIdx.x == 0 && blockIdx.x == 0) off[m] = m > 0 ? off[m - 1] + (unsigned long long)len[m - 1] : 0ull;
}

__global__ void k_narrow_off(int32_t n, const unsigned long long *__restrict__ w, int32_t *o) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) o[i] = (int32_t)w[i];
}

// exclusive scan of device int32 lengths into device int32 offsets (m + 1),
// on the device in 64-bit (dscan.h), one 8-byte read for the total
int scan_lengths(const int32_t *d_len, int32_t m, int32_t **d_off, int64_t *total) {
    unsigned long long *w = nullptr, *tmp = nullptr;
    hipError_t e;
    int rc = AIJHIP_OK;
    unsigned long long t = 0;
    *d_off = nullptr;
    if ((e = dalloc(&w, (int64_t)m + 1)) != hipSuccess ||
        (e = dalloc(&tmp, aijhip_dscan::scan_tmp_elems(std::max<int64_t>(m, 1)))) != hipSuccess ||
        (m > 0 && (e = aijhip_dscan::exclusive_scan(d_len, w, (int64_t)m, tmp, nullptr)) != hipSuccess)) {
        rc = gerr(e, "lengths");
        goto done;
    }
    hipLaunchKernelGGL(k_len_total, dim3(1), dim3(64), 0, nullptr, m, d_len, w);
    if ((e = hipMemcpy(&t, w + m, sizeof(t), hipMemcpyDeviceToHost)) != hipSuccess) {
        rc = gerr(e, "lengths");
        goto done;
    }
    if (t > (unsigned long long)INT32_MAX) {
        rc = mfail(AIJHIP_ERR_STATE, "distributed GAMG: a local operator past int32 entries");
        goto done;
    }
    *total = (int64_t)t;
    if ((e = dalloc(d_off, (int64_t)m + 1)) != hipSuccess) {
        rc = gerr(e, "offsets");
        goto done;
    }
    hipLaunchKernelGGL(k_narrow_off, dim3(nblk((int64_t)m + 1)), dim3(256), 0, nullptr, m + 1, w, *d_off);
    if ((e = hipGetLastError()) != hipSuccess) rc = gerr(e, "offsets");
done:
    hipFree(w);
    hipFree(tmp);
    if (rc) {
        hipFree(*d_off);
        *d_off = nullptr;
    }
    return rc;
}

// C = [A | B] (B: full row pointer bi, columns shifted by boff); bi may be null
int hcat(const DCsr &A, const int32_t *bi, const int32_t *bj, const double *ba, int32_t boff, int32_t ncols,
         DCsr &C) {
    C = DCsr();
    C.m = A.m;
    C.n = ncols;
    int32_t *len = nullptr;
    hipError_t e;
    if ((e = dalloc(&len, A.m)) != hipSuccess) return gerr(e, "alloc");
    if (A.m > 0) hipLaunchKernelGGL(k_hcat_len, dim3(nblk(A.m)), dim3(256), 0, nullptr, A.m, A.ai, bi, len);
    int rc = scan_lengths(len, A.m, &C.ai, &C.nz);
    hipFree(len);
    if (rc) return rc;
    if ((e = dalloc(&C.aj, C.nz + 2)) != hipSuccess || (e = dalloc(&C.aa, C.nz + 2)) != hipSuccess) {
        C.release();
        return gerr(e, "alloc");
    }
    if (A.m > 0)
        hipLaunchKernelGGL(k_hcat_fill, dim3(nblk(A.m)), dim3(256), 0, nullptr, A.m, A.ai, A.aj, A.aa, bi, bj, ba,
                           boff, C.ai, C.aj, C.aa);
    if ((e = hipGetLastError()) != hipSuccess) {
        C.release();
        return gerr(e, "concatenate");
    }
    return AIJHIP_OK;
}

// C = A + B (same shape, sorted rows)
int csr_add(const DCsr &A, const DCsr &B, DCsr &C) {
    C = DCsr();
    C.m = A.m;
    C.n = A.n;
    int32_t *len = nullptr;
    hipError_t e;
    if ((e = dalloc(&len, A.m)) != hipSuccess) return gerr(e, "alloc");
    if (A.m > 0)
        hipLaunchKernelGGL(k_add_len, dim3(nblk(A.m)), dim3(256), 0, nullptr, A.m, A.ai, A.aj, A.aa, B.ai, B.aj, B.aa,
                           len);
    int rc = scan_lengths(len, A.m, &C.ai, &C.nz);
    hipFree(len);
    if (rc) return rc;
    if ((e = dalloc(&C.aj, C.nz + 2)) != hipSuccess || (e = dalloc(&C.aa, C.nz + 2)) != hipSuccess) {
        C.release();
        return gerr(e, "alloc");
    }
    if (A.m > 0)
        hipLaunchKernelGGL(k_add_fill, dim3(nblk(A.m)), dim3(256), 0, nullptr, A.m, A.ai, A.aj, A.aa, B.ai, B.aj, B.aa,
                           C.ai, C.aj, C.aa);
    if ((e = hipGetLastError()) != hipSuccess) {
        C.release();
        return gerr(e, "sum");
    }
    return AIJHIP_OK;
}

// D = columns < nloc, O = the others shifted by -nloc (nghost columns)
int csr_split(const DCsr &C, int32_t nloc, int32_t nghost, DCsr &D, DCsr &O) {
    D = DCsr();
    O = DCsr();
    D.m = O.m = C.m;
    D.n = nloc;
    O.n = nghost;
    int32_t *ld = nullptr, *lo = nullptr;
    hipError_t e;
    if ((e = dalloc(&ld, C.m)) != hipSuccess || (e = dalloc(&lo, C.m)) != hipSuccess) {
        hipFree(ld);
        return gerr(e, "alloc");
    }
    if (C.m > 0)
        hipLaunchKernelGGL(k_split_len, dim3(nblk(C.m)), dim3(256), 0, nullptr, C.m, C.ai, C.aj, nloc, ld, lo);
    int rc = scan_lengths(ld, C.m, &D.ai, &D.nz);
    if (!rc) rc = scan_lengths(lo, C.m, &O.ai, &O.nz);
    hipFree(ld);
    hipFree(lo);
    if (rc) {
        D.release();
        O.release();
        return rc;
    }
    if ((e = dalloc(&D.aj, D.nz + 2)) != hipSuccess || (e = dalloc(&D.aa, D.nz + 2)) != hipSuccess ||
        (e = dalloc(&O.aj, O.nz + 2)) != hipSuccess || (e = dalloc(&O.aa, O.nz + 2)) != hipSuccess) {
        D.release();
        O.release();
        return gerr(e, "alloc");
    }
    if (C.m > 0)
        hipLaunchKernelGGL(k_split_fill, dim3(nblk(C.m)), dim3(256), 0, nullptr, C.m, C.ai, C.aj, C.aa, nloc, D.ai,
                           D.aj, D.aa, O.ai, O.aj, O.aa);
    if ((e = hipGetLastError()) != hipSuccess) {
        D.release();
        O.release();
        return gerr(e, "split");
    }
    return AIJHIP_OK;
}

int remap_cols(DCsr &C, const std::vector<int32_t> &table) {
    if (C.nz == 0) return AIJHIP_OK;
    int32_t *d_t = nullptr;
    hipError_t e;
    if ((e = dalloc(&d_t, (int64_t)table.size())) != hipSuccess ||
        (e = hipMemcpy(d_t, table.data(), sizeof(int32_t) * table.size(), hipMemcpyHostToDevice)) != hipSuccess) {
        hipFree(d_t);
        return gerr(e, "column map");
    }
    hipLaunchKernelGGL(k_remap, dim3(nblk(C.nz)), dim3(256), 0, nullptr, C.nz, d_t, C.aj);
    e = hipGetLastError();
    hipFree(d_t);
    return e == hipSuccess ? AIJHIP_OK : gerr(e, "column map");
}

// copy a handle's CSR into a DCsr view (not owned)
DCsr view(const aijhip_mat &A) {
    DCsr v;
    v.m = A.m;
    v.n = A.n;
    v.nz = A.nz;
    v.ai = A.d_ai;
    v.aj = A.d_aj;
    v.aa = A.d_aa;
    return v;
}

// A handle's CSR on the host with a full row pointer (compressed-row form expanded)
int host_full_rows(const aijhip_mat &A, std::vector<int32_t> &ai, std::vector<int32_t> &aj,
                   std::vector<double> &aa) {
    ai.assign((size_t)A.m + 1, 0);
    aj.resize((size_t)A.nz);
    aa.resize((size_t)A.nz);
    hipError_t e;
    if (A.nz > 0 && ((e = hipMemcpy(aj.data(), A.d_aj, sizeof(int32_t) * (size_t)A.nz, hipMemcpyDeviceToHost)) !=
                         hipSuccess ||
                     (e = hipMemcpy(aa.data(), A.d_aa, sizeof(double) * (size_t)A.nz, hipMemcpyDeviceToHost)) !=
                         hipSuccess))
        return gerr(e, "read block");
    if (!A.compressed) {
        if ((e = hipMemcpy(ai.data(), A.d_ai, sizeof(int32_t) * ai.size(), hipMemcpyDeviceToHost)) != hipSuccess)
            return gerr(e, "read block");
        return AIJHIP_OK;
    }
    std::vector<int32_t> cai((size_t)A.n_crow + 1), ridx((size_t)A.n_crow);
    if ((e = hipMemcpy(cai.data(), A.d_cai, sizeof(int32_t) * cai.size(), hipMemcpyDeviceToHost)) != hipSuccess ||
        (A.n_crow > 0 &&
         (e = hipMemcpy(ridx.data(), A.d_ridx, sizeof(int32_t) * ridx.size(), hipMemcpyDeviceToHost)) != hipSuccess))
        return gerr(e, "read block");
    std::vector<int32_t> len((size_t)A.m, 0);
    for (int32_t q = 0; q < A.n_crow; ++q) len[ridx[q]] = cai[q + 1] - cai[q];
    for (int32_t i = 0; i < A.m; ++i) ai[i + 1] = ai[i] + len[i];
    return AIJHIP_OK;
}

// Ghost values of a device vector through an operator's halo (host copy).
int halo_values(aijhip_mpiaij *M, const double *d_x, std::vector<double> &out) {
    out.assign((size_t)M->n_ghost, 0.0);
    int rc = aijhip_mpi::halo_post(M, d_x, nullptr);
    if (!rc) rc = aijhip_mpi::halo_finish(M, nullptr);
    if (rc) return rc;
    hipError_t e;
    if ((e = hipStreamSynchronize(nullptr)) != hipSuccess ||
        (M->n_ghost > 0 && (e = hipMemcpy(out.data(), M->d_ghost, sizeof(double) * out.size(),
                                          hipMemcpyDeviceToHost)) != hipSuccess))
        return gerr(e, "ghost values");
    return AIJHIP_OK;
}

// sqrt of the sum over all ranks of the 256-blocked local sums of squares
// sum a . b over the ranks: each rank's 256-entry block sums left to right,
// then the ranks' sums (the same order as global_norm)
int global_dot(aijhip_comm *C, const double *d_a, const double *d_b, int32_t m, double *d_part, double *out) {
    const int64_t nb = (m + kDotBlock - 1) / kDotBlock;
    std::vector<double> h((size_t)nb);
    hipError_t e;
    if (nb > 0) {
        hipLaunchKernelGGL(k_dot_blocks, dim3(nblk(nb, 64)), dim3(64), 0, nullptr, (int64_t)m, d_a, d_b, d_part);
        if ((e = hipMemcpy(h.data(), d_part, sizeof(double) * (size_t)nb, hipMemcpyDeviceToHost)) != hipSuccess)
            return gerr(e, "dot");
    }
    double s = 0.0;
    for (int64_t q = 0; q < nb; ++q) s += h[q];
    int rc = aijhip_mpi::comm_allreduce_host(C, &s, 1);
    if (rc) return rc;
    *out = s;
    return AIJHIP_OK;
}

int global_norm(aijhip_comm *C, const double *d_v, int32_t m, double *d_part, double *out) {
    const int64_t nb = (m + kDotBlock - 1) / kDotBlock;
    std::vector<double> h((size_t)nb);
    hipError_t e;
    if (nb > 0) {
        hipLaunchKernelGGL(k_sumsq_blocks, dim3(nblk(nb, 64)), dim3(64), 0, nullptr, (int64_t)m, d_v, d_part);
        if ((e = hipMemcpy(h.data(), d_part, sizeof(double) * (size_t)nb, hipMemcpyDeviceToHost)) != hipSuccess)
            return gerr(e, "norm");
    }
    double s = 0.0;
    for (int64_t q = 0; q < nb; ++q) s += h[q];
    int rc = aijhip_mpi::comm_allreduce_host(C, &s, 1);
    if (rc) return rc;
    *out = std::sqrt(s);
    return AIJHIP_OK;
}


// ---- the distributed MIS (coarsen 1; kernels k_dm_*): see the kernels'
// comment. In: the level (handles, halo, ghost ids), its strength graph S_d
// and diagonal from aggregate_level, the near-null space B. Out: the own
// roots' count na and every rank's (cstarts), per local node the coarse
// global id of its aggregate (cg, -1 removed), its local aggregate (agg: own
// roots' aggregates, -1 otherwise), p0 = B_i / Bc, and the own aggregates'
// Bc; on the host the local nodes whose aggregate is rooted on another rank
// (PETSc's mis.c: a node deleted by a selected ghost joins that ghost's
// aggregate, lid_parent_gid) with their coarse ids. Bc sums B^2 over the
// members: its own in ascending order, then the other ranks' (each a sum in
// their ascending order) in rank order.
struct DistMis {
    int32_t na = 0, rounds = 0;
    std::vector<int64_t> cstarts;
    double *d_cg = nullptr, *d_p0 = nullptr, *d_Bc = nullptr;
    int32_t *d_agg = nullptr;
    std::vector<int32_t> rnode;
    std::vector<int64_t> rcg;
    ~DistMis() { release(); }
    void release() {
        hipFree(d_cg); hipFree(d_p0); hipFree(d_Bc); hipFree(d_agg);
        d_cg = d_p0 = d_Bc = nullptr;
        d_agg = nullptr;
    }
};

// the ghost values of d_x in M->d_ghost, ordered on the null stream
int halo_device(aijhip_mpiaij *M, const double *d_x) {
    int rc = aijhip_mpi::halo_post(M, d_x, nullptr);
    if (!rc) rc = aijhip_mpi::halo_finish(M, nullptr);
    return rc;
}

int dist_mis(aijhip_comm *C, aijhip_gamg_mpi::Level &L, const aijhip_gamg_params_t &p, int32_t level,
             const aijhip_gamg::StrengthGraph &S, const double *d_B, bool b_ones, DistMis &out) {
    const int32_t m = L.m, ng = (int32_t)L.ghost_gid.size();
    const int P = C->nranks, me = C->rank;
    const int64_t rstart = L.rstart, M = L.starts[P];
    const bool square = level < p.square_graph;
    const bool log = std::getenv("AIJHIP_GAMG_LOG") != nullptr;
    aijhip_mpiaij *op = L.op;
    const unsigned g = nblk(m);
    int rc = AIJHIP_OK;
    hipError_t e = hipSuccess;
    double *gd = nullptr, *val = nullptr, *amin = nullptr;
    int32_t *cnt = nullptr, *soi = nullptr, *soj = nullptr, *flag = nullptr, *idx = nullptr;
    int32_t *rnode_d = nullptr;
    int64_t *ggid = nullptr, *hi = nullptr, *parent = nullptr, *rpar_d = nullptr;
    uint32_t *hk = nullptr;
    dmis_t *state = nullptr;
    unsigned *wcount = nullptr, *rcount = nullptr;
    unsigned long long *left = nullptr;
    int64_t nso = 0;
#define DM(call, what) do { if ((e = (call)) != hipSuccess) { rc = gerr(e, what); goto done; } } while (0)
#define DMRC(call) do { if ((rc = (call))) goto done; } while (0)
    // ---- S_o: the ghosts' diagonal through the halo, then the filter
    DM(dalloc(&gd, std::max(ng, 1)), "alloc");
    DMRC(halo_device(op, S.d));
    if (ng > 0) DM(hipMemcpyAsync(gd, op->d_ghost, sizeof(double) * (size_t)ng, hipMemcpyDeviceToDevice, nullptr), "copy");
    DM(dalloc(&cnt, m), "alloc");
    DM(hipMemsetAsync(cnt, 0, sizeof(int32_t) * (size_t)std::max(m, 1), nullptr), "memset");
    if (L.Ao && ng > 0) {
        const aijhip::RowList R = aijhip::row_list(*L.Ao);
        if (R.nr > 0)
            hipLaunchKernelGGL(k_dm_so_count, dim3(nblk(R.nr)), dim3(256), 0, nullptr, R.nr, R.rai, R.ridx,
                               L.Ao->d_aa, S.d, gd, L.Ao->d_aj, p.threshold, cnt);
        DMRC(scan_lengths(cnt, m, &soi, &nso));
        DM(dalloc(&soj, std::max<int64_t>(nso, 1)), "alloc");
        if (R.nr > 0)
            hipLaunchKernelGGL(k_dm_so_fill, dim3(nblk(R.nr)), dim3(256), 0, nullptr, R.nr, R.rai, R.ridx,
                               L.Ao->d_aa, S.d, gd, L.Ao->d_aj, p.threshold, soi, soj);
    } else {
        DMRC(scan_lengths(cnt, m, &soi, &nso));
        DM(dalloc(&soj, 1), "alloc");
    }
    // ---- the rounds
    DM(dalloc(&state, m), "alloc");
    DM(dalloc(&hk, m), "alloc");
    DM(dalloc(&val, m), "alloc");
    DM(dalloc(&amin, m), "alloc");
    DM(dalloc(&wcount, g), "alloc");
    DM(dalloc(&left, 1), "alloc");
    if (m > 0) hipLaunchKernelGGL(k_dm_init, dim3(g), dim3(256), 0, nullptr, m, rstart, level, S.si, soi, state, hk);
    {
        constexpr int32_t kBatch = 4;
        bool done_all = false;
        for (int64_t r0 = 0; !done_all && r0 <= M; r0 += kBatch) {
            for (int32_t r = 0; r < kBatch; ++r) {
                if (m > 0) hipLaunchKernelGGL(k_dm_value, dim3(g), dim3(256), 0, nullptr, m, rstart, state, hk, false, val);
                DMRC(halo_device(op, val));
                if (m > 0)
                    hipLaunchKernelGGL(k_dm_closed_min, dim3(g), dim3(256), 0, nullptr, m, rstart, S.si, S.sj, soi, soj,
                                       state, hk, op->d_ghost, false, amin);
                DMRC(halo_device(op, amin));
                if (m > 0)
                    hipLaunchKernelGGL(k_dm_decide, dim3(g), dim3(256), 0, nullptr, m, rstart, S.si, S.sj, soi, soj,
                                       square, hk, amin, op->d_ghost, state, wcount);
            }
            unsigned long long h_left = 0;
            if (m > 0) {
                hipLaunchKernelGGL(k_dm_total, dim3(1), dim3(1024), 0, nullptr, wcount, (int32_t)g, left);
                DM(hipMemcpy(&h_left, left, sizeof(h_left), hipMemcpyDeviceToHost), "count");
            }
            double tot = (double)h_left;
            DMRC(aijhip_mpi::comm_allreduce_host(C, &tot, 1));
            out.rounds = (int32_t)(r0 + kBatch);
            if (log)
                std::fprintf(stderr, "[rank %d] distributed MIS level %d rounds %lld-%lld: %.0f undecided\n", me, level,
                             (long long)r0, (long long)(r0 + kBatch - 1), tot);
            done_all = tot == 0.0;
        }
        if (!done_all) {
            rc = mfail(AIJHIP_ERR_STATE, "distributed GAMG: the MIS rounds did not finish");
            goto done;
        }
    }
    // ---- parents: the roots' keys within reach (and smoothAggs' neighbours)
    DM(dalloc(&ggid, std::max(ng, 1)), "alloc");
    if (ng > 0) DM(hipMemcpy(ggid, L.ghost_gid.data(), sizeof(int64_t) * (size_t)ng, hipMemcpyHostToDevice), "ghost ids");
    DM(dalloc(&hi, m), "alloc");
    DM(dalloc(&parent, m), "alloc");
    DM(dalloc(&flag, m), "alloc");
    if (m > 0) hipLaunchKernelGGL(k_dm_value, dim3(g), dim3(256), 0, nullptr, m, rstart, state, hk, true, val);
    DMRC(halo_device(op, val));
    if (m > 0) {
        hipLaunchKernelGGL(k_dm_hiroot, dim3(g), dim3(256), 0, nullptr, m, rstart, S.si, S.sj, soi, soj, state,
                           op->d_ghost, ggid, hi);
        hipLaunchKernelGGL(k_dm_closed_min, dim3(g), dim3(256), 0, nullptr, m, rstart, S.si, S.sj, soi, soj, state, hk,
                           op->d_ghost, true, amin);
    }
    DMRC(halo_device(op, amin));
    if (m > 0)
        hipLaunchKernelGGL(k_dm_parent, dim3(g), dim3(256), 0, nullptr, m, rstart, S.si, S.sj, soi, soj, square, amin,
                           op->d_ghost, state, hi, parent, flag);
    {
        int64_t na64 = 0;
        DMRC(scan_lengths(flag, m, &idx, &na64));
        out.na = (int32_t)na64;
    }
    {
        std::vector<int64_t> all;
        DMRC(all_values(C, out.na, all));
        out.cstarts.assign((size_t)P + 1, 0);
        for (int q = 0; q < P; ++q) out.cstarts[q + 1] = out.cstarts[q] + all[q];
    }
    {
        const int64_t cstart = out.cstarts[me];
        DM(dalloc(&out.d_cg, m), "alloc");
        DM(dalloc(&out.d_agg, m), "alloc");
        DM(dalloc(&out.d_p0, m), "alloc");
        DM(dalloc(&out.d_Bc, std::max(out.na, 1)), "alloc");
        DM(dalloc(&rnode_d, m), "alloc");
        DM(dalloc(&rpar_d, m), "alloc");
        DM(dalloc(&rcount, 1), "alloc");
        DM(hipMemset(rcount, 0, sizeof(unsigned)), "memset");
        if (m > 0)
            hipLaunchKernelGGL(k_dm_coarse, dim3(g), dim3(256), 0, nullptr, m, rstart, cstart, parent, idx, out.d_cg,
                               out.d_agg, rnode_d, rpar_d, rcount);
        unsigned nr = 0;
        DM(hipMemcpy(&nr, rcount, sizeof(nr), hipMemcpyDeviceToHost), "remote count");
        // own members' sums of squares, ascending (the single-GPU Bc before its root)
        DM(aijhip_gamg::aggregate_sumsq_device(m, out.na, out.d_agg, b_ones ? nullptr : d_B, out.d_Bc, b_ones),
           "aggregate sums");
        // the members on this rank of other ranks' aggregates: sorted by node
        std::vector<int32_t> rn(nr);
        std::vector<int64_t> rp(nr);
        std::vector<double> rb(nr, 1.0);
        if (nr > 0) {
            DM(hipMemcpy(rn.data(), rnode_d, sizeof(int32_t) * nr, hipMemcpyDeviceToHost), "remote nodes");
            DM(hipMemcpy(rp.data(), rpar_d, sizeof(int64_t) * nr, hipMemcpyDeviceToHost), "remote parents");
            std::vector<uint32_t> ord(nr);
            std::iota(ord.begin(), ord.end(), 0u);
            std::sort(ord.begin(), ord.end(), [&](uint32_t a, uint32_t b) { return rn[a] < rn[b]; });
            std::vector<int32_t> rn2(nr);
            std::vector<int64_t> rp2(nr);
            for (unsigned k = 0; k < nr; ++k) { rn2[k] = rn[ord[k]]; rp2[k] = rp[ord[k]]; }
            rn.swap(rn2);
            rp.swap(rp2);
            if (!b_ones) {  // B at those nodes
                double *bv = nullptr;
                DM(dalloc(&bv, nr), "alloc");
                DM(hipMemcpy(rnode_d, rn.data(), sizeof(int32_t) * nr, hipMemcpyHostToDevice), "remote nodes");
                hipLaunchKernelGGL(k_dm_gather_f64, dim3(nblk(nr)), dim3(256), 0, nullptr, (int32_t)nr, rnode_d, d_B, bv);
                e = hipMemcpy(rb.data(), bv, sizeof(double) * nr, hipMemcpyDeviceToHost);
                hipFree(bv);
                if (e != hipSuccess) { rc = gerr(e, "remote B"); goto done; }
            }
        }
        // requests: per owner, per parent (ascending) the sum of B^2 of its
        // members here (in ascending node order)
        std::vector<std::vector<uint64_t>> req((size_t)P), got;
        std::vector<std::vector<int64_t>> asked((size_t)P);  // the parents asked of each owner, in order
        {
            std::vector<uint32_t> ord(nr);
            std::iota(ord.begin(), ord.end(), 0u);
            std::stable_sort(ord.begin(), ord.end(), [&](uint32_t a, uint32_t b) { return rp[a] < rp[b]; });
            for (unsigned k = 0; k < nr;) {
                const int64_t par = rp[ord[k]];
                double s2 = 0.0;
                unsigned j = k;
                for (; j < nr && rp[ord[j]] == par; ++j) s2 += rb[ord[j]] * rb[ord[j]];
                const int q = owner_of(L.starts, par);
                uint64_t bits;
                std::memcpy(&bits, &s2, 8);
                req[q].push_back((uint64_t)par);
                req[q].push_back(bits);
                asked[q].push_back(par);
                k = j;
            }
        }
        DMRC(aijhip_mpi::comm_sendrecv(C, req, got));
        // owner: the requested roots' local aggregates, the other ranks'
        // contributions added (rank order), then Bc and the replies
        std::vector<int32_t> rroot;  // every requested root (local index), in (rank, message) order
        for (int q = 0; q < P; ++q) {
            if (q == me) continue;
            for (size_t k = 0; k + 1 < got[q].size(); k += 2) {
                const int64_t par = (int64_t)got[q][k];
                if (par < rstart || par >= rstart + m) {
                    rc = mfail(AIJHIP_ERR_COMM, "distributed GAMG: a root request for another rank's node");
                    goto done;
                }
                rroot.push_back((int32_t)(par - rstart));
            }
        }
        std::vector<int32_t> ragg(rroot.size());
        if (!rroot.empty()) {
            int32_t *at = nullptr, *o = nullptr;
            const int32_t n = (int32_t)rroot.size();
            if ((e = dalloc(&at, n)) == hipSuccess && (e = dalloc(&o, n)) == hipSuccess &&
                (e = hipMemcpy(at, rroot.data(), sizeof(int32_t) * (size_t)n, hipMemcpyHostToDevice)) == hipSuccess) {
                hipLaunchKernelGGL(k_dm_gather_i32, dim3(nblk(n)), dim3(256), 0, nullptr, n, at, idx, o);
                e = hipMemcpy(ragg.data(), o, sizeof(int32_t) * (size_t)n, hipMemcpyDeviceToHost);
            }
            hipFree(at);
            hipFree(o);
            if (e != hipSuccess) { rc = gerr(e, "requested roots"); goto done; }
        }
        {
            // per aggregate the other ranks' sums, added in rank order
            std::vector<std::pair<int32_t, double>> adds;
            size_t t = 0;
            for (int q = 0; q < P; ++q) {
                if (q == me) continue;
                for (size_t k = 0; k + 1 < got[q].size(); k += 2, ++t) {
                    double v;
                    std::memcpy(&v, &got[q][k + 1], 8);
                    adds.emplace_back(ragg[t], v);
                }
            }
            std::stable_sort(adds.begin(), adds.end(),
                             [](const std::pair<int32_t, double> &a, const std::pair<int32_t, double> &b) {
                                 return a.first < b.first;
                             });
            std::vector<int32_t> aa_i;
            std::vector<double> aa_v;
            for (size_t k = 0; k < adds.size();) {
                double v = 0.0;
                size_t j = k;
                for (; j < adds.size() && adds[j].first == adds[k].first; ++j) v += adds[j].second;
                aa_i.push_back(adds[k].first);
                aa_v.push_back(v);
                k = j;
            }
            if (!aa_i.empty()) {
                int32_t *di = nullptr;
                double *dv = nullptr;
                const int32_t n = (int32_t)aa_i.size();
                if ((e = dalloc(&di, n)) == hipSuccess && (e = dalloc(&dv, n)) == hipSuccess &&
                    (e = hipMemcpy(di, aa_i.data(), sizeof(int32_t) * (size_t)n, hipMemcpyHostToDevice)) == hipSuccess &&
                    (e = hipMemcpy(dv, aa_v.data(), sizeof(double) * (size_t)n, hipMemcpyHostToDevice)) == hipSuccess)
                    hipLaunchKernelGGL(k_dm_add_at, dim3(nblk(n)), dim3(256), 0, nullptr, n, di, dv, out.d_Bc);
                if (e == hipSuccess) e = hipStreamSynchronize(nullptr);
                hipFree(di);
                hipFree(dv);
                if (e != hipSuccess) { rc = gerr(e, "remote sums"); goto done; }
            }
        }
        if (out.na > 0) hipLaunchKernelGGL(k_dm_sqrt, dim3(nblk(out.na)), dim3(256), 0, nullptr, out.na, out.d_Bc);
        if (m > 0)
            hipLaunchKernelGGL(k_dm_p0, dim3(g), dim3(256), 0, nullptr, m, out.d_agg, b_ones ? nullptr : d_B, out.d_Bc,
                               out.d_p0);
        // replies: per request (in its order) the coarse id and Bc
        std::vector<double> rbc(ragg.size());
        if (!ragg.empty()) {
            int32_t *at = nullptr;
            double *o = nullptr;
            const int32_t n = (int32_t)ragg.size();
            if ((e = dalloc(&at, n)) == hipSuccess && (e = dalloc(&o, n)) == hipSuccess &&
                (e = hipMemcpy(at, ragg.data(), sizeof(int32_t) * (size_t)n, hipMemcpyHostToDevice)) == hipSuccess) {
                hipLaunchKernelGGL(k_dm_gather_f64, dim3(nblk(n)), dim3(256), 0, nullptr, n, at, out.d_Bc, o);
                e = hipMemcpy(rbc.data(), o, sizeof(double) * (size_t)n, hipMemcpyDeviceToHost);
            }
            hipFree(at);
            hipFree(o);
            if (e != hipSuccess) { rc = gerr(e, "replies"); goto done; }
        }
        std::vector<std::vector<uint64_t>> rep((size_t)P), back;
        {
            size_t t = 0;
            for (int q = 0; q < P; ++q) {
                if (q == me) continue;
                for (size_t k = 0; k + 1 < got[q].size(); k += 2, ++t) {
                    uint64_t bits;
                    std::memcpy(&bits, &rbc[t], 8);
                    rep[q].push_back((uint64_t)(cstart + ragg[t]));
                    rep[q].push_back(bits);
                }
            }
        }
        DMRC(aijhip_mpi::comm_sendrecv(C, rep, back));
        // this rank's members of other ranks' aggregates: coarse id, p0
        std::vector<int64_t> pcg;  // per parent asked (owner order, then ascending)
        std::vector<double> pbc;
        std::vector<int64_t> plist;
        for (int q = 0; q < P; ++q) {
            if (q == me) continue;
            if (back[q].size() != 2 * asked[q].size()) {
                rc = mfail(AIJHIP_ERR_COMM, "distributed GAMG: short root reply");
                goto done;
            }
            for (size_t k = 0; k < asked[q].size(); ++k) {
                plist.push_back(asked[q][k]);
                pcg.push_back((int64_t)back[q][2 * k]);
                double v;
                std::memcpy(&v, &back[q][2 * k + 1], 8);
                pbc.push_back(v);
            }
        }
        std::vector<uint32_t> pord(plist.size());
        std::iota(pord.begin(), pord.end(), 0u);
        std::sort(pord.begin(), pord.end(), [&](uint32_t a, uint32_t b) { return plist[a] < plist[b]; });
        out.rnode = rn;
        out.rcg.assign(nr, -1);
        std::vector<double> cgv(nr), p0v(nr);
        for (unsigned k = 0; k < nr; ++k) {
            const auto it = std::lower_bound(pord.begin(), pord.end(), rp[k],
                                             [&](uint32_t a, int64_t v) { return plist[a] < v; });
            if (it == pord.end() || plist[*it] != rp[k]) {
                rc = mfail(AIJHIP_ERR_COMM, "distributed GAMG: a root without a reply");
                goto done;
            }
            out.rcg[k] = pcg[*it];
            cgv[k] = (double)pcg[*it];
            const double c = pbc[*it];
            p0v[k] = c > 0.0 ? rb[k] / c : 0.0;
        }
        if (nr > 0) {
            double *dc = nullptr, *dp = nullptr;
            if ((e = dalloc(&dc, nr)) == hipSuccess && (e = dalloc(&dp, nr)) == hipSuccess &&
                (e = hipMemcpy(rnode_d, rn.data(), sizeof(int32_t) * nr, hipMemcpyHostToDevice)) == hipSuccess &&
                (e = hipMemcpy(dc, cgv.data(), sizeof(double) * nr, hipMemcpyHostToDevice)) == hipSuccess &&
                (e = hipMemcpy(dp, p0v.data(), sizeof(double) * nr, hipMemcpyHostToDevice)) == hipSuccess)
                hipLaunchKernelGGL(k_dm_set_remote, dim3(nblk(nr)), dim3(256), 0, nullptr, (int32_t)nr, rnode_d, dc, dp,
                                   out.d_cg, out.d_p0);
            if (e == hipSuccess) e = hipStreamSynchronize(nullptr);
            hipFree(dc);
            hipFree(dp);
            if (e != hipSuccess) { rc = gerr(e, "remote members"); goto done; }
        }
        if (log)
            std::fprintf(stderr, "[rank %d] distributed MIS level %d: %d rounds, %d own aggregates, %u members of "
                         "other ranks' aggregates\n", me, level, out.rounds, out.na, nr);
    }
    DM(hipGetLastError(), "distributed MIS");
done:
#undef DM
#undef DMRC
    hipFree(gd); hipFree(val); hipFree(amin); hipFree(cnt); hipFree(soi); hipFree(soj); hipFree(flag); hipFree(idx);
    hipFree(rnode_d); hipFree(ggid); hipFree(hi); hipFree(parent); hipFree(rpar_d); hipFree(hk); hipFree(state);
    hipFree(wcount); hipFree(rcount); hipFree(left);
    if (rc) out.release();
    return rc;
}

}  // namespace

namespace aijhip_gamg_mpi {

void Hierarchy::destroy() {
    for (size_t l = 0; l < lv.size(); ++l) {
        Level &L = lv[l];
        if (L.op && l > 0) aijhip_mpiaij_destroy(L.op);
        if (l > 0) {
            aijhip_mat_destroy(L.Ad);
            aijhip_mat_destroy(L.Ao);
        }
        aijhip_mat_destroy(L.Pd);
        aijhip_mat_destroy(L.Po);
        aijhip_mat_destroy(L.Ro);
        hipFree(L.dinv); hipFree(L.b); hipFree(L.x); hipFree(L.r);
    }
    lv.clear();
}

// The p2p halo plan of a level from its sorted ghost list: requests to the
// owners (ghost order = owner order), send lists from what others request.
static int make_operator(aijhip_comm *C, aijhip_mat *Ad, aijhip_mat *Ao, const std::vector<int64_t> &ghosts,
                         const std::vector<int64_t> &starts, aijhip_mpiaij **out) {
    const int P = C->nranks;
    std::vector<std::vector<uint64_t>> req((size_t)P), got;
    std::vector<int32_t> recv_peer;
    std::vector<int64_t> recv_off{0};
    for (size_t s = 0; s < ghosts.size();) {
        const int q = owner_of(starts, ghosts[s]);
        size_t e = s;
        while (e < ghosts.size() && owner_of(starts, ghosts[e]) == q) {
            req[q].push_back((uint64_t)(ghosts[e] - starts[q]));
            ++e;
        }
        recv_peer.push_back(q);
        recv_off.push_back((int64_t)e);
        s = e;
    }
    int rc = aijhip_mpi::comm_sendrecv(C, req, got);
    if (rc) return rc;
    std::vector<int32_t> send_peer, send_rows;
    std::vector<int64_t> send_off{0};
    for (int q = 0; q < P; ++q) {
        if (q == C->rank || got[q].empty()) continue;
        send_peer.push_back(q);
        for (uint64_t r : got[q]) send_rows.push_back((int32_t)r);
        send_off.push_back((int64_t)send_rows.size());
    }
    return aijhip_mpiaij_create(C, Ad, Ao, AIJHIP_HALO_P2P, (int32_t)send_peer.size(), send_peer.data(),
                                send_off.data(), send_rows.empty() ? nullptr : send_rows.data(),
                                (int32_t)recv_peer.size(), recv_peer.data(), recv_off.data(), 0, out);
}

// A level's interpolation handles (P_d with R_d = P_d^T attached, and P_o)
// made on a second host thread, as the single-GPU set-up does: planning
// P_d's STREAM handle reads its row offsets back to the host, and nothing
// needs the handles before the V-cycle. No communication inside.
struct PJob {
    std::thread th;
    size_t level = 0;
    int rc = AIJHIP_OK;
    std::string err;
    aijhip_mat *Pd = nullptr, *Po = nullptr;
    void start(int device, size_t l, DCsr pd, DCsr po) {
        level = l;
        th = std::thread([this, device, pd, po]() mutable {
            (void)hipSetDevice(device);
            rc = aijhip_gamg::make_level_handle(device, pd, &Pd);
            if (!rc) {
                int32_t *ti = nullptr, *tj = nullptr;
                double *ta = nullptr;
                const hipError_t e = aijhip::build_transpose(*Pd, &ti, &tj, &ta, nullptr);
                rc = e != hipSuccess ? gerr(e, "P^T") : aijhip::attach_transpose(Pd, ti, tj, ta);
            }
            if (!rc && po.nz > 0) rc = aijhip_gamg::make_level_handle(device, po, &Po);
            if (!rc && Po) {  // P_o^T for the restriction's off-rank share (vcycle)
                int32_t *ti = nullptr, *tj = nullptr;
                double *ta = nullptr;
                const hipError_t e = aijhip::build_transpose(*Po, &ti, &tj, &ta, nullptr);
                rc = e != hipSuccess ? gerr(e, "P_o^T") : aijhip::attach_transpose(Po, ti, tj, ta);
            }
            po.release();
            pd.release();
            if (rc) {
                err = aijhip_last_error();
                aijhip_mat_destroy(Pd);
                aijhip_mat_destroy(Po);
                Pd = Po = nullptr;
            }
        });
    }
    void join() {
        if (th.joinable()) th.join();
    }
    ~PJob() {
        join();
        aijhip_mat_destroy(Pd);
        aijhip_mat_destroy(Po);
    }
};

int build(aijhip_mpiaij *M0, const aijhip_gamg_params_t &p, Hierarchy &H) {
    aijhip::Range range("PCSetUp_GAMG (MPIAIJ)");
    H.destroy();
    aijhip_comm *C = M0->comm;
    if (M0->halo != AIJHIP_HALO_P2P)
        return mfail(AIJHIP_ERR_ARG, "distributed GAMG: the operator needs the p2p halo (AIJHIP_HALO_P2P)");
    const bool log = std::getenv("AIJHIP_GAMG_LOG") != nullptr;
    auto t0 = std::chrono::steady_clock::now();
    auto lap = [&](size_t l, const char *what) {
        if (!log) return;
        (void)hipDeviceSynchronize();
        const auto t = std::chrono::steady_clock::now();
        std::fprintf(stderr, "[rank %d] gamg mpi level %zu %-22s %8.3f s\n", C->rank, l, what,
                     std::chrono::duration<double>(t - t0).count());
        t0 = t;
    };
    const int P = C->nranks, me = C->rank;
    const int n_cu = std::max(M0->Ad->n_cu, 1);
    constexpr bool in_line = false;  // the interpolation handles come from a second host thread
    std::vector<std::unique_ptr<PJob>> jobs;
    hipError_t e;
    int rc = AIJHIP_OK;
    // ---- level 0: the caller's operator and its ghost global ids
    H.lv.emplace_back();
    {
        Level &L0 = H.lv[0];
        L0.Ad = M0->Ad;
        L0.Ao = M0->Ao;
        L0.op = M0;
        L0.m = M0->mloc;
        std::vector<int64_t> all;
        if ((rc = all_values(C, L0.m, all))) return rc;
        L0.starts.assign((size_t)P + 1, 0);
        for (int q = 0; q < P; ++q) L0.starts[q + 1] = L0.starts[q] + all[q];
        L0.rstart = L0.starts[me];
        double *gid = nullptr;
        if ((e = dalloc(&gid, L0.m)) != hipSuccess) return gerr(e, "alloc");
        std::vector<int32_t> agg_id;  // gid = rstart + i
        int32_t *iota = nullptr;
        if ((e = dalloc(&iota, (int64_t)L0.m + 1)) != hipSuccess) {
            hipFree(gid);
            return gerr(e, "alloc");
        }
        hipLaunchKernelGGL(k_iota32, dim3(nblk((int64_t)L0.m + 1)), dim3(256), 0, nullptr, L0.m, iota);
        if (L0.m > 0) hipLaunchKernelGGL(k_coarse_gid, dim3(nblk(L0.m)), dim3(256), 0, nullptr, L0.m, L0.rstart, iota, gid);
        std::vector<double> g;
        rc = halo_values(M0, gid, g);
        hipFree(gid);
        hipFree(iota);
        if (rc) return rc;
        L0.ghost_gid.resize(g.size());
        for (size_t s = 0; s < g.size(); ++s) L0.ghost_gid[s] = (int64_t)g[s];
    }
    // the near-null space of the current level (ones at the top)
    double *d_B = nullptr;
    if ((e = dalloc(&d_B, H.lv[0].m)) != hipSuccess) return gerr(e, "alloc");
    if (H.lv[0].m > 0)
        hipLaunchKernelGGL(k_fill_value, dim3(nblk(H.lv[0].m)), dim3(256), 0, nullptr, H.lv[0].m, 1.0, d_B);
    lap(0, "ghost ids, B");
    for (;;) {
        const size_t l = H.lv.size() - 1;
        Level &L = H.lv[l];
        const int32_t m = L.m;
        const int64_t M = L.starts[P];
        if ((int32_t)H.lv.size() >= p.max_levels || M <= p.coarse_eq_limit) break;
        // ---- emax(D^-1 A) of the distributed operator, on a second host
        // thread while this one forms the local aggregates (which need no
        // communication; the thread's halo exchanges and all-reduces are the
        // only collectives in flight, in the same order on every rank, and it
        // is joined before the next one below)
        double emax = 1.0;
        int emax_rc = AIJHIP_OK;
        std::string emax_err;
        double *dinv_e = nullptr;
        std::thread emax_th;
        if (p.nsmooths > 0) {
            if ((e = dalloc(&dinv_e, m)) != hipSuccess) {
                rc = gerr(e, "alloc");
                break;
            }
            if (m > 0)
                hipLaunchKernelGGL(k_diag_inv, dim3(nblk(m)), dim3(256), 0, nullptr, m, L.Ad->d_ai, L.Ad->d_aj,
                                   L.Ad->d_aa, dinv_e);
            emax_th = std::thread([&, dev = L.Ad->device]() {
                (void)hipSetDevice(dev);
                if (p.eig_ksp == 1) {  // CG's Lanczos estimate (PETSc's; gamg_setup.cpp estimate_emax_cg)
                    double *r = nullptr, *z = nullptr, *pv = nullptr, *w = nullptr, *part = nullptr;
                    hipError_t x;
                    if ((x = dalloc(&r, m)) != hipSuccess || (x = dalloc(&z, m)) != hipSuccess ||
                        (x = dalloc(&pv, m)) != hipSuccess || (x = dalloc(&w, m)) != hipSuccess ||
                        (x = dalloc(&part, (m + kDotBlock - 1) / kDotBlock)) != hipSuccess)
                        emax_rc = gerr(x, "alloc");
                    std::vector<double> alpha, beta;
                    double rz = 0.0;
                    if (!emax_rc) {
                        if (m > 0)
                            hipLaunchKernelGGL(k_cgest_start_off, dim3(nblk(m)), dim3(256), 0, nullptr, m, L.rstart,
                                               dinv_e, r, z, pv);
                        emax_rc = global_dot(C, z, r, m, part, &rz);
                    }
                    for (int it = 0; !emax_rc && it < p.eig_its; ++it) {
                        if ((emax_rc = aijhip_mpi::mpiaij_apply(L.op, pv, w, nullptr, nullptr, nullptr, nullptr, false)))
                            break;
                        double pw = 0.0;
                        if ((emax_rc = global_dot(C, pv, w, m, part, &pw))) break;
                        if (!(pw != 0.0 && rz != 0.0)) break;
                        const double a = rz / pw;
                        alpha.push_back(a);
                        if (m > 0)
                            hipLaunchKernelGGL(k_cgest_update, dim3(nblk(m)), dim3(256), 0, nullptr, m, a, w, dinv_e, r, z);
                        double rzn = 0.0;
                        if ((emax_rc = global_dot(C, z, r, m, part, &rzn))) break;
                        const double b = rzn / rz;
                        beta.push_back(b);
                        if (m > 0) hipLaunchKernelGGL(k_cgest_dir, dim3(nblk(m)), dim3(256), 0, nullptr, m, b, z, pv);
                        rz = rzn;
                    }
                    (void)hipStreamSynchronize(nullptr);
                    if (!emax_rc && !alpha.empty()) emax = aijhip_gamg::lanczos_emax(alpha, beta);
                    hipFree(r); hipFree(z); hipFree(pv); hipFree(w); hipFree(part);
                    if (emax_rc) emax_err = aijhip_last_error();
                    return;
                }
                double *v = nullptr, *w = nullptr, *part = nullptr;
                hipError_t x;
                if ((x = dalloc(&v, m)) != hipSuccess || (x = dalloc(&w, m)) != hipSuccess ||
                    (x = dalloc(&part, (m + kDotBlock - 1) / kDotBlock)) != hipSuccess)
                    emax_rc = gerr(x, "alloc");
                double nv = 0.0;
                if (!emax_rc) {
                    if (m > 0) hipLaunchKernelGGL(k_power_start_off, dim3(nblk(m)), dim3(256), 0, nullptr, m, L.rstart, v);
                    emax_rc = global_norm(C, v, m, part, &nv);
                }
                if (!emax_rc && m > 0) hipLaunchKernelGGL(k_divide, dim3(nblk(m)), dim3(256), 0, nullptr, m, v, nv, v);
                for (int it = 0; !emax_rc && it < p.eig_its; ++it) {
                    if ((emax_rc = aijhip_mpi::mpiaij_apply(L.op, v, w, nullptr, nullptr, nullptr, nullptr, false))) break;
                    if (m > 0) hipLaunchKernelGGL(k_scale_by, dim3(nblk(m)), dim3(256), 0, nullptr, m, dinv_e, w);
                    double nw = 0.0;
                    if ((emax_rc = global_norm(C, w, m, part, &nw))) break;
                    if (!(nw > 0.0)) break;
                    emax = nw;
                    if (m > 0) hipLaunchKernelGGL(k_divide, dim3(nblk(m)), dim3(256), 0, nullptr, m, w, nw, v);
                }
                (void)hipStreamSynchronize(nullptr);
                hipFree(v); hipFree(w); hipFree(part);
                if (emax_rc) emax_err = aijhip_last_error();
            });
        }
        // ---- aggregates: PETSc's parallel MIS across the ranks (coarsen 1,
        // dist_mis: the strength graph of A_d from the single-GPU steps, the
        // rounds over the level's halo), or the greedy pass on each rank's
        // diagonal block (coarsen 0; aggregates local)
        int32_t *d_agg = nullptr, na = 0;
        double *dinv = nullptr;
        const bool dmis = p.coarsen == 1;
        aijhip_gamg::StrengthGraph S;
        DistMis DMo;
        rc = aijhip_gamg::aggregate_level(*L.Ad, p, &d_agg, &na, &dinv, 0, nullptr, nullptr, l, dmis ? &S : nullptr);
        if (emax_th.joinable()) emax_th.join();
        hipFree(dinv_e);
        if (!rc && emax_rc) {
            rc = emax_rc;
            aijhip::set_error(emax_err);
        }
        if (dmis) {
            // every rank's outcome so far, before the rounds' collectives
            std::vector<int64_t> ok_all;
            const int lrc = rc;
            const int crc = all_values(C, lrc ? -1 : 0, ok_all);
            bool peer = false;
            if (!crc)
                for (int64_t v : ok_all) peer = peer || v < 0;
            if (!lrc && !crc && !peer) rc = dist_mis(C, L, p, (int32_t)l, S, d_B, l == 0, DMo);
            else rc = lrc ? lrc : crc ? crc : mfail(AIJHIP_ERR_COMM, ("distributed GAMG: another rank failed at level " +
                                                                    std::to_string(l)).c_str());
            hipFree(S.si); hipFree(S.sj); hipFree(S.d);
            hipFree(d_agg);
            d_agg = DMo.d_agg;
            DMo.d_agg = nullptr;
            na = DMo.na;
        }
        // the level's first collective carries this rank's outcome (-1 =
        // failed): a failure on one rank (allocation, aggregation, emax) ends
        // the set-up on every rank here, instead of leaving the others in the
        // level's exchanges until the communicator times out
        std::vector<int64_t> na_all;
        {
            const int lrc = rc;
            const int crc = all_values(C, lrc ? -1 : (int64_t)na, na_all);
            bool peer = false;
            if (!crc)
                for (int64_t v : na_all) peer = peer || v < 0;
            if (lrc || crc || peer) {
                hipFree(d_agg); hipFree(dinv);
                rc = lrc ? lrc : crc ? crc : mfail(AIJHIP_ERR_COMM, ("distributed GAMG: another rank failed at level " +
                                                                   std::to_string(l)).c_str());
                break;
            }
        }
        int64_t NA = 0, cstart = 0;
        std::vector<int64_t> cstarts((size_t)P + 1, 0);
        for (int q = 0; q < P; ++q) cstarts[q + 1] = cstarts[q] + na_all[q];
        NA = cstarts[P];
        cstart = cstarts[me];
        lap(l, "aggregates");
        if (NA == 0 || NA >= M) {  // no coarsening anywhere: this is the coarsest level
            hipFree(d_agg); hipFree(dinv);
            break;
        }
        lap(l, "emax");
        const double alpha = -p.smooth_scale / emax;
        // ---- tentative prolongator and its ghost rows (aggregate gid, value)
        double *d_p0 = nullptr, *d_Bc = nullptr, *d_v = nullptr;
        std::vector<double> g_agg, g_p0;
        if (dmis) {  // (dist_mis made them: coarse ids cover the members of other ranks' aggregates)
            d_p0 = DMo.d_p0;
            d_Bc = DMo.d_Bc;
            d_v = DMo.d_cg;
            DMo.d_p0 = DMo.d_Bc = DMo.d_cg = nullptr;
            rc = halo_values(L.op, d_v, g_agg);
        } else if ((e = dalloc(&d_p0, m)) != hipSuccess || (e = dalloc(&d_Bc, na)) != hipSuccess ||
            (e = dalloc(&d_v, m)) != hipSuccess || (e = aijhip_gamg::tentative_device(m, na, d_agg, d_B, d_Bc, d_p0, l == 0)) !=
                                                       hipSuccess) {
            rc = gerr(e, "tentative prolongator");
        } else {
            if (m > 0) hipLaunchKernelGGL(k_coarse_gid, dim3(nblk(m)), dim3(256), 0, nullptr, m, cstart, d_agg, d_v);
            rc = halo_values(L.op, d_v, g_agg);
        }
        if (!rc) rc = halo_values(L.op, d_p0, g_p0);
        hipFree(d_v);
        const int32_t ng = (int32_t)L.ghost_gid.size();
        // extended coarse numbering E1: own aggregates, then the off-rank ones of the ghosts (sorted)
        std::vector<int64_t> e1_off;
        bool ghost_removed = false;  // a ghost fine node MIS removed (no aggregate)
        for (int32_t s = 0; s < ng; ++s) {
            const int64_t ga = (int64_t)g_agg[s];
            if (ga < 0) ghost_removed = true;
            else if (ga < cstart || ga >= cstart + na) e1_off.push_back(ga);  // (a ghost may sit in an own aggregate)
        }
        for (int64_t c : DMo.rcg) e1_off.push_back(c);  // this rank's members of other ranks' aggregates
        std::sort(e1_off.begin(), e1_off.end());
        e1_off.erase(std::unique(e1_off.begin(), e1_off.end()), e1_off.end());
        auto e1_id = [&](int64_t gidc) -> int32_t {
            if (gidc >= cstart && gidc < cstart + na) return (int32_t)(gidc - cstart);
            return na + (int32_t)(std::lower_bound(e1_off.begin(), e1_off.end(), gidc) - e1_off.begin());
        };
        // their P0 column: the E1 slot of that aggregate
        if (!rc && !DMo.rnode.empty()) {
            const int32_t n = (int32_t)DMo.rnode.size();
            std::vector<int32_t> col((size_t)n);
            for (int32_t k = 0; k < n; ++k) col[k] = e1_id(DMo.rcg[k]);
            int32_t *dn = nullptr, *dc = nullptr;
            if ((e = dalloc(&dn, n)) != hipSuccess || (e = dalloc(&dc, n)) != hipSuccess ||
                (e = hipMemcpy(dn, DMo.rnode.data(), sizeof(int32_t) * (size_t)n, hipMemcpyHostToDevice)) != hipSuccess ||
                (e = hipMemcpy(dc, col.data(), sizeof(int32_t) * (size_t)n, hipMemcpyHostToDevice)) != hipSuccess)
                rc = gerr(e, "P0 columns");
            if (!rc) {
                hipLaunchKernelGGL(k_dm_set_i32, dim3(nblk(n)), dim3(256), 0, nullptr, n, dn, dc, d_agg);
                if ((e = hipStreamSynchronize(nullptr)) != hipSuccess) rc = gerr(e, "P0 columns");
            }
            hipFree(dn);
            hipFree(dc);
        }
        DMo.release();
        // A_ext = [A_d | A_o] (ghost columns after the local ones)
        DCsr Aext, P0ext, T, Plocal;
        std::vector<int32_t> oai, oaj;
        std::vector<double> oaa;
        bool aext_owned = false;
        if (!rc && L.Ao && ng > 0) {
            rc = host_full_rows(*L.Ao, oai, oaj, oaa);
            DCsr Ofull;
            if (!rc) rc = upload_csr(m, ng, oai, oaj, oaa, Ofull);
            if (!rc) rc = hcat(view(*L.Ad), Ofull.ai, Ofull.aj, Ofull.aa, m, m + ng, Aext);
            Ofull.release();
            aext_owned = true;
        } else if (!rc) {
            Aext = view(*L.Ad);
            Aext.n = m + ng;
        }
        lap(l, "A_ext");
        // P0 extended by the ghost rows: rows m + ng, columns E1. A node MIS
        // removed (agg -1, the single-GPU set-up's empty P0 row) has no
        // entry: such levels (rare: isolated rows, e.g. the reference point
        // row 0 at level 0) are compacted on the host; the others keep one
        // entry per row, built on the device
        bool local_removed = false;
        if (!rc && m > 0) {
            unsigned long long *d_n = nullptr, h_n = 0;
            if ((e = dalloc(&d_n, 1)) != hipSuccess || (e = hipMemset(d_n, 0, sizeof(h_n))) != hipSuccess) {
                rc = gerr(e, "alloc");
            } else {
                hipLaunchKernelGGL(k_count_negative, dim3(nblk(m)), dim3(256), 0, nullptr, m, d_agg, d_n);
                if ((e = hipMemcpy(&h_n, d_n, sizeof(h_n), hipMemcpyDeviceToHost)) != hipSuccess) rc = gerr(e, "count");
            }
            hipFree(d_n);
            local_removed = h_n > 0;
        }
        if (!rc && (local_removed || ghost_removed)) {
            std::vector<int32_t> h_agg((size_t)m), ai, aj;
            std::vector<double> h_p0((size_t)m), aa;
            if (m > 0 && ((e = hipMemcpy(h_agg.data(), d_agg, sizeof(int32_t) * (size_t)m, hipMemcpyDeviceToHost)) !=
                              hipSuccess ||
                          (e = hipMemcpy(h_p0.data(), d_p0, sizeof(double) * (size_t)m, hipMemcpyDeviceToHost)) !=
                              hipSuccess))
                rc = gerr(e, "P0 rows");
            ai.push_back(0);
            for (int32_t i = 0; i < m; ++i) {
                if (h_agg[i] >= 0) {
                    aj.push_back(h_agg[i]);
                    aa.push_back(h_p0[i]);
                }
                ai.push_back((int32_t)aj.size());
            }
            for (int32_t s = 0; s < ng; ++s) {
                if (g_agg[s] >= 0) {
                    aj.push_back(e1_id((int64_t)g_agg[s]));
                    aa.push_back(g_p0[s]);
                }
                ai.push_back((int32_t)aj.size());
            }
            if (!rc) rc = upload_csr(m + ng, na + (int32_t)e1_off.size(), ai, aj, aa, P0ext);
        } else if (!rc) {
            std::vector<int32_t> gcol((size_t)ng);
            for (int32_t s = 0; s < ng; ++s) gcol[s] = e1_id((int64_t)g_agg[s]);
            P0ext.m = m + ng;
            P0ext.n = na + (int32_t)e1_off.size();
            P0ext.nz = m + ng;
            if ((e = dalloc(&P0ext.ai, (int64_t)m + ng + 1)) != hipSuccess ||
                (e = dalloc(&P0ext.aj, (int64_t)m + ng + 2)) != hipSuccess ||
                (e = dalloc(&P0ext.aa, (int64_t)m + ng + 2)) != hipSuccess ||
                (e = hipMemset(P0ext.aj, 0, sizeof(int32_t) * (size_t)(m + ng + 2))) != hipSuccess ||
                (e = hipMemset(P0ext.aa, 0, sizeof(double) * (size_t)(m + ng + 2))) != hipSuccess ||
                (m > 0 && ((e = hipMemcpy(P0ext.aj, d_agg, sizeof(int32_t) * (size_t)m, hipMemcpyDeviceToDevice)) !=
                               hipSuccess ||
                           (e = hipMemcpy(P0ext.aa, d_p0, sizeof(double) * (size_t)m, hipMemcpyDeviceToDevice)) !=
                               hipSuccess)) ||
                (ng > 0 && ((e = hipMemcpy(P0ext.aj + m, gcol.data(), sizeof(int32_t) * (size_t)ng,
                                           hipMemcpyHostToDevice)) != hipSuccess ||
                            (e = hipMemcpy(P0ext.aa + m, g_p0.data(), sizeof(double) * (size_t)ng,
                                           hipMemcpyHostToDevice)) != hipSuccess)))
                rc = gerr(e, "P0 extended");
            if (!rc) hipLaunchKernelGGL(k_iota32, dim3(nblk((int64_t)m + ng + 1)), dim3(256), 0, nullptr, m + ng,
                                        P0ext.ai);
        }
        // ---- P = P0 + alpha D^-1 (A P0) on the local rows (columns E1)
        int cols_used = 0;
        if (!rc) {
            if (p.nsmooths > 0) {
                rc = aijhip_gamg::rowprod_device(Aext, P0ext, T, n_cu, &cols_used);
                if (!rc) rc = aijhip_gamg::prolong_from_T(T, d_agg, d_p0, dinv, alpha, Plocal);
                T.release();
            } else {  // P = P0 (local rows)
                std::vector<int32_t> ai((size_t)m + 1), aj((size_t)m);
                std::vector<double> aa((size_t)m);
                std::iota(ai.begin(), ai.end(), 0);
                if ((m > 0 && ((e = hipMemcpy(aj.data(), d_agg, sizeof(int32_t) * (size_t)m, hipMemcpyDeviceToHost)) !=
                                   hipSuccess ||
                               (e = hipMemcpy(aa.data(), d_p0, sizeof(double) * (size_t)m, hipMemcpyDeviceToHost)) !=
                                   hipSuccess)))
                    rc = gerr(e, "P0");
                if (!rc && local_removed) {  // (MIS-removed nodes: empty rows)
                    std::vector<int32_t> ci(1, 0), cj;
                    std::vector<double> ca;
                    for (int32_t i = 0; i < m; ++i) {
                        if (aj[i] >= 0) {
                            cj.push_back(aj[i]);
                            ca.push_back(aa[i]);
                        }
                        ci.push_back((int32_t)cj.size());
                    }
                    ai.swap(ci);
                    aj.swap(cj);
                    aa.swap(ca);
                }
                if (!rc) rc = upload_csr(m, P0ext.n, ai, aj, aa, Plocal);
            }
        }
        P0ext.release();
        lap(l, "prolongator");
        // ---- P's rows of the ghost fine nodes (global coarse ids): each
        // rank sends the rows its neighbours hold as ghosts
        auto e1_gid = [&](int32_t c) -> int64_t { return c < na ? cstart + c : e1_off[c - na]; };
        std::vector<std::vector<int64_t>> gcols((size_t)ng);  // ghost row s: global coarse ids
        std::vector<std::vector<double>> gvals((size_t)ng);
        if (!rc) {
            std::vector<std::vector<uint64_t>> out((size_t)P), in;
            for (size_t q = 0; q < L.op->send_peer.size() && !rc; ++q) {
                const int64_t a = L.op->send_off[q], b = L.op->send_off[q + 1];
                std::vector<int32_t> rows(L.op->h_send_rows.begin() + a, L.op->h_send_rows.begin() + b), off, cols;
                std::vector<double> vals;
                if ((rc = download_rows(Plocal.ai, Plocal.aj, Plocal.aa, rows, off, cols, vals))) break;
                auto &o = out[L.op->send_peer[q]];
                for (size_t r = 0; r < rows.size(); ++r) {
                    o.push_back((uint64_t)(off[r + 1] - off[r]));
                    for (int32_t k = off[r]; k < off[r + 1]; ++k) {
                        o.push_back((uint64_t)e1_gid(cols[k]));
                        uint64_t bitsv;
                        std::memcpy(&bitsv, &vals[k], 8);
                        o.push_back(bitsv);
                    }
                }
            }
            if (!rc) rc = aijhip_mpi::comm_sendrecv(C, out, in);
            for (size_t pp = 0; !rc && pp < L.op->recv_peer.size(); ++pp) {
                const auto &w = in[L.op->recv_peer[pp]];
                size_t k = 0;
                for (int64_t s = L.op->recv_off[pp]; s < L.op->recv_off[pp + 1]; ++s) {
                    if (k >= w.size()) {
                        rc = mfail(AIJHIP_ERR_COMM, "distributed GAMG: short ghost-row message");
                        break;
                    }
                    const uint64_t len = w[k++];
                    for (uint64_t t = 0; t < len; ++t) {
                        gcols[s].push_back((int64_t)w[k++]);
                        double v;
                        std::memcpy(&v, &w[k++], 8);
                        gvals[s].push_back(v);
                    }
                }
            }
        }
        lap(l, "ghost rows of P");
        // extended coarse numbering E2: own, then every off-rank id of P's local and ghost rows
        std::vector<int64_t> e2_off(e1_off);
        for (int32_t s = 0; s < ng; ++s)
            for (int64_t c : gcols[s])
                if (c < cstart || c >= cstart + na) e2_off.push_back(c);
        std::sort(e2_off.begin(), e2_off.end());
        e2_off.erase(std::unique(e2_off.begin(), e2_off.end()), e2_off.end());
        const int32_t n2 = na + (int32_t)e2_off.size();
        auto e2_id = [&](int64_t gidc) -> int32_t {
            if (gidc >= cstart && gidc < cstart + na) return (int32_t)(gidc - cstart);
            return na + (int32_t)(std::lower_bound(e2_off.begin(), e2_off.end(), gidc) - e2_off.begin());
        };
        // P_local: E1 -> E2; P_ext2 = [P_local; P_ghost]
        DCsr Pext, AP, PT, Cext;
        if (!rc) {
            std::vector<int32_t> t1((size_t)P0ext.n);
            for (int32_t c = 0; c < (int32_t)t1.size(); ++c) t1[c] = c < na ? c : e2_id(e1_off[c - na]);
            rc = remap_cols(Plocal, t1);
            Plocal.n = n2;
        }
        if (!rc) {
            std::vector<int32_t> gi{0}, gj;
            std::vector<double> ga;
            for (int32_t s = 0; s < ng; ++s) {
                std::vector<std::pair<int32_t, double>> row;
                for (size_t k = 0; k < gcols[s].size(); ++k) row.emplace_back(e2_id(gcols[s][k]), gvals[s][k]);
                std::sort(row.begin(), row.end(),
                          [](const std::pair<int32_t, double> &a, const std::pair<int32_t, double> &b) {
                              return a.first < b.first;
                          });
                for (auto &x : row) {
                    gj.push_back(x.first);
                    ga.push_back(x.second);
                }
                gi.push_back((int32_t)gj.size());
            }
            // vertical stack on the device
            const int64_t nzl = Plocal.nz, nzg = (int64_t)gj.size();
            Pext.m = m + ng;
            Pext.n = n2;
            Pext.nz = nzl + nzg;
            int32_t *d_gi = nullptr;
            if ((e = dalloc(&Pext.ai, (int64_t)m + ng + 1)) != hipSuccess || (e = dalloc(&Pext.aj, Pext.nz + 2)) != hipSuccess ||
                (e = dalloc(&Pext.aa, Pext.nz + 2)) != hipSuccess ||
                (e = hipMemset(Pext.aj, 0, sizeof(int32_t) * (size_t)(Pext.nz + 2))) != hipSuccess ||
                (e = hipMemset(Pext.aa, 0, sizeof(double) * (size_t)(Pext.nz + 2))) != hipSuccess ||
                (e = hipMemcpy(Pext.ai, Plocal.ai, sizeof(int32_t) * ((size_t)m + 1), hipMemcpyDeviceToDevice)) != hipSuccess ||
                (nzl > 0 && ((e = hipMemcpy(Pext.aj, Plocal.aj, sizeof(int32_t) * (size_t)nzl, hipMemcpyDeviceToDevice)) !=
                                 hipSuccess ||
                             (e = hipMemcpy(Pext.aa, Plocal.aa, sizeof(double) * (size_t)nzl, hipMemcpyDeviceToDevice)) !=
                                 hipSuccess)) ||
                (nzg > 0 && ((e = hipMemcpy(Pext.aj + nzl, gj.data(), sizeof(int32_t) * (size_t)nzg,
                                            hipMemcpyHostToDevice)) != hipSuccess ||
                             (e = hipMemcpy(Pext.aa + nzl, ga.data(), sizeof(double) * (size_t)nzg,
                                            hipMemcpyHostToDevice)) != hipSuccess)) ||
                (e = dalloc(&d_gi, (int64_t)ng + 1)) != hipSuccess ||
                (e = hipMemcpy(d_gi, gi.data(), sizeof(int32_t) * gi.size(), hipMemcpyHostToDevice)) != hipSuccess)
                rc = gerr(e, "P extended");
            if (!rc && ng > 0)
                hipLaunchKernelGGL(k_add_offset, dim3(nblk(ng)), dim3(256), 0, nullptr, ng, (int32_t)nzl, d_gi + 1,
                                   Pext.ai + m + 1);
            hipFree(d_gi);
        }
        lap(l, "P extended");
        // ---- A P and P^T (A P)
        if (!rc) rc = aijhip_gamg::rowprod_device(Aext, Pext, AP, n_cu, &cols_used);
        Pext.release();
        if (aext_owned) Aext.release();
        lap(l, "A*P");
        if (!rc) {
            aijhip_mat pv;  // non-owning view for the transpose builder
            pv.m = Plocal.m;
            pv.n = Plocal.n;
            pv.nz = Plocal.nz;
            pv.d_ai = Plocal.ai;
            pv.d_aj = Plocal.aj;
            pv.d_aa = Plocal.aa;
            PT.m = Plocal.n;
            PT.n = Plocal.m;
            PT.nz = Plocal.nz;
            e = aijhip::build_transpose(pv, &PT.ai, &PT.aj, &PT.aa, nullptr);
            pv.d_ai = pv.d_aj = nullptr;
            pv.d_aa = nullptr;
            if (e != hipSuccess) rc = gerr(e, "transpose");
        }
        if (!rc) rc = aijhip_gamg::rowprod_device(PT, AP, Cext, n_cu, &cols_used);
        PT.release();
        AP.release();
        lap(l, "P^T*(AP)");
        // ---- rows [na, n2) of Cext belong to other ranks: send them to their owners
        std::vector<int64_t> gnew;  // level l+1 ghost list
        std::vector<int32_t> corr_i{0}, corr_j;
        std::vector<double> corr_a;
        if (!rc) {
            std::vector<int32_t> rows;
            for (int32_t r = na; r < n2; ++r) rows.push_back(r);
            std::vector<int32_t> off, cols;
            std::vector<double> vals;
            rc = download_rows(Cext.ai, Cext.aj, Cext.aa, rows, off, cols, vals);
            auto e2_gid = [&](int32_t c) -> int64_t { return c < na ? cstart + c : e2_off[c - na]; };
            std::vector<std::vector<uint64_t>> out((size_t)P), in;
            for (size_t q = 0; !rc && q < rows.size(); ++q) {
                const int64_t rg = e2_off[q];
                auto &o = out[owner_of(cstarts, rg)];
                o.push_back((uint64_t)rg);
                o.push_back((uint64_t)(off[q + 1] - off[q]));
                for (int32_t k = off[q]; k < off[q + 1]; ++k) {
                    o.push_back((uint64_t)e2_gid(cols[k]));
                    uint64_t bitsv;
                    std::memcpy(&bitsv, &vals[k], 8);
                    o.push_back(bitsv);
                }
            }
            if (!rc) rc = aijhip_mpi::comm_sendrecv(C, out, in);
            // received (row, col, value) for own rows, in (peer, message) order
            struct Trip {
                int32_t r, cu;  // own coarse row; column in the unified numbering (set below)
                int64_t c;
                double v;
            };
            std::vector<Trip> trips;
            for (int q = 0; !rc && q < P; ++q) {
                if (q == me) continue;
                const auto &w = in[q];
                size_t k = 0;
                while (k < w.size()) {
                    const int64_t rg = (int64_t)w[k++];
                    const uint64_t len = w[k++];
                    for (uint64_t t = 0; t < len; ++t) {
                        Trip tr;
                        tr.r = (int32_t)(rg - cstart);
                        tr.c = (int64_t)w[k++];
                        std::memcpy(&tr.v, &w[k++], 8);
                        trips.push_back(tr);
                    }
                }
            }
            // level l+1 ghosts: E2's off-rank ids and every off-rank column received
            gnew = e2_off;
            for (const Trip &t : trips)
                if (t.c < cstart || t.c >= cstart + na) gnew.push_back(t.c);
            std::sort(gnew.begin(), gnew.end());
            gnew.erase(std::unique(gnew.begin(), gnew.end()), gnew.end());
            auto u_id = [&](int64_t gidc) -> int32_t {  // unified: own [0, na), ghost slot na + s
                if (gidc >= cstart && gidc < cstart + na) return (int32_t)(gidc - cstart);
                return na + (int32_t)(std::lower_bound(gnew.begin(), gnew.end(), gidc) - gnew.begin());
            };
            for (Trip &t : trips) t.cu = u_id(t.c);
            std::stable_sort(trips.begin(), trips.end(), [](const Trip &a, const Trip &b) {
                return a.r != b.r ? a.r < b.r : a.cu < b.cu;
            });
            std::vector<int32_t> cnt((size_t)na, 0);
            for (size_t k = 0; k < trips.size();) {
                size_t j = k;
                double v = 0.0;
                const int32_t cu = trips[k].cu;
                while (j < trips.size() && trips[j].r == trips[k].r && trips[j].cu == cu) v += trips[j++].v;
                ++cnt[trips[k].r];
                corr_j.push_back(cu);
                corr_a.push_back(v);
                k = j;
            }
            corr_i.assign((size_t)na + 1, 0);
            for (int32_t r = 0; r < na; ++r) corr_i[r + 1] = corr_i[r] + cnt[r];
            // E2 -> unified numbering for the own rows of Cext and for P
            std::vector<int32_t> t2((size_t)n2);
            for (int32_t c = 0; c < n2; ++c) t2[c] = c < na ? c : u_id(e2_off[c - na]);
            if (!rc) rc = remap_cols(Cext, t2);
            if (!rc) rc = remap_cols(Plocal, t2);
        }
        lap(l, "Galerkin contributions");
        // ---- the coarse operator's own rows: Cext[0, na) + received, split
        DCsr Cown, Corr, Ctot, Cd, Co, Pd, Po;
        const int32_t ngn = (int32_t)gnew.size();
        if (!rc) {
            Cown.m = na;
            Cown.n = na + ngn;
            Cown.ai = Cext.ai;
            Cown.aj = Cext.aj;
            Cown.aa = Cext.aa;
            int32_t nz_own = 0;
            if ((e = hipMemcpy(&nz_own, Cext.ai + na, sizeof(int32_t), hipMemcpyDeviceToHost)) != hipSuccess)
                rc = gerr(e, "coarse rows");
            Cown.nz = nz_own;
            if (!rc) rc = upload_csr(na, na + ngn, corr_i, corr_j, corr_a, Corr);
            if (!rc) rc = csr_add(Cown, Corr, Ctot);
            Cown = DCsr();  // a view of Cext
            Corr.release();
            if (!rc) rc = csr_split(Ctot, na, ngn, Cd, Co);
            Ctot.release();
            Plocal.n = na + ngn;
            if (!rc) rc = csr_split(Plocal, na, ngn, Pd, Po);
        }
        Cext.release();
        Plocal.release();
        // ---- handles of level l+1 and the transfer operators of level l
        aijhip_mat *Adn = nullptr, *Aon = nullptr;
        if (!rc) rc = aijhip_gamg::make_level_handle(L.Ad->device, Cd, &Adn);
        if (!rc && Co.nz > 0) rc = aijhip_gamg::make_level_handle(L.Ad->device, Co, &Aon);
        Co.release();
        if (!rc && !in_line) {  // P_d (with R_d = P_d^T) and P_o on a second host thread
            jobs.emplace_back(new PJob());
            jobs.back()->start(L.Ad->device, l, Pd, Po);
            Pd = DCsr();  // owned by the job now
            Po = DCsr();
        }
        if (!rc && in_line) rc = aijhip_gamg::make_level_handle(L.Ad->device, Pd, &L.Pd);
        if (!rc && in_line) {  // R_d = P_d^T attached for the restriction
            int32_t *ti = nullptr, *tj = nullptr;
            double *ta = nullptr;
            if ((e = aijhip::build_transpose(*L.Pd, &ti, &tj, &ta, nullptr)) != hipSuccess) rc = gerr(e, "P^T");
            else rc = aijhip::attach_transpose(L.Pd, ti, tj, ta);
        }
        if (!rc && in_line && Po.nz > 0) rc = aijhip_gamg::make_level_handle(L.Ad->device, Po, &L.Po);
        Po.release();
        Pd.release();
        Cd.release();
        hipFree(d_agg);
        hipFree(dinv);
        hipFree(d_p0);
        lap(l, "handles");
        if (rc) {
            aijhip_mat_destroy(Adn);
            aijhip_mat_destroy(Aon);
            hipFree(d_Bc);
            break;
        }
        H.lv.emplace_back();
        Level &N = H.lv.back();
        Level &Lp = H.lv[l];  // (reference refreshed after the push)
        N.Ad = Adn;
        N.Ao = Aon;
        N.m = na;
        N.starts = cstarts;
        N.rstart = cstart;
        N.ghost_gid = gnew;
        rc = make_operator(C, Adn, Aon, gnew, cstarts, &N.op);
        Lp.emax = emax;
        std::swap(d_B, d_Bc);
        hipFree(d_Bc);
        lap(l, "halo plan");
        if (rc) break;
    }
    hipFree(d_B);
    for (auto &j : jobs) {  // the interpolation handles made meanwhile
        j->join();
        if (j->rc) {
            if (!rc) {
                rc = j->rc;
                aijhip::set_error(j->err);
            }
            continue;
        }
        H.lv[j->level].Pd = j->Pd;
        H.lv[j->level].Po = j->Po;
        j->Pd = j->Po = nullptr;
    }
    jobs.clear();
    // level vectors and D^-1
    for (size_t l = 0; !rc && l < H.lv.size(); ++l) {
        Level &L = H.lv[l];
        const size_t vb = sizeof(double) * (size_t)std::max<int32_t>(L.m, 1);
        if ((e = hipMalloc(&L.dinv, vb)) != hipSuccess || (e = hipMalloc(&L.r, vb)) != hipSuccess ||
            (l > 0 && ((e = hipMalloc(&L.b, vb)) != hipSuccess || (e = hipMalloc(&L.x, vb)) != hipSuccess))) {
            rc = gerr(e, "level vectors");
            break;
        }
        if (L.m > 0)
            hipLaunchKernelGGL(k_diag_inv, dim3(nblk(L.m)), dim3(256), 0, nullptr, L.m, L.Ad->d_ai, L.Ad->d_aj,
                               L.Ad->d_aa, L.dinv);
    }
    if (!rc && (e = hipDeviceSynchronize()) != hipSuccess) rc = gerr(e, "set-up");
    if (rc) H.destroy();
    return rc;
}

// Rows of [Bd | Bo] on the host with global columns: Bd's column c -> doff +
// c, Bo's column s -> ghost[s]; each row sorted by global column.
int level_rows(const aijhip_mat *Bd, const aijhip_mat *Bo, int64_t doff, const std::vector<int64_t> &ghost,
               std::vector<int64_t> &ai, std::vector<int64_t> &aj, std::vector<double> &aa) {
    std::vector<int32_t> di, dj, oi, oj;
    std::vector<double> da, oa;
    int rc = host_full_rows(*Bd, di, dj, da);
    if (!rc && Bo) rc = host_full_rows(*Bo, oi, oj, oa);
    if (rc) return rc;
    const int32_t m = Bd->m;
    ai.assign((size_t)m + 1, 0);
    aj.clear();
    aa.clear();
    std::vector<std::pair<int64_t, double>> row;
    for (int32_t i = 0; i < m; ++i) {
        row.clear();
        for (int32_t k = di[i]; k < di[i + 1]; ++k) row.emplace_back(doff + dj[k], da[k]);
        if (Bo)
            for (int32_t k = oi[i]; k < oi[i + 1]; ++k) row.emplace_back(ghost[oj[k]], oa[k]);
        std::sort(row.begin(), row.end(), [](const std::pair<int64_t, double> &a, const std::pair<int64_t, double> &b) {
            return a.first < b.first;
        });
        for (auto &x : row) {
            aj.push_back(x.first);
            aa.push_back(x.second);
        }
        ai[i + 1] = (int64_t)aj.size();
    }
    return AIJHIP_OK;
}

int get_level(const Hierarchy &H, int32_t l, char which, int64_t *rstart, int32_t *m, std::vector<int64_t> &ai,
              std::vector<int64_t> &aj, std::vector<double> &aa) {
    if (l < 0 || l >= (int32_t)H.lv.size()) return mfail(AIJHIP_ERR_ARG, "no such level");
    const Level &L = H.lv[l];
    *rstart = L.rstart;
    *m = L.m;
    if (which == 'A') return level_rows(L.Ad, L.Ao, L.rstart, L.ghost_gid, ai, aj, aa);
    if (which == 'P') {
        if (l + 1 >= (int32_t)H.lv.size()) return mfail(AIJHIP_ERR_ARG, "the coarsest level has no interpolation");
        const Level &N = H.lv[l + 1];
        return level_rows(L.Pd, L.Po, N.rstart, N.ghost_gid, ai, aj, aa);
    }
    return mfail(AIJHIP_ERR_ARG, "which: 'A' or 'P'");
}

// y = B x (+ z) through the halo of `halo_op`: the exchange of x overlaps B_d x
static int transfer(aijhip_mpiaij *halo_op, const aijhip_mat *Bd, const aijhip_mat *Bo, const double *x,
                    const double *z, double *y, bool add, hipStream_t s, const int *stop) {
    const bool exch = halo_op->n_send > 0 || halo_op->n_ghost > 0;
    int rc = exch ? aijhip_mpi::halo_post(halo_op, x, s) : AIJHIP_OK;
    if (rc) return rc;
    hipError_t e = aijhip::launch_mult(*Bd, x, z, y, add, s, stop);
    if (e != hipSuccess)
        return exch ? aijhip_mpi::halo_abort(halo_op, s, gerr(e, "transfer product")) : gerr(e, "transfer product");
    if (exch && (rc = aijhip_mpi::halo_finish(halo_op, s))) return rc;
    if (Bo && (e = aijhip::launch_mult(*Bo, halo_op->d_ghost, y, y, true, s, stop)) != hipSuccess)
        return gerr(e, "transfer ghost product");
    return AIJHIP_OK;
}

// MatRestrict as MatMultTranspose_MPIAIJ: b = P_d^T r, then P_o^T r (one
// value per ghost coarse slot of level l+1, in that level's ghost vector)
// sent back to the slots' owners and added (halo_reverse_add). An aggregate
// may have members on other ranks up to two steps from its root (PETSc's
// parallel MIS), and P's smoothing reaches one more, so the fine rows with
// entries in a rank's coarse columns are not all ghosts of its level-l halo:
// the sums travel with the coarse level's plan instead.
static int restrict_to(const Level &L, Level &N, const double *r, double *b, hipStream_t s, const int *stop) {
    hipError_t e = aijhip::launch_mult(*L.Pd->transpose, r, nullptr, b, false, s, stop);
    if (e != hipSuccess) return gerr(e, "restriction");
    aijhip_mpiaij *M = N.op;
    if (M->n_send == 0 && M->n_ghost == 0) return AIJHIP_OK;
    double *t = M->d_ghost;
    if (L.Po && L.Po->transpose) e = aijhip::launch_mult(*L.Po->transpose, r, nullptr, t, false, s, stop);
    else if (M->n_ghost > 0) e = hipMemsetAsync(t, 0, sizeof(double) * (size_t)M->n_ghost, s);
    if (e != hipSuccess) return gerr(e, "restriction (off-rank share)");
    return aijhip_mpi::halo_reverse_add(M, t, b, s);
}

// The A_o correction of a fused smoothing launch (after the halo landed).
static int offdiag_axpy(const Level &L, const double *scale, double *y, hipStream_t s, const int *stop) {
    if (!L.Ao) return AIJHIP_OK;
    const aijhip::RowList R = aijhip::row_list(*L.Ao);
    if (R.nr == 0) return AIJHIP_OK;
    hipLaunchKernelGGL(k_offdiag_axpy, dim3(nblk(R.nr)), dim3(256), 0, s, R.nr, R.rai, R.ridx, L.Ao->d_aj,
                       L.Ao->d_aa, L.op->d_ghost, scale, y, stop);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? AIJHIP_OK : gerr(e, "off-diagonal smoothing share");
}

int vcycle(Hierarchy &H, const double *b0, double *x0, hipStream_t s, const int *stop) {
    const int nl = (int)H.lv.size();
    auto B = [&](int l) { return l == 0 ? b0 : (const double *)H.lv[l].b; };
    auto X = [&](int l) { return l == 0 ? x0 : H.lv[l].x; };
    auto grid = [](int64_t n) { return dim3((unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 2048))); };
    // smoothing SpMVs fused with their vector passes on STREAM-planned blocks
    // (ksp.hip's launch_mg_resid / launch_mg_post over A_d while the halo
    // moves, then A_o's share on the boundary rows); AIJHIP_MG_UNFUSED=1 for A/B
    static const bool unfused = std::getenv("AIJHIP_MG_UNFUSED") != nullptr;
    auto fused = [&](const Level &L) { return !unfused && aijhip::stream_mg_fusable(*L.Ad); };
    auto exchanges = [](const aijhip_mpiaij *M) { return M->n_send > 0 || M->n_ghost > 0; };
    int rc;
    hipError_t e;
    for (int l = 0; l < nl; ++l) {
        Level &L = H.lv[l];
        hipLaunchKernelGGL(k_mg_jacobi, grid(L.m), dim3(256), 0, s, (int64_t)L.m, L.dinv, B(l), X(l), stop);
        if (l == nl - 1) break;  // coarse: preonly + Jacobi
        // r = b - A x
        if (fused(L)) {
            const bool ex = exchanges(L.op);
            if (ex && (rc = aijhip_mpi::halo_post(L.op, X(l), s))) return rc;
            if ((e = aijhip::launch_mg_resid(*L.Ad, X(l), B(l), L.r, s, true, stop)) != hipSuccess)
                return ex ? aijhip_mpi::halo_abort(L.op, s, gerr(e, "residual")) : gerr(e, "residual");
            if (ex && (rc = aijhip_mpi::halo_finish(L.op, s))) return rc;
            if ((rc = offdiag_axpy(L, nullptr, L.r, s, stop))) return rc;
        } else {  // MatMult_MPIAIJ, then the residual
            if ((rc = aijhip_mpi::mpiaij_apply(L.op, X(l), L.r, s, nullptr, nullptr, nullptr, false, stop))) return rc;
            hipLaunchKernelGGL(k_mg_resid, grid(L.m), dim3(256), 0, s, (int64_t)L.m, B(l), L.r, stop);
        }
        // MatRestrict: b_{l+1} = P^T r = P_d^T r + R_o r_ghost
        if ((rc = restrict_to(L, H.lv[l + 1], L.r, H.lv[l + 1].b, s, stop))) return rc;
    }
    for (int l = nl - 2; l >= 0; --l) {
        Level &L = H.lv[l];
        if (fused(L)) {
            // MatInterpolateAdd into the scratch: t = x + P x_c, then smoothu
            // x = t + D^-1 (b - A t) in the SpMV epilogue over A_d
            if ((rc = transfer(H.lv[l + 1].op, L.Pd, L.Po, X(l + 1), X(l), L.r, true, s, stop))) return rc;
            const bool ex = exchanges(L.op);
            if (ex && (rc = aijhip_mpi::halo_post(L.op, L.r, s))) return rc;
            if ((e = aijhip::launch_mg_post(*L.Ad, L.r, B(l), L.dinv, X(l), nullptr, s, true, stop)) != hipSuccess)
                return ex ? aijhip_mpi::halo_abort(L.op, s, gerr(e, "post-smoothing")) : gerr(e, "post-smoothing");
            if (ex && (rc = aijhip_mpi::halo_finish(L.op, s))) return rc;
            if ((rc = offdiag_axpy(L, L.dinv, X(l), s, stop))) return rc;
        } else {
            // MatInterpolateAdd: x = x + P x_c (P_d x_c + P_o x_c ghost)
            if ((rc = transfer(H.lv[l + 1].op, L.Pd, L.Po, X(l + 1), X(l), X(l), true, s, stop))) return rc;
            // smoothu: x = x + D^-1 (b - A x)
            if ((rc = aijhip_mpi::mpiaij_apply(L.op, X(l), L.r, s, nullptr, nullptr, nullptr, false, stop))) return rc;
            hipLaunchKernelGGL(k_mg_richardson, grid(L.m), dim3(256), 0, s, (int64_t)L.m, L.dinv, B(l), L.r, X(l),
                               stop);
        }
    }
    e = hipGetLastError();
    return e == hipSuccess ? AIJHIP_OK : gerr(e, "V-cycle");
}

}  // namespace aijhip_gamg_mpi
