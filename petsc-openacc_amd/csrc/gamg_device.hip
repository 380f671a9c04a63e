// gamg_device.hip — the smoothed-aggregation set-up on the device
// (gamg_internal.h build_device). Same steps, same summation orders and so
// the same hierarchy, bit for bit, as the host builder (gamg_setup.cpp,
// itself pinned to oracle/gamg.py):
//   diagonal / D^-1               one lane per row
//   strength graph S (+ S^T)      atomic slots, then per-row sort + unique
//   aggregation                   greedy, natural order: phase 1 as a
//                                 device sweep (gamg_aggregate.hip) or the
//                                 host pass, phase 2 on the device, phase 3
//                                 sequential over the nodes left
//   emax(D^-1 A)                  power iteration on the STREAM SpMV in
//                                 PETSc order; 256-entry blocked dots
//   P = (I - 1.4/emax D^-1 A) P0  row-wise product A*P0, union with P0
//   A_c = P^T (A P)               row-wise products (below), P^T by the
//                                 stable radix-sort transpose
// Row-wise product C = A*B (scipy csr_matmat order): one lane per output row
// keeps the row's distinct columns sorted in LDS and adds each product
// a_ik * b_kj to its column's accumulator in traversal order, starting from
// 0.0. A row with more distinct columns than the lane's capacity retries
// with a larger capacity; past the largest the level goes to the host.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "dscan.h"
#include "gamg_device.h"

namespace {

using aijhip::set_error;

int herr(hipError_t e, const char *what) {
    set_error(std::string("GAMG device set-up: ") + what + ": " + hipGetErrorString(e));
    return AIJHIP_ERR_HIP;
}

inline unsigned blocks_for(int64_t n, int t) { return (unsigned)std::max<int64_t>(1, (n + t - 1) / t); }

// ---------------------------------------------------------------- kernels

__global__ void k_diag_dinv(int32_t m, const int32_t *__restrict__ ai, const int32_t *__restrict__ aj,
                            const double *__restrict__ aa, double *d, double *dinv) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    double v = 0.0;
    for (int32_t k = ai[i]; k < ai[i + 1]; ++k)
        if (aj[k] == i) { v = aa[k]; break; }
    d[i] = v;
    dinv[i] = 1.0 / (v == 0.0 ? 1.0 : v);
}

__device__ __forceinline__ bool strong(int32_t i, int32_t j, double a, const double *d, double theta) {
    return j != i && fabs(a) > theta * sqrt(fabs(d[i] * d[j]));
}

__global__ void k_strong_count(int32_t m, const int32_t *__restrict__ ai, const int32_t *__restrict__ aj,
                               const double *__restrict__ aa, const double *__restrict__ d, double theta,
                               unsigned long long *cnt) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    unsigned long long own = 0;
    for (int32_t k = ai[i]; k < ai[i + 1]; ++k)
        if (strong(i, aj[k], aa[k], d, theta)) {
            ++own;
            atomicAdd(&cnt[aj[k]], 1ull);
        }
    if (own) atomicAdd(&cnt[i], own);
}

__global__ void k_strong_fill(int32_t m, const int32_t *__restrict__ ai, const int32_t *__restrict__ aj,
                              const double *__restrict__ aa, const double *__restrict__ d, double theta,
                              const unsigned long long *__restrict__ off, unsigned int *pos, int32_t *tmp) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    for (int32_t k = ai[i]; k < ai[i + 1]; ++k) {
        const int32_t j = aj[k];
        if (!strong(i, j, aa[k], d, theta)) continue;
        tmp[off[i] + atomicAdd(&pos[i], 1u)] = j;
        tmp[off[j] + atomicAdd(&pos[j], 1u)] = i;
    }
}

// The weight of S entry (i, j): |a_ij| of the stored entry, or -1 when A
// stores no (i, j) (the entry came from S^T). SORTED: A's row columns strictly
// increase (binary search); otherwise the max over a scan of the row.
template <bool SORTED>
__device__ __forceinline__ double stored_weight(int32_t j, int32_t a0, int32_t a1, const int32_t *__restrict__ aj,
                                                const double *__restrict__ aa) {
    if (SORTED) {
        int32_t lo = a0, hi = a1;
        while (lo < hi) {
            const int32_t q = (lo + hi) >> 1;
            if (aj[q] < j) lo = q + 1;
            else hi = q;
        }
        return (lo < a1 && aj[lo] == j) ? fabs(aa[lo]) : -1.0;
    }
    double v = -1.0;
    for (int32_t e = a0; e < a1; ++e)
        if (aj[e] == j) v = fmax(v, fabs(aa[e]));
    return v;
}

// flag = 1 when some row of A has columns that do not strictly increase
__global__ void k_rows_unsorted(int32_t m, const int32_t *__restrict__ ai, const int32_t *__restrict__ aj,
                                int32_t *flag) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    for (int32_t k = ai[i] + 1; k < ai[i + 1]; ++k)
        if (aj[k] <= aj[k - 1]) { atomicOr(flag, 1); return; }
}

// S straight from A when A's rows are sorted and the strong pattern is
// symmetric (Galerkin operators of a symmetric operand, the 7-point one):
// then S u S^T = S, already sorted and unique, every entry a stored one.
// G lanes per row (rows of up to a few G entries; a wave holds 64 / G rows).
#define AIJHIP_ROW_LANES                                                                                      \
    const int lane = threadIdx.x & 63;                                                                        \
    const int l = lane & (G - 1);                                                                             \
    const unsigned long long segmask = (G == 64 ? ~0ull : ((1ull << G) - 1ull)) << (lane & ~(G - 1));         \
    const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;                                                \
    for (int64_t base = (((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6) * (64 / G); base < m;         \
         base += nw * (64 / G))

// Also: flag[0] = 1 when a row's columns do not strictly increase (the
// neighbouring entry's column is a neighbouring lane's load), and *updown +=
// (strong entries above the diagonal) - (below it), one atomic per wavefront:
// with every upper entry mirrored (k_strong_asymmetric) a zero tally makes S
// symmetric (the mirror map is injective from the upper entries into the
// lower ones; equal counts make it onto).
template <int G>
__global__ __launch_bounds__(256) void k_strong_direct_count(int32_t m, const int32_t *__restrict__ ai,
                                                             const int32_t *__restrict__ aj,
                                                             const double *__restrict__ aa,
                                                             const double *__restrict__ d, double theta,
                                                             int32_t *cnt, int32_t *flag,
                                                             unsigned long long *updown) {
    long long ud = 0;
    bool unsorted = false;
    AIJHIP_ROW_LANES {
        const int64_t i = base + lane / G;
        const bool on = i < m;
        const int32_t a0 = on ? ai[i] : 0, a1 = on ? ai[i + 1] : 0;
        int32_t c = 0;
        for (int32_t k = a0 + l; k < a1; k += G) {
            const int32_t j = aj[k];
            unsorted |= k > a0 && aj[k - 1] >= j;
            if (strong((int32_t)i, j, aa[k], d, theta)) {
                ++c;
                ud += j > i ? 1 : -1;
            }
        }
        for (int o = G / 2; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
        if (on && l == 0) cnt[i] = c;
    }
    (void)segmask;
    for (int o = 32; o > 0; o >>= 1) ud += __shfl_xor(ud, o, 64);
    if (__ballot(unsorted) && (threadIdx.x & 63) == 0) atomicOr(flag, 1);
    if (ud != 0 && (threadIdx.x & 63) == 0) atomicAdd(updown, (unsigned long long)ud);
}

// the strong entries in A's order: lanes take entries l, l + G, ... and
// place them by a ballot over the row's lanes
template <int G>
__global__ __launch_bounds__(256) void k_strong_direct_fill(int32_t m, const int32_t *__restrict__ ai,
                                                            const int32_t *__restrict__ aj,
                                                            const double *__restrict__ aa,
                                                            const double *__restrict__ d, double theta,
                                                            const int32_t *__restrict__ si, int32_t *sj,
                                                            double *sval) {
    AIJHIP_ROW_LANES {
        const int64_t i = base + lane / G;
        const bool on = i < m;
        const int32_t a0 = on ? ai[i] : 0, a1 = on ? ai[i + 1] : 0;
        int32_t len = a1 - a0;
        for (int o = 32; o > 0; o >>= 1) len = max(len, __shfl_xor(len, o, 64));
        int32_t o = on ? si[i] : 0;
        for (int32_t r = 0; r < len; r += G) {  // wavefront-uniform rounds
            const int32_t k = a0 + r + l;
            const bool in = k < a1;
            const int32_t j = in ? aj[k] : 0;
            const double a = in ? aa[k] : 0.0;
            const bool keep = in && strong((int32_t)i, j, a, d, theta);
            const unsigned long long bal = __ballot(keep) & segmask;
            if (keep) {
                const int pos = __popcll(bal & ((1ull << lane) - 1ull));
                sj[o + pos] = j;
                sval[o + pos] = fabs(a);
            }
            o += __popcll(bal);
        }
    }
}

// flag = 1 when some (i, j) of S with j > i has no (j, i) (the entries below
// the diagonal are covered by the tally of k_strong_direct_count)
template <int G>
__global__ __launch_bounds__(256) void k_strong_asymmetric(int32_t m, const int32_t *__restrict__ si,
                                                           const int32_t *__restrict__ sj, int32_t *flag) {
    AIJHIP_ROW_LANES {
        const int64_t i = base + lane / G;
        if (i >= m) continue;
        (void)segmask;
        bool bad = false;
        for (int32_t k = si[i] + l; k < si[i + 1] && !bad; k += G) {
            const int32_t j = sj[k];
            if (j < (int32_t)i) continue;
            const int32_t e = si[j + 1];
            int32_t lo = si[j], hi = e;
            while (lo < hi) {
                const int32_t q = (lo + hi) >> 1;
                if (sj[q] < (int32_t)i) lo = q + 1;
                else hi = q;
            }
            bad = lo == e || sj[lo] != (int32_t)i;
        }
        if (bad) atomicOr(flag, 1);
    }
}
#undef AIJHIP_ROW_LANES

// Each gathered neighbour list of at most G entries sorted and made unique
// by G lanes (bitonic across the segment's lanes, unique by ballot), with the
// kept entries' weights: written back in place (tmp, tval), count to ucnt.
// Longer lists are k_strength_rows_long's / k_strength_rows_huge's.
template <int G, bool SORTED>
__global__ __launch_bounds__(256) void k_strength_rows(int32_t m, const unsigned long long *__restrict__ off,
                                                       int32_t *tmp, double *tval, int32_t *ucnt,
                                                       const int32_t *__restrict__ ai,
                                                       const int32_t *__restrict__ aj,
                                                       const double *__restrict__ aa) {
    const int lane = threadIdx.x & 63;
    const int l = lane & (G - 1);
    const unsigned long long segmask = (G == 64 ? ~0ull : ((1ull << G) - 1ull)) << (lane & ~(G - 1));
    const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t base = (((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6) * (64 / G); base < m;
         base += nw * (64 / G)) {
        const int64_t i = base + lane / G;
        unsigned long long o = 0;
        int n = G + 1;
        if (i < m) {
            o = off[i];
            n = (int)(off[i + 1] - o);
        }
        const bool mine = n <= G;
        int32_t v = (mine && l < n) ? tmp[o + l] : INT32_MAX;
#pragma unroll
        for (int k = 2; k <= G; k <<= 1) {
#pragma unroll
            for (int j = k >> 1; j > 0; j >>= 1) {
                const int32_t u = __shfl_xor(v, j, 64);
                const bool up = (l & k) == 0, low = (l & j) == 0;
                v = (up == low) ? min(v, u) : max(v, u);
            }
        }
        const int32_t prev = __shfl_up(v, 1, 64);
        const bool keep = mine && l < n && (l == 0 || v != prev);
        const unsigned long long bal = __ballot(keep);
        if (keep) {
            const int pos = __popcll(bal & segmask & ((1ull << lane) - 1ull));
            tmp[o + pos] = v;
            tval[o + pos] = stored_weight<SORTED>(v, ai[i], ai[i + 1], aj, aa);
        }
        if (mine && l == 0) ucnt[i] = __popcll(bal & segmask);
    }
}

// the rows whose gathered list is longer than lo entries and at most hi
__global__ void k_collect_rows(int32_t m, const unsigned long long *__restrict__ off, int lo, int hi,
                               int32_t *rows, unsigned int *count) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const int64_t n = (int64_t)(off[i + 1] - off[i]);
    if (n > lo && n <= hi) rows[atomicAdd(count, 1u)] = i;
}

constexpr int kLongList = 1024;  // k_strength_rows_long's LDS list

// The same for lists of 65..1024 entries, one workgroup per row: bitonic in
// LDS, unique by ballot with per-wave counts.
template <bool SORTED>
__global__ __launch_bounds__(256) void k_strength_rows_long(int32_t nrows, const int32_t *__restrict__ rows,
                                                            const unsigned long long *__restrict__ off,
                                                            int32_t *tmp, double *tval, int32_t *ucnt,
                                                            const int32_t *__restrict__ ai,
                                                            const int32_t *__restrict__ aj,
                                                            const double *__restrict__ aa) {
    __shared__ int32_t sv[kLongList];
    __shared__ int wsum[4];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    for (int32_t q = blockIdx.x; q < nrows; q += gridDim.x) {
        const int32_t i = rows[q];
        const unsigned long long o = off[i];
        const int n = (int)(off[i + 1] - o);
        int P = 128;
        while (P < n) P <<= 1;
        for (int x = t; x < P; x += 256) sv[x] = x < n ? tmp[o + x] : INT32_MAX;
        __syncthreads();
        for (int k = 2; k <= P; k <<= 1) {
            for (int j = k >> 1; j > 0; j >>= 1) {
                for (int x = t; x < P; x += 256) {
                    const int y = x ^ j;
                    if (y > x) {
                        const int32_t a = sv[x], b = sv[y];
                        if ((a > b) == ((x & k) == 0)) { sv[x] = b; sv[y] = a; }
                    }
                }
                __syncthreads();
            }
        }
        const int32_t a0 = ai[i], a1 = ai[i + 1];
        int kept = 0;
        for (int r = 0; r < P; r += 256) {
            const int x = r + t;
            const bool keep = x < n && (x == 0 || sv[x] != sv[x - 1]);
            const unsigned long long bal = __ballot(keep);
            if (lane == 0) wsum[w] = __popcll(bal);
            __syncthreads();
            int before = kept;
            for (int z = 0; z < w; ++z) before += wsum[z];
            const int total = wsum[0] + wsum[1] + wsum[2] + wsum[3];
            if (keep) {
                const int pos = before + __popcll(bal & ((1ull << lane) - 1ull));
                tmp[o + pos] = sv[x];
                tval[o + pos] = stored_weight<SORTED>(sv[x], a0, a1, aj, aa);
            }
            kept += total;
            __syncthreads();  // wsum is rewritten by the next round
        }
        if (t == 0) ucnt[i] = kept;
        __syncthreads();  // sv is refilled for the next row
    }
}

// Lists longer than kLongList: one lane per row, insertion sort in place.
template <bool SORTED>
__global__ void k_strength_rows_huge(int32_t nrows, const int32_t *__restrict__ rows,
                                     const unsigned long long *__restrict__ off, int32_t *tmp, double *tval,
                                     int32_t *ucnt, const int32_t *__restrict__ ai,
                                     const int32_t *__restrict__ aj, const double *__restrict__ aa) {
    const int32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nrows) return;
    const int32_t i = rows[q];
    int32_t *r = tmp + off[i];
    const int64_t n = (int64_t)(off[i + 1] - off[i]);
    for (int64_t a = 1; a < n; ++a) {
        const int32_t v = r[a];
        int64_t b = a - 1;
        while (b >= 0 && r[b] > v) { r[b + 1] = r[b]; --b; }
        r[b + 1] = v;
    }
    int64_t u = 0;
    for (int64_t a = 0; a < n; ++a)
        if (u == 0 || r[a] != r[u - 1]) r[u++] = r[a];
    for (int64_t a = 0; a < u; ++a) tval[off[i] + a] = stored_weight<SORTED>(r[a], ai[i], ai[i + 1], aj, aa);
    ucnt[i] = (int32_t)u;
}

// S = the unique lists compacted (G lanes per row)
template <int G>
__global__ __launch_bounds__(256) void k_strength_copy(int32_t m, const unsigned long long *__restrict__ off,
                                                       const int32_t *__restrict__ tmp,
                                                       const double *__restrict__ tval,
                                                       const int32_t *__restrict__ si, int32_t *sj,
                                                       double *sval) {
    const int lane = threadIdx.x & 63;
    const int l = lane & (G - 1);
    const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t base = (((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6) * (64 / G); base < m;
         base += nw * (64 / G)) {
        const int64_t i = base + lane / G;
        if (i >= m) continue;
        const unsigned long long o = off[i];
        const int32_t s0 = si[i], n = si[i + 1] - s0;
        for (int32_t k = l; k < n; k += G) {
            sj[s0 + k] = tmp[o + k];
            sval[s0 + k] = tval[o + k];
        }
    }
}

// Aggregation phase 2 (gamg_setup.cpp aggregate): a node phase 1 left free
// joins the aggregate of its strongest stored phase-1 neighbour, lowest
// index on ties.
__global__ void k_agg_phase2(int32_t m, const int32_t *__restrict__ si, const int32_t *__restrict__ sj,
                             const double *__restrict__ sval, const int32_t *__restrict__ phase1, int32_t *agg) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    int32_t a = phase1[i];
    if (a == -1) {
        int32_t best = -1;
        double bv = -1.0;
        for (int32_t k = si[i]; k < si[i + 1]; ++k) {
            const int32_t j = sj[k];
            const double v = sval[k];
            if (phase1[j] == -1 || v < 0.0) continue;
            if (v > bv || (v == bv && j < best)) { bv = v; best = j; }
        }
        if (best >= 0) a = phase1[best];
    }
    agg[i] = a;
}

__global__ void k_count_value(int32_t m, const int32_t *__restrict__ x, int32_t v, unsigned long long *count) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const bool hit = i < m && x[i] == v;
    const unsigned long long b = __ballot(hit);
    if ((threadIdx.x & 63) == 0 && b) atomicAdd(count, (unsigned long long)__popcll(b));
}

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

// the power iteration's start (gamg_setup.cpp estimate_emax)
__global__ void k_power_start(int32_t m, double *v) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    v[i] = 2.0 * ((double)(mix64(0x5EEDULL + (uint64_t)(i + 1) * 0x9E3779B97F4A7C15ULL) >> 11) *
                  (1.0 / 9007199254740992.0)) - 1.0;
}

constexpr int64_t kDotBlock = 256;  // gamg_setup.cpp kDotBlock

// One wavefront per 256-entry block: the lanes load the block coalesced (4
// entries each), stage the products in LDS, and lane 0 adds them left to
// right — the host builder's order (the host sums the blocks). One lane per
// block reading its 256 entries alone measured ~150 us per 27 M-entry dot
// (strided, uncoalesced loads) against ~55 us of bytes.
template <bool SQUARE>
__global__ __launch_bounds__(256) void k_block_dot_wave(int64_t n, const double *__restrict__ a,
                                                         const double *__restrict__ b, double *part) {
    static_assert(kDotBlock == 256, "four entries per lane");
    __shared__ double prod[4][kDotBlock];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t q = (int64_t)blockIdx.x * 4 + w;
    const int64_t i0 = q * kDotBlock;
    if (i0 >= n) return;  // (wave-uniform; no workgroup barrier below)
    const int64_t e = min(n, i0 + kDotBlock);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int64_t i = i0 + lane + 64 * j;
        double v = 0.0;
        if (i < e) v = SQUARE ? a[i] * a[i] : a[i] * b[i];
        prod[w][lane + 64 * j] = v;
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    if (lane == 0) {
        const int len = (int)(e - i0);
        double s = 0.0;
        int k = 0;
        for (; k + 8 <= len; k += 8) {
            double v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = prod[w][k + u];
#pragma unroll
            for (int u = 0; u < 8; ++u) s += v[u];
        }
        for (; k < len; ++k) s += prod[w][k];
        part[q] = s;
    }
}

// CG's emax estimate (gamg_setup.cpp estimate_emax_cg): the start, r -= a w
// with z = D^-1 r, and p = z + b p
__global__ void k_cgest_start(int32_t m, const double *__restrict__ dinv, double *r, double *z, double *p) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const double v = 2.0 * ((double)(mix64(0x5EEDULL + (uint64_t)(i + 1) * 0x9E3779B97F4A7C15ULL) >> 11) *
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

__global__ void k_div(int32_t m, const double *w, double nw, double *v) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < m) v[i] = w[i] / nw;
}

// head[i][t] = row i's t-th column of S, or i past its end (the host phase-1
// pass tests a free node's first columns from this dense array first)
__global__ void k_phase1_head(int32_t m, const int32_t *__restrict__ si, const int32_t *__restrict__ sj,
                              int32_t *__restrict__ head) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= (int64_t)m * aijhip_gamg::kPhase1Head) return;
    const int32_t i = (int32_t)(q / aijhip_gamg::kPhase1Head), t = (int32_t)(q % aijhip_gamg::kPhase1Head);
    const int64_t k = (int64_t)si[i] + t;
    head[q] = k < si[i + 1] ? sj[k] : i;
}

__global__ void k_fill(int32_t m, double v, double *x) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < m) x[i] = v;
}

// seg[a] = first position of aggregate a in the sorted aggregate keys
// The tentative prolongator's near-null space (gamg_setup.cpp prolongator):
// B_c[a] = sqrt of the sum of B[i]^2 over the members of aggregate a in
// ascending row order (the stable sort's order), p0[i] = B[i] / B_c[agg[i]].
__global__ void k_agg_norm(int32_t na, const int32_t *__restrict__ seg, const double *__restrict__ bm,
                           double *Bc) {
    const int32_t a = blockIdx.x * blockDim.x + threadIdx.x;
    if (a >= na) return;
    double s = 0.0;
    for (int32_t q = seg[a]; q < seg[a + 1]; ++q) {
        const double b = bm[q];
        s += b * b;
    }
    Bc[a] = sqrt(s);
}

// B = 1 (the finest level): the member counts, and B_c = sqrt(count) (the sum
// of count ones is count exactly, whatever the order)
__global__ void k_agg_count(int32_t m, const int32_t *__restrict__ agg, int32_t *count) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < m && agg[i] >= 0) atomicAdd(&count[agg[i]], 1);  // (-1: MIS's removed singleton)
}

__global__ void k_agg_norm_count(int32_t na, const int32_t *__restrict__ count, double *Bc) {
    const int32_t a = blockIdx.x * blockDim.x + threadIdx.x;
    if (a < na) Bc[a] = sqrt((double)count[a]);
}

// the sums of squares themselves (the distributed set-up adds the members
// other ranks hold before the square root): k_agg_norm / k_agg_norm_count
// without it
__global__ void k_agg_sumsq(int32_t na, const int32_t *__restrict__ seg, const double *__restrict__ bm, double *s2) {
    const int32_t a = blockIdx.x * blockDim.x + threadIdx.x;
    if (a >= na) return;
    double s = 0.0;
    for (int32_t q = seg[a]; q < seg[a + 1]; ++q) {
        const double b = bm[q];
        s += b * b;
    }
    s2[a] = s;
}

__global__ void k_agg_count_d(int32_t na, const int32_t *__restrict__ count, double *s2) {
    const int32_t a = blockIdx.x * blockDim.x + threadIdx.x;
    if (a < na) s2[a] = (double)count[a];
}

__global__ void k_tentative(int32_t m, const int32_t *__restrict__ agg, const double *__restrict__ B,
                            const double *__restrict__ Bc, double *p0) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const double c = agg[i] >= 0 ? Bc[agg[i]] : 0.0;
    p0[i] = c > 0.0 ? (B ? B[i] : 1.0) / c : 0.0;  // B == nullptr: the constant near-null space
}

// P0 with empty rows for the nodes no aggregate took (agg -1, MIS's removed
// singletons): flag / scan, then the compacted entries.
__global__ void k_member_flags(int32_t m, const int32_t *__restrict__ agg, int32_t *flag) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < m) flag[i] = agg[i] >= 0;
}

__global__ void k_member_compact(int32_t m, const int32_t *__restrict__ agg, const double *__restrict__ v,
                                 const int32_t *__restrict__ ai, int32_t *aj, double *aa) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m || agg[i] < 0) return;
    aj[ai[i]] = agg[i];
    aa[ai[i]] = v ? v[i] : 1.0;
}

__global__ void k_iota(int32_t n, int32_t *v) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i <= n) v[i] = i;
}

__global__ void k_widen(int32_t m, const int32_t *__restrict__ c, unsigned long long *w) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < m) w[i] = (unsigned long long)c[i];
}

__global__ void k_narrow(int32_t n, const unsigned long long *__restrict__ w, int32_t *c) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) c[i] = (int32_t)w[i];
}

// The same product, G lanes per output row sharing an LDS hash table of T
// column slots (round 3). The row's terms a_ik are taken in order; for each,
// the G lanes cover B row k's entries side by side, each adding its product
// to its column's slot. A row of B holds every column once, so no two lanes
// of one step touch the same slot, and the steps run in k order (the group
// is one wavefront's lanes, whose LDS operations complete in program order):
// per column, the sum runs in traversal order from 0.0, as with one lane
// alone — the same bits. Keys are claimed with an LDS compare-and-swap and
// linear probing; values need no atomics. A_i's terms come in chunks of G
// (one lane each: a_ik, k and B row k's extent) and are broadcast by shuffle.
// Each lane loads its first entry of the next D steps' B rows together
// before the first of them goes in (one load latency per D steps, not per
// step: the coarse Galerkin rows take hundreds of steps of ~15-entry B rows);
// the LDS order is unchanged.
// Count mode: cnt[i] = distinct columns, or -1 when they could pass keys_max
// (< T; checked against an upper bound, recounted exactly only when it says
// so);
// klass[i] = myclass when it fits. Write mode: the rows of myclass, their
// keys compacted and ranked (sorted columns) and written with the sums.
template <int G, int T, int NG, bool WRITE>
__global__ __launch_bounds__(G *NG) void k_rowprod_hash(int32_t m, const int32_t *__restrict__ ai,
                                                        const int32_t *__restrict__ aj,
                                                        const double *__restrict__ aa,
                                                        const int32_t *__restrict__ bi,
                                                        const int32_t *__restrict__ bj,
                                                        const double *__restrict__ ba, const int32_t *__restrict__ ci,
                                                        int32_t *cj, double *ca, int32_t *cnt, int32_t *klass,
                                                        int32_t myclass, bool redo, int keys_max) {
    static_assert(G >= 1 && G <= 64 && 64 % G == 0, "a group lies within one wavefront");
    static_assert((T & (T - 1)) == 0 && T >= 2 * G, "power-of-two table, at least two slots per lane");
    constexpr int LOGT = __builtin_ctz(T);
    constexpr int DM = WRITE ? 4 : 8;  // (write mode at 8: 82-98 VGPRs, 5 waves/SIMD; at 4: 58-76)
    constexpr int D = G < DM ? G : DM;  // steps whose first entries are loaded together
    __shared__ int32_t s_key[NG * T];
    __shared__ double s_val[WRITE ? NG * T : 1];
    __shared__ int32_t s_ck[WRITE ? NG * T : 1];
    const int g = threadIdx.x / G, l = threadIdx.x % G;
    const int gbase = (threadIdx.x & 63) - l;  // the group's first lane within the wavefront
    int32_t *key = s_key + g * T;
    double *val = s_val + (WRITE ? g * T : 0);
    int32_t *ck = s_ck + (WRITE ? g * T : 0);
    auto group_sum = [&](int v) {
#pragma unroll
        for (int off = G / 2; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
        return v;
    };
    for (int64_t i = (int64_t)blockIdx.x * NG + g; i < m; i += (int64_t)gridDim.x * NG) {
        if (!WRITE && redo && cnt[i] >= 0) continue;  // counted by a smaller class
        if (WRITE && klass[i] != myclass) continue;    // another class's row
        for (int s = l; s < T; s += G) {
            key[s] = -1;
            if (WRITE) val[s] = 0.0;
        }
        __builtin_amdgcn_wave_barrier();
        int mine = 0;     // keys this lane claimed
        int bound = 0;    // (group-uniform) at least the keys in the table
        bool over = false;
        const int32_t k1 = ai[i + 1];
        for (int32_t kc = ai[i]; kc < k1 && !over; kc += G) {
            int32_t q0 = 0, q1 = 0;
            double a = 0.0;
            if (kc + l < k1) {
                const int32_t j = aj[kc + l];
                if (WRITE) a = aa[kc + l];
                q0 = bi[j];
                q1 = bi[j + 1];
            }
            const int nk = min(G, k1 - kc);
            auto insert = [&](int32_t c, double p) {
                uint32_t h = ((uint32_t)c * 0x9E3779B1u) >> (32 - LOGT);
                for (;;) {
                    const int32_t old = atomicCAS(&key[h], -1, c);
                    if (old == -1) {
                        ++mine;
                        break;
                    }
                    if (old == c) break;
                    h = (h + 1) & (T - 1);
                }
                if (WRITE) val[h] += p;
            };
            for (int t0 = 0; t0 < nk && !over; t0 += D) {
                // steps t0 .. t0 + D - 1: extents, a_ik and this lane's first
                // entry of each B row, all loads in flight together
                int32_t pb0[D], pb1[D], pc[D];
                double pa[D], pv[D];
#pragma unroll
                for (int u = 0; u < D; ++u) {
                    const int src = gbase + (t0 + u < nk ? t0 + u : 0);
                    pb0[u] = __shfl(q0, src, 64);
                    pb1[u] = t0 + u < nk ? __shfl(q1, src, 64) : pb0[u];
                    pa[u] = WRITE ? __shfl(a, src, 64) : 0.0;
                    pc[u] = -1;
                    pv[u] = 0.0;
                    if (pb0[u] + l < pb1[u]) {
                        pc[u] = bj[pb0[u] + l];
                        if (WRITE) pv[u] = ba[pb0[u] + l];
                    }
                }
#pragma unroll
                for (int u = 0; u < D; ++u) {
                    if (t0 + u >= nk) break;  // group-uniform
                    const int len = pb1[u] - pb0[u];
                    if (bound + len > keys_max) {  // the table could fill: count exactly
                        bound = group_sum(mine);
                        if (bound + len > keys_max) {
                            over = true;
                            break;
                        }
                    }
                    bound += len;
                    if (pc[u] >= 0) insert(pc[u], WRITE ? pa[u] * pv[u] : 0.0);
                    for (int32_t q = pb0[u] + l + G; q < pb1[u]; q += G) insert(bj[q], WRITE ? pa[u] * ba[q] : 0.0);
                    __builtin_amdgcn_wave_barrier();
                }
            }
        }
        if (!WRITE) {
            const int tot = group_sum(mine);
            if (l == 0) {
                cnt[i] = over ? -1 : tot;
                if (!over) klass[i] = myclass;
            }
            __builtin_amdgcn_wave_barrier();  // the table is cleared for the group's next row
            continue;
        }
        // compact the keys, rank each against them (sorted columns), write
        const unsigned long long gmask = G == 64 ? ~0ull : ((1ull << G) - 1ull);
        const unsigned long long below = (1ull << l) - 1ull;
        int n = 0;
        for (int s0 = 0; s0 < T; s0 += G) {
            const int32_t c = key[s0 + l];
            const bool occ = c != -1;
            const unsigned long long b = (__ballot(occ) >> gbase) & gmask;
            if (occ) ck[n + __popcll(b & below)] = c;
            n += __popcll(b);
        }
        __builtin_amdgcn_wave_barrier();
        const int32_t o = ci[i];
        for (int s0 = 0; s0 < T; s0 += G) {
            const int32_t c = key[s0 + l];
            if (c != -1) {
                int r = 0;
                for (int z = 0; z < n; ++z) r += ck[z] < c;
                cj[o + r] = c;
                ca[o + r] = val[s0 + l];
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// T = A * P0 where P0 has one entry per row (column agg[k], value p0[k]):
// one lane per row, the row's distinct columns (at most CAP) in registers,
// each product added to its column in traversal order from 0.0 (the order
// of the general forms, so the same bits); sorted by rank on the way out.
// Count mode: cnt[i] = distinct columns, or -1 past CAP (the general form
// takes the product then).
template <int CAP, bool WRITE>
__global__ __launch_bounds__(256) void k_rowprod_p0(int32_t m, const int32_t *__restrict__ ai,
                                                    const int32_t *__restrict__ aj, const double *__restrict__ aa,
                                                    const int32_t *__restrict__ agg, const double *__restrict__ p0,
                                                    const int32_t *__restrict__ ci, int32_t *cj, double *ca,
                                                    int32_t *cnt) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    int32_t col[CAP];
    double val[CAP];
#pragma unroll
    for (int e = 0; e < CAP; ++e) {
        col[e] = -1;
        val[e] = 0.0;
    }
    int n = 0;
    bool over = false;
    const int32_t k1 = ai[i + 1];
    for (int32_t k = ai[i]; k < k1; ++k) {
        const int32_t j = aj[k];
        const int32_t c = agg[j];
        if (c < 0) continue;  // an empty row of P0
        const double p = WRITE ? aa[k] * p0[j] : 0.0;
        bool hit = false;
#pragma unroll
        for (int e = 0; e < CAP; ++e)
            if (col[e] == c) {
                if (WRITE) val[e] += p;
                hit = true;
            }
        if (hit) continue;
        if (n == CAP) {
            over = true;
            break;
        }
#pragma unroll
        for (int e = 0; e < CAP; ++e)
            if (e == n) {
                col[e] = c;
                if (WRITE) val[e] += p;  // from 0.0
            }
        ++n;
    }
    if (!WRITE) {
        cnt[i] = over ? -1 : n;
        return;
    }
    if (cnt[i] < 0) return;  // the general form's row
    const int32_t o = ci[i];
#pragma unroll
    for (int e = 0; e < CAP; ++e) {
        if (e < n) {
            int r = 0;
#pragma unroll
            for (int z = 0; z < CAP; ++z) r += (z < n && col[z] < col[e]);
            cj[o + r] = col[e];
            ca[o + r] = val[e];
        }
    }
}

// P = alpha (D^-1 T) + P0 on the union pattern (gamg_setup.cpp prolongator):
// lengths, then entries.
__global__ void k_prolong_len(int32_t m, const int32_t *__restrict__ ti, const int32_t *__restrict__ tj,
                              const int32_t *__restrict__ agg, int32_t *len) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    bool has = agg[i] < 0;  // (no P0 entry)
    for (int32_t k = ti[i]; k < ti[i + 1]; ++k) has |= tj[k] == agg[i];
    len[i] = ti[i + 1] - ti[i] + (has ? 0 : 1);
}

__global__ void k_prolong_fill(int32_t m, const int32_t *__restrict__ ti, const int32_t *__restrict__ tj,
                               const double *__restrict__ ta, const int32_t *__restrict__ agg,
                               const double *__restrict__ p0v, const double *__restrict__ dinv, double alpha,
                               const int32_t *__restrict__ pi, int32_t *pj, double *pa) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    int32_t p = pi[i];
    const int32_t g = agg[i];
    bool placed = g < 0;  // (no P0 entry to place)
    const double p0 = p0v[i];
    for (int32_t k = ti[i]; k < ti[i + 1]; ++k) {
        const int32_t c = tj[k];
        if (!placed && g < c) { pj[p] = g; pa[p] = p0; ++p; placed = true; }
        const double t = dinv[i] * ta[k];
        pj[p] = c;
        pa[p] = alpha * t + (c == g ? p0 : 0.0);
        if (c == g) placed = true;
        ++p;
    }
    if (!placed) { pj[p] = g; pa[p] = p0; }
}

// ---------------------------------------------------------------- host side

using aijhip_gamg::DCsr;
using aijhip_gamg::dalloc;

// exclusive scan of int32 counts into int32 offsets (m+1); false on overflow
hipError_t scan_offsets(const int32_t *cnt, int32_t m, int32_t *off, int64_t *total) {
    unsigned long long *w = nullptr, *o = nullptr, *stmp = nullptr;
    hipError_t e;
    if ((e = dalloc(&w, (int64_t)m + 1)) != hipSuccess || (e = dalloc(&o, (int64_t)m + 1)) != hipSuccess) goto done;
    if ((e = hipMemset(w, 0, sizeof(unsigned long long) * ((size_t)m + 1))) != hipSuccess) goto done;
    if (m > 0) hipLaunchKernelGGL(k_widen, dim3(blocks_for(m, 256)), dim3(256), 0, nullptr, m, cnt, w);
    if ((e = dalloc(&stmp, aijhip_dscan::scan_tmp_elems((int64_t)m + 1))) != hipSuccess) goto done;
    if ((e = aijhip_dscan::exclusive_scan(w, o, (int64_t)m + 1, stmp, nullptr)) != hipSuccess) goto done;
    {
        unsigned long long t = 0;
        if ((e = hipMemcpy(&t, o + m, sizeof(t), hipMemcpyDeviceToHost)) != hipSuccess) goto done;
        *total = (int64_t)t;
        if (t <= (unsigned long long)INT32_MAX) {  // narrow to int32 offsets (PetscInt)
            hipLaunchKernelGGL(k_narrow, dim3(blocks_for((int64_t)m + 1, 256)), dim3(256), 0, nullptr, m + 1, o, off);
            e = hipGetLastError();
        }
    }
done:
    hipFree(w); hipFree(o); hipFree(stmp);
    return e;
}

// P0 (na columns) as a CSR: row i holds (agg[i], v[i]) (v nullptr: 1.0), or
// nothing where agg[i] = -1 (MIS's removed singletons). Without such rows
// the arrays are agg and v themselves (borrowed: *own false, only P0.ai
// allocated); else compacted copies (*own true).
hipError_t p0_csr(int32_t m, int32_t na, const int32_t *agg, const double *v, DCsr &P0, bool *own) {
    P0 = DCsr();
    P0.m = m;
    P0.n = na;
    *own = false;
    unsigned long long *nfree = nullptr;
    unsigned long long h = 0;
    hipError_t e = dalloc(&nfree, 1);
    if (e == hipSuccess) e = hipMemset(nfree, 0, sizeof(h));
    if (e == hipSuccess && m > 0) {
        hipLaunchKernelGGL(k_count_value, dim3(blocks_for(m, 256)), dim3(256), 0, nullptr, m, agg, -1, nfree);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpy(&h, nfree, sizeof(h), hipMemcpyDeviceToHost);
    hipFree(nfree);
    if (e != hipSuccess) return e;
    if ((e = dalloc(&P0.ai, (int64_t)m + 1)) != hipSuccess) return e;
    if (h == 0 && v) {
        hipLaunchKernelGGL(k_iota, dim3(blocks_for((int64_t)m + 1, 256)), dim3(256), 0, nullptr, m, P0.ai);
        P0.nz = m;
        P0.aj = const_cast<int32_t *>(agg);
        P0.aa = const_cast<double *>(v);
        return hipGetLastError();
    }
    *own = true;
    int32_t *flag = nullptr;
    if ((e = dalloc(&flag, m)) == hipSuccess) {
        if (m > 0) hipLaunchKernelGGL(k_member_flags, dim3(blocks_for(m, 256)), dim3(256), 0, nullptr, m, agg, flag);
        e = scan_offsets(flag, m, P0.ai, &P0.nz);
    }
    hipFree(flag);
    if (e == hipSuccess && (e = dalloc(&P0.aj, P0.nz + 2)) == hipSuccess && (e = dalloc(&P0.aa, P0.nz + 2)) == hipSuccess &&
        m > 0) {
        hipLaunchKernelGGL(k_member_compact, dim3(blocks_for(m, 256)), dim3(256), 0, nullptr, m, agg, v, P0.ai, P0.aj,
                           P0.aa);
        e = hipGetLastError();
    }
    if (e != hipSuccess) P0.release();
    return e;
}

// C = A * B. Returns AIJHIP_OK, or AIJHIP_ERR_STATE when a row's distinct
// columns exceed every device capacity (the caller falls back to the host).
// The hash-table classes (k_rowprod_hash): table sizes tried in order; a
// row counted -1 at one size is recounted at the next. Groups per workgroup:
// at least a wavefront, at most 256 lanes and 64 KiB of LDS (16 B per slot
// in the numeric pass).
constexpr int kHashClasses = 6;
constexpr int kHashT[kHashClasses] = {16, 32, 64, 128, 256, 1024};
constexpr int kHashClassId = 16;  // klass ids kHashClassId + t

template <int G, int T>
constexpr int hash_groups() {
    return std::max(64 / G, std::min(256 / G, 65536 / (16 * T)));
}

template <int G, int T>
hipError_t rowprod_hash_pass(const DCsr &A, const DCsr &B, int32_t *cnt, int32_t *klass, int32_t myclass, bool redo,
                             const int32_t *ci, DCsr *C, bool numeric, int n_cu) {
    // A product of few rows (a coarse level's: 744 at 300^3) leaves most CUs
    // idle, and each group's time is its probes: at most half-full tables
    // there (linear probing at load ~0.9 walks several slots per insert);
    // many rows keep the fuller tables and their occupancy.
    const int keys_max = A.m < 64 * n_cu ? T / 2 : T - 1;
    constexpr int NG = hash_groups<G, T>();
    static_assert(NG * T * 16 <= 65536, "LDS per workgroup");
    const unsigned grid = (unsigned)std::min<int64_t>(blocks_for(A.m, NG), (int64_t)n_cu * 32);
    if (!numeric)
        hipLaunchKernelGGL((k_rowprod_hash<G, T, NG, false>), dim3(grid), dim3(G * NG), 0, nullptr, A.m, A.ai, A.aj,
                           A.aa, B.ai, B.aj, B.aa, nullptr, nullptr, nullptr, cnt, klass, myclass, redo, keys_max);
    else
        hipLaunchKernelGGL((k_rowprod_hash<G, T, NG, true>), dim3(grid), dim3(G * NG), 0, nullptr, A.m, A.ai, A.aj,
                           A.aa, B.ai, B.aj, B.aa, ci, C->aj, C->aa, cnt, klass, myclass, false, keys_max);
    return hipGetLastError();
}

// lanes per row for table t given the preferred G (at most half the table;
// at least 16 for the largest table, whose groups would not fit otherwise)
int hash_lanes(int G, int t) {
    const int T = kHashT[t];
    if (G > T / 2) G = T / 2;
    if (T == 1024 && G < 16) G = 16;
    return G;
}

hipError_t rowprod_hash_class(int t, int G, const DCsr &A, const DCsr &B, int32_t *cnt, int32_t *klass, bool redo,
                              const int32_t *ci, DCsr *C, bool numeric, int n_cu) {
    const int id = kHashClassId + t;
#define AIJHIP_HASH(GG, TT)                                                                                   \
    if (G == GG && kHashT[t] == TT) return rowprod_hash_pass<GG, TT>(A, B, cnt, klass, id, redo, ci, C, numeric, n_cu)
    AIJHIP_HASH(4, 16); AIJHIP_HASH(8, 16); AIJHIP_HASH(4, 32); AIJHIP_HASH(8, 32); AIJHIP_HASH(16, 32);
    AIJHIP_HASH(4, 64); AIJHIP_HASH(4, 128); AIJHIP_HASH(4, 256);
    AIJHIP_HASH(8, 64); AIJHIP_HASH(8, 128); AIJHIP_HASH(8, 256);
    AIJHIP_HASH(16, 64); AIJHIP_HASH(16, 128); AIJHIP_HASH(16, 256); AIJHIP_HASH(16, 1024);
    AIJHIP_HASH(32, 64); AIJHIP_HASH(32, 128); AIJHIP_HASH(32, 256); AIJHIP_HASH(32, 1024);
    AIJHIP_HASH(64, 128); AIJHIP_HASH(64, 256); AIJHIP_HASH(64, 1024);
#undef AIJHIP_HASH
    return hipErrorInvalidValue;
}

// the minimum of cnt[0..m) (0 when m = 0)
hipError_t min_of(const int32_t *cnt, int32_t m, int32_t *mn) {
    *mn = 0;
    if (m == 0) return hipSuccess;
    int32_t *dmin = nullptr;
    int dev = 0, cus = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    hipError_t r;
    if ((r = dalloc(&dmin, 1)) == hipSuccess &&
        (r = aijhip_dscan::extreme<int32_t, false>(cnt, m, dmin, cus, nullptr)) == hipSuccess)
        r = hipMemcpy(mn, dmin, sizeof(int32_t), hipMemcpyDeviceToHost);
    hipFree(dmin);
    return r;
}

int rowprod(const DCsr &A, const DCsr &B, DCsr &C, int n_cu, int *cols_used = nullptr);

// T = A * P0 (P0: one entry per row, column agg, value p0) by k_rowprod_p0;
// a row with more than kP0Cap distinct columns sends the whole product to
// the general form (same bits either way).
constexpr int kP0Cap = 8;
int rowprod_p0(const DCsr &A, const DCsr &P0, const int32_t *agg, const double *p0, DCsr &C, int n_cu,
               int *cols_used) {
    // (rows of A longer than the list on average: the hash form directly)
    if (A.nz > (int64_t)kP0Cap * std::max<int32_t>(A.m, 1)) return rowprod(A, P0, C, n_cu, cols_used);
    C = DCsr();
    C.m = A.m;
    C.n = P0.n;
    int32_t *cnt = nullptr;
    hipError_t e;
    const unsigned g = blocks_for(A.m, 256);
    if ((e = dalloc(&cnt, A.m)) != hipSuccess) return herr(e, "product counts");
    if (A.m > 0)
        hipLaunchKernelGGL((k_rowprod_p0<kP0Cap, false>), dim3(g), dim3(256), 0, nullptr, A.m, A.ai, A.aj, A.aa,
                           agg, p0, nullptr, nullptr, nullptr, cnt);
    int32_t mn = 0;
    if ((e = hipGetLastError()) != hipSuccess || (e = min_of(cnt, A.m, &mn)) != hipSuccess) {
        hipFree(cnt);
        return herr(e, "symbolic product");
    }
    if (mn < 0) {
        hipFree(cnt);
        return rowprod(A, P0, C, n_cu, cols_used);
    }
    int64_t total = 0;
    if ((e = dalloc(&C.ai, (int64_t)A.m + 1)) != hipSuccess || (e = scan_offsets(cnt, A.m, C.ai, &total)) != hipSuccess ||
        (e = dalloc(&C.aj, total + 2)) != hipSuccess || (e = dalloc(&C.aa, total + 2)) != hipSuccess ||
        (e = hipMemset(C.aj + total, 0, 2 * sizeof(int32_t))) != hipSuccess ||
        (e = hipMemset(C.aa + total, 0, 2 * sizeof(double))) != hipSuccess) {
        hipFree(cnt);
        C.release();
        return herr(e, "product alloc");
    }
    C.nz = total;
    if (A.m > 0)
        hipLaunchKernelGGL((k_rowprod_p0<kP0Cap, true>), dim3(g), dim3(256), 0, nullptr, A.m, A.ai, A.aj, A.aa,
                           agg, p0, C.ai, C.aj, C.aa, cnt);
    e = hipGetLastError();
    hipFree(cnt);
    if (e != hipSuccess) {
        C.release();
        return herr(e, "numeric product");
    }
    if (cols_used) *cols_used = std::max(*cols_used, kP0Cap);
    return AIJHIP_OK;
}

int rowprod(const DCsr &A, const DCsr &B, DCsr &C, int n_cu, int *cols_used) {
    C = DCsr();
    C.m = A.m;
    C.n = B.n;
    int32_t *cnt = nullptr;
    hipError_t e;
    if ((e = dalloc(&cnt, A.m)) != hipSuccess) return herr(e, "product counts");
    // products per row (mean): A's row length x B's
    double per_row = 0.0, b_row = 0.0;
    {
        int32_t bnz = 0;
        if ((e = hipMemcpy(&bnz, B.ai + B.m, sizeof(int32_t), hipMemcpyDeviceToHost)) != hipSuccess) {
            hipFree(cnt);
            return herr(e, "product sizes");
        }
        per_row = B.m > 0 ? (double)A.nz * ((double)bnz / (double)B.m) / std::max<int32_t>(A.m, 1) : 0.0;
        b_row = B.m > 0 ? (double)bnz / (double)B.m : 0.0;
    }
    {
        // G lanes per row: B's mean row length rounded up to a power of two
        int G = 4;
        while (G < 64 && G < b_row) G <<= 1;
        const bool log = std::getenv("AIJHIP_GAMG_LOG") != nullptr;
        const auto t0 = std::chrono::steady_clock::now();
        int32_t *klass = nullptr;
        auto bail = [&](hipError_t r, const char *what) {
            hipFree(cnt);
            hipFree(klass);
            C.release();
            return herr(r, what);
        };
        if ((e = dalloc(&klass, A.m)) != hipSuccess) return bail(e, "product classes");
        // the first table: the smallest above the mean products per row
        // (their bound on the distinct columns; twice that for few rows),
        // at most 64 slots (128); rows that overflow it are recounted with
        // the next. The table size never changes the sums (traversal order)
        int first = 0;
        const int fill = A.m < 64 * n_cu ? 2 : 1;  // few rows: half-full tables (rowprod_hash_pass)
        while (first + 1 < kHashClasses && kHashT[first] <= fill * std::min(per_row, 48.0)) ++first;
        int last = -1;
        for (int t = first; t < kHashClasses; ++t) {
            if ((e = rowprod_hash_class(t, hash_lanes(G, t), A, B, cnt, klass, t > first, nullptr, nullptr, false,
                                        n_cu)) != hipSuccess)
                return bail(e, "symbolic product");
            int32_t mn = 0;
            if ((e = min_of(cnt, A.m, &mn)) != hipSuccess) return bail(e, "symbolic product");
            if (mn >= 0) {
                last = t;
                break;
            }
        }
        if (last < 0) {  // a row past the largest table: the host builder takes the level
            hipFree(cnt);
            hipFree(klass);
            return AIJHIP_ERR_STATE;
        }
        if ((e = dalloc(&C.ai, (int64_t)A.m + 1)) != hipSuccess) return bail(e, "product rows");
        int64_t total = 0;
        if ((e = scan_offsets(cnt, A.m, C.ai, &total)) != hipSuccess) return bail(e, "scan");
        if (total > INT32_MAX) {
            hipFree(cnt);
            hipFree(klass);
            C.release();
            set_error("GAMG device set-up: product exceeds int32 indices");
            return AIJHIP_ERR_ARG;
        }
        C.nz = total;
        if ((e = dalloc(&C.aj, total + 2)) != hipSuccess || (e = dalloc(&C.aa, total + 2)) != hipSuccess ||
            (e = hipMemset(C.aj + total, 0, 2 * sizeof(int32_t))) != hipSuccess ||
            (e = hipMemset(C.aa + total, 0, 2 * sizeof(double))) != hipSuccess)
            return bail(e, "product alloc");
        for (int t = first; t <= last && e == hipSuccess; ++t)
            e = rowprod_hash_class(t, hash_lanes(G, t), A, B, cnt, klass, false, C.ai, &C, true, n_cu);
        if (e != hipSuccess) return bail(e, "numeric product");
        hipFree(cnt);
        hipFree(klass);
        if (cols_used) *cols_used = std::max(*cols_used, kHashT[last]);
        if (log) {
            (void)hipDeviceSynchronize();
            std::fprintf(stderr, "  product %d x %d: %.0f products per row, B rows %.1f -> hash, %d lanes, "
                         "tables %d-%d: %.2f ms\n", A.m, B.n, per_row, b_row, G, kHashT[first], kHashT[last],
                         std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() * 1e3);
        }
        return AIJHIP_OK;
    }
}

// S directly from A (k_strong_direct_*): *ok = false, nothing allocated,
// when A has an unsorted row or the strong pattern is not symmetric (the
// caller then gathers S u S^T).
int strength_direct(const aijhip_mat &A, const double *d, double theta, int32_t **si, int32_t **sj,
                    double **sval, int64_t *nzs, bool *ok) {
    const int32_t m = A.m;
    int32_t *cnt = nullptr, *flag = nullptr;
    unsigned long long *updown = nullptr;  // flag (int32) and the tally, one allocation
    struct { int32_t flag, pad; long long updown; } h = {0, 0, 0};
    hipError_t e;
    int rc = AIJHIP_OK;
    *ok = false;
    *si = *sj = nullptr;
    *sval = nullptr;
#define DTRY(call, what) do { if ((e = (call)) != hipSuccess) { rc = herr(e, what); goto done; } } while (0)
    DTRY(dalloc(&updown, 2), "alloc");
    flag = reinterpret_cast<int32_t *>(updown);
    ++updown;
    DTRY(hipMemset(flag, 0, 2 * sizeof(unsigned long long)), "memset");
    {
        // lanes per row: the mean row length rounded up to a power of two
        const double mean = m > 0 ? (double)A.nz / m : 1.0;
        int G = 4;
        while (G < 64 && G < mean) G <<= 1;
        const unsigned grid = (unsigned)std::min<int64_t>(blocks_for((int64_t)m * G, 256), (int64_t)A.n_cu * 64);
        DTRY(dalloc(&cnt, m), "alloc");
#define AIJHIP_SD(GG)                                                                                         \
    case GG:                                                                                                  \
        hipLaunchKernelGGL((k_strong_direct_count<GG>), dim3(grid), dim3(256), 0, nullptr, m, A.d_ai, A.d_aj,  \
                           A.d_aa, d, theta, cnt, flag, updown);                                              \
        break
        switch (G) { AIJHIP_SD(4); AIJHIP_SD(8); AIJHIP_SD(16); AIJHIP_SD(32); AIJHIP_SD(64); }
#undef AIJHIP_SD
        DTRY(hipGetLastError(), "strength kernels");
        DTRY(hipMemcpy(&h, flag, sizeof(h), hipMemcpyDeviceToHost), "read");
        if (h.flag || h.updown != 0) goto done;  // unsorted rows, or S cannot be symmetric
        DTRY(dalloc(si, (int64_t)m + 1), "alloc");
        DTRY(scan_offsets(cnt, m, *si, nzs), "scan");
        if (*nzs > INT32_MAX) { rc = AIJHIP_ERR_ARG; set_error("GAMG: strength graph exceeds int32"); goto done; }
        DTRY(dalloc(sj, *nzs), "alloc");
        DTRY(dalloc(sval, *nzs), "alloc");
#define AIJHIP_SD(GG)                                                                                         \
    case GG:                                                                                                  \
        hipLaunchKernelGGL((k_strong_direct_fill<GG>), dim3(grid), dim3(256), 0, nullptr, m, A.d_ai, A.d_aj,   \
                           A.d_aa, d, theta, *si, *sj, *sval);                                                \
        hipLaunchKernelGGL((k_strong_asymmetric<GG>), dim3(grid), dim3(256), 0, nullptr, m, *si, *sj, flag);  \
        break
        switch (G) { AIJHIP_SD(4); AIJHIP_SD(8); AIJHIP_SD(16); AIJHIP_SD(32); AIJHIP_SD(64); }
#undef AIJHIP_SD
    }
    DTRY(hipGetLastError(), "strength kernels");
    DTRY(hipMemcpy(&h.flag, flag, sizeof(h.flag), hipMemcpyDeviceToHost), "read");
    *ok = h.flag == 0;
done:
#undef DTRY
    hipFree(cnt);
    hipFree(flag);  // (and the tally: one allocation)
    if (rc || !*ok) {
        hipFree(*si); hipFree(*sj); hipFree(*sval);
        *si = *sj = nullptr;
        *sval = nullptr;
    }
    return rc;
}

// S from the gathered lists (tmp, rows at off, cnt entries each): sorted,
// unique, weighted, compacted into (si, sj, sval) of *nzs entries.
int strength_lists(const aijhip_mat &A, const unsigned long long *cnt, const unsigned long long *off,
                   int32_t *tmp, int64_t ntmp, int n_cu, int32_t **si, int32_t **sj, double **sval, int64_t *nzs) {
    const int32_t m = A.m;
    double *tval = nullptr;
    int32_t *ucnt = nullptr, *rows = nullptr, *flag = nullptr;
    unsigned long long *dmax = nullptr;
    unsigned int *nrows = nullptr;
    unsigned long long maxn = 0;
    int32_t unsorted = 0;
    int G = 8;
    hipError_t e;
    const unsigned g256 = blocks_for(m, 256);
    *si = *sj = nullptr;
    *sval = nullptr;
#define STRY(call, what) do { if ((e = (call)) != hipSuccess) { rc = herr(e, what); goto done; } } while (0)
    int rc = AIJHIP_OK;
    STRY(dalloc(&tval, ntmp), "alloc");
    STRY(dalloc(&ucnt, m), "alloc");
    STRY(dalloc(&flag, 1), "alloc");
    STRY(dalloc(&dmax, 1), "alloc");
    STRY(hipMemset(flag, 0, sizeof(int32_t)), "memset");
    STRY(hipMemset(dmax, 0, sizeof(unsigned long long)), "memset");
    hipLaunchKernelGGL(k_rows_unsorted, dim3(g256), dim3(256), 0, nullptr, m, A.d_ai, A.d_aj, flag);
    if (m > 0) STRY((aijhip_dscan::extreme<unsigned long long, true>(cnt, m, dmax, n_cu, nullptr)), "reduce");
    STRY(hipMemcpy(&maxn, dmax, sizeof(maxn), hipMemcpyDeviceToHost), "read");
    STRY(hipMemcpy(&unsorted, flag, sizeof(unsorted), hipMemcpyDeviceToHost), "read");
    while (G < 64 && (unsigned long long)G < maxn) G <<= 1;
    {
        const unsigned grid = (unsigned)std::min<int64_t>(blocks_for((int64_t)m * G, 256), (int64_t)n_cu * 32);
#define AIJHIP_SR(GG)                                                                                          \
    case GG:                                                                                                   \
        if (unsorted)                                                                                          \
            hipLaunchKernelGGL((k_strength_rows<GG, false>), dim3(grid), dim3(256), 0, nullptr, m, off, tmp,   \
                               tval, ucnt, A.d_ai, A.d_aj, A.d_aa);                                            \
        else                                                                                                   \
            hipLaunchKernelGGL((k_strength_rows<GG, true>), dim3(grid), dim3(256), 0, nullptr, m, off, tmp,    \
                               tval, ucnt, A.d_ai, A.d_aj, A.d_aa);                                            \
        break
        switch (G) { AIJHIP_SR(8); AIJHIP_SR(16); AIJHIP_SR(32); AIJHIP_SR(64); }
#undef AIJHIP_SR
    }
    if (maxn > 64) {  // the long lists: a workgroup per row, past kLongList a lane per row
        STRY(dalloc(&rows, m), "alloc");
        STRY(dalloc(&nrows, 2), "alloc");
        STRY(hipMemset(nrows, 0, 2 * sizeof(unsigned int)), "memset");
        hipLaunchKernelGGL(k_collect_rows, dim3(g256), dim3(256), 0, nullptr, m, off, 64, kLongList, rows, nrows);
        unsigned int nl = 0, nh = 0;
        STRY(hipMemcpy(&nl, nrows, sizeof(nl), hipMemcpyDeviceToHost), "read");
        if (nl > 0) {
            const unsigned grid = (unsigned)std::min<int64_t>(nl, (int64_t)n_cu * 8);
            if (unsorted)
                hipLaunchKernelGGL(k_strength_rows_long<false>, dim3(grid), dim3(256), 0, nullptr, (int32_t)nl, rows,
                                   off, tmp, tval, ucnt, A.d_ai, A.d_aj, A.d_aa);
            else
                hipLaunchKernelGGL(k_strength_rows_long<true>, dim3(grid), dim3(256), 0, nullptr, (int32_t)nl, rows,
                                   off, tmp, tval, ucnt, A.d_ai, A.d_aj, A.d_aa);
        }
        if (maxn > (unsigned long long)kLongList) {
            hipLaunchKernelGGL(k_collect_rows, dim3(g256), dim3(256), 0, nullptr, m, off, kLongList, INT32_MAX,
                               rows, nrows + 1);
            STRY(hipMemcpy(&nh, nrows + 1, sizeof(nh), hipMemcpyDeviceToHost), "read");
            if (nh > 0) {
                if (unsorted)
                    hipLaunchKernelGGL(k_strength_rows_huge<false>, dim3(blocks_for(nh, 64)), dim3(64), 0, nullptr,
                                       (int32_t)nh, rows, off, tmp, tval, ucnt, A.d_ai, A.d_aj, A.d_aa);
                else
                    hipLaunchKernelGGL(k_strength_rows_huge<true>, dim3(blocks_for(nh, 64)), dim3(64), 0, nullptr,
                                       (int32_t)nh, rows, off, tmp, tval, ucnt, A.d_ai, A.d_aj, A.d_aa);
            }
        }
    }
    STRY(hipGetLastError(), "strength kernels");
    STRY(dalloc(si, (int64_t)m + 1), "alloc");
    STRY(scan_offsets(ucnt, m, *si, nzs), "scan");
    if (*nzs > INT32_MAX) { rc = AIJHIP_ERR_ARG; set_error("GAMG: strength graph exceeds int32"); goto done; }
    STRY(dalloc(sj, *nzs), "alloc");
    STRY(dalloc(sval, *nzs), "alloc");
    {
        const unsigned grid = (unsigned)std::min<int64_t>(blocks_for((int64_t)m * G, 256), (int64_t)n_cu * 32);
        switch (G) {
            case 8: hipLaunchKernelGGL(k_strength_copy<8>, dim3(grid), dim3(256), 0, nullptr, m, off, tmp, tval, *si, *sj, *sval); break;
            case 16: hipLaunchKernelGGL(k_strength_copy<16>, dim3(grid), dim3(256), 0, nullptr, m, off, tmp, tval, *si, *sj, *sval); break;
            case 32: hipLaunchKernelGGL(k_strength_copy<32>, dim3(grid), dim3(256), 0, nullptr, m, off, tmp, tval, *si, *sj, *sval); break;
            default: hipLaunchKernelGGL(k_strength_copy<64>, dim3(grid), dim3(256), 0, nullptr, m, off, tmp, tval, *si, *sj, *sval); break;
        }
    }
    STRY(hipGetLastError(), "strength copy");
done:
#undef STRY
    hipFree(tval); hipFree(ucnt); hipFree(rows); hipFree(flag); hipFree(dmax); hipFree(nrows);
    if (rc) {
        hipFree(*si); hipFree(*sj); hipFree(*sval);
        *si = *sj = nullptr;
        *sval = nullptr;
    }
    return rc;
}

// B_c and p0 of the tentative prolongator from the aggregates (device).
// The members of each aggregate in ascending row order, with their B, are
// the transpose of P0's pattern (one entry per row, column agg[i], value
// B[i]): the library's stable transpose gives exactly that.
hipError_t tentative(int32_t m, int32_t na, const int32_t *agg, const double *B, double *Bc, double *p0,
                     bool b_ones = false, bool sumsq = false) {
    // sumsq: Bc gets the sums of squares (no square root) and p0 is untouched
    if (m == 0) return hipSuccess;
    int32_t *ai = nullptr, *tai = nullptr, *taj = nullptr;
    double *taa = nullptr;
    hipError_t e;
    if (b_ones) {  // B = 1: each sum of B^2 is its member count, exact in any order
        int32_t *count = nullptr;
        if ((e = dalloc(&count, std::max(na, 1))) != hipSuccess) return e;
        if ((e = hipMemset(count, 0, sizeof(int32_t) * (size_t)std::max(na, 1))) == hipSuccess) {
            hipLaunchKernelGGL(k_agg_count, dim3(blocks_for(m, 256)), dim3(256), 0, nullptr, m, agg, count);
            if (sumsq) {
                if (na > 0) hipLaunchKernelGGL(k_agg_count_d, dim3(blocks_for(na, 256)), dim3(256), 0, nullptr, na, count, Bc);
            } else {
                if (na > 0)
                    hipLaunchKernelGGL(k_agg_norm_count, dim3(blocks_for(na, 256)), dim3(256), 0, nullptr, na, count, Bc);
                hipLaunchKernelGGL(k_tentative, dim3(blocks_for(m, 256)), dim3(256), 0, nullptr, m, agg, B, Bc, p0);
            }
            e = hipGetLastError();
        }
        hipFree(count);
        return e;
    }
    DCsr P0;
    bool own = false;
    if ((e = p0_csr(m, na, agg, B, P0, &own)) != hipSuccess) return e;
    ai = P0.ai;
    {
        aijhip_mat v;  // non-owning view
        v.m = m;
        v.n = na;
        v.nz = P0.nz;
        v.d_ai = P0.ai;
        v.d_aj = P0.aj;
        v.d_aa = P0.aa;
        e = aijhip::build_transpose(v, &tai, &taj, &taa, nullptr);
        v.d_ai = v.d_aj = nullptr;
        v.d_aa = nullptr;
    }
    if (own) {
        hipFree(P0.aj);
        hipFree(P0.aa);
    }
    if (e == hipSuccess && sumsq) {
        if (na > 0) hipLaunchKernelGGL(k_agg_sumsq, dim3(blocks_for(na, 256)), dim3(256), 0, nullptr, na, tai, taa, Bc);
        e = hipGetLastError();
    } else if (e == hipSuccess) {
        if (na > 0) hipLaunchKernelGGL(k_agg_norm, dim3(blocks_for(na, 256)), dim3(256), 0, nullptr, na, tai, taa, Bc);
        hipLaunchKernelGGL(k_tentative, dim3(blocks_for(m, 256)), dim3(256), 0, nullptr, m, agg, B, Bc, p0);
        e = hipGetLastError();
    }
    hipFree(ai); hipFree(tai); hipFree(taj); hipFree(taa);
    return e;
}

// a . b in the host builder's blocked order (block sums on the device, then
// summed left to right on the host)
// (s: the emax job's own stream — its copies wait for its kernels only, not
// for the aggregation the set-up thread runs meanwhile on the null stream)
// Block partials come down into h_part: pinned (the emax job's) — a
// pageable copy goes through the runtime's staging and, measured, kept the
// job in step with the aggregation on the null stream (r05j: the CG estimate
// was the level's critical path) — or a vector grown here (other callers).
struct HostPart {
    double *pinned = nullptr;
    int64_t cap = 0;
    std::vector<double> pageable;
    double *get(int64_t nb) {
        if (pinned && nb <= cap) return pinned;
        pageable.resize((size_t)std::max<int64_t>(nb, 1));
        return pageable.data();
    }
};

double host_blocked_dot(const double *d_a, const double *d_b, int64_t n, double *d_part, HostPart &hp,
                        hipError_t *e, hipStream_t s = nullptr) {
    const int64_t nb = (n + kDotBlock - 1) / kDotBlock;
    if (nb > 0)
        hipLaunchKernelGGL(k_block_dot_wave<false>, dim3(blocks_for(nb, 4)), dim3(256), 0, s, n, d_a, d_b, d_part);
    double *h = hp.get(nb);
    *e = hipSuccess;
    if (nb > 0 && (*e = hipMemcpyAsync(h, d_part, sizeof(double) * (size_t)nb, hipMemcpyDeviceToHost, s)) == hipSuccess)
        *e = hipStreamSynchronize(s);
    double sum = 0.0;
    for (int64_t q = 0; q < nb; ++q) sum += h[q];
    return sum;
}

double host_blocked_norm(const double *d_v, int64_t n, double *d_part, HostPart &hp, hipError_t *e,
                         hipStream_t s = nullptr) {
    const int64_t nb = (n + kDotBlock - 1) / kDotBlock;
    if (nb > 0)
        hipLaunchKernelGGL(k_block_dot_wave<true>, dim3(blocks_for(nb, 4)), dim3(256), 0, s, n, d_v, d_v, d_part);
    double *h = hp.get(nb);
    *e = hipSuccess;
    if (nb > 0 && (*e = hipMemcpyAsync(h, d_part, sizeof(double) * (size_t)nb, hipMemcpyDeviceToHost, s)) == hipSuccess)
        *e = hipStreamSynchronize(s);
    double sum = 0.0;
    for (int64_t q = 0; q < nb; ++q) sum += h[q];
    return std::sqrt(sum);
}

// Pinned host staging for the strength graph and the aggregates, grown as
// needed and reused across levels and set-ups (measured at 300^3: level-0
// strength phase 0.14 s pinned vs 0.22 s through pageable copies, allocation
// included; the 0.86 GB allocation alone is 35 ms, paid once per process).
struct Staging {
    void *p = nullptr;
    size_t bytes = 0;
    hipError_t reserve(size_t b) {
        if (b <= bytes) return hipSuccess;
        if (p) hipHostFree(p);
        p = nullptr;
        bytes = 0;
        const hipError_t e = hipHostMalloc(&p, b);
        if (e == hipSuccess) bytes = b;
        return e;
    }
    int32_t *i32() { return static_cast<int32_t *>(p); }
};

// One per process, never freed (static destructors may run after the HIP
// runtime is gone); set-ups take turns on it.
Staging &process_staging(std::unique_lock<std::mutex> &lock) {
    static std::mutex mu;
    static Staging *st = new Staging();
    lock = std::unique_lock<std::mutex>(mu);
    return *st;
}

DCsr view_of(const aijhip_mat &A) {
    DCsr v;
    v.m = A.m;
    v.n = A.n;
    v.nz = A.nz;
    v.ai = A.d_ai;
    v.aj = A.d_aj;
    v.aa = A.d_aa;
    return v;
}

// The power iteration for emax(D^-1 A) (10 steps from a fixed start, norms
// summed on the host in 256-entry blocks: the host builder's order) on a
// host thread of its own.
// cg: CG's Lanczos estimate instead (gamg_setup.cpp estimate_emax_cg: the
// same start, A p in PETSc's row order, the same blocked dots, the
// tridiagonal's emax by the host's bisection).
// Both run on the set-up's stream slot 2 (a queue of its own beside the
// aggregation's kernels on the null stream), after `ready` (D^-1 written).
struct EmaxJob {
    std::thread th;
    double emax = 1.0;
    hipError_t e = hipSuccess;
    double *v = nullptr, *w = nullptr, *part = nullptr, *r = nullptr, *z = nullptr;
    double *h_pin = nullptr;  // pinned host partials
    hipStream_t js = nullptr;
    void start(const aijhip_mat &A, const double *dinv, int its, bool cg, hipEvent_t ready) {
        js = aijhip_gamg::setup_stream(A.device, 2);
        if (js && ready) e = hipStreamWaitEvent(js, ready, 0);
        if (cg) {
            th = std::thread([this, &A, dinv, its] {
                (void)hipSetDevice(A.device);
                const int32_t m = A.m;
                const unsigned g256 = blocks_for(m, 256);
                std::vector<double> alpha, beta;
                HostPart h_part;
                const int64_t nb = (m + kDotBlock - 1) / kDotBlock;
                if ((e = dalloc(&v, m)) != hipSuccess || (e = dalloc(&w, m)) != hipSuccess ||
                    (e = dalloc(&r, m)) != hipSuccess || (e = dalloc(&z, m)) != hipSuccess ||
                    (e = dalloc(&part, nb)) != hipSuccess)
                    return;
                if (hipHostMalloc(reinterpret_cast<void **>(&h_pin), sizeof(double) * (size_t)std::max<int64_t>(nb, 1)) ==
                    hipSuccess) {
                    h_part.pinned = h_pin;
                    h_part.cap = nb;
                }
                if (m == 0) return;
                double *p = v;
                hipLaunchKernelGGL(k_cgest_start, dim3(g256), dim3(256), 0, js, m, dinv, r, z, p);
                double rz = host_blocked_dot(z, r, m, part, h_part, &e, js);
                if (e != hipSuccess) return;
                for (int it = 0; it < its; ++it) {
                    if ((e = aijhip::launch_mult_exact(A, p, w, js)) != hipSuccess) return;
                    const double pw = host_blocked_dot(p, w, m, part, h_part, &e, js);
                    if (e != hipSuccess) return;
                    if (!(pw != 0.0 && rz != 0.0)) break;
                    const double a = rz / pw;
                    alpha.push_back(a);
                    hipLaunchKernelGGL(k_cgest_update, dim3(g256), dim3(256), 0, js, m, a, w, dinv, r, z);
                    const double rzn = host_blocked_dot(z, r, m, part, h_part, &e, js);
                    if (e != hipSuccess) return;
                    const double b = rzn / rz;
                    beta.push_back(b);
                    hipLaunchKernelGGL(k_cgest_dir, dim3(g256), dim3(256), 0, js, m, b, z, p);
                    rz = rzn;
                }
                e = hipStreamSynchronize(js);
                if (e == hipSuccess && !alpha.empty()) emax = aijhip_gamg::lanczos_emax(alpha, beta);
            });
            return;
        }
        th = std::thread([this, &A, dinv, its] {
            const bool log = std::getenv("AIJHIP_GAMG_LOG") != nullptr;
            auto c0 = std::chrono::steady_clock::now();
            auto mark = [&](const char *what) {
                if (!log) return;
                const auto now = std::chrono::steady_clock::now();
                std::fprintf(stderr, "  emax job %-12s %8.3f ms\n", what,
                             std::chrono::duration<double, std::milli>(now - c0).count());
                c0 = now;
            };
            (void)hipSetDevice(A.device);
            const int32_t m = A.m;
            const unsigned g256 = blocks_for(m, 256);
            HostPart h_part;
            const int64_t nb = (m + kDotBlock - 1) / kDotBlock;
            if ((e = dalloc(&v, m)) != hipSuccess || (e = dalloc(&w, m)) != hipSuccess ||
                (e = dalloc(&part, nb)) != hipSuccess)
                return;
            if (hipHostMalloc(reinterpret_cast<void **>(&h_pin), sizeof(double) * (size_t)std::max<int64_t>(nb, 1)) ==
                hipSuccess) {
                h_part.pinned = h_pin;
                h_part.cap = nb;
            }
            mark("alloc");
            hipLaunchKernelGGL(k_power_start, dim3(g256), dim3(256), 0, js, m, v);
            const double nv = host_blocked_norm(v, m, part, h_part, &e, js);
            if (e != hipSuccess) return;
            mark("start");
            hipLaunchKernelGGL(k_div, dim3(g256), dim3(256), 0, js, m, v, nv, v);
            for (int it = 0; it < its; ++it) {
                if ((e = aijhip::launch_dinv_mult(A, dinv, v, w, js)) != hipSuccess) return;
                const double nw = host_blocked_norm(w, m, part, h_part, &e, js);
                if (e != hipSuccess) return;
                if (it == 0) mark("iteration 0");
                if (!(nw > 0.0)) break;
                emax = nw;
                hipLaunchKernelGGL(k_div, dim3(g256), dim3(256), 0, js, m, w, nw, v);
            }
            e = hipStreamSynchronize(js);
            mark("iterations");
        });
    }
    void join() {
        if (th.joinable()) th.join();
    }
    void release() {
        hipFree(v); hipFree(w); hipFree(part); hipFree(r); hipFree(z);
        if (h_pin) (void)hipHostFree(h_pin);
        v = w = part = r = z = h_pin = nullptr;
    }
    ~EmaxJob() {
        join();
        release();
    }
};

// The level's handle adopts the set-up's device arrays (no copy, no host
// column check: they were made here).
int make_handle(int device, DCsr &C, aijhip_mat **out) {
    const int rc = aijhip::adopt_device_csr(device, C.m, C.n, C.nz, C.ai, C.aj, C.aa, nullptr, out);
    C.ai = C.aj = nullptr;  // owned by the handle now (or freed on failure)
    C.aa = nullptr;
    return rc;
}

// The interpolation handle of one level (P, with P^T attached for
// MatRestrict) made on a second host thread: its planning reads P's row
// offsets back to the host (27 M rows at 300^3, ~14 ms) and nothing before
// the V-cycle needs it, so it overlaps the next level's aggregation, whose
// phase 1 keeps the GPU idle on coarse levels. Joined before build_device
// returns.
struct HandleJob {
    std::thread th;
    size_t level = 0;
    int rc = AIJHIP_OK;
    std::string err;
    aijhip_mat *P = nullptr;
    void start(int device, size_t l, DCsr Pm, DCsr PTm) {
        level = l;
        th = std::thread([this, device, Pm, PTm]() mutable {
            (void)hipSetDevice(device);
            rc = make_handle(device, Pm, &P);
            if (!rc) rc = aijhip::attach_transpose(P, PTm.ai, PTm.aj, PTm.aa);  // consumes PT
            else PTm.release();
            if (rc) {
                err = aijhip_last_error();
                if (P) aijhip_mat_destroy(P);
                P = nullptr;
            }
        });
    }
    void join() {
        if (th.joinable()) th.join();
    }
    ~HandleJob() {
        join();
        if (P) aijhip_mat_destroy(P);
    }
};


// Which side runs aggregation phase 1 (both give the same aggregates): the
// device sweep for levels of at least 2^20 rows whose S averages at most 16
// strong neighbours (the sweep follows walks of length 2, ~deg^2 per node),
// with a round budget near the host pass's cost (a round ~ 10-20 us, the pass
// ~ 3 ns per node); AIJHIP_GAMG_AGG=host|device overrides (device: no round
// budget).
bool device_phase1(int32_t m, int64_t nzs, int32_t *max_rounds) {
    const char *f = std::getenv("AIJHIP_GAMG_AGG");
    if (f && std::string(f) == "host") return false;
    if (f && std::string(f) == "device") {
        *max_rounds = m + 2;
        return true;
    }
    *max_rounds = std::max<int32_t>(256, m / 8192);
    return m >= (1 << 20) && nzs <= 16 * (int64_t)m;
}

}  // namespace

namespace aijhip_gamg {

// Process-wide set-up streams, per device and slot (0: the phase-1 sweep,
// 1: the host pass's staging copies, 2: the emax job): created once, kept for the life of the
// process like the pinned staging (a first stream creation costs ~5 ms on the
// MI355X; set_pc_type(GAMG) makes them ahead of the set-up).
hipStream_t setup_stream(int device, int slot) {
    static std::mutex mu;
    static std::vector<hipStream_t> *cache = new std::vector<hipStream_t>();
    std::lock_guard<std::mutex> g(mu);
    const size_t k = (size_t)device * 3 + (size_t)std::min(std::max(slot, 0), 2);
    if (cache->size() <= k) cache->resize(k + 1, nullptr);
    if (!(*cache)[k]) {
        int cur = 0;
        (void)hipGetDevice(&cur);
        if (cur != device) (void)hipSetDevice(device);
        hipStream_t st = nullptr;
        if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) == hipSuccess) (*cache)[k] = st;
        if (cur != device) (void)hipSetDevice(cur);
    }
    return (*cache)[k];
}

void free_device_levels(std::vector<DeviceLevel> &levels) {
    for (size_t l = 0; l < levels.size(); ++l) {
        if (l > 0) aijhip_mat_destroy(levels[l].A);
        aijhip_mat_destroy(levels[l].P);
    }
    levels.clear();
}

// Diagonal, strength graph and aggregates of one level (the first half of a
// coarsening; build_device's and the distributed set-up's). With emax_its >
// 0 the power iteration for emax(D^-1 A) runs on a second host thread
// meanwhile (*emax on return).
int aggregate_level(aijhip_mat &A, const aijhip_gamg_params_t &p, int32_t **d_agg_out, int32_t *na_out,
                    double **dinv_out, int emax_its, double *emax, hipError_t *emax_err, size_t level,
                    StrengthGraph *keep_S) {
    *d_agg_out = nullptr;
    *dinv_out = nullptr;
    *na_out = 0;
    const int32_t m = A.m;
    const int n_cu = std::max(A.n_cu, 1);
    const bool log = std::getenv("AIJHIP_GAMG_LOG") != nullptr;
    auto t0 = std::chrono::steady_clock::now();
    auto lap = [&](const char *what) {
        if (!log) return;
        (void)hipDeviceSynchronize();
        const auto t = std::chrono::steady_clock::now();
        std::fprintf(stderr, "gamg device level %zu %-14s %8.3f s\n", level, what,
                     std::chrono::duration<double>(t - t0).count());
        t0 = t;
    };
    std::unique_lock<std::mutex> stage_lock;  // taken by the host pass only
    int rc = AIJHIP_OK;
    hipError_t e = hipSuccess;
    const unsigned g256 = blocks_for(m, 256);
    double *d = nullptr, *dinv = nullptr, *sval = nullptr;
    unsigned long long *cnt = nullptr, *off = nullptr;
    unsigned int *pos = nullptr;
    int32_t *tmp = nullptr, *si = nullptr, *sj = nullptr;
    unsigned long long *scan_tmp = nullptr;
    int64_t nzs = 0;
    int32_t *h_si = nullptr, *agg = nullptr, *d_ph = nullptr, *d_head = nullptr;
    int32_t *d_aggv = nullptr;  // the aggregates (device), handed to the prolongator
    unsigned long long *d_left = nullptr;
    int32_t na = 0;
    bool dev_agg = false;  // phase 1 ran on the device (else the host pass)
    int32_t sweep_rounds = 0;
    // emax(D^-1 A) needs only A: its power iteration runs from a second
    // host thread while this one stages S and aggregates on the CPU
    EmaxJob job;
    hipEvent_t ev_dinv = nullptr;
#define GTRY(call, what) do { if ((e = (call)) != hipSuccess) { rc = herr(e, what); goto level_done; } } while (0)
    GTRY(dalloc(&d, m), "alloc");
    GTRY(dalloc(&dinv, m), "alloc");
    hipLaunchKernelGGL(k_diag_dinv, dim3(g256), dim3(256), 0, nullptr, m, A.d_ai, A.d_aj, A.d_aa, d, dinv);
    // the emax job starts as soon as D^-1 is queued: it overlaps the strength
    // graph as well as the aggregation (round 5: started after the strength
    // graph, the level-0 CG estimate still held the level ~8 ms past the MIS)
    if (emax_its > 0) {  // (D^-1 is written on the null stream: the job's stream waits for it)
        if (hipEventCreateWithFlags(&ev_dinv, hipEventDisableTiming) != hipSuccess ||
            hipEventRecord(ev_dinv, nullptr) != hipSuccess) {
            if (ev_dinv) (void)hipEventDestroy(ev_dinv);
            ev_dinv = nullptr;
            GTRY(hipDeviceSynchronize(), "D^-1");
        }
        job.start(A, dinv, emax_its, p.eig_ksp == 1, ev_dinv);
    }
    {
        bool direct = false;  // S straight from A (sorted rows, symmetric strong pattern)
        if ((rc = strength_direct(A, d, p.threshold, &si, &sj, &sval, &nzs, &direct))) goto level_done;
        if (log)
            std::fprintf(stderr, "gamg device level %zu strength graph: %s\n", level,
                         direct ? "direct (symmetric)" : "gathered (S u S^T)");
        if (direct) goto strength_done;
    }
    GTRY(dalloc(&cnt, (int64_t)m + 1), "alloc");
    GTRY(dalloc(&off, (int64_t)m + 1), "alloc");
    GTRY(hipMemset(cnt, 0, sizeof(unsigned long long) * ((size_t)m + 1)), "memset");
    hipLaunchKernelGGL(k_strong_count, dim3(g256), dim3(256), 0, nullptr, m, A.d_ai, A.d_aj, A.d_aa, d,
                       p.threshold, cnt);
    GTRY(dalloc(&scan_tmp, aijhip_dscan::scan_tmp_elems((int64_t)m + 1)), "alloc");
    GTRY(aijhip_dscan::exclusive_scan(cnt, off, (int64_t)m + 1, scan_tmp, nullptr), "scan");
    {
        unsigned long long t = 0;
        GTRY(hipMemcpy(&t, off + m, sizeof(t), hipMemcpyDeviceToHost), "read");
        nzs = (int64_t)t;
    }
    GTRY(dalloc(&tmp, nzs), "alloc");
    GTRY(dalloc(&pos, m), "alloc");
    GTRY(hipMemset(pos, 0, sizeof(unsigned int) * (size_t)std::max(m, 1)), "memset");
    hipLaunchKernelGGL(k_strong_fill, dim3(g256), dim3(256), 0, nullptr, m, A.d_ai, A.d_aj, A.d_aa, d,
                       p.threshold, off, pos, tmp);
    if ((rc = strength_lists(A, cnt, off, tmp, nzs, n_cu, &si, &sj, &sval, &nzs))) goto level_done;
strength_done:
    GTRY(hipGetLastError(), "strength kernels");
    if (keep_S) {  // the distributed MIS aggregates across ranks itself (gamg_mpi.hip)
        keep_S->si = si;
        keep_S->sj = sj;
        keep_S->nz = nzs;
        keep_S->d = d;
        si = sj = nullptr;
        d = nullptr;
        goto level_done;
    }
    // ---- aggregation. Phase 1: the device sweep (gamg_aggregate.hip) on
    // large levels with a sparse S, else -- or when the sweep would run too
    // deep -- the sequential pass on the host from S staged in pinned
    // memory; the same aggregates either way. Phase 2 on the device; phase
    // 3 (sequential) over the nodes left.
    lap("strength kernels");
    GTRY(dalloc(&d_aggv, m), "alloc");
    if (p.coarsen == 1) {  // PETSc 3.7 agg's MIS (gamg_aggregate.hip), node for node the host's
        int32_t rounds = 0;
        GTRY(aijhip_gamg::aggregate_mis_device(m, si, sj, (int32_t)level < p.square_graph, (int32_t)level, d_aggv,
                                               &na, &rounds),
             "MIS aggregation");
        if (log)
            std::fprintf(stderr, "gamg device level %zu MIS%s: %d rounds, %d aggregates\n", level,
                         (int32_t)level < p.square_graph ? " (squared graph)" : "", rounds, na);
        lap("aggregate");
        goto level_done;
    }
    GTRY(dalloc(&d_ph, m), "alloc");
    GTRY(dalloc(&d_left, 1), "alloc");
    {
        int32_t max_rounds = 0;
        if (device_phase1(m, nzs, &max_rounds)) {
            GTRY(aijhip_gamg::aggregate_phase1_device(m, si, sj, max_rounds, d_ph, &na, &sweep_rounds, &dev_agg),
                 "phase 1 sweep");
            if (log)
                std::fprintf(stderr, "gamg device level %zu phase 1 sweep: %d rounds%s\n", level, sweep_rounds,
                             dev_agg ? "" : " (too deep: host pass)");
        }
    }
    if (!dev_agg) {
        // S's columns come down in row chunks through two pinned slots while
        // the pass works through the rows already here (a node reads only its
        // own row of S; the aggregate ids of all). Pinned: the row offsets,
        // the ids and the two slots (~50 MB at 300^3 level 1, where a whole
        // copy of S took 0.37 GB and 20 ms to pin on first use). (Phase 1
        // measured on the MI355X host at 300^3 level 0: this int32 form
        // 83 ms; bitmap or byte flags with or without early exits 87-121 ms.)
        constexpr int kChunks = 32;
        int32_t r[kChunks + 1];
        for (int c = 0; c <= kChunks; ++c) r[c] = (int32_t)((int64_t)m * c / kChunks);
        int32_t *h_off = nullptr;
        GTRY(hipHostMalloc(reinterpret_cast<void **>(&h_off), sizeof(int32_t) * (kChunks + 1)), "pinned offsets");
        for (int c = 0; c <= kChunks && e == hipSuccess; ++c)
            e = hipMemcpyAsync(h_off + c, si + r[c], sizeof(int32_t), hipMemcpyDeviceToHost, nullptr);
        if (e == hipSuccess) e = hipStreamSynchronize(nullptr);
        int64_t slot = 0;
        for (int c = 0; c < kChunks; ++c) slot = std::max<int64_t>(slot, (int64_t)h_off[c + 1] - h_off[c]);
        (void)hipHostFree(h_off);
        GTRY(e, "read S offsets");
        constexpr int H = aijhip_gamg::kPhase1Head;
        GTRY(dalloc(&d_head, (int64_t)m * H), "alloc");
        hipLaunchKernelGGL(k_phase1_head, dim3(blocks_for((int64_t)m * H, 256)), dim3(256), 0, nullptr, m, si, sj,
                           d_head);
        Staging &stage = process_staging(stage_lock);
        GTRY(stage.reserve(sizeof(int32_t) * ((2 + (size_t)H) * (size_t)m + 1 + 2 * (size_t)slot)), "pinned staging");
        lap("staging alloc");
        h_si = stage.i32();
        agg = h_si + m + 1;
        int32_t *h_head = agg + m;
        int32_t *h_slot[2] = {h_head + (size_t)H * m, h_head + (size_t)H * m + slot};
        GTRY(hipMemcpy(h_si, si, sizeof(int32_t) * ((size_t)m + 1), hipMemcpyDeviceToHost), "read S");
        lap("strength");
        {
            hipEvent_t ev[2] = {};
            hipStream_t cs = setup_stream(A.device, 1);
            if (!cs) GTRY(hipErrorOutOfMemory, "stream");
            auto fetch = [&](int c) {  // chunk c into slot c % 2 (its rows' heads first)
                const int64_t a = h_si[r[c]], b = h_si[r[c + 1]];
                hipError_t x = hipSuccess;
                if (r[c + 1] > r[c])
                    x = hipMemcpyAsync(h_head + (size_t)H * r[c], d_head + (size_t)H * r[c],
                                       sizeof(int32_t) * H * (size_t)(r[c + 1] - r[c]), hipMemcpyDeviceToHost, cs);
                if (x == hipSuccess && b > a)
                    x = hipMemcpyAsync(h_slot[c & 1], sj + a, sizeof(int32_t) * (size_t)(b - a),
                                       hipMemcpyDeviceToHost, cs);
                if (x == hipSuccess) x = hipEventRecord(ev[c & 1], cs);
                return x;
            };
            for (int z = 0; z < 2 && e == hipSuccess; ++z) e = hipEventCreateWithFlags(&ev[z], hipEventDisableTiming);
            for (int c = 0; c < 2 && c < kChunks && e == hipSuccess; ++c) e = fetch(c);
            std::fill(agg, agg + m, -1);
            std::vector<uint64_t> taken(((size_t)m + 63) / 64, 0);
            na = 0;
            double t_wait = 0.0, t_pass = 0.0;  // (logged: copy-bound or pass-bound)
            for (int c = 0; c < kChunks && e == hipSuccess; ++c) {
                const auto w0 = std::chrono::steady_clock::now();
                if ((e = hipEventSynchronize(ev[c & 1])) != hipSuccess) break;
                const auto w1 = std::chrono::steady_clock::now();
                na = aijhip_gamg::aggregate_phase1_rows(r[c], r[c + 1], h_si, h_slot[c & 1], agg, taken.data(), na,
                                                        h_si[r[c]], h_head);
                if (c + 2 < kChunks) e = fetch(c + 2);
                t_wait += std::chrono::duration<double, std::milli>(w1 - w0).count();
                t_pass += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - w1).count();
            }
            if (log)
                std::fprintf(stderr, "gamg device level %zu host phase 1: %.1f MB of S, waits %.2f ms, pass %.2f ms\n",
                             level, 4e-6 * (double)nzs, t_wait, t_pass);
            (void)hipStreamSynchronize(cs);
            for (hipEvent_t x : ev)
                if (x) (void)hipEventDestroy(x);
            GTRY(e, "read S");
        }
        GTRY(hipMemcpy(d_ph, agg, sizeof(int32_t) * (size_t)m, hipMemcpyHostToDevice), "upload phase 1");
    }
    lap("phase 1");
    hipLaunchKernelGGL(k_agg_phase2, dim3(g256), dim3(256), 0, nullptr, m, si, sj, sval, d_ph, d_aggv);
    GTRY(hipMemset(d_left, 0, sizeof(unsigned long long)), "memset");
    hipLaunchKernelGGL(k_count_value, dim3(g256), dim3(256), 0, nullptr, m, d_aggv, -1, d_left);
    {
        unsigned long long left = 0;
        GTRY(hipMemcpy(&left, d_left, sizeof(left), hipMemcpyDeviceToHost), "read phase 2");
        lap("phase 2");
        if (left > 0)  // phase 3 over the left-over nodes' rows only (the host pass's order)
            GTRY(aijhip_gamg::aggregate_phase3_device(m, si, sj, d_aggv, &na), "phase 3");
    }
    lap("aggregate");
level_done:
#undef GTRY
    job.join();
    if (ev_dinv) (void)hipEventDestroy(ev_dinv);
    lap("emax joined");
    hipFree(cnt); hipFree(off); hipFree(pos); hipFree(tmp); hipFree(si); hipFree(sj);
    hipFree(sval); hipFree(scan_tmp); hipFree(d); hipFree(d_ph); hipFree(d_left); hipFree(d_head);
    lap("freed");
    if (emax_its > 0) {
        *emax = job.emax;
        if (emax_err) *emax_err = job.e;
    }
    job.release();
    if (rc) {
        hipFree(dinv);
        hipFree(d_aggv);
        return rc;
    }
    *d_agg_out = d_aggv;
    *dinv_out = dinv;
    *na_out = na;
    return AIJHIP_OK;
}

// The tentative prolongator (near-null space B normalised per aggregate:
// Bc = the next level's B, p0) and the smoothed P = P0 + alpha D^-1 (A P0)
// with local columns (agg ids). d_p0 (m) and d_Bc (na) are returned for the
// caller to free; P owns its arrays.
int smooth_level(const DCsr &Av, int32_t na, int32_t *d_agg, const double *d_B, const double *dinv, double alpha,
                 int nsmooths, int n_cu, double **d_p0_out, double **d_Bc_out, DCsr &P, int *cols_used,
                 bool b_ones) {
    const int32_t m = Av.m;
    const unsigned g256 = blocks_for(m, 256);
    int rc = AIJHIP_OK;
    hipError_t e = hipSuccess;
    double *d_p0 = nullptr, *d_Bc = nullptr;
    int32_t *plen = nullptr;
    DCsr P0, T;
    bool p0_own = false;  // P0's aj / aa compacted copies (MIS singletons) rather than d_agg / d_p0
    const bool log = std::getenv("AIJHIP_GAMG_LOG") != nullptr;
    auto t0 = std::chrono::steady_clock::now();
    auto lap = [&](const char *what) {
        if (!log) return;
        (void)hipDeviceSynchronize();
        const auto t = std::chrono::steady_clock::now();
        std::fprintf(stderr, "  smooth %-12s %8.3f ms\n", what, std::chrono::duration<double, std::milli>(t - t0).count());
        t0 = t;
    };
#define GTRY(call, what) do { if ((e = (call)) != hipSuccess) { rc = herr(e, what); goto done; } } while (0)
    GTRY(dalloc(&d_p0, m), "alloc");
    GTRY(dalloc(&d_Bc, na), "alloc");
    GTRY(tentative(m, na, d_agg, d_B, d_Bc, d_p0, b_ones), "tentative prolongator");
    lap("tentative");
    GTRY(p0_csr(m, na, d_agg, d_p0, P0, &p0_own), "tentative prolongator");
    if (nsmooths > 0) {
        if ((rc = rowprod_p0(Av, P0, d_agg, d_p0, T, n_cu, cols_used))) goto done;
        lap("A*P0");
        P.m = m;
        P.n = na;
        GTRY(dalloc(&plen, m), "alloc");
        hipLaunchKernelGGL(k_prolong_len, dim3(g256), dim3(256), 0, nullptr, m, T.ai, T.aj, d_agg, plen);
        GTRY(dalloc(&P.ai, (int64_t)m + 1), "alloc");
        GTRY(scan_offsets(plen, m, P.ai, &P.nz), "scan");
        GTRY(dalloc(&P.aj, P.nz + 2), "alloc");
        GTRY(dalloc(&P.aa, P.nz + 2), "alloc");
        hipLaunchKernelGGL(k_prolong_fill, dim3(g256), dim3(256), 0, nullptr, m, T.ai, T.aj, T.aa, d_agg, d_p0,
                           dinv, alpha, P.ai, P.aj, P.aa);
        GTRY(hipGetLastError(), "prolongator");
        lap("P fill");
    } else {
        P.m = m;
        P.n = na;
        P.nz = P0.nz;
        GTRY(dalloc(&P.ai, (int64_t)m + 1), "alloc");
        GTRY(dalloc(&P.aj, P0.nz + 2), "alloc");
        GTRY(dalloc(&P.aa, P0.nz + 2), "alloc");
        GTRY(hipMemcpy(P.ai, P0.ai, sizeof(int32_t) * ((size_t)m + 1), hipMemcpyDeviceToDevice), "copy");
        GTRY(hipMemcpy(P.aj, P0.aj, sizeof(int32_t) * (size_t)P0.nz, hipMemcpyDeviceToDevice), "copy");
        GTRY(hipMemcpy(P.aa, P0.aa, sizeof(double) * (size_t)P0.nz, hipMemcpyDeviceToDevice), "copy");
    }
done:
#undef GTRY
    hipFree(P0.ai);
    if (p0_own) {
        hipFree(P0.aj);
        hipFree(P0.aa);
    }
    hipFree(plen);
    T.release();
    lap("freed");
    if (rc) {
        P.release();
        hipFree(d_p0);
        hipFree(d_Bc);
        return rc;
    }
    *d_p0_out = d_p0;
    *d_Bc_out = d_Bc;
    return AIJHIP_OK;
}

// The Galerkin operator A_c = P^T (A P) of local blocks (PT = P^T returned:
// the MatRestrict operator); AP is released unless ap_out is given.
int galerkin_level(const DCsr &Av, const DCsr &P, DCsr &PT, DCsr &Ac, int n_cu, int *cols_used, DCsr *ap_out) {
    const bool log = std::getenv("AIJHIP_GAMG_LOG") != nullptr;
    auto t0 = std::chrono::steady_clock::now();
    auto lap = [&](const char *what) {
        if (!log) return;
        (void)hipDeviceSynchronize();
        const auto t = std::chrono::steady_clock::now();
        std::fprintf(stderr, "  galerkin %-12s %8.3f ms\n", what, std::chrono::duration<double, std::milli>(t - t0).count());
        t0 = t;
    };
    DCsr AP;
    int rc = rowprod(Av, P, AP, n_cu, cols_used);
    lap("A*P");
    if (rc) return rc;
    {
        aijhip_mat pv;  // non-owning view for the transpose builder
        pv.m = P.m;
        pv.n = P.n;
        pv.nz = P.nz;
        pv.d_ai = P.ai;
        pv.d_aj = P.aj;
        pv.d_aa = P.aa;
        PT.m = P.n;
        PT.n = P.m;
        PT.nz = P.nz;
        const hipError_t e = aijhip::build_transpose(pv, &PT.ai, &PT.aj, &PT.aa, nullptr);
        pv.d_ai = pv.d_aj = nullptr;
        pv.d_aa = nullptr;
        lap("P^T");
        if (e != hipSuccess) {
            AP.release();
            return herr(e, "transpose");
        }
    }
    if ((rc = rowprod(PT, AP, Ac, n_cu, cols_used))) {
        AP.release();
        PT.release();
        return rc;
    }
    lap("P^T*(AP)");
    if (ap_out) *ap_out = AP;
    else AP.release();
    lap("released");
    return AIJHIP_OK;
}

int make_level_handle(int device, DCsr &C, aijhip_mat **out) { return make_handle(device, C, out); }

int rowprod_device(const DCsr &A, const DCsr &B, DCsr &C, int n_cu, int *cols_used) {
    return rowprod(A, B, C, n_cu, cols_used);
}

hipError_t tentative_device(int32_t m, int32_t na, const int32_t *agg, const double *B, double *Bc, double *p0,
                            bool b_ones) {
    return tentative(m, na, agg, B, Bc, p0, b_ones);
}

hipError_t aggregate_sumsq_device(int32_t m, int32_t na, const int32_t *agg, const double *B, double *s2,
                                  bool b_ones) {
    return tentative(m, na, agg, B, s2, nullptr, b_ones, true);
}

int prolong_from_T(const DCsr &T, const int32_t *d_agg, const double *d_p0, const double *dinv, double alpha,
                   DCsr &P) {
    const int32_t m = T.m;
    const unsigned g256 = blocks_for(m, 256);
    int32_t *plen = nullptr;
    hipError_t e;
    P = DCsr();
    P.m = m;
    P.n = T.n;
    if ((e = dalloc(&plen, m)) != hipSuccess) return herr(e, "alloc");
    if (m > 0) hipLaunchKernelGGL(k_prolong_len, dim3(g256), dim3(256), 0, nullptr, m, T.ai, T.aj, d_agg, plen);
    if ((e = dalloc(&P.ai, (int64_t)m + 1)) != hipSuccess || (e = scan_offsets(plen, m, P.ai, &P.nz)) != hipSuccess ||
        (e = dalloc(&P.aj, P.nz + 2)) != hipSuccess || (e = dalloc(&P.aa, P.nz + 2)) != hipSuccess) {
        hipFree(plen);
        P.release();
        return herr(e, "prolongator");
    }
    if (m > 0)
        hipLaunchKernelGGL(k_prolong_fill, dim3(g256), dim3(256), 0, nullptr, m, T.ai, T.aj, T.aa, d_agg, d_p0, dinv,
                           alpha, P.ai, P.aj, P.aa);
    e = hipGetLastError();
    hipFree(plen);
    if (e != hipSuccess) {
        P.release();
        return herr(e, "prolongator");
    }
    return AIJHIP_OK;
}

int build_device(aijhip_mat *A0, const aijhip_gamg_params_t &p, std::vector<DeviceLevel> &levels,
                 std::vector<double> &B, bool *more, bool *overflow) {
    levels.clear();
    *more = false;
    if (overflow) *overflow = false;
    const bool log = std::getenv("AIJHIP_GAMG_LOG") != nullptr;
    auto t0 = std::chrono::steady_clock::now();
    auto lap = [&](const char *what) {
        if (!log) return;
        (void)hipDeviceSynchronize();
        const auto t = std::chrono::steady_clock::now();
        std::fprintf(stderr, "gamg device level %zu %-14s %8.3f s\n", levels.size() - 1, what,
                     std::chrono::duration<double>(t - t0).count());
        t0 = t;
    };
    levels.push_back(DeviceLevel{A0, nullptr, 0.0});
    const int n_cu = std::max(A0->n_cu, 1);
    int rc = AIJHIP_OK;
    hipError_t e = hipSuccess;
    constexpr bool in_line = false;  // (in line measured ~14 ms slower at 300^3)
    std::vector<std::unique_ptr<HandleJob>> jobs;
    // the near-null space of the current level, on the device; the finest
    // level's (all ones) is implicit — nullptr, read as 1.0 by k_tentative —
    // which spares a first set-up a 216 MB allocation and fill at 300^3 (5 ms)
    double *d_B = nullptr;
    // A finest level the device sweep aggregates leaves the first host pass
    // to level 1: its pinned staging (S row chunks and ids and row heads,
    // ~31 B per level-1 row, ~4 B per finest row at aggregates of ~8) is reserved on a host
    // thread meanwhile (6 ms of pinning at 300^3 on a first set-up)
    std::thread prestage;
    {
        int32_t rounds = 0;
        if (p.coarsen == 0 && A0->m >= p.device_min_rows && device_phase1(A0->m, A0->nz - A0->m, &rounds))
            prestage = std::thread([bytes = (size_t)A0->m * 9 / 2, device = A0->device] {
                (void)hipSetDevice(device);
                std::unique_lock<std::mutex> lock;
                (void)process_staging(lock).reserve(bytes);
            });
    }
    struct Joiner {
        std::thread &t;
        ~Joiner() { if (t.joinable()) t.join(); }
    } prestage_join{prestage};
    lap("first kernel");
    while ((int32_t)levels.size() < p.max_levels && levels.back().A->m > p.coarse_eq_limit) {
        aijhip_mat &A = *levels.back().A;
        const int32_t m = A.m;
        aijhip::Range range("PCGAMG device level");
        // the device while the level has device_min_rows rows or 25 x as many
        // entries (PETSc's MIS hierarchy reaches a few thousand rows of ~200
        // entries: 82 ms of host set-up at 300^3 against ~15 on the device)
        if ((m < p.device_min_rows && A.nz < 25 * (int64_t)p.device_min_rows) || !aijhip::stream_mg_fusable(A)) {
            *more = true;  // the host takes it from here
            break;
        }
        int32_t *d_agg = nullptr, na = 0;
        double *dinv = nullptr, emax = 1.0;
        hipError_t emax_err = hipSuccess;
        rc = aggregate_level(A, p, &d_agg, &na, &dinv, p.nsmooths > 0 ? p.eig_its : 0, &emax, &emax_err,
                             levels.size() - 1);
        if (rc || na >= m || na == 0) {  // an error, or no coarsening: this is the coarsest level
            hipFree(dinv);
            hipFree(d_agg);
            break;
        }
        if (emax_err != hipSuccess) {
            hipFree(dinv);
            hipFree(d_agg);
            rc = herr(emax_err, "power iteration");
            break;
        }
        lap("emax");
        int cols_used = 0;
        const DCsr Av = view_of(A);
        DCsr P, PT, Ac;
        double *d_p0 = nullptr, *d_Bc = nullptr;
        aijhip_mat *Ph = nullptr, *Ach = nullptr;
        // ---- tentative + smoothed prolongator
        rc = smooth_level(Av, na, d_agg, d_B, dinv, -p.smooth_scale / emax, p.nsmooths, n_cu, &d_p0, &d_Bc, P,
                          &cols_used, levels.size() == 1);
        lap("prolongator");
        // ---- Galerkin operator A_c = P^T (A P)
        if (!rc) rc = galerkin_level(Av, P, PT, Ac, n_cu, &cols_used, nullptr);
        lap("P^T*(AP)");
        // ---- handles: P (with P^T attached for MatRestrict) and A_c
        if (!rc && !in_line) {
            jobs.emplace_back(new HandleJob());
            jobs.back()->start(A.device, levels.size() - 1, P, PT);
            P = DCsr();  // owned by the job now
            PT = DCsr();
        }
        if (!rc && in_line) rc = make_handle(A.device, P, &Ph);
        if (!rc && in_line) {
            rc = aijhip::attach_transpose(Ph, PT.ai, PT.aj, PT.aa);
            PT = DCsr();  // consumed by attach_transpose (freed on failure)
        }
        if (!rc) rc = make_handle(A.device, Ac, &Ach);
        if (!rc) {
            levels.back().P = Ph;
            levels.back().emax = emax;
            levels.back().product_cols = cols_used;
            Ph = nullptr;
            levels.push_back(DeviceLevel{Ach, nullptr, 0.0});
            Ach = nullptr;
            std::swap(d_B, d_Bc);
            lap("handles");
        }
        hipFree(dinv); hipFree(d_agg); hipFree(d_p0); hipFree(d_Bc);
        P.release(); PT.release(); Ac.release();
        if (Ph) aijhip_mat_destroy(Ph);
        if (Ach) aijhip_mat_destroy(Ach);
        if (rc == AIJHIP_ERR_STATE) {  // a row past the device accumulators
            rc = AIJHIP_OK;
            *more = true;
            if (overflow) *overflow = true;
            break;
        }
        if (rc) break;
    }
    for (auto &j : jobs) {  // the interpolation handles made meanwhile
        j->join();
        if (j->rc) {
            if (!rc) {
                rc = j->rc;
                set_error(j->err);
            }
            continue;
        }
        levels[j->level].P = j->P;
        j->P = nullptr;
    }
    jobs.clear();
    lap("P handles");
    if (!rc) {  // the coarsest device level's near-null space, for the host levels
        B.resize((size_t)levels.back().A->m);
        if (!d_B) std::fill(B.begin(), B.end(), 1.0);  // (no level made: still the implicit ones)
        else if (!B.empty() &&
                 (e = hipMemcpy(B.data(), d_B, sizeof(double) * B.size(), hipMemcpyDeviceToHost)) != hipSuccess)
            rc = herr(e, "read near-null space");
    }
    hipFree(d_B);
    if (rc) free_device_levels(levels);
    return rc;
}

}  // namespace aijhip_gamg
