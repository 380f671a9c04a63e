// gamg_aggregate.hip — phases 1 and 3 of the greedy aggregation
// (gamg_setup.cpp aggregate) on the device, with the same result as the
// sequential passes, node for node.
//
// Phase 1 walks the nodes in natural order and roots an aggregate at a free
// node whose strong neighbours are all free; the root takes them. A node is
// free at its turn exactly when no earlier root lies within two steps of it
// in S (a root at distance 1 took it, one at distance 2 took a neighbour), so
// the roots are the lexicographically-first distance-2 independent set of
// the nodes with strong neighbours, and that set is unique: node i is a root
// iff every lower node within two steps of it is not. That rule runs in
// parallel as an event-driven sweep (a topological order on the "lower
// node within two steps" relation):
//   cnt[i]  = the number of walks of length 1 and 2 from i to lower nodes;
//   a root marks every higher node within two steps OUT (compare-and-swap:
//           the first root to reach it wins; all that matters is that it is
//           OUT);
//   an OUT node takes one off cnt[k] for every walk to a higher, still
//           undecided k; the walk that brings cnt[k] to 0 makes k a root
//           (all its lower neighbours are decided and none is a root: a
//           root never decrements, so a node next to one never gets to 0).
// Decisions are final, so the order in which concurrent lanes act cannot
// change the outcome. Each round is one launch (k_lf_round: OUT nodes count
// down, and each new root is marked by the workgroup that made it); the
// rounds needed grow with the longest chain of roots the natural order
// forces (about 2.35 N on an N^3 grid: 704 at 300^3). Deep chains (a path
// graph needs m / 3 rounds) are handed back to the host pass past a round
// budget. A workgroup gathers its list appends in LDS and combines its
// count-downs per node in an LDS hash table, so the global atomics are one
// per workgroup and pass on the list tails and one per distinct node on the
// counts (the middle rounds, whose frontiers are the largest, are where the
// time goes).
// Aggregate numbers follow the roots' index order (a scan), as the host's
// counter does.
//
// Phase 3 (the few nodes phases 1 and 2 leave) stays the host's sequential
// pass, over those nodes and their S rows only, gathered on the device.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "dscan.h"
#include "gamg_device.h"

namespace {

constexpr int32_t kUndecided = 0, kRoot = 1, kOut = 2;
constexpr unsigned kRoundGrid = 2048;  // workgroups of 256 lanes per round launch (512: 10 % slower)

inline unsigned blocks_for(int64_t n, int t) { return (unsigned)std::max<int64_t>(1, (n + t - 1) / t); }

// f(k) for every walk i -> j (k = j) and i -> j -> k (k != i) in S
template <class F>
__device__ __forceinline__ void for_walks(int32_t i, const int32_t *__restrict__ si, const int32_t *__restrict__ sj,
                                          F f) {
    const int32_t a1 = si[i + 1];
    for (int32_t a = si[i]; a < a1; ++a) {
        const int32_t j = sj[a];
        f(j);
        const int32_t b1 = si[j + 1];
        for (int32_t b = si[j]; b < b1; ++b) {
            const int32_t k = sj[b];
            if (k != i) f(k);
        }
    }
}

__global__ void k_lf_init(int32_t m, const int32_t *__restrict__ si, const int32_t *__restrict__ sj, int32_t *state,
                          int32_t *cnt) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    if (si[i] == si[i + 1]) {  // no strong neighbour: never a root, in nobody's walks
        state[i] = kOut;
        cnt[i] = 0;
        return;
    }
    int32_t c = 0;
    for_walks(i, si, sj, [&](int32_t k) { c += k < i; });
    state[i] = kUndecided;
    cnt[i] = c;
}

// round 0's roots: undecided nodes with no lower node within two steps
__global__ void k_lf_seed(int32_t m, int32_t *state, const int32_t *__restrict__ cnt, int32_t *roots,
                          unsigned *tails) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m || state[i] != kUndecided || cnt[i] != 0) return;
    state[i] = kRoot;
    roots[atomicAdd(&tails[0], 1u)] = i;
}

constexpr int kGroup = 8;   // lanes per frontier node: its strong neighbours split over them
constexpr int kBatch2 = 8;  // second-step nodes loaded together before acting on them

// A workgroup's appends gather in LDS and go to the global list with one
// atomic on its tail per workgroup and pass (the tails are single counters
// every workgroup of a round appends to; per-lane or per-wavefront atomics on
// them serialise the middle rounds, whose frontiers are the largest).
constexpr int kWgBuf = 2048;
struct WgList {
    int32_t v[kWgBuf];
    unsigned n, base;
};

// Append k[u] for every (lane, u) with p[u] set: one LDS atomic per
// wavefront and batch; past the buffer, straight to the global list.
__device__ __forceinline__ void wg_add(WgList &L, const bool (&p)[kBatch2], const int32_t (&k)[kBatch2],
                                       int32_t *list, unsigned *tail) {
    unsigned long long mask[kBatch2];
    unsigned total = 0;
#pragma unroll
    for (int u = 0; u < kBatch2; ++u) {
        mask[u] = __ballot(p[u]);
        total += (unsigned)__popcll(mask[u]);
    }
    if (total == 0) return;
    const int lane = threadIdx.x & 63;
    const unsigned long long below = (1ull << lane) - 1ull;
    unsigned long long any = 0;
#pragma unroll
    for (int u = 0; u < kBatch2; ++u) any |= mask[u];
    const int leader = __ffsll(any) - 1;
    unsigned pos = 0;
    if (lane == leader) pos = atomicAdd(&L.n, total);
    pos = (unsigned)__shfl((int)pos, leader, 64);
#pragma unroll
    for (int u = 0; u < kBatch2; ++u) {
        if (p[u]) {
            const unsigned idx = pos + (unsigned)__popcll(mask[u] & below);
            if (idx < (unsigned)kWgBuf) L.v[idx] = k[u];
            else list[atomicAdd(tail, 1u)] = k[u];
        }
        pos += (unsigned)__popcll(mask[u]);
    }
}

// Append k to list when p (one element per lane; every lane of the
// workgroup calls it at the same point).
__device__ __forceinline__ void wg_add1(WgList &L, bool p, int32_t k, int32_t *list, unsigned *tail) {
    const unsigned long long mask = __ballot(p);
    if (!mask) return;
    const int lane = threadIdx.x & 63;
    const int leader = __ffsll(mask) - 1;
    unsigned pos = 0;
    if (lane == leader) pos = atomicAdd(&L.n, (unsigned)__popcll(mask));
    pos = (unsigned)__shfl((int)pos, leader, 64);
    if (p) {
        const unsigned idx = pos + (unsigned)__popcll(mask & ((1ull << lane) - 1ull));
        if (idx < (unsigned)kWgBuf) L.v[idx] = k;
        else list[atomicAdd(tail, 1u)] = k;
    }
}

// A workgroup's count-downs of one pass, combined per node in an LDS hash
// table (open addressing, 8 probes) and applied with one global atomic per
// distinct node (the OUT nodes of a round share most of their higher
// neighbours): 35 -> 31 ms over the 704 rounds at 300^3.
constexpr int kHashBits = 11, kHash = 1 << kHashBits;
struct WgCounts {
    int32_t key[kHash];
    int32_t n[kHash];
};

__device__ __forceinline__ bool wg_count_add(WgCounts &H, int32_t k) {
    const uint32_t h = ((uint32_t)k * 0x9E3779B1u) >> (32 - kHashBits);
    for (int probe = 0; probe < 8; ++probe) {
        const uint32_t s = (h + (uint32_t)probe) & (kHash - 1);
        const int32_t prev = atomicCAS(&H.key[s], -1, k);
        if (prev == -1 || prev == k) {
            atomicAdd(&H.n[s], 1);
            return true;
        }
    }
    return false;  // the caller counts down in global memory directly
}

// Workgroup-uniform: the buffered appends to list[tail ...), coalesced.
__device__ __forceinline__ void wg_flush(WgList &L, int32_t *list, unsigned *tail) {
    __syncthreads();
    const unsigned n = min(L.n, (unsigned)kWgBuf);
    if (threadIdx.x == 0) L.base = n ? atomicAdd(tail, n) : 0u;
    __syncthreads();
    for (unsigned i = threadIdx.x; i < n; i += blockDim.x) list[L.base + i] = L.v[i];
    __syncthreads();
    if (threadIdx.x == 0) L.n = 0;
    __syncthreads();
}

// The walks of frontier node i handled by one lane of its group: neighbours
// j = S(i)[l], S(i)[l + kGroup], ... and their rows, in batches of kBatch2:
// the batch's nodes, then their states, then act(k, st) on the whole batch,
// whose atomics are independent of one another (a lane's chain is a few
// dependent steps per batch, not per node).
template <class Act>
__device__ __forceinline__ void group_walks(int32_t i, int l, bool on, const int32_t *__restrict__ si,
                                            const int32_t *__restrict__ sj, const int32_t *state, bool pre, Act act) {
    const int32_t a0 = on ? si[i] : 0, a1 = on ? si[i + 1] : 0;
    // every lane of the wavefront runs the same number of batches, so that
    // act() may vote across the wavefront
    int32_t deg = a1 - a0;
    for (int o = 32; o > 0; o >>= 1) deg = max(deg, __shfl_xor(deg, o, 64));
    for (int32_t a_base = 0; a_base < deg; a_base += kGroup) {
        const int32_t a = a_base + l;
        const bool has_j = a < a1 - a0;
        const int32_t j = has_j ? sj[a0 + a] : 0;
        const int32_t b0 = has_j ? si[j] : 0, b1 = has_j ? si[j + 1] : 0;
        const int32_t len = has_j ? b1 - b0 + 1 : 0;  // the neighbour itself, then its row
        int32_t mx = len;
        for (int o = 32; o > 0; o >>= 1) mx = max(mx, __shfl_xor(mx, o, 64));
        for (int32_t c = 0; c < mx; c += kBatch2) {
            int32_t k[kBatch2], st[kBatch2];
#pragma unroll
            for (int u = 0; u < kBatch2; ++u) {
                const int32_t e = c + u;
                k[u] = e < len ? (e == 0 ? j : sj[b0 + e - 1]) : -1;
            }
#pragma unroll
            for (int u = 0; u < kBatch2; ++u) st[u] = k[u] > i ? (pre ? state[k[u]] : kUndecided) : kOut;
            act(k, st);
        }
    }
}

// Root appends (one element per lane; every lane of the workgroup calls it at
// the same point) to the workgroup's LDS root list; past its capacity the
// sweep is abandoned (*overflow: the host pass takes the level; never seen:
// a workgroup's share of a round makes a few roots at most).
__device__ __forceinline__ void wg_root(WgList &L, bool p, int32_t k, unsigned *overflow) {
    const unsigned long long mask = __ballot(p);
    if (!mask) return;
    const int lane = threadIdx.x & 63;
    const int leader = __ffsll(mask) - 1;
    unsigned pos = 0;
    if (lane == leader) pos = atomicAdd(&L.n, (unsigned)__popcll(mask));
    pos = (unsigned)__shfl((int)pos, leader, 64);
    if (p) {
        const unsigned idx = pos + (unsigned)__popcll(mask & ((1ull << lane) - 1ull));
        if (idx < (unsigned)kWgBuf) L.v[idx] = k;
        else atomicOr(overflow, 1u);
    }
}

// Roots R.v[0, nr) mark every higher node within two steps OUT (first
// compare-and-swap wins), appended to `next` through the LDS list M; a
// group per root. Workgroup-uniform (nr is read after a barrier).
__device__ __forceinline__ void mark_roots(const WgList &R, unsigned nr, WgList &M, const int32_t *__restrict__ si,
                                           const int32_t *__restrict__ sj, int32_t *state, int32_t *next,
                                           unsigned *ntail) {
    const int l = threadIdx.x % kGroup;
    const unsigned gpw = blockDim.x / kGroup, g = threadIdx.x / kGroup;
    for (unsigned r0 = 0; r0 < nr; r0 += gpw) {
        const bool on = r0 + g < nr;
        const int32_t r = on ? R.v[r0 + g] : 0;
        group_walks(r, l, on, si, sj, state, false, [&](const int32_t (&k)[kBatch2], const int32_t (&st)[kBatch2]) {
            bool p[kBatch2];
#pragma unroll
            for (int u = 0; u < kBatch2; ++u)
                p[u] = on && st[u] == kUndecided && atomicCAS(&state[k[u]], kUndecided, kOut) == kUndecided;
            wg_add(M, p, k, next, ntail);
        });
        wg_flush(M, next, ntail);
    }
}

// Round 0's roots (the seeds, k_lf_seed) mark their higher nodes OUT into
// out-list 0, which round 0 reads.
__global__ __launch_bounds__(256) void k_lf_seed_mark(const int32_t *__restrict__ seeds, const unsigned *nseeds,
                                                      const int32_t *__restrict__ si, const int32_t *__restrict__ sj,
                                                      int32_t *state, int32_t *outs0, unsigned *tail0) {
    __shared__ WgList R, M;
    const unsigned n = *nseeds, gpw = blockDim.x / kGroup;
    if (threadIdx.x == 0) M.n = 0;
    for (unsigned b0 = blockIdx.x * gpw; b0 < n; b0 += gridDim.x * gpw) {  // grid-uniform per workgroup
        const unsigned nr = min(gpw, n - b0);
        __syncthreads();
        for (unsigned i = threadIdx.x; i < nr; i += blockDim.x) R.v[i] = seeds[b0 + i];
        __syncthreads();
        mark_roots(R, nr, M, si, sj, state, outs0, tail0);
    }
}

// Round t of the sweep, one launch. The OUT nodes of out-list t % 2
// (marked in round t - 1) count down their higher undecided nodes; a count
// reaching 0 makes a root, and the workgroup that made it marks its higher
// nodes within two steps OUT at once, into out-list (t + 1) % 2 for round
// t + 1. Marking inside the round is safe: a node a new root can mark has
// that root among its lower two-step nodes, whose walk never counts down,
// so no concurrent count-down can make it a root; decisions stay final and
// only their timing moves (the roots are the same set). The two out-lists
// alternate, so the list a round reads gets no appends while it runs;
// ostart[t] = where round t's part of its list begins, recorded by round
// t - 2. One launch per round instead of two (mark, then count).
__global__ __launch_bounds__(256) void k_lf_round(int t, const int32_t *__restrict__ si,
                                                  const int32_t *__restrict__ sj, int32_t *state, int32_t *cnt,
                                                  int32_t *outs0, int32_t *outs1, unsigned *tails, unsigned *ostart,
                                                  unsigned *overflow) {
    const int P = t & 1;
    const int32_t *outs = P ? outs1 : outs0;
    int32_t *next = P ? outs0 : outs1;
    unsigned *ntail = &tails[P ^ 1];
    const unsigned lo = ostart[t], hi = tails[P];
    if (blockIdx.x == 0 && threadIdx.x == 0) ostart[t + 2] = hi;
    if (lo >= hi) return;  // grid-uniform
    __shared__ WgList R, M;
    __shared__ WgCounts H;
    if (threadIdx.x == 0) {
        R.n = 0;
        M.n = 0;
    }
    for (int s = threadIdx.x; s < kHash; s += blockDim.x) {
        H.key[s] = -1;
        H.n[s] = 0;
    }
    __syncthreads();
    const int l = threadIdx.x % kGroup;
    const unsigned groups = gridDim.x * (blockDim.x / kGroup);
    const unsigned g0 = blockIdx.x * (blockDim.x / kGroup) + threadIdx.x / kGroup;
    for (unsigned q0 = lo; q0 < hi; q0 += groups) {  // workgroup-uniform trip count
        const unsigned q = q0 + g0;
        const bool on = q < hi;
        const int32_t j = on ? outs[q] : 0;
        group_walks(j, l, on, si, sj, state, false, [&](const int32_t (&k)[kBatch2], const int32_t (&st)[kBatch2]) {
            bool p[kBatch2];
#pragma unroll
            for (int u = 0; u < kBatch2; ++u) {
                p[u] = false;
                if (on && st[u] == kUndecided && !wg_count_add(H, k[u])) p[u] = atomicSub(&cnt[k[u]], 1) == 1;
            }
#pragma unroll
            for (int u = 0; u < kBatch2; ++u) {
                if (p[u]) state[k[u]] = kRoot;
                wg_root(R, p[u], k[u], overflow);
            }
        });
        __syncthreads();
        // the combined count-downs: the one that brings a count to 0 (its old
        // value equals what it subtracts) makes the root
        for (int s0 = 0; s0 < kHash; s0 += blockDim.x) {
            const int s = s0 + threadIdx.x;
            const int32_t key = s < kHash ? H.key[s] : -1;
            bool pr = false;
            if (key >= 0) {
                const int32_t c = H.n[s];
                pr = atomicSub(&cnt[key], c) == c;
                if (pr) state[key] = kRoot;
                H.key[s] = -1;
                H.n[s] = 0;
            }
            wg_root(R, pr, key, overflow);
        }
        __syncthreads();
        mark_roots(R, min(R.n, (unsigned)kWgBuf), M, si, sj, state, next, ntail);
        __syncthreads();
        if (threadIdx.x == 0) R.n = 0;
        __syncthreads();
    }
}

__global__ void k_lf_flags(int32_t m, const int32_t *__restrict__ state, int32_t *flag, unsigned *undecided) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const int32_t s = state[i];
    flag[i] = s == kRoot;
    if (s == kUndecided) atomicAdd(undecided, 1u);
}

// phase-1 aggregates: the root and its strong neighbours (disjoint: roots
// are at least three steps apart)
__global__ void k_lf_assign(int32_t m, const int32_t *__restrict__ si, const int32_t *__restrict__ sj,
                            const int32_t *__restrict__ state, const int32_t *__restrict__ id, int32_t *agg) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m || state[i] != kRoot) return;
    const int32_t a = id[i];
    agg[i] = a;
    for (int32_t k = si[i]; k < si[i + 1]; ++k) agg[sj[k]] = a;
}

__global__ void k_fill_i32(int32_t m, int32_t v, int32_t *x) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < m) x[i] = v;
}

__global__ void k_free_flags(int32_t m, const int32_t *__restrict__ agg, int32_t *flag) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < m) flag[i] = agg[i] == -1;
}

// the free nodes in index order, and their S row lengths
__global__ void k_free_list(int32_t m, const int32_t *__restrict__ flag, const int32_t *__restrict__ pos,
                            const int32_t *__restrict__ si, int32_t *list, int32_t *len) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m || !flag[i]) return;
    list[pos[i]] = i;
    len[pos[i]] = si[i + 1] - si[i];
}

__global__ void k_free_rows(int32_t nf, const int32_t *__restrict__ list, const int32_t *__restrict__ roff,
                            const int32_t *__restrict__ si, const int32_t *__restrict__ sj, int32_t *rows) {
    const int32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nf) return;
    const int32_t i = list[q], s0 = si[i], n = si[i + 1] - s0, o = roff[q];
    for (int32_t k = 0; k < n; ++k) rows[o + k] = sj[s0 + k];
}

__global__ void k_scatter_i32(int32_t nf, const int32_t *__restrict__ list, const int32_t *__restrict__ v,
                              int32_t *agg) {
    const int32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q < nf) agg[list[q]] = v[q];
}

template <class T>
hipError_t dalloc(T **p, int64_t n) {
    return hipMalloc(reinterpret_cast<void **>(p), sizeof(T) * (size_t)std::max<int64_t>(n, 1));
}

// exclusive sum of n int32 (temp allocated here)
hipError_t exclusive_sum(const int32_t *in, int32_t *out, int32_t n, hipStream_t s) {
    int32_t *tmp = nullptr;
    hipError_t e = dalloc(&tmp, aijhip_dscan::scan_tmp_elems(n));
    if (e == hipSuccess) e = aijhip_dscan::exclusive_scan(in, out, (int64_t)n, tmp, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    hipFree(tmp);
    return e;
}

// ---- PETSc 3.7 agg's MIS (gamg_internal.h aggregate_mis) on the device.
// The sequential pass visits the nodes in key order and roots an aggregate
// at every node no earlier root lies within reach of (G2: two steps of S
// when squared, one otherwise), so the roots are the lexicographically-first
// independent set of G2 by key, unique: node i is a root iff no lower-key
// node within reach of it is one. Rounds decide it: an undecided node with a
// root within reach is OUT (that root has the lower key: it was decided with
// i undecided in its reach); one whose lower-key nodes within reach are all
// OUT is a root; otherwise it waits. Decisions are final, so the rounds reach
// the sequential pass's set whatever their number (random keys: ~16-20).
//
// A round is two flat one-hop passes rather than one two-hop walk: pass A
// takes, for every node u, the minimum over its closed neighbourhood N[u] of
// a value that is 0 for a root, key + 1 for an undecided node and all-ones
// otherwise; pass B takes each undecided node's minimum over its neighbours'
// pass-A values (squared) or its own (not) — that covers its reach and
// itself — and decides: 0 → OUT, its own key + 1 → root, else it waits.
// Round 5's first form walked the two-hop reach per lane (~50 visits, each a
// dependent sj → state → key load chain): ~5 ms a round at 300^3 against
// two neighbour-list passes' worth of bytes here.
// one byte per node: a squared 7-point neighbourhood spans +-2 planes, 360 KB
// of byte states against 1.4 MB of int32 ones (per-XCD L2: 4 MB)
typedef uint8_t mis_state_t;
constexpr mis_state_t kMisUndecided = 0, kMisRoot = 1, kMisOut = 2, kMisSingle = 3;

// hk[i]: the high word of mis_key(i, level); its low word is i.
__device__ __forceinline__ uint64_t mis_key_of(uint32_t h, int32_t i) {
    return (uint64_t)h << 32 | (uint32_t)i;
}

// roots = false: a round's decision value; true: a root's key (parents)
__device__ __forceinline__ uint64_t mis_value(mis_state_t st, uint32_t h, int32_t w, bool roots) {
    if (roots) return st == kMisRoot ? mis_key_of(h, w) : ~0ull;
    return st == kMisRoot ? 0ull : st == kMisUndecided ? mis_key_of(h, w) + 1 : ~0ull;
}

__global__ void k_mis_init(int32_t m, int32_t level, const int32_t *__restrict__ si, mis_state_t *state,
                           uint32_t *hk) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < m) {
        state[i] = si[i] == si[i + 1] ? kMisSingle : kMisUndecided;
        hk[i] = static_cast<uint32_t>(aijhip_gamg::mis_key(i, level) >> 32);
    }
}

// Pass A: amin[u] = min over N[u] of mis_value. Neighbour lists go four at a
// time (clamped, so a repeat only re-reads the last one), their loads issued
// together.
__global__ __launch_bounds__(256) void k_mis_closed_min(int32_t m, const int32_t *__restrict__ si,
                                                        const int32_t *__restrict__ sj,
                                                        const uint32_t *__restrict__ hk,
                                                        const mis_state_t *__restrict__ state, bool roots,
                                                        uint64_t *__restrict__ amin) {
    const int32_t u = blockIdx.x * blockDim.x + threadIdx.x;
    if (u >= m) return;
    uint64_t best = mis_value(state[u], hk[u], u, roots);
    const int32_t a0 = si[u], a1 = si[u + 1];
    for (int32_t a = a0; a < a1; a += 4) {
        int32_t j[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) j[q] = sj[min(a + q, a1 - 1)];
        mis_state_t st[4];
        uint32_t h[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            st[q] = state[j[q]];
            h[q] = hk[j[q]];
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) best = min(best, mis_value(st[q], h[q], j[q], roots));
    }
    amin[u] = best;
}

// min over i's neighbours of amin (squared reach), or amin[i] itself
__device__ __forceinline__ uint64_t reach_min(int32_t i, bool square, const int32_t *__restrict__ si,
                                              const int32_t *__restrict__ sj, const uint64_t *__restrict__ amin) {
    if (!square) return amin[i];
    uint64_t b = ~0ull;
    const int32_t a0 = si[i], a1 = si[i + 1];
    for (int32_t a = a0; a < a1; a += 4) {
        int32_t j[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) j[q] = sj[min(a + q, a1 - 1)];
        uint64_t v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = amin[j[q]];
#pragma unroll
        for (int q = 0; q < 4; ++q) b = min(b, v[q]);
    }
    return b;
}

// Pass B: the decisions (only this node's state is written; every read is
// of pass A's output, so a round is the same whatever the lane order).
__global__ __launch_bounds__(256) void k_mis_decide(int32_t m, const int32_t *__restrict__ si,
                                                    const int32_t *__restrict__ sj, bool square,
                                                    const uint32_t *__restrict__ hk,
                                                    const uint64_t *__restrict__ amin, mis_state_t *state,
                                                    unsigned *wcount) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    bool waits = false;
    if (i < m && state[i] == kMisUndecided) {
        const uint64_t b = reach_min(i, square, si, sj, amin);
        if (b == 0) state[i] = kMisOut;
        else if (b == mis_key_of(hk[i], i) + 1) state[i] = kMisRoot;
        else waits = true;
    }
    // the workgroup's count of waiting nodes, one plain store per workgroup
    // (k_mis_total sums them once a batch): one atomic per wave on a single
    // counter serialised ~420 K atomics a round at 300^3, ~2 ms
    __shared__ unsigned wc[4];
    const unsigned nw = (unsigned)__popcll(__ballot(waits));
    if ((threadIdx.x & 63) == 0) wc[threadIdx.x >> 6] = nw;
    __syncthreads();
    if (threadIdx.x == 0) wcount[blockIdx.x] = wc[0] + wc[1] + wc[2] + wc[3];
}

// total = the sum of n per-workgroup counts (one workgroup of 1024)
__global__ __launch_bounds__(1024) void k_mis_total(const unsigned *__restrict__ wcount, int32_t n,
                                                    unsigned long long *total) {
    __shared__ unsigned long long part[16];
    unsigned long long s = 0;
    for (int32_t q = threadIdx.x; q < n; q += 1024) s += wcount[q];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s += __shfl_down(s, off, 64);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long t = 0;
        for (int w = 0; w < 16; ++w) t += part[w];
        *total = t;
    }
}

// parent: a root itself; an OUT node the lowest-key root within reach (the
// first root of the pass to take it: amin over roots' keys, whose low word is
// the root), then (squared: smoothAggs) the highest-index root among its S
// neighbours when it has one; singletons -1. flag[i] = 1 for the roots
// (their scan numbers the aggregates).
__global__ __launch_bounds__(256) void k_mis_parent(int32_t m, const int32_t *__restrict__ si,
                                                    const int32_t *__restrict__ sj, bool square,
                                                    const uint64_t *__restrict__ amin,
                                                    const mis_state_t *__restrict__ state, int32_t *parent,
                                                    int32_t *flag) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const mis_state_t st = state[i];
    flag[i] = st == kMisRoot;
    if (st == kMisRoot) { parent[i] = i; return; }
    if (st != kMisOut) { parent[i] = -1; return; }
    const uint64_t b = reach_min(i, square, si, sj, amin);  // an OUT node has a root within reach
    int32_t best = static_cast<int32_t>(static_cast<uint32_t>(b));
    if (square) {
        int32_t hi = -1;
        for (int32_t a = si[i]; a < si[i + 1]; ++a) {
            const int32_t j = sj[a];
            if (state[j] == kMisRoot && j > hi) hi = j;
        }
        if (hi >= 0) best = hi;
    }
    parent[i] = best;
}

__global__ void k_mis_number(int32_t m, const int32_t *__restrict__ parent, const int32_t *__restrict__ cidx,
                             int32_t *agg) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < m) agg[i] = parent[i] >= 0 ? cidx[parent[i]] : -1;
}

}  // namespace

namespace aijhip_gamg {

// MIS scratch: stream-ordered allocations on the rounds' stream (hipFree
// would wait for the whole device, the emax job's and the handle jobs' work
// included)
template <class T>
hipError_t salloc(T **p, int64_t n, hipStream_t s) {
    return hipMallocAsync(reinterpret_cast<void **>(p), sizeof(T) * (size_t)std::max<int64_t>(n, 1), s);
}

hipError_t aggregate_mis_device(int32_t m, const int32_t *si, const int32_t *sj, bool square, int32_t level,
                                int32_t *agg, int32_t *na, int32_t *rounds) {
    *na = 0;
    *rounds = 0;
    if (m == 0) return hipSuccess;
    // The rounds run on set-up stream slot 0 (the greedy sweep's), after the
    // null stream's strength graph (an event, no host wait): round 5 measured
    // a 15 ms stall of the level-1 rounds on the null stream while the handle
    // job built P_0's plan (its copies and syncs go through the null stream).
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    hipStream_t ms = e == hipSuccess ? aijhip_gamg::setup_stream(dev, 0) : nullptr;
    if (!ms) return e == hipSuccess ? hipErrorInvalidValue : e;
    hipEvent_t ready = nullptr;
    if ((e = hipEventCreateWithFlags(&ready, hipEventDisableTiming)) != hipSuccess) return e;
    if ((e = hipEventRecord(ready, nullptr)) == hipSuccess) e = hipStreamWaitEvent(ms, ready, 0);
    mis_state_t *state = nullptr;
    uint32_t *hk = nullptr;
    uint64_t *amin = nullptr;
    int32_t *parent = nullptr, *flag = nullptr, *cidx = nullptr, *tmp = nullptr;
    unsigned long long *left = nullptr, *h_ctl = nullptr;  // h_ctl: [0] the count, [1] the aggregates
    unsigned *wcount = nullptr;
    const unsigned g = blocks_for(m, 256);
    if (e == hipSuccess) e = salloc(&state, m, ms);
    if (e == hipSuccess) e = salloc(&hk, m, ms);
    if (e == hipSuccess) e = salloc(&amin, m, ms);
    if (e == hipSuccess) e = salloc(&left, 1, ms);
    if (e == hipSuccess) e = salloc(&wcount, g, ms);
    // pinned, one per host thread and never freed (hipHostFree waits for the device)
    static thread_local unsigned long long *t_ctl = nullptr;
    if (e == hipSuccess && !t_ctl) e = hipHostMalloc(reinterpret_cast<void **>(&t_ctl), 2 * sizeof(unsigned long long));
    h_ctl = t_ctl;
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_mis_init, dim3(g), dim3(256), 0, ms, m, level, si, state, hk);
        e = hipGetLastError();
    }
    // Every round decides at least the lowest-key undecided node, so m rounds
    // always suffice. They go out in batches of kBatch with one count read
    // per batch (a round past the last is a no-op), the count through pinned
    // memory.
    static const bool log = std::getenv("AIJHIP_GAMG_LOG") != nullptr;
    constexpr int32_t kBatch = 4;
    for (int32_t r0 = 0; e == hipSuccess && r0 < m; r0 += kBatch) {
        const auto t0 = std::chrono::steady_clock::now();
        for (int32_t r = r0; r < r0 + kBatch && e == hipSuccess; ++r) {
            hipLaunchKernelGGL(k_mis_closed_min, dim3(g), dim3(256), 0, ms, m, si, sj, hk, state, false, amin);
            hipLaunchKernelGGL(k_mis_decide, dim3(g), dim3(256), 0, ms, m, si, sj, square, hk, amin, state, wcount);
            e = hipGetLastError();
        }
        if (e == hipSuccess) {
            hipLaunchKernelGGL(k_mis_total, dim3(1), dim3(1024), 0, ms, wcount, (int32_t)g, left);
            e = hipGetLastError();
        }
        if (e == hipSuccess) e = hipMemcpyAsync(h_ctl, left, sizeof(unsigned long long), hipMemcpyDeviceToHost, ms);
        if (e == hipSuccess) e = hipStreamSynchronize(ms);
        if (e != hipSuccess) break;
        *rounds = r0 + kBatch;
        if (log)
            std::fprintf(stderr, "  MIS rounds %d-%d: %llu undecided after, %.3f ms\n", r0, r0 + kBatch - 1, h_ctl[0],
                         std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
        if (h_ctl[0] == 0) break;
    }
    if (e == hipSuccess) e = salloc(&parent, m, ms);
    if (e == hipSuccess) e = salloc(&flag, m, ms);
    if (e == hipSuccess) e = salloc(&cidx, m, ms);
    if (e == hipSuccess) e = salloc(&tmp, aijhip_dscan::scan_tmp_elems(m), ms);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_mis_closed_min, dim3(g), dim3(256), 0, ms, m, si, sj, hk, state, true, amin);
        hipLaunchKernelGGL(k_mis_parent, dim3(g), dim3(256), 0, ms, m, si, sj, square, amin, state, parent, flag);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = aijhip_dscan::exclusive_scan(flag, cidx, (int64_t)m, tmp, ms);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_mis_number, dim3(g), dim3(256), 0, ms, m, parent, cidx, agg);
        e = hipGetLastError();
    }
    int32_t *h_na = reinterpret_cast<int32_t *>(h_ctl + 1);  // [0] the last scan value, [1] the last flag
    if (e == hipSuccess) e = hipMemcpyAsync(h_na, cidx + (m - 1), sizeof(int32_t), hipMemcpyDeviceToHost, ms);
    if (e == hipSuccess) e = hipMemcpyAsync(h_na + 1, flag + (m - 1), sizeof(int32_t), hipMemcpyDeviceToHost, ms);
    for (void *q : {(void *)state, (void *)hk, (void *)amin, (void *)parent, (void *)flag, (void *)cidx,
                    (void *)tmp, (void *)left, (void *)wcount})
        if (q) (void)hipFreeAsync(q, ms);
    const hipError_t es = hipStreamSynchronize(ms);  // agg and the count are ready; the scratch went back
    if (e == hipSuccess) e = es;
    if (e == hipSuccess) *na = h_na[0] + h_na[1];
    (void)hipEventDestroy(ready);
    return e;
}

hipError_t aggregate_phase1_device(int32_t m, const int32_t *si, const int32_t *sj, int32_t max_rounds,
                                   int32_t *phase1, int32_t *na, int32_t *rounds, bool *done) {
    *done = false;
    *na = 0;
    *rounds = 0;
    if (m <= 0) {
        *done = true;
        return hipSuccess;
    }
    const bool log = std::getenv("AIJHIP_GAMG_LOG") != nullptr;
    const unsigned grid = kRoundGrid;
    auto clk = std::chrono::steady_clock::now();
    hipStream_t s = nullptr;
    int32_t *state = nullptr, *cnt = nullptr, *roots = nullptr, *outs = nullptr, *outs1 = nullptr;
    // tails: [0], [1] the out-lists' ends, [2] the seeds (round 0's roots),
    // [3] the root-list overflow flag
    unsigned *tails = nullptr, *ostart = nullptr, *h_ctl = nullptr;
    const unsigned g = blocks_for(m, 256);
    constexpr int kBatch = 32;  // rounds launched between two looks at the tails
    // s does not synchronise with the null stream, on which the strength
    // kernels wrote si/sj: drain it first, so the sweep's reads are ordered
    // after their producers explicitly
    hipError_t e = hipStreamSynchronize(nullptr);
    auto mark = [&](const char *what) {
        if (!log) return;
        const auto now = std::chrono::steady_clock::now();
        std::fprintf(stderr, "  phase 1 sweep %-10s %8.3f ms (host)\n", what,
                     std::chrono::duration<double, std::milli>(now - clk).count());
    };
    mark("drained");
    if (e == hipSuccess) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        s = aijhip_gamg::setup_stream(dev, 0);
        if (!s) e = hipErrorOutOfMemory;
    }
    mark("stream");
    if (e == hipSuccess) e = dalloc(&state, m);
    if (e == hipSuccess) e = dalloc(&cnt, m);
    if (e == hipSuccess) e = dalloc(&roots, m);
    if (e == hipSuccess) e = dalloc(&outs, m);
    if (e == hipSuccess) e = dalloc(&outs1, m);
    if (e == hipSuccess) e = dalloc(&tails, 4);
    if (e == hipSuccess) e = dalloc(&ostart, (int64_t)max_rounds + kBatch + 3);
    if (e == hipSuccess) e = hipHostMalloc(reinterpret_cast<void **>(&h_ctl), sizeof(unsigned) * 8);
    mark("allocs");
    if (e == hipSuccess) e = hipMemsetAsync(tails, 0, sizeof(unsigned) * 4, s);
    if (e == hipSuccess) e = hipMemsetAsync(ostart, 0, sizeof(unsigned) * 2, s);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_lf_init, dim3(g), dim3(256), 0, s, m, si, sj, state, cnt);
        hipLaunchKernelGGL(k_lf_seed, dim3(g), dim3(256), 0, s, m, state, cnt, roots, tails + 2);
        hipLaunchKernelGGL(k_lf_seed_mark, dim3(grid), dim3(256), 0, s, roots, tails + 2, si, sj, state, outs,
                           tails);
        e = hipGetLastError();
    }
    mark("launched");
    auto lap = [&](const char *what) {
        if (!log) return;
        (void)hipStreamSynchronize(s);
        const auto now = std::chrono::steady_clock::now();
        std::fprintf(stderr, "  phase 1 sweep %-10s %8.3f ms\n", what,
                     std::chrono::duration<double, std::milli>(now - clk).count());
        clk = now;
    };
    lap("init");
    int t = 0;
    while (e == hipSuccess && t < max_rounds) {
        for (int b = 0; b < kBatch; ++b, ++t)
            hipLaunchKernelGGL(k_lf_round, dim3(grid), dim3(256), 0, s, t, si, sj, state, cnt, outs, outs1, tails,
                               ostart, tails + 3);
        // finished when round t would find its part of its out-list empty
        // (ostart[t], recorded by round t - 2, equals the list's end): no
        // OUT node left to count down, so no root can follow
        if ((e = hipGetLastError()) != hipSuccess) break;
        if ((e = hipMemcpyAsync(h_ctl, tails, sizeof(unsigned) * 4, hipMemcpyDeviceToHost, s)) != hipSuccess) break;
        if ((e = hipMemcpyAsync(h_ctl + 4, ostart + t, sizeof(unsigned), hipMemcpyDeviceToHost, s)) != hipSuccess)
            break;
        if ((e = hipStreamSynchronize(s)) != hipSuccess) break;
        if (h_ctl[3] != 0) break;  // a workgroup's root list overflowed: the host pass
        if (h_ctl[t & 1] == h_ctl[4]) {
            *done = true;
            break;
        }
    }
    *rounds = t;
    lap("rounds");
    if (e == hipSuccess && *done) {
        // every node decided (a check on the rule above), aggregate numbers in
        // root order
        int32_t *flag = cnt, *id = outs;  // reused: the sweep is over
        if ((e = hipMemsetAsync(tails + 2, 0, sizeof(unsigned), s)) == hipSuccess) {
            hipLaunchKernelGGL(k_lf_flags, dim3(g), dim3(256), 0, s, m, state, flag, tails + 2);
            e = hipGetLastError();
        }
        if (e == hipSuccess) e = exclusive_sum(flag, id, m, s);
        if (e == hipSuccess) e = hipMemcpyAsync(h_ctl + 2, tails + 2, sizeof(unsigned), hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e == hipSuccess && h_ctl[2] != 0) *done = false;  // unreachable if the rule holds: the host redoes it
        int32_t last_id = 0, last_flag = 0;
        if (e == hipSuccess && *done) {
            e = hipMemcpy(&last_id, id + (m - 1), sizeof(int32_t), hipMemcpyDeviceToHost);
            if (e == hipSuccess) e = hipMemcpy(&last_flag, flag + (m - 1), sizeof(int32_t), hipMemcpyDeviceToHost);
        }
        if (e == hipSuccess && *done) {
            *na = last_id + last_flag;
            hipLaunchKernelGGL(k_fill_i32, dim3(g), dim3(256), 0, s, m, -1, phase1);
            hipLaunchKernelGGL(k_lf_assign, dim3(g), dim3(256), 0, s, m, si, sj, state, id, phase1);
            e = hipGetLastError();
            if (e == hipSuccess) e = hipStreamSynchronize(s);
        }
    }
    lap("numbering");
    hipFree(state); hipFree(cnt); hipFree(roots); hipFree(outs);
    hipFree(outs1); hipFree(tails); hipFree(ostart);
    if (h_ctl) hipHostFree(h_ctl);
    // (s is the process's set-up stream: kept)
    return e;
}

hipError_t aggregate_phase3_device(int32_t m, const int32_t *si, const int32_t *sj, int32_t *agg, int32_t *na) {
    int32_t *flag = nullptr, *pos = nullptr, *list = nullptr, *len = nullptr, *roff = nullptr, *rows = nullptr,
            *val = nullptr;
    const unsigned g = blocks_for(m, 256);
    int32_t nf = 0, nrow = 0;
    std::vector<int32_t> h_list, h_roff, h_rows, h_val;
    hipError_t e = dalloc(&flag, m);
    if (e == hipSuccess) e = dalloc(&pos, m);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_free_flags, dim3(g), dim3(256), 0, nullptr, m, agg, flag);
        e = exclusive_sum(flag, pos, m, nullptr);
    }
    if (e == hipSuccess) {
        int32_t lp = 0, lf = 0;
        e = hipMemcpy(&lp, pos + (m - 1), sizeof(int32_t), hipMemcpyDeviceToHost);
        if (e == hipSuccess) e = hipMemcpy(&lf, flag + (m - 1), sizeof(int32_t), hipMemcpyDeviceToHost);
        nf = lp + lf;
    }
    if (e == hipSuccess && nf > 0) {
        if ((e = dalloc(&list, nf)) == hipSuccess && (e = dalloc(&len, nf)) == hipSuccess &&
            (e = dalloc(&roff, nf)) == hipSuccess) {
            hipLaunchKernelGGL(k_free_list, dim3(g), dim3(256), 0, nullptr, m, flag, pos, si, list, len);
            e = exclusive_sum(len, roff, nf, nullptr);
        }
        if (e == hipSuccess) {
            int32_t lo = 0, ll = 0;
            e = hipMemcpy(&lo, roff + (nf - 1), sizeof(int32_t), hipMemcpyDeviceToHost);
            if (e == hipSuccess) e = hipMemcpy(&ll, len + (nf - 1), sizeof(int32_t), hipMemcpyDeviceToHost);
            nrow = lo + ll;
        }
        if (e == hipSuccess && (e = dalloc(&rows, nrow)) == hipSuccess) {
            hipLaunchKernelGGL(k_free_rows, dim3(blocks_for(nf, 256)), dim3(256), 0, nullptr, nf, list, roff, si, sj,
                               rows);
            e = hipGetLastError();
        }
        if (e == hipSuccess) {
            h_list.resize(nf);
            h_roff.resize((size_t)nf + 1);
            h_rows.resize((size_t)std::max(nrow, 1));
            e = hipMemcpy(h_list.data(), list, sizeof(int32_t) * (size_t)nf, hipMemcpyDeviceToHost);
            if (e == hipSuccess) e = hipMemcpy(h_roff.data(), roff, sizeof(int32_t) * (size_t)nf, hipMemcpyDeviceToHost);
            if (e == hipSuccess && nrow > 0)
                e = hipMemcpy(h_rows.data(), rows, sizeof(int32_t) * (size_t)nrow, hipMemcpyDeviceToHost);
            h_roff[nf] = nrow;
        }
        if (e == hipSuccess) {
            // gamg_setup.cpp aggregate phase 3 over the free nodes alone: a node
            // outside the list already has an aggregate
            h_val.assign(nf, -1);
            int32_t n = *na;
            for (int32_t q = 0; q < nf; ++q) {
                if (h_val[q] != -1) continue;
                h_val[q] = n;
                for (int32_t k = h_roff[q]; k < h_roff[q + 1]; ++k) {
                    const auto it = std::lower_bound(h_list.begin(), h_list.end(), h_rows[k]);
                    if (it != h_list.end() && *it == h_rows[k] && h_val[it - h_list.begin()] == -1)
                        h_val[it - h_list.begin()] = n;
                }
                ++n;
            }
            *na = n;
            if ((e = dalloc(&val, nf)) == hipSuccess &&
                (e = hipMemcpy(val, h_val.data(), sizeof(int32_t) * (size_t)nf, hipMemcpyHostToDevice)) ==
                    hipSuccess) {
                hipLaunchKernelGGL(k_scatter_i32, dim3(blocks_for(nf, 256)), dim3(256), 0, nullptr, nf, list, val,
                                   agg);
                e = hipGetLastError();
            }
        }
    }
    hipFree(flag); hipFree(pos); hipFree(list); hipFree(len); hipFree(roff); hipFree(rows); hipFree(val);
    return e;
}

}  // namespace aijhip_gamg
