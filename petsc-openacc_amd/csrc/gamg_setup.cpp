// gamg_setup.cpp — host construction of the smoothed-aggregation hierarchy
// (include/aijhip_gamg.h). Set-up only: the solve-phase V-cycle runs on the
// device (ksp.hip). OpenMP over rows where the work is row-parallel; every
// floating-point sum is accumulated in a fixed (row-traversal) order, so the
// result does not depend on the thread count, and equals a scipy CSR
// restatement (oracle/gamg.py) bit for bit.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <new>
#include <stdexcept>
#include <vector>

#ifdef _OPENMP
#include <omp.h>
#endif

#include "aijhip.h"
#include "aijhip_gamg.h"
#include "gamg_internal.h"

namespace {

struct CSR {
    int32_t m = 0, n = 0;
    std::vector<int32_t> ai, aj;
    std::vector<double> aa;
    int64_t nnz() const { return ai.empty() ? 0 : ai[m]; }
};

// Read-only view of a CSR (the caller's level-0 arrays or a stored level).
struct View {
    int32_t m, n;
    const int32_t *ai, *aj;
    const double *aa;
};

View view(const CSR &c) { return View{c.m, c.n, c.ai.data(), c.aj.data(), c.aa.data()}; }

double wtime() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int nthreads(int req) {
#ifdef _OPENMP
    return req > 0 ? req : omp_get_max_threads();
#else
    (void)req;
    return 1;
#endif
}

// First stored diagonal entry of each row (0 if none) — MatGetDiagonal.
std::vector<double> diagonal(const View &A, int nt) {
    std::vector<double> d(A.m, 0.0);
#pragma omp parallel for schedule(static) num_threads(nt)
    for (int32_t i = 0; i < A.m; ++i)
        for (int32_t k = A.ai[i]; k < A.ai[i + 1]; ++k)
            if (A.aj[k] == i) { d[i] = A.aa[k]; break; }
    return d;
}

// Symmetric strength graph: j != i with |a_ij| > theta * sqrt(|a_ii a_jj|),
// united with its transpose; rows sorted, unique. Each row's set gathers its
// own strong entries and the rows strong towards it into atomically taken
// slots, then is sorted, so the result does not depend on the thread count.
void strength_graph(const View &A, const std::vector<double> &d, double theta,
                    std::vector<int32_t> &si, std::vector<int32_t> &sj, int nt) {
    const int32_t m = A.m;
    auto strong = [&](int32_t i, int32_t k) {
        const int32_t j = A.aj[k];
        if (j == i) return false;
        const double v = std::fabs(A.aa[k]);
        return v > theta * std::sqrt(std::fabs(d[i] * d[j]));
    };
    std::vector<int32_t> cnt(m, 0);  // out-degree + in-degree
#pragma omp parallel for schedule(dynamic, 4096) num_threads(nt)
    for (int32_t i = 0; i < m; ++i)
        for (int32_t k = A.ai[i]; k < A.ai[i + 1]; ++k)
            if (strong(i, k)) {
#pragma omp atomic
                ++cnt[i];
#pragma omp atomic
                ++cnt[A.aj[k]];
            }
    std::vector<int64_t> off((size_t)m + 1, 0);
    for (int32_t i = 0; i < m; ++i) off[i + 1] = off[i] + cnt[i];
    std::vector<int32_t> tmp(off[m]);
    std::vector<int64_t> pos(off.begin(), off.end() - 1);
#pragma omp parallel for schedule(dynamic, 4096) num_threads(nt)
    for (int32_t i = 0; i < m; ++i)
        for (int32_t k = A.ai[i]; k < A.ai[i + 1]; ++k)
            if (strong(i, k)) {
                const int32_t j = A.aj[k];
                int64_t a, b;
#pragma omp atomic capture
                a = pos[i]++;
#pragma omp atomic capture
                b = pos[j]++;
                tmp[a] = j;
                tmp[b] = i;
            }
#pragma omp parallel for schedule(dynamic, 4096) num_threads(nt)
    for (int32_t i = 0; i < m; ++i) {
        auto b = tmp.begin() + off[i], e = tmp.begin() + off[i + 1];
        std::sort(b, e);
        cnt[i] = (int32_t)(std::unique(b, e) - b);
    }
    si.assign((size_t)m + 1, 0);
    for (int32_t i = 0; i < m; ++i) si[i + 1] = si[i] + cnt[i];
    sj.resize(si[m]);
#pragma omp parallel for schedule(static) num_threads(nt)
    for (int32_t i = 0; i < m; ++i) std::copy_n(tmp.begin() + off[i], cnt[i], sj.begin() + si[i]);
}

// Greedy aggregation in natural order (Vanek et al.): (1) a free node whose
// strong neighbours are all free roots an aggregate with them; (2) a free
// node joins the phase-1 aggregate of its strongest phase-1 neighbour
// (lowest index on ties); (3) what is left roots aggregates with its free
// neighbours. Isolated nodes are singletons.
int32_t aggregate(const View &A, const std::vector<int32_t> &si, const std::vector<int32_t> &sj,
                  std::vector<int32_t> &agg) {
    const int32_t m = A.m;
    agg.assign(m, -1);
    int32_t na = 0;
    for (int32_t i = 0; i < m; ++i) {
        if (agg[i] != -1 || si[i] == si[i + 1]) continue;
        bool free_all = true;
        for (int32_t k = si[i]; k < si[i + 1] && free_all; ++k) free_all = agg[sj[k]] == -1;
        if (!free_all) continue;
        agg[i] = na;
        for (int32_t k = si[i]; k < si[i + 1]; ++k) agg[sj[k]] = na;
        ++na;
    }
    const std::vector<int32_t> phase1 = agg;
    for (int32_t i = 0; i < m; ++i) {
        if (phase1[i] != -1) continue;
        int32_t best = -1;
        double bv = -1.0;
        for (int32_t k = A.ai[i]; k < A.ai[i + 1]; ++k) {
            const int32_t j = A.aj[k];
            if (j == i || phase1[j] == -1) continue;
            if (!std::binary_search(sj.begin() + si[i], sj.begin() + si[i + 1], j)) continue;
            const double v = std::fabs(A.aa[k]);
            if (v > bv || (v == bv && j < best)) { bv = v; best = j; }
        }
        if (best >= 0) agg[i] = phase1[best];
    }
    for (int32_t i = 0; i < m; ++i) {
        if (agg[i] != -1) continue;
        agg[i] = na;
        for (int32_t k = si[i]; k < si[i + 1]; ++k)
            if (agg[sj[k]] == -1) agg[sj[k]] = na;
        ++na;
    }
    return na;
}

uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

// y = D^-1 A x (row-parallel, each row summed in storage order)
void dinv_apply(const View &A, const std::vector<double> &dinv, const std::vector<double> &x,
                std::vector<double> &y, int nt) {
#pragma omp parallel for schedule(static) num_threads(nt)
    for (int32_t i = 0; i < A.m; ++i) {
        double s = 0.0;
        for (int32_t k = A.ai[i]; k < A.ai[i + 1]; ++k) s += A.aa[k] * x[A.aj[k]];
        y[i] = dinv[i] * s;
    }
}

// Deterministic blocked dot: left to right inside fixed kDotBlock-entry
// blocks, then the block sums left to right (oracle/gamg.py _blockdot).
constexpr int64_t kDotBlock = 256;

double dot(const std::vector<double> &a, const std::vector<double> &b, int nt) {
    const int64_t n = (int64_t)a.size(), nb = (n + kDotBlock - 1) / kDotBlock;
    std::vector<double> part(nb);
#pragma omp parallel for schedule(static) num_threads(nt)
    for (int64_t q = 0; q < nb; ++q) {
        double s = 0.0;
        for (int64_t i = q * kDotBlock, e = std::min(n, i + kDotBlock); i < e; ++i) s += a[i] * b[i];
        part[q] = s;
    }
    double s = 0.0;
    for (int64_t q = 0; q < nb; ++q) s += part[q];
    return s;
}

// emax(D^-1 A) by power iteration from a counter-based random start.
double estimate_emax(const View &A, const std::vector<double> &dinv, int its, int nt) {
    const int32_t m = A.m;
    if (m == 0) return 1.0;
    std::vector<double> v(m), w(m);
#pragma omp parallel for schedule(static) num_threads(nt)
    for (int32_t i = 0; i < m; ++i)
        v[i] = 2.0 * ((double)(mix64(0x5EEDULL + (uint64_t)(i + 1) * 0x9E3779B97F4A7C15ULL) >> 11) *
                      (1.0 / 9007199254740992.0)) - 1.0;
    const double nv = std::sqrt(dot(v, v, nt));
#pragma omp parallel for schedule(static) num_threads(nt)
    for (int32_t i = 0; i < m; ++i) v[i] /= nv;
    double lam = 1.0;
    for (int it = 0; it < its; ++it) {
        dinv_apply(A, dinv, v, w, nt);
        const double nw = std::sqrt(dot(w, w, nt));
        if (!(nw > 0.0)) break;
        lam = nw;
#pragma omp parallel for schedule(static) num_threads(nt)
        for (int32_t i = 0; i < m; ++i) v[i] = w[i] / nw;
    }
    return lam;
}

// emax(D^-1 A) from CG's Lanczos tridiagonal (PETSc 3.7's estimate for the
// smoother: KSPCG + PC Jacobi, norm none, `its` iterations from x = 0 on a
// random b, KSPComputeExtremeSingularValues; oracle/gamg.py
// estimate_emax_cg): the same b as the power iteration's start (not
// normalised), dots in the blocked order, w = A p summed in storage order.
double estimate_emax_cg(const View &A, const std::vector<double> &dinv, int its, int nt) {
    const int32_t m = A.m;
    if (m == 0) return 1.0;
    std::vector<double> r(m), z(m), p(m), w(m);
#pragma omp parallel for schedule(static) num_threads(nt)
    for (int32_t i = 0; i < m; ++i) {
        r[i] = 2.0 * ((double)(mix64(0x5EEDULL + (uint64_t)(i + 1) * 0x9E3779B97F4A7C15ULL) >> 11) *
                      (1.0 / 9007199254740992.0)) - 1.0;
        z[i] = dinv[i] * r[i];
        p[i] = z[i];
    }
    double rz = dot(z, r, nt);
    std::vector<double> alpha, beta;
    for (int it = 0; it < its; ++it) {
#pragma omp parallel for schedule(static) num_threads(nt)
        for (int32_t i = 0; i < m; ++i) {
            double s = 0.0;
            for (int32_t k = A.ai[i]; k < A.ai[i + 1]; ++k) s += A.aa[k] * p[A.aj[k]];
            w[i] = s;
        }
        const double pw = dot(p, w, nt);
        if (!(pw != 0.0 && rz != 0.0)) break;
        const double a = rz / pw;
        alpha.push_back(a);
#pragma omp parallel for schedule(static) num_threads(nt)
        for (int32_t i = 0; i < m; ++i) {
            r[i] = r[i] - a * w[i];
            z[i] = dinv[i] * r[i];
        }
        const double rzn = dot(z, r, nt);
        const double b = rzn / rz;
        beta.push_back(b);
#pragma omp parallel for schedule(static) num_threads(nt)
        for (int32_t i = 0; i < m; ++i) p[i] = z[i] + b * p[i];
        rz = rzn;
    }
    return alpha.empty() ? 1.0 : aijhip_gamg::lanczos_emax(alpha, beta);
}

// C = A * B (CSR x CSR). Row-parallel; per row, each product is added into
// its column's accumulator in (A entry, B entry) traversal order starting
// from 0.0 (the order of scipy's csr_matmat), then columns sorted.
void spgemm(const View &A, const View &B, CSR &C, int nt) {
    const int32_t m = A.m, n = B.n;
    C.m = m;
    C.n = n;
    C.ai.assign((size_t)m + 1, 0);
    std::vector<int32_t> cnt(m, 0);
#pragma omp parallel num_threads(nt)
    {
        std::vector<int32_t> mark(n, -1);
#pragma omp for schedule(dynamic, 4096)
        for (int32_t i = 0; i < m; ++i) {
            int32_t c = 0;
            for (int32_t k = A.ai[i]; k < A.ai[i + 1]; ++k) {
                const int32_t j = A.aj[k];
                for (int32_t q = B.ai[j]; q < B.ai[j + 1]; ++q)
                    if (mark[B.aj[q]] != i) { mark[B.aj[q]] = i; ++c; }
            }
            cnt[i] = c;
        }
    }
    int64_t total = 0;
    for (int32_t i = 0; i < m; ++i) total += cnt[i];
    if (total > INT32_MAX) throw std::length_error("spgemm: product exceeds int32 indices");
    for (int32_t i = 0; i < m; ++i) C.ai[i + 1] = C.ai[i] + cnt[i];
    C.aj.resize(C.ai[m]);
    C.aa.resize(C.ai[m]);
#pragma omp parallel num_threads(nt)
    {
        std::vector<int32_t> mark(n, -1);
        std::vector<double> acc(n, 0.0);
        std::vector<int32_t> cols;
#pragma omp for schedule(dynamic, 4096)
        for (int32_t i = 0; i < m; ++i) {
            cols.clear();
            for (int32_t k = A.ai[i]; k < A.ai[i + 1]; ++k) {
                const int32_t j = A.aj[k];
                const double a = A.aa[k];
                for (int32_t q = B.ai[j]; q < B.ai[j + 1]; ++q) {
                    const int32_t c = B.aj[q];
                    if (mark[c] != i) { mark[c] = i; acc[c] = 0.0; cols.push_back(c); }
                    acc[c] += a * B.aa[q];
                }
            }
            std::sort(cols.begin(), cols.end());
            int64_t p = C.ai[i];
            for (int32_t c : cols) { C.aj[p] = c; C.aa[p] = acc[c]; ++p; }
        }
    }
}

// Transpose: each output row lists the input rows ascending. The input rows
// are cut into one contiguous chunk per thread; per-(chunk, column) counts
// give every chunk its own slots in each output row, so each thread fills
// its slots in row order and no sort or atomic is needed.
void transpose(const View &A, CSR &T, int nt) {
    T.m = A.n;
    T.n = A.m;
    const int64_t nz = A.ai[A.m];
    nt = std::max(1, std::min<int>(nt, A.m / 4096 + 1));
    std::vector<int32_t> cnt((size_t)nt * A.n, 0);  // [chunk][column]
    auto chunk = [&](int t) { return std::make_pair((int32_t)((int64_t)A.m * t / nt),
                                                    (int32_t)((int64_t)A.m * (t + 1) / nt)); };
#pragma omp parallel for schedule(static, 1) num_threads(nt)
    for (int t = 0; t < nt; ++t) {
        const auto [r0, r1] = chunk(t);
        int32_t *c = cnt.data() + (size_t)t * A.n;
        for (int64_t k = A.ai[r0]; k < A.ai[r1]; ++k) ++c[A.aj[k]];
    }
    T.ai.assign((size_t)A.n + 1, 0);
    int64_t run = 0;
    for (int32_t col = 0; col < A.n; ++col) {
        T.ai[col] = (int32_t)run;
        for (int t = 0; t < nt; ++t) {  // counts -> starting slots
            const int32_t k = cnt[(size_t)t * A.n + col];
            cnt[(size_t)t * A.n + col] = (int32_t)run;
            run += k;
        }
    }
    T.ai[A.n] = (int32_t)run;
    T.aj.resize(nz);
    T.aa.resize(nz);
#pragma omp parallel for schedule(static, 1) num_threads(nt)
    for (int t = 0; t < nt; ++t) {
        const auto [r0, r1] = chunk(t);
        int32_t *pos = cnt.data() + (size_t)t * A.n;
        for (int32_t i = r0; i < r1; ++i)
            for (int32_t k = A.ai[i]; k < A.ai[i + 1]; ++k) {
                const int32_t p = pos[A.aj[k]]++;
                T.aj[p] = i;
                T.aa[p] = A.aa[k];
            }
    }
}

// Smoothed prolongator P = alpha * (D^-1 A P0) + P0, alpha = -scale/emax,
// with P0(i, agg[i]) = B_i / |B restricted to agg[i]| (QR of the near-null
// space per aggregate); returns the coarse near-null space |B|_agg.
void prolongator(const View &A, const std::vector<double> &dinv, const std::vector<int32_t> &agg,
                 int32_t na, const std::vector<double> &B, double alpha, int nsmooths, CSR &P,
                 std::vector<double> &Bc, int nt) {
    // (agg[i] = -1: a node no aggregate took, MIS's removed singleton: an
    // empty row of P0)
    const int32_t m = A.m;
    Bc.assign(na, 0.0);
    for (int32_t i = 0; i < m; ++i)
        if (agg[i] >= 0) Bc[agg[i]] += B[i] * B[i];
    for (int32_t a = 0; a < na; ++a) Bc[a] = std::sqrt(Bc[a]);
    CSR P0;
    P0.m = m;
    P0.n = na;
    P0.ai.resize((size_t)m + 1);
    P0.ai[0] = 0;
    for (int32_t i = 0; i < m; ++i) P0.ai[i + 1] = P0.ai[i] + (agg[i] >= 0 ? 1 : 0);
    P0.aj.resize(P0.ai[m]);
    P0.aa.resize(P0.ai[m]);
#pragma omp parallel for schedule(static) num_threads(nt)
    for (int32_t i = 0; i < m; ++i) {
        if (agg[i] < 0) continue;
        P0.aj[P0.ai[i]] = agg[i];
        P0.aa[P0.ai[i]] = Bc[agg[i]] > 0.0 ? B[i] / Bc[agg[i]] : 0.0;
    }
    if (nsmooths <= 0) { P = std::move(P0); return; }
    CSR T;
    spgemm(A, view(P0), T, nt);
    // P = alpha * (dinv_i * T_ic) + P0_ic on the union pattern (P0's column
    // agg[i] is in T's row whenever a_ii is stored)
    P.m = m;
    P.n = na;
    P.ai.assign((size_t)m + 1, 0);
    std::vector<int32_t> len(m);
#pragma omp parallel for schedule(static) num_threads(nt)
    for (int32_t i = 0; i < m; ++i) {
        const bool has = agg[i] < 0 ||
                         std::binary_search(T.aj.begin() + T.ai[i], T.aj.begin() + T.ai[i + 1], agg[i]);
        len[i] = (T.ai[i + 1] - T.ai[i]) + (has ? 0 : 1);
    }
    for (int32_t i = 0; i < m; ++i) P.ai[i + 1] = P.ai[i] + len[i];
    P.aj.resize(P.ai[m]);
    P.aa.resize(P.ai[m]);
#pragma omp parallel for schedule(static) num_threads(nt)
    for (int32_t i = 0; i < m; ++i) {
        int64_t p = P.ai[i];
        const int32_t g = agg[i];
        bool placed = g < 0;  // (no P0 entry to place)
        const double p0 = g < 0 ? 0.0 : P0.aa[P0.ai[i]];
        for (int32_t k = T.ai[i]; k < T.ai[i + 1]; ++k) {
            const int32_t c = T.aj[k];
            if (!placed && g < c) { P.aj[p] = g; P.aa[p] = p0; ++p; placed = true; }
            const double t = dinv[i] * T.aa[k];
            P.aj[p] = c;
            P.aa[p] = alpha * t + (c == g ? p0 : 0.0);
            if (c == g) placed = true;
            ++p;
        }
        if (!placed) { P.aj[p] = g; P.aa[p] = p0; }
    }
}

}  // namespace

namespace aijhip_gamg {

int32_t aggregate_phase1_rows(int32_t r0, int32_t r1, const int32_t *si, const int32_t *sj, int32_t *agg,
                              uint64_t *taken, int32_t na, int64_t sj0, const int32_t *head) {
    // The pass is a chain of dependent loads (row start, its columns, their
    // state). The state it tests is `taken`, one bit per node (agg[j] != -1):
    // 400 KB for the 3.27 M nodes of 300^3's level 1, so the random tests hit
    // the core's L2 instead of the 13 MB agg array; agg is only written.
    auto is_taken = [taken](int32_t j) { return (taken[j >> 6] >> (j & 63)) & 1u; };
    auto take = [taken, agg](int32_t j, int32_t a) {
        agg[j] = a;
        taken[j >> 6] |= uint64_t(1) << (j & 63);
    };
    auto visit = [&](int32_t i) {  // the pass's step for a free node with a row
        const int32_t *row = sj + (si[i] - sj0);
        const int32_t len = si[i + 1] - si[i];
        for (int32_t k = 0; k < len; ++k)
            if (is_taken(row[k])) return;
        take(i, na);
        for (int32_t k = 0; k < len; ++k) take(row[k], na);
        ++na;
    };
    if (!head) {  // rows of nodes still free are prefetched 64 ahead (an aggregated node's row is never read)
        constexpr int32_t kAhead = 64;
        for (int32_t i = r0; i < r1; ++i) {
            if (i + kAhead < r1) {
                const int32_t ib = i + kAhead;
                if (!is_taken(ib)) __builtin_prefetch(sj + (si[ib] - sj0), 0, 3);
            }
            if (!is_taken(i) && si[i] != si[i + 1]) visit(i);
        }
        return na;
    }
    // With `head` (each row's first columns, the lowest: settled, mostly
    // taken -- at 300^3's level 1 they rule out 89 % of the free nodes), a
    // look-ahead kLook nodes in front of the pass drops every node that is
    // already taken or has a taken head column, and queues the rest with
    // their rows prefetched; the pass visits only the queue, in order. Exact:
    // a node only ever becomes taken, so what the look-ahead drops the pass
    // would drop too, and each queued node is tested in full at its turn.
    // (Host benchmark of that S: 85-91 ms plain, 55-62 ms this way.)
    constexpr int32_t kLook = 32, kQueue = 64;  // kQueue > kLook + 1, a power of two
    auto head_free = [head, &is_taken](int32_t i) {
        const int32_t *h = head + (size_t)i * kPhase1Head;
        bool f = true;
        for (int t = 0; t < kPhase1Head; ++t) f &= !is_taken(h[t]);
        return f;
    };
    int32_t queue[kQueue];
    uint32_t qh = 0, qt = 0;
    for (int32_t ib = r0; ib < r1; ++ib) {
        if (!is_taken(ib) && si[ib] != si[ib + 1] && head_free(ib)) {
            queue[qt++ & (kQueue - 1)] = ib;
            __builtin_prefetch(sj + (si[ib] - sj0), 0, 3);
        }
        while (qh != qt && queue[qh & (kQueue - 1)] <= ib - kLook) {
            const int32_t i = queue[qh++ & (kQueue - 1)];
            if (!is_taken(i)) visit(i);
        }
    }
    while (qh != qt) {
        const int32_t i = queue[qh++ & (kQueue - 1)];
        if (!is_taken(i)) visit(i);
    }
    return na;
}

int32_t aggregate_mis(int32_t m, const int32_t *si, const int32_t *sj, bool square, int32_t level, int32_t *agg) {
    // the visiting order: ascending key (the key's low half is the node)
    std::vector<uint64_t> order((size_t)m);
    for (int32_t i = 0; i < m; ++i) order[i] = mis_key(i, level);
    std::sort(order.begin(), order.end());
    enum : int8_t { kNotDone = 0, kDeleted = 1, kSelected = 2, kRemoved = 3 };
    std::vector<int8_t> state((size_t)m, kNotDone);
    std::vector<int32_t> parent((size_t)m, -1);
    for (const uint64_t key : order) {
        const int32_t r = (int32_t)(uint32_t)key;
        if (state[r] != kNotDone) continue;
        if (si[r] == si[r + 1]) {  // G2 row = {r}: a singleton, removed
            state[r] = kRemoved;
            continue;
        }
        state[r] = kSelected;
        parent[r] = r;
        auto take = [&](int32_t j) {
            if (state[j] == kNotDone) {
                state[j] = kDeleted;
                parent[j] = r;
            }
        };
        for (int32_t a = si[r]; a < si[r + 1]; ++a) {  // G2 = G1 o G1, G1 = S + I
            const int32_t u = sj[a];
            take(u);
            if (square)
                for (int32_t b = si[u]; b < si[u + 1]; ++b) take(sj[b]);
        }
    }
    if (square)  // smoothAggs
        for (int32_t r = 0; r < m; ++r) {
            if (state[r] != kSelected) continue;
            for (int32_t a = si[r]; a < si[r + 1]; ++a) {
                const int32_t j = sj[a];
                if (state[j] == kDeleted && parent[j] != r) parent[j] = r;
            }
        }
    std::vector<int32_t> cidx((size_t)m, -1);
    int32_t na = 0;
    for (int32_t i = 0; i < m; ++i)
        if (state[i] == kSelected) cidx[i] = na++;
    for (int32_t i = 0; i < m; ++i) agg[i] = parent[i] >= 0 ? cidx[parent[i]] : -1;
    return na;
}

double tridiag_max_eig(const std::vector<double> &d, const std::vector<double> &e) {
    const size_t n = d.size();
    double lo = d[0], hi = d[0];
    for (size_t k = 0; k < n; ++k) {
        const double r = (k > 0 ? std::fabs(e[k - 1]) : 0.0) + (k + 1 < n ? std::fabs(e[k]) : 0.0);
        lo = std::min(lo, d[k] - r);
        hi = std::max(hi, d[k] + r);
    }
    auto below = [&](double x) {  // Sturm count of eigenvalues < x
        size_t c = 0;
        double q = 1.0;
        for (size_t k = 0; k < n; ++k) {
            q = (d[k] - x) - (k > 0 ? (e[k - 1] * e[k - 1]) / q : 0.0);
            if (q == 0.0) q = -1e-300;
            if (q < 0.0) ++c;
        }
        return c;
    };
    for (int it = 0; it < 200; ++it) {
        const double mid = 0.5 * (lo + hi);
        if (!(lo < mid && mid < hi)) break;
        if (below(mid) >= n) hi = mid;
        else lo = mid;
    }
    return hi;
}

double lanczos_emax(const std::vector<double> &alpha, const std::vector<double> &beta) {
    const size_t n = alpha.size();
    std::vector<double> d(n), e(n > 0 ? n - 1 : 0);
    d[0] = 1.0 / alpha[0];
    for (size_t k = 1; k < n; ++k) d[k] = 1.0 / alpha[k] + beta[k - 1] / alpha[k - 1];
    for (size_t k = 0; k + 1 < n; ++k) e[k] = std::sqrt(std::fabs(beta[k])) / alpha[k];
    return tridiag_max_eig(d, e);
}

int32_t aggregate_phase1(int32_t m, const int32_t *si, const int32_t *sj, int32_t *agg) {
    std::fill(agg, agg + m, -1);
    std::vector<uint64_t> taken(((size_t)m + 63) / 64, 0);
    return aggregate_phase1_rows(0, m, si, sj, agg, taken.data(), 0);
}

int32_t aggregate_phase3(int32_t m, const int32_t *si, const int32_t *sj, int32_t *agg, int32_t na) {
    for (int32_t i = 0; i < m; ++i) {
        if (agg[i] != -1) continue;
        agg[i] = na;
        for (int32_t k = si[i]; k < si[i + 1]; ++k)
            if (agg[sj[k]] == -1) agg[sj[k]] = na;
        ++na;
    }
    return na;
}

}  // namespace aijhip_gamg

struct aijhip_gamg_host {
    std::vector<int32_t> m;          // rows per level
    std::vector<int64_t> nnz_a;
    std::vector<CSR> A;              // A[0] unused (the input); A[l], l >= 1
    std::vector<CSR> P;              // P[l]: m[l] x m[l+1]
    std::vector<std::vector<int32_t>> agg;
    std::vector<double> emax;
};

extern "C" {

int aijhip_gamg_params_default(aijhip_gamg_params_t *p) {
    if (!p) return AIJHIP_ERR_ARG;
    p->threshold = 0.0;
    p->coarse_eq_limit = 50;
    p->max_levels = 10;
    p->nsmooths = 1;
    p->smooth_scale = 1.4;
    p->eig_its = 10;
    p->threads = 0;
    p->device_min_rows = 20000;
    p->coarsen = 1;  // PETSc 3.7 agg's MIS (round 5: faster to solution than greedy)
    p->square_graph = 1;
    p->eig_ksp = 1;
    p->pad0 = 0;
    return AIJHIP_OK;
}

int aijhip_gamg_build_host(int32_t m, const int32_t *ai, const int32_t *aj, const double *aa,
                           const aijhip_gamg_params_t *pp, aijhip_gamg_host_t *out) {
    aijhip_gamg_params_t p;
    aijhip_gamg_params_default(&p);
    if (pp) p = *pp;
    return aijhip_gamg::build_host_nns(m, ai, aj, aa, nullptr, p, out);
}

}  // extern "C"

int aijhip_gamg::build_host_nns(int32_t m, const int32_t *ai, const int32_t *aj, const double *aa, const double *B0,
                                const aijhip_gamg_params_t &p, aijhip_gamg_host_t *out, int32_t level0) {
    if (!out || m < 0 || !ai || (ai[m] > 0 && (!aj || !aa))) return AIJHIP_ERR_ARG;
    *out = nullptr;
    if (p.max_levels < 1) return AIJHIP_ERR_ARG;
    const int nt = nthreads(p.threads);
    aijhip_gamg_host *H = new (std::nothrow) aijhip_gamg_host();
    if (!H) return AIJHIP_ERR_ALLOC;
    try {
        H->m.push_back(m);
        H->nnz_a.push_back(ai[m]);
        H->A.emplace_back();
        // near-null space: the constant vector of the scalar operator, or
        // the one the levels above handed down
        std::vector<double> B = B0 ? std::vector<double>(B0, B0 + m) : std::vector<double>(m, 1.0);
        View cur{m, m, ai, aj, aa};
        const bool log = std::getenv("AIJHIP_GAMG_LOG") != nullptr;
        double t0 = wtime();
        auto lap = [&](const char *what) {
            if (!log) return;
            const double t = wtime();
            std::fprintf(stderr, "gamg level %zu %-12s %8.3f s\n", H->m.size() - 1, what, t - t0);
            t0 = t;
        };
        while ((int32_t)H->m.size() < p.max_levels && cur.m > p.coarse_eq_limit) {
            const std::vector<double> d = diagonal(cur, nt);
            std::vector<double> dinv(cur.m);
            for (int32_t i = 0; i < cur.m; ++i) dinv[i] = 1.0 / (d[i] == 0.0 ? 1.0 : d[i]);
            std::vector<int32_t> si, sj, agg;
            lap("diagonal");
            strength_graph(cur, d, p.threshold, si, sj, nt);
            lap("strength");
            const int32_t level = level0 + (int32_t)H->P.size();
            int32_t na;
            if (p.coarsen == 1) {
                agg.resize(cur.m);
                na = aijhip_gamg::aggregate_mis(cur.m, si.data(), sj.data(), level < p.square_graph, level,
                                                agg.data());
            } else {
                na = aggregate(cur, si, sj, agg);
            }
            lap("aggregate");
            if (na >= cur.m || na == 0) break;  // no coarsening
            const double emax = p.nsmooths <= 0 ? 1.0
                                : p.eig_ksp == 1 ? estimate_emax_cg(cur, dinv, p.eig_its, nt)
                                                 : estimate_emax(cur, dinv, p.eig_its, nt);
            lap("emax");
            CSR P;
            std::vector<double> Bc;
            prolongator(cur, dinv, agg, na, B, -p.smooth_scale / emax, p.nsmooths, P, Bc, nt);
            lap("prolongator");
            CSR AP, PT, Ac;
            spgemm(cur, view(P), AP, nt);
            lap("A*P");
            transpose(view(P), PT, nt);
            lap("P^T");
            spgemm(view(PT), view(AP), Ac, nt);
            lap("P^T*(AP)");
            H->P.push_back(std::move(P));
            H->agg.push_back(std::move(agg));
            H->emax.push_back(emax);
            H->m.push_back(Ac.m);
            H->nnz_a.push_back(Ac.nnz());
            H->A.push_back(std::move(Ac));
            B.swap(Bc);
            cur = view(H->A.back());
        }
    } catch (const std::bad_alloc &) {
        delete H;
        return AIJHIP_ERR_ALLOC;
    } catch (const std::exception &) {
        delete H;
        return AIJHIP_ERR_ARG;
    }
    *out = H;
    return AIJHIP_OK;
}

extern "C" {

int aijhip_gamg_host_num_levels(aijhip_gamg_host_t h, int32_t *n) {
    if (!h || !n) return AIJHIP_ERR_ARG;
    *n = (int32_t)h->m.size();
    return AIJHIP_OK;
}

int aijhip_gamg_host_level_info(aijhip_gamg_host_t h, int32_t l, int32_t *m, int64_t *nnz_a, int64_t *nnz_p,
                                double *emax) {
    if (!h || l < 0 || l >= (int32_t)h->m.size()) return AIJHIP_ERR_ARG;
    if (m) *m = h->m[l];
    if (nnz_a) *nnz_a = h->nnz_a[l];
    const bool hasp = l < (int32_t)h->P.size();
    if (nnz_p) *nnz_p = hasp ? h->P[l].nnz() : 0;
    if (emax) *emax = hasp ? h->emax[l] : 0.0;
    return AIJHIP_OK;
}

int aijhip_gamg_host_get_A(aijhip_gamg_host_t h, int32_t l, int32_t *ai, int32_t *aj, double *aa) {
    if (!h || l < 1 || l >= (int32_t)h->m.size() || !ai) return AIJHIP_ERR_ARG;
    const CSR &c = h->A[l];
    std::copy(c.ai.begin(), c.ai.end(), ai);
    if (aj) std::copy(c.aj.begin(), c.aj.end(), aj);
    if (aa) std::copy(c.aa.begin(), c.aa.end(), aa);
    return AIJHIP_OK;
}

int aijhip_gamg_host_get_P(aijhip_gamg_host_t h, int32_t l, int32_t *ai, int32_t *aj, double *aa) {
    if (!h || l < 0 || l >= (int32_t)h->P.size() || !ai) return AIJHIP_ERR_ARG;
    const CSR &c = h->P[l];
    std::copy(c.ai.begin(), c.ai.end(), ai);
    if (aj) std::copy(c.aj.begin(), c.aj.end(), aj);
    if (aa) std::copy(c.aa.begin(), c.aa.end(), aa);
    return AIJHIP_OK;
}

int aijhip_gamg_host_get_aggregates(aijhip_gamg_host_t h, int32_t l, int32_t *agg) {
    if (!h || l < 0 || l >= (int32_t)h->agg.size() || !agg) return AIJHIP_ERR_ARG;
    std::copy(h->agg[l].begin(), h->agg[l].end(), agg);
    return AIJHIP_OK;
}

int aijhip_gamg_host_view(aijhip_gamg_host_t h, int32_t l, char which, const int32_t **ai, const int32_t **aj,
                          const double **aa) {
    if (!h || !ai || !aj || !aa || l < 0) return AIJHIP_ERR_ARG;
    const CSR *c = nullptr;
    if (which == 'A' && l >= 1 && l < (int32_t)h->A.size()) c = &h->A[l];
    if (which == 'P' && l < (int32_t)h->P.size()) c = &h->P[l];
    if (!c) return AIJHIP_ERR_ARG;
    *ai = c->ai.data();
    *aj = c->aj.data();
    *aa = c->aa.data();
    return AIJHIP_OK;
}

int aijhip_gamg_host_destroy(aijhip_gamg_host_t h) {
    delete h;
    return AIJHIP_OK;
}

}  // extern "C"
