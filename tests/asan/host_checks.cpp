// Host-side code of the library under AddressSanitizer + UBSan (SURVEY.md §5:
// "run the fixtures under AddressSanitizer on the host path"): the operand
// producers (harness.cpp), the MPIAIJ row split, the host GAMG hierarchy
// (gamg_setup.cpp) and the oracle's C MatMult, on small inputs including
// ragged and degenerate ones. Built and run by tests/test_asan.py; exits
// non-zero on a failed check, the sanitizers abort on a memory error.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "aijhip.h"
#include "aijhip_gamg.h"
#include "aijhip_harness.h"
#include "gamg_internal.h"

extern "C" void oracle_matmult_seqaij(int32_t m, const int32_t *ai, const int32_t *aj, const double *aa,
                                      const double *x, double *y);

#define CHECK(c)                                                        \
    do {                                                                \
        if (!(c)) {                                                     \
            std::fprintf(stderr, "check failed: %s (line %d)\n", #c, __LINE__); \
            std::exit(1);                                               \
        }                                                               \
    } while (0)

static void poisson_case(int nx, int ny, int nz, int z0, int z1) {
    int64_t nnz = 0;
    CHECK(aijhip_poisson_nnz(nx, ny, nz, z0, z1, &nnz) == AIJHIP_OK);
    const int64_t m = (int64_t)nx * ny * (z1 - z0);
    std::vector<int32_t> ai(m + 1), aj(nnz);
    const int64_t n = (int64_t)nx * ny * nz;  // columns are global
    std::vector<double> aa(nnz), rhs(m), ex(m), x(n), y(m);
    double sc = 0.0;
    CHECK(aijhip_poisson_fill(nx, ny, nz, z0, z1, 1, ai.data(), aj.data(), aa.data(), &sc) == AIJHIP_OK);
    CHECK(ai[m] == nnz);
    CHECK(aijhip_poisson_vectors(nx, ny, nz, z0, z1, 1, rhs.data(), ex.data()) == AIJHIP_OK);
    aijhip_splitmix_uniform(n, 42, 0, x.data());
    oracle_matmult_seqaij((int32_t)m, ai.data(), aj.data(), aa.data(), x.data(), y.data());
    // MPIAIJ split of the slab's rows (columns outside the slab go off-diagonal)
    const int32_t lo = z0 * nx * ny, hi = z1 * nx * ny;
    int64_t nzd = 0, nzo = 0;
    int32_t ng = 0;
    CHECK(aijhip_split_rows((int32_t)m, ai.data(), aj.data(), aa.data(), lo, hi, &nzd, &nzo, &ng, nullptr, nullptr,
                            nullptr, nullptr, nullptr, nullptr, nullptr) == AIJHIP_OK);
    CHECK(nzd + nzo == nnz);
    std::vector<int32_t> dai(m + 1), daj(nzd + 1), oai(m + 1), oaj(nzo + 1), garray(ng + 1);
    std::vector<double> daa(nzd + 1), oaa(nzo + 1);
    CHECK(aijhip_split_rows((int32_t)m, ai.data(), aj.data(), aa.data(), lo, hi, &nzd, &nzo, &ng, dai.data(),
                            daj.data(), daa.data(), oai.data(), oaj.data(), oaa.data(), garray.data()) == AIJHIP_OK);
}

static void gamg_case(int n, int threads) {
    int64_t nnz = 0;
    CHECK(aijhip_poisson_nnz(n, n, n, 0, n, &nnz) == AIJHIP_OK);
    const int64_t m = (int64_t)n * n * n;
    std::vector<int32_t> ai(m + 1), aj(nnz);
    std::vector<double> aa(nnz);
    CHECK(aijhip_poisson_fill(n, n, n, 0, n, 1, ai.data(), aj.data(), aa.data(), nullptr) == AIJHIP_OK);
    aijhip_gamg_params_t p;
    aijhip_gamg_params_default(&p);
    p.coarse_eq_limit = 10;
    p.threads = threads;
    aijhip_gamg_host_t h = nullptr;
    CHECK(aijhip_gamg_build_host((int32_t)m, ai.data(), aj.data(), aa.data(), &p, &h) == AIJHIP_OK);
    int32_t nl = 0;
    CHECK(aijhip_gamg_host_num_levels(h, &nl) == AIJHIP_OK && nl >= 2);
    int32_t prev = (int32_t)m;
    for (int32_t l = 0; l < nl; ++l) {
        int32_t ml = 0;
        int64_t na = 0, np = 0;
        double emax = 0.0;
        CHECK(aijhip_gamg_host_level_info(h, l, &ml, &na, &np, &emax) == AIJHIP_OK);
        CHECK(l == 0 || ml < prev);
        prev = ml;
        if (l + 1 < nl) {
            std::vector<int32_t> pi(ml + 1), pj(np + 1), agg(ml);
            std::vector<double> pa(np + 1);
            CHECK(aijhip_gamg_host_get_P(h, l, pi.data(), pj.data(), pa.data()) == AIJHIP_OK);
            CHECK(aijhip_gamg_host_get_aggregates(h, l, agg.data()) == AIJHIP_OK);
            CHECK(emax > 0.0 && std::isfinite(emax));
        }
        if (l >= 1) {
            std::vector<int32_t> xi(ml + 1), xj(na + 1);
            std::vector<double> xa(na + 1);
            CHECK(aijhip_gamg_host_get_A(h, l, xi.data(), xj.data(), xa.data()) == AIJHIP_OK);
        }
    }
    CHECK(aijhip_gamg_host_level_info(h, nl, nullptr, nullptr, nullptr, nullptr) == AIJHIP_ERR_ARG);
    CHECK(aijhip_gamg_host_destroy(h) == AIJHIP_OK);
}

// The device set-up's host phase-1 pass (gamg_device.hip: S's rows arrive in
// chunks, each chunk's columns in a buffer of its own, with the dense head
// array of each row's first columns; the pass runs behind a look-ahead) gives
// the plain sequential pass's aggregates on random symmetric graphs with
// empty rows, for several chunk counts.
static void phase1_case(int32_t m, int deg, uint64_t seed, int chunks) {
    std::vector<std::vector<int32_t>> adj(m);
    uint64_t z = seed;
    auto next = [&z]() { z = z * 6364136223846793005ULL + 1442695040888963407ULL; return z >> 33; };
    for (int32_t i = 0; i < m; ++i) {
        if (next() % 7 == 0) continue;  // some rows stay empty unless a neighbour picks them
        const int d = (int)(next() % (uint64_t)(2 * deg + 1));
        for (int e = 0; e < d; ++e) {
            const int32_t span = 1 + (int32_t)(next() % 3 == 0 ? m : 40);
            int32_t j = i + (int32_t)(next() % (uint64_t)(2 * span + 1)) - span;
            if (j < 0 || j >= m || j == i) continue;
            adj[i].push_back(j);
            adj[j].push_back(i);
        }
    }
    std::vector<int32_t> si(m + 1, 0), sj;
    for (int32_t i = 0; i < m; ++i) {
        std::sort(adj[i].begin(), adj[i].end());
        adj[i].erase(std::unique(adj[i].begin(), adj[i].end()), adj[i].end());
        sj.insert(sj.end(), adj[i].begin(), adj[i].end());
        si[i + 1] = (int32_t)sj.size();
    }
    std::vector<int32_t> ref(m), agg(m, -1);
    const int32_t nref = aijhip_gamg::aggregate_phase1(m, si.data(), sj.data(), ref.data());
    constexpr int H = aijhip_gamg::kPhase1Head;
    std::vector<int32_t> head((size_t)m * H);
    for (int32_t i = 0; i < m; ++i)
        for (int t = 0; t < H; ++t) head[(size_t)i * H + t] = si[i] + t < si[i + 1] ? sj[si[i] + t] : i;
    std::vector<uint64_t> taken(((size_t)m + 63) / 64, 0);
    int32_t na = 0;
    for (int c = 0; c < chunks; ++c) {
        const int32_t r0 = (int32_t)((int64_t)m * c / chunks), r1 = (int32_t)((int64_t)m * (c + 1) / chunks);
        std::vector<int32_t> slot(sj.begin() + si[r0], sj.begin() + si[r1]);  // the chunk's own buffer
        na = aijhip_gamg::aggregate_phase1_rows(r0, r1, si.data(), slot.data(), agg.data(), taken.data(), na, si[r0],
                                                head.data());
    }
    CHECK(na == nref);
    CHECK(agg == ref);
    for (int32_t i = 0; i < m; ++i) CHECK(((taken[i >> 6] >> (i & 63)) & 1u) == (agg[i] != -1));
}

int main() {
    poisson_case(6, 5, 4, 0, 4);
    poisson_case(7, 3, 9, 2, 6);
    poisson_case(1, 1, 5, 0, 5);
    poisson_case(5, 5, 5, 4, 5);
    poisson_case(4, 4, 4, 2, 2);  // empty slab
    int64_t nnz = 0;
    CHECK(aijhip_skewed_csr(3000, 1565, &nnz, nullptr, nullptr, nullptr) == AIJHIP_OK);
    std::vector<int32_t> si(3001), sj(nnz);
    std::vector<double> sa(nnz);
    CHECK(aijhip_skewed_csr(3000, 1565, &nnz, si.data(), sj.data(), sa.data()) == AIJHIP_OK);
    phase1_case(5000, 6, 1, 1);
    phase1_case(5000, 6, 2, 7);
    phase1_case(20000, 15, 3, 32);
    phase1_case(300, 2, 4, 32);  // chunks shorter than the look-ahead
    phase1_case(1, 0, 5, 1);
    gamg_case(10, 1);
    gamg_case(9, 4);
    CHECK(aijhip_poisson_nnz(0, 3, 3, 0, 3, &nnz) == AIJHIP_ERR_ARG);
    std::puts("host checks ok");
    return 0;
}
