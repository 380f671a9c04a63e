// Host-side code of the library under AddressSanitizer + UBSan (SURVEY.md §5:
// "run the fixtures under AddressSanitizer on the host path"): the operand
// producers (harness.cpp), the MPIAIJ row split, the host GAMG hierarchy
// (gamg_setup.cpp) and the oracle's C MatMult, on small inputs including
// ragged and degenerate ones. Built and run by tests/test_asan.py; exits
// non-zero on a failed check, the sanitizers abort on a memory error.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "aijhip.h"
#include "aijhip_gamg.h"
#include "aijhip_harness.h"

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
    gamg_case(10, 1);
    gamg_case(9, 4);
    CHECK(aijhip_poisson_nnz(0, 3, 3, 0, 3, &nnz) == AIJHIP_ERR_ARG);
    std::puts("host checks ok");
    return 0;
}
