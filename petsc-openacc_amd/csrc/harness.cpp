// harness.cpp — operand producers for the SpMV path (include/aijhip_harness.h).
// Restates /root/reference/src/helper.cpp on the host, directly into CSR
// (no DMDA, no MatSetValues), slab by slab. Not the hot path.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <algorithm>
#include <vector>

#include "aijhip.h"
#include "aijhip_harness.h"
#include "poisson_grid.h"

namespace {

using namespace aijhip_poisson;

inline uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
inline uint64_t rnd(uint64_t seed, uint64_t stream, uint64_t idx) {
    return mix64(seed + stream * 0xD1B54A32D192ED03ULL + (idx + 1) * 0x9E3779B97F4A7C15ULL);
}
inline double unit(uint64_t z) { return (double)(z >> 11) * (1.0 / 9007199254740992.0); }

// Skewed stand-in. Flan_1565 is a 3-D hexahedral FEM model with 3 dofs per
// node, so a row's columns come in runs of 3 (one per neighbouring node's
// dofs): ordinary rows couple 15..33 nodes (45..99 entries, mean 72 ~ Flan's
// 114.2M / 1.565M) within a band of +-kBandNodes nodes; a 1e-4 fraction of
// hub rows (log-uniform 1e3..2e5 scattered entries) stresses load balance.
constexpr int32_t kBandNodes = 700;
inline bool skew_is_hub(int32_t r, uint64_t seed) { return rnd(seed, 1, (uint64_t)r) % 10000 == 0; }
inline void skew_band(int32_t r, int32_t m, int64_t *lo, int64_t *hi) {
    const int64_t nn = m / 3, node = std::min<int64_t>((int64_t)r / 3, std::max<int64_t>(nn - 1, 0));
    *lo = std::max<int64_t>(0, node - kBandNodes);
    *hi = std::min<int64_t>(nn, node + kBandNodes + 1);
}
inline int32_t skew_len(int32_t r, int32_t m, uint64_t seed) {
    if (skew_is_hub(r, seed)) {
        const int64_t L = (int64_t)(1000.0 * std::pow(200.0, unit(rnd(seed, 2, (uint64_t)r))));
        return (int32_t)std::min<int64_t>(L, m);
    }
    int64_t lo, hi;
    skew_band(r, m, &lo, &hi);
    const int64_t nodes = 15 + (int64_t)((rnd(seed, 1, (uint64_t)r) >> 20) % 19);
    return (int32_t)(3 * std::min<int64_t>(nodes, hi - lo));
}

}  // namespace

extern "C" {

int aijhip_poisson_nnz(int32_t nx, int32_t ny, int32_t nz, int32_t z0, int32_t z1, int64_t *nnz) {
    Grid g;
    if (!nnz || make_grid(nx, ny, nz, z0, z1, &g)) return AIJHIP_ERR_ARG;
    // per row 1 + (#in-domain neighbours); separable over the three axes
    const int64_t rows = (int64_t)(z1 - z0) * g.nxy;
    int64_t nb_x = 2 * (int64_t)(nx - 1) * ny;  // x-neighbour entries per plane
    int64_t nb_y = 2 * (int64_t)(ny - 1) * nx;
    int64_t total = rows + (int64_t)(z1 - z0) * (nb_x + nb_y);
    for (int32_t k = z0; k < z1; ++k) total += g.nxy * ((k > 0) + (k < nz - 1));
    *nnz = total;
    return AIJHIP_OK;
}

int aijhip_poisson_fill(int32_t nx, int32_t ny, int32_t nz, int32_t z0, int32_t z1, int ref_point,
                        int32_t *ai, int32_t *aj, double *aa, double *scale) {
    Grid g;
    if (!ai || make_grid(nx, ny, nz, z0, z1, &g)) return AIJHIP_ERR_ARG;
    if (z1 > z0 && (!aj || !aa)) return AIJHIP_ERR_ARG;  // an empty slab needs only ai
    const int64_t row0 = (int64_t)z0 * g.nxy;
    int64_t p = 0;
    int64_t lr = 0;
    ai[0] = 0;
    // helper.cpp:198-240, natural ordering; SeqAIJ keeps each row's columns
    // sorted, so the stencil is stored as k-1, j-1, i-1, c, i+1, j+1, k+1.
    for (int32_t k = z0; k < z1; ++k)
        for (int32_t j = 0; j < ny; ++j)
            for (int32_t i = 0; i < nx; ++i) {
                const int64_t r = i + (int64_t)nx * (j + (int64_t)ny * k);
                if (k > 0) { aj[p] = (int32_t)(r - g.nxy); aa[p++] = g.vz; }
                if (j > 0) { aj[p] = (int32_t)(r - nx); aa[p++] = g.vy; }
                if (i > 0) { aj[p] = (int32_t)(r - 1); aa[p++] = g.vx; }
                aj[p] = (int32_t)r; aa[p++] = diag_value(g, i, j, k);
                if (i < nx - 1) { aj[p] = (int32_t)(r + 1); aa[p++] = g.vx; }
                if (j < ny - 1) { aj[p] = (int32_t)(r + nx); aa[p++] = g.vy; }
                if (k < nz - 1) { aj[p] = (int32_t)(r + g.nxy); aa[p++] = g.vz; }
                ai[++lr] = (int32_t)p;
            }
    double sc = 0.0;
    if (ref_point) {
        // setRefPoint, helper.cpp:250-279: MatZeroRowsColumns(A,1,{0},scale,...)
        // zeroes row 0 and column 0, keeping the entries as explicit zeros,
        // and sets a_00 = scale.
        sc = ref_scale(g);
        const int64_t mloc = (int64_t)(z1 - z0) * g.nxy;
        const int64_t cand[3] = {1, (int64_t)nx, g.nxy};
        for (int64_t c : cand) {
            const int64_t l = c - row0;
            if (c >= g.m || l < 0 || l >= mloc) continue;
            for (int32_t q = ai[l]; q < ai[l + 1]; ++q)
                if (aj[q] == 0) aa[q] = 0.0;
        }
        if (row0 == 0 && mloc > 0)
            for (int32_t q = ai[0]; q < ai[1]; ++q) aa[q] = (aj[q] == 0) ? sc : 0.0;
    }
    if (scale) *scale = sc;
    return AIJHIP_OK;
}

int aijhip_poisson_vectors(int32_t nx, int32_t ny, int32_t nz, int32_t z0, int32_t z1, int ref_point,
                           double *rhs, double *exact) {
    Grid g;
    if (make_grid(nx, ny, nz, z0, z1, &g)) return AIJHIP_ERR_ARG;
    const double dx = kL / nx, dy = kL / ny, dz = kL / nz;
    std::vector<double> cx(nx), cy(ny), cz(nz);
    for (int32_t i = 0; i < nx; ++i) cx[i] = cfac(i, dx);
    for (int32_t j = 0; j < ny; ++j) cy[j] = cfac(j, dy);
    for (int32_t k = 0; k < nz; ++k) cz[k] = cfac(k, dz);
    int64_t p = 0;
    for (int32_t k = z0; k < z1; ++k)
        for (int32_t j = 0; j < ny; ++j)
            for (int32_t i = 0; i < nx; ++i, ++p) {
                // helper.cpp:107-110 (c2 expanded textually) and :148-151
                if (rhs) rhs[p] = -3.0 * 2.0 * 1.0 * M_PI * 2.0 * 1.0 * M_PI * cx[i] * cy[j] * cz[k];
                if (exact) exact[p] = cx[i] * cy[j] * cz[k];
            }
    if (ref_point && rhs) {
        const int64_t row0 = (int64_t)z0 * g.nxy, mloc = (int64_t)(z1 - z0) * g.nxy;
        const double ex0 = cx[0] * cy[0] * cz[0];
        // rows holding column 0: b_i -= a_i0 * exact_0 (MatZeroRowsColumns [ext])
        const int64_t cand[3] = {1, (int64_t)nx, g.nxy};
        const double coef[3] = {g.vx, g.vy, g.vz};
        for (int q = 0; q < 3; ++q) {
            const int64_t c = cand[q];
            if (c >= g.m || c - row0 < 0 || c - row0 >= mloc) continue;
            if (q == 0 && nx < 2) continue;
            if (q == 1 && ny < 2) continue;
            if (q == 2 && nz < 2) continue;
            rhs[c - row0] -= coef[q] * ex0;
        }
        if (row0 == 0 && mloc > 0) rhs[0] = ref_scale(g) * ex0;
    }
    return AIJHIP_OK;
}

void aijhip_splitmix_uniform(int64_t n, uint64_t seed, int64_t offset, double *x) {
    for (int64_t i = 0; i < n; ++i) {
        const uint64_t z = mix64(seed + (uint64_t)(offset + i + 1) * 0x9E3779B97F4A7C15ULL);
        x[i] = 2.0 * unit(z) - 1.0;
    }
}

int aijhip_skewed_csr(int32_t m, uint64_t seed, int64_t *nnz, int32_t *ai, int32_t *aj, double *aa) {
    if (m < 0 || !nnz) return AIJHIP_ERR_ARG;
    int64_t total = 0;
    for (int32_t r = 0; r < m; ++r) total += skew_len(r, m, seed);
    if (total > INT32_MAX) return AIJHIP_ERR_ARG;
    *nnz = total;
    if (!ai) return AIJHIP_OK;
    if (!aj || !aa) return AIJHIP_ERR_ARG;
    int64_t p = 0;
    ai[0] = 0;
    for (int32_t r = 0; r < m; ++r) {
        const int32_t L = skew_len(r, m, seed);
        if (skew_is_hub(r, seed)) {
            // one distinct column per bucket [q*m/L, (q+1)*m/L): sorted, unique
            for (int32_t q = 0; q < L; ++q) {
                const int64_t b0 = (int64_t)q * m / L, b1 = (int64_t)(q + 1) * m / L;
                aj[p] = (int32_t)(b0 + (int64_t)(rnd(seed, 4, (uint64_t)p) % (uint64_t)(b1 - b0)));
                aa[p] = 2.0 * unit(rnd(seed, 3, (uint64_t)p)) - 1.0;
                ++p;
            }
        } else {
            int64_t lo, hi;
            skew_band(r, m, &lo, &hi);
            const int64_t W = hi - lo, nodes = L / 3;
            // one node per bucket of the node band, its 3 dofs consecutive
            for (int64_t q = 0; q < nodes; ++q) {
                const int64_t b0 = lo + q * W / nodes, b1 = lo + (q + 1) * W / nodes;
                const int64_t node = b0 + (int64_t)(rnd(seed, 4, (uint64_t)p) % (uint64_t)(b1 - b0));
                for (int d = 0; d < 3; ++d) {
                    aj[p] = (int32_t)(3 * node + d);
                    aa[p] = 2.0 * unit(rnd(seed, 3, (uint64_t)p)) - 1.0;
                    ++p;
                }
            }
        }
        ai[r + 1] = (int32_t)p;
    }
    return AIJHIP_OK;
}

int aijhip_fem_hex_csr(int32_t nx, int32_t ny, int32_t nz, int32_t dofs, uint64_t seed, int64_t *nnz,
                       int32_t *ai, int32_t *aj, double *aa) {
    if (nx < 1 || ny < 1 || nz < 1 || dofs < 1 || !nnz) return AIJHIP_ERR_ARG;
    // couplings per axis: 3 neighbours inside, 2 at a face (1 on a 1-wide axis)
    auto pairs = [](int64_t n) { return n == 1 ? (int64_t)1 : 3 * n - 2; };
    const int64_t nodes = (int64_t)nx * ny * nz, m = nodes * dofs;
    const int64_t total = pairs(nx) * pairs(ny) * pairs(nz) * dofs * dofs;
    if (m > INT32_MAX || total > INT32_MAX) return AIJHIP_ERR_ARG;
    *nnz = total;
    if (!ai) return AIJHIP_OK;
    if (!aj || !aa) return AIJHIP_ERR_ARG;
    int64_t p = 0, r = 0;
    ai[0] = 0;
    for (int32_t k = 0; k < nz; ++k)
        for (int32_t j = 0; j < ny; ++j)
            for (int32_t i = 0; i < nx; ++i)
                for (int32_t d = 0; d < dofs; ++d) {
                    // the 27 neighbouring nodes in ascending node order, all
                    // their dofs: the row's columns come out sorted
                    for (int32_t dk = -1; dk <= 1; ++dk) {
                        if (k + dk < 0 || k + dk >= nz) continue;
                        for (int32_t dj = -1; dj <= 1; ++dj) {
                            if (j + dj < 0 || j + dj >= ny) continue;
                            for (int32_t di = -1; di <= 1; ++di) {
                                if (i + di < 0 || i + di >= nx) continue;
                                const int64_t node = (i + di) + (int64_t)nx * ((j + dj) + (int64_t)ny * (k + dk));
                                for (int32_t e = 0; e < dofs; ++e, ++p) {
                                    aj[p] = (int32_t)(node * dofs + e);
                                    aa[p] = 2.0 * unit(rnd(seed, 5, (uint64_t)p)) - 1.0;
                                }
                            }
                        }
                    }
                    ai[++r] = (int32_t)p;
                }
    return AIJHIP_OK;
}

int aijhip_split_rows(int32_t m, const int32_t *ai, const int32_t *aj, const double *aa,
                      int32_t col_lo, int32_t col_hi, int64_t *nz_d, int64_t *nz_o,
                      int32_t *n_garray, int32_t *d_ai, int32_t *d_aj, double *d_aa,
                      int32_t *o_ai, int32_t *o_aj, double *o_aa, int32_t *garray) {
    if (m < 0 || !ai || !nz_d || !nz_o || !n_garray || col_lo > col_hi) return AIJHIP_ERR_ARG;
    std::vector<int32_t> g;
    int64_t cd = 0, co = 0;
    for (int64_t k = 0; k < ai[m]; ++k) {
        if (aj[k] >= col_lo && aj[k] < col_hi) ++cd;
        else { ++co; g.push_back(aj[k]); }
    }
    std::sort(g.begin(), g.end());
    g.erase(std::unique(g.begin(), g.end()), g.end());
    *nz_d = cd;
    *nz_o = co;
    *n_garray = (int32_t)g.size();
    if (!d_ai) return AIJHIP_OK;
    if (!o_ai || (cd && (!d_aj || !d_aa)) || (co && (!o_aj || !o_aa)) || (!g.empty() && !garray))
        return AIJHIP_ERR_ARG;
    std::copy(g.begin(), g.end(), garray);
    int64_t pd = 0, po = 0;
    d_ai[0] = 0;
    o_ai[0] = 0;
    for (int32_t i = 0; i < m; ++i) {
        for (int32_t k = ai[i]; k < ai[i + 1]; ++k) {
            const int32_t c = aj[k];
            if (c >= col_lo && c < col_hi) { d_aj[pd] = c - col_lo; d_aa[pd++] = aa[k]; }
            else {
                o_aj[po] = (int32_t)(std::lower_bound(g.begin(), g.end(), c) - g.begin());
                o_aa[po++] = aa[k];
            }
        }
        d_ai[i + 1] = (int32_t)pd;
        o_ai[i + 1] = (int32_t)po;
    }
    return AIJHIP_OK;
}

}  // extern "C"
