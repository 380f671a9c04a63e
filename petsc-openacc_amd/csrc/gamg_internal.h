// gamg_internal.h — host pieces of the smoothed-aggregation set-up shared by
// the host builder (gamg_setup.cpp) and the device builder (gamg_device.hip,
// gamg_device.h).
#pragma once

#include <cstdint>
#include <vector>

#include "aijhip_gamg.h"

namespace aijhip_gamg {

// Greedy aggregation (gamg_setup.cpp aggregate) split around its parallel
// middle phase, from the symmetric strength graph S (rows sorted, unique):
// phase 1 roots aggregates at free nodes whose strong neighbours are all
// free (returns the aggregate count so far); phase 2 (device) joins each
// left-over node to its strongest stored phase-1 neighbour's aggregate;
// phase 3 roots aggregates at what is left (returns the final count).
int32_t aggregate_phase1(int32_t m, const int32_t *si, const int32_t *sj, int32_t *agg);
// The same pass over rows [r0, r1) (agg already holds rows < r0's result, -1
// elsewhere; taken: one bit per node, set exactly where agg != -1; na = the
// count so far): a node reads only its own row of S, so rows may arrive in
// order while earlier ones are processed.
// (sj holds S's columns from entry sj0 on: sj[k - sj0] is entry k)
// head (optional): each row's first kPhase1Head columns (padded with the row's
// own index), kPhase1Head per row from row 0; most free nodes meet a taken
// neighbour among them, so their rows of sj are never read.
constexpr int kPhase1Head = 4;
int32_t aggregate_phase1_rows(int32_t r0, int32_t r1, const int32_t *si, const int32_t *sj, int32_t *agg,
                              uint64_t *taken, int32_t na, int64_t sj0 = 0, const int32_t *head = nullptr);
int32_t aggregate_phase3(int32_t m, const int32_t *si, const int32_t *sj, int32_t *agg, int32_t na);

// PETSc 3.7 agg's MIS coarsening (coarsen 1; oracle/gamg.py aggregate_mis):
// nodes are visited in ascending mis_key order (a counter-based hash per
// node and level; PETSc's own shuffle uses its rand48 stream, not
// reproduced); an undone node with a neighbour in G2 becomes a root and takes
// every undone G2 neighbour; G1 = S + I, G2 = G1^2 when `square`, else G1; a
// node with no strong neighbour is removed (agg -1: a zero row of P0). With
// `square`, smoothAggs: the roots in natural order take every G1 neighbour
// sitting in another root's aggregate. Aggregates are numbered by their
// roots' index order. The device form (gamg_aggregate.hip
// aggregate_mis_device) gives the same aggregates, node for node.
constexpr uint64_t kMisSeed = 0x4D495332ULL;  // "MIS2"
#if defined(__HIPCC__)
__host__ __device__
#endif
inline uint64_t mis_key(int32_t i, int32_t level) {
    uint64_t z = kMisSeed + (uint64_t)level * 0x632BE59BD9B4E019ULL + (uint64_t)(i + 1) * 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    z ^= z >> 31;
    return ((z >> 32) << 32) | (uint32_t)i;
}
int32_t aggregate_mis(int32_t m, const int32_t *si, const int32_t *sj, bool square, int32_t level, int32_t *agg);

// emax of the symmetric tridiagonal (d[0..n), e[0..n-1)) by bisection from
// its Gershgorin bounds (oracle/gamg.py tridiag_max_eig: same steps, same bits).
double tridiag_max_eig(const std::vector<double> &d, const std::vector<double> &e);
// CG's Lanczos tridiagonal from its alphas / betas (oracle estimate_emax_cg):
// T_kk = 1/a_k + b_(k-1)/a_(k-1), T_(k+1)k = sqrt|b_k| / a_k; its emax.
double lanczos_emax(const std::vector<double> &alpha, const std::vector<double> &beta);

// Host continuation: the hierarchy below operator (m, ai, aj, aa) whose
// near-null space is B (NULL = ones), at most p.max_levels levels counting
// this one, which is level `level0` of the whole hierarchy (the MIS order
// and square_graph count levels from the finest).
int build_host_nns(int32_t m, const int32_t *ai, const int32_t *aj, const double *aa, const double *B,
                   const aijhip_gamg_params_t &p, aijhip_gamg_host_t *out, int32_t level0 = 0);

}  // namespace aijhip_gamg
