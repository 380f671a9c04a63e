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

// Host continuation: the hierarchy below operator (m, ai, aj, aa) whose
// near-null space is B (NULL = ones), at most p.max_levels levels counting
// this one.
int build_host_nns(int32_t m, const int32_t *ai, const int32_t *aj, const double *aa, const double *B,
                   const aijhip_gamg_params_t &p, aijhip_gamg_host_t *out);

}  // namespace aijhip_gamg
