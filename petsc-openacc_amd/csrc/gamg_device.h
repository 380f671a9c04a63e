// gamg_device.h — the device-side smoothed-aggregation set-up
// (gamg_device.hip), used by the KSP set-up (ksp.hip).
#pragma once

#include <vector>

#include "aijhip_internal.h"
#include "gamg_internal.h"

namespace aijhip_gamg {

// One level of the device hierarchy.
struct DeviceLevel {
    aijhip_mat *A = nullptr;  // level operator (level 0: the caller's, borrowed)
    aijhip_mat *P = nullptr;  // prolongator to the next level, P^T attached
    double emax = 0.0;
    // the widest accumulator class the Galerkin products building P and
    // A_{l+1} needed: 0 = wavefront form, else 32 / 64 / 128 / 256 LDS columns
    int product_cols = 0;
};

// Device set-up: levels are built on the device while the level has at least
// p.device_min_rows rows; the greedy aggregation runs on the host from the
// device strength graph. On return `levels` holds every level built
// (levels[0].A = A0). *more is true when the hierarchy continues below the
// last level (too small for the device, or a Galerkin row beyond the device
// accumulators): B is then that level's near-null space for build_host_nns.
// *overflow is true when that hand-over happened at a level the device
// would otherwise have built (a product row past every device class).
int build_device(aijhip_mat *A0, const aijhip_gamg_params_t &p, std::vector<DeviceLevel> &levels,
                 std::vector<double> &B, bool *more, bool *overflow = nullptr);

void free_device_levels(std::vector<DeviceLevel> &levels);

// Aggregation phase 1 on the device (gamg_aggregate.hip), from the symmetric
// strength graph S (device CSR, rows sorted, unique, no diagonal): phase1[i]
// = the phase-1 aggregate of node i or -1, *na = their count, identical to
// aggregate_phase1. *done is false when the sweep needed more than
// max_rounds rounds (the caller then runs the host pass).
hipError_t aggregate_phase1_device(int32_t m, const int32_t *si, const int32_t *sj, int32_t max_rounds,
                                   int32_t *phase1, int32_t *na, int32_t *rounds, bool *done);
// Phase 3 for the nodes agg[] still has at -1 (aggregate_phase3 restricted to
// them): their S rows are gathered on the device, the sequential pass runs on
// the host, the result is scattered back. *na in: the count so far; out: the
// final count.
hipError_t aggregate_phase3_device(int32_t m, const int32_t *si, const int32_t *sj, int32_t *agg, int32_t *na);

}  // namespace aijhip_gamg
