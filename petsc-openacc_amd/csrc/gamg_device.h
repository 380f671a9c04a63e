// gamg_device.h — the device-side smoothed-aggregation set-up
// (gamg_device.hip), used by the KSP set-up (ksp.hip).
#pragma once

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "aijhip_internal.h"
#include "gamg_internal.h"

namespace aijhip_gamg {

// Device CSR owned by a set-up (nz + 2 entries: the SpMV handles' tail pad).
struct DCsr {
    int32_t m = 0, n = 0;
    int64_t nz = 0;
    int32_t *ai = nullptr, *aj = nullptr;
    double *aa = nullptr;
    void release() {
        hipFree(ai); hipFree(aj); hipFree(aa);
        ai = aj = nullptr;
        aa = nullptr;
    }
};

template <class T>
hipError_t dalloc(T **p, int64_t count) {
    static const bool log = std::getenv("AIJHIP_GAMG_LOG") != nullptr;
    const size_t bytes = sizeof(T) * (size_t)std::max<int64_t>(count, 1);
    if (!log) return hipMalloc(reinterpret_cast<void **>(p), bytes);
    const auto t0 = std::chrono::steady_clock::now();
    const hipError_t e = hipMalloc(reinterpret_cast<void **>(p), bytes);
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (ms > 1.0) std::fprintf(stderr, "  slow hipMalloc %.1f MB: %.2f ms\n", bytes / 1e6, ms);
    return e;
}

// The set-up's process-wide streams (device, slot 0 or 1), created on first
// use and kept.
hipStream_t setup_stream(int device, int slot);

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

// The steps of one coarsening, shared by build_device and the distributed
// set-up (gamg_mpi.hip):
//  aggregate_level: D^-1, strength graph and aggregates of A's rows (device
//    agg ids in [0, *na)); with emax_its > 0 also emax(D^-1 A) of A itself
//    (the power iteration on a second host thread);
//  smooth_level: the tentative P0 from the near-null space B (Bc = the next
//    level's) and P = P0 + alpha D^-1 (A P0), columns = agg ids;
//  galerkin_level: A_c = P^T (A P) and P^T (ap_out: keep A P as well).
//    keep_S: the strength graph (S of A's rows, symmetric, no diagonal) and
//    the diagonal handed to the caller instead of aggregating (*d_agg NULL)
struct StrengthGraph {
    int32_t *si = nullptr, *sj = nullptr;
    int64_t nz = 0;
    double *d = nullptr;
};
int aggregate_level(aijhip_mat &A, const aijhip_gamg_params_t &p, int32_t **d_agg, int32_t *na, double **dinv,
                    int emax_its, double *emax, hipError_t *emax_err, size_t level, StrengthGraph *keep_S = nullptr);
int smooth_level(const DCsr &Av, int32_t na, int32_t *d_agg, const double *d_B, const double *dinv, double alpha,
                 int nsmooths, int n_cu, double **d_p0, double **d_Bc, DCsr &P, int *cols_used,
                 bool b_ones = false);  // b_ones: d_B is all 1.0 (the finest level's near-null space)
int galerkin_level(const DCsr &Av, const DCsr &P, DCsr &PT, DCsr &Ac, int n_cu, int *cols_used, DCsr *ap_out);
// A handle adopting C's arrays (C is emptied).
int make_level_handle(int device, DCsr &C, aijhip_mat **out);
// C = A B, the row-traversal product (scipy csr_matmat order).
int rowprod_device(const DCsr &A, const DCsr &B, DCsr &C, int n_cu, int *cols_used);
// The tentative prolongator's values: Bc[a] = ||B over aggregate a||, p0[i] =
// B[i] / Bc[agg[i]] (device arrays).
hipError_t tentative_device(int32_t m, int32_t na, const int32_t *agg, const double *B, double *Bc, double *p0,
                            bool b_ones = false);  // b_ones: B is all 1.0
// Per aggregate the sum of B_i^2 over its members (agg[i] in [0, na); -1
// not a member), in ascending member order: tentative_device's Bc before
// the square root (B == nullptr or b_ones: the member counts).
hipError_t aggregate_sumsq_device(int32_t m, int32_t na, const int32_t *agg, const double *B, double *s2,
                                  bool b_ones = false);
// P = P0 + alpha D^-1 T on the union pattern of T and P0 (P0: one entry per
// row, column agg[i], value p0[i]); T's columns may extend past the local
// aggregates (the distributed set-up's ghost coarse columns).
int prolong_from_T(const DCsr &T, const int32_t *d_agg, const double *d_p0, const double *dinv, double alpha,
                   DCsr &P);

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
// PETSc 3.7 agg's MIS aggregates (gamg_internal.h aggregate_mis, node for
// node) from the symmetric strength graph S: agg[0, m) in [-1, *na).
hipError_t aggregate_mis_device(int32_t m, const int32_t *si, const int32_t *sj, bool square, int32_t level,
                                int32_t *agg, int32_t *na, int32_t *rounds);

}  // namespace aijhip_gamg
