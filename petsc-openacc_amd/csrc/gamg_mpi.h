// gamg_mpi.h — PCGAMG across ranks (gamg_mpi.hip), used by the distributed
// KSP (ksp_mpi.hip) for AIJHIP_PC_GAMG at more than one rank.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

#include "aijhip.h"
#include "aijhip_gamg.h"
#include "aijhip_mpi.h"

namespace aijhip_gamg_mpi {

// One level of the distributed hierarchy on this rank.
struct Level {
    int32_t m = 0;                 // own rows
    int64_t rstart = 0;            // first global row
    std::vector<int64_t> starts;   // ownership: rank q owns [starts[q], starts[q+1])
    aijhip_mat *Ad = nullptr;      // own columns
    aijhip_mat *Ao = nullptr;      // ghost columns (slots of op's ghost vector); may be NULL
    aijhip_mpiaij *op = nullptr;   // MatMult_MPIAIJ + the level's p2p halo (level 0: the caller's)
    std::vector<int64_t> ghost_gid;  // global row of every ghost slot
    // transfer to level l+1: P = [Pd | Po] (Po's columns: level l+1's ghost
    // slots); R = P^T as MatMultTranspose_MPIAIJ: Pd^T (attached to Pd) and
    // Po^T (attached to Po) whose ghost-slot sums go back to their owners
    // (Ro: unused since round 6, always NULL)
    aijhip_mat *Pd = nullptr, *Po = nullptr, *Ro = nullptr;
    double emax = 0.0;
    double *dinv = nullptr, *b = nullptr, *x = nullptr, *r = nullptr;
};

struct Hierarchy {
    std::vector<Level> lv;  // finest first
    void destroy();
};

// PCSetUp_GAMG over the distributed operator M0 (p2p halo). Collective.
int build(aijhip_mpiaij *M0, const aijhip_gamg_params_t &p, Hierarchy &H);
// This rank's rows of level l's operator ('A') or interpolation ('P') on the
// host, columns in the global numbering of their level (tests).
int get_level(const Hierarchy &H, int32_t l, char which, int64_t *rstart, int32_t *m, std::vector<int64_t> &ai,
              std::vector<int64_t> &aj, std::vector<double> &aa);
// One multiplicative V-cycle x = B b on `s` (every halo exchange is issued on
// every rank whatever the stop flag says; the kernels return at once past it).
int vcycle(Hierarchy &H, const double *b, double *x, hipStream_t s, const int *stop);

}  // namespace aijhip_gamg_mpi
