// poisson_grid.h — the grid constants of /root/reference/src/helper.cpp
// shared by the host operand producer (harness.cpp) and the device assembly
// (poisson.hip), so both compute bit-identical values.
#pragma once

#include <cmath>
#include <cstdint>

#include "aijhip.h"

namespace aijhip_poisson {

// helper.cpp:14-18. The macros are textual; c1*(i+0.5)*dx and
// c2*cos*cos*cos below are written out so they round exactly as the
// expanded reference expressions do (left to right).
constexpr double kL = 1.0;

inline double cfac(int32_t i, double d) { return std::cos(2.0 * 1.0 * M_PI * (i + 0.5) * d); }

struct Grid {
    int32_t nx, ny, nz;
    int64_t nxy, m;
    double vx, vy, vz;  // 1/dx^2, 1/dy^2, 1/dz^2 (helper.cpp:193-195)
};

inline int make_grid(int32_t nx, int32_t ny, int32_t nz, int32_t z0, int32_t z1, Grid *g) {
    if (nx <= 0 || ny <= 0 || nz <= 0 || z0 < 0 || z1 > nz || z0 > z1) return AIJHIP_ERR_ARG;
    const int64_t m = (int64_t)nx * ny * nz;
    if (m > INT32_MAX) return AIJHIP_ERR_ARG;  // PetscInt is int32 in the reference build
    g->nx = nx; g->ny = ny; g->nz = nz;
    g->nxy = (int64_t)nx * ny;
    g->m = m;
    const double dx = kL / nx, dy = kL / ny, dz = kL / nz;  // helper.cpp:188-190
    g->vx = 1.0 / (dx * dx);
    g->vy = 1.0 / (dy * dy);
    g->vz = 1.0 / (dz * dz);
    return AIJHIP_OK;
}

// Diagonal of cell (i,j,k): values[0] = 0; values[0] -= values[idx] for the
// in-domain neighbours in stencil order i-1, i+1, j-1, j+1, k-1, k+1
// (helper.cpp:229-233).
inline double diag_value(const Grid &g, int32_t i, int32_t j, int32_t k) {
    double d = 0.0;
    if (i > 0) d -= g.vx;
    if (i < g.nx - 1) d -= g.vx;
    if (j > 0) d -= g.vy;
    if (j < g.ny - 1) d -= g.vy;
    if (k > 0) d -= g.vz;
    if (k < g.nz - 1) d -= g.vz;
    return d;
}

// setRefPoint scale: VecSum(diag)/n over the GLOBAL diagonal (helper.cpp:264-272),
// VecSum [ext] being a sequential loop in row order.
inline double ref_scale(const Grid &g) {
    double s = 0.0;
    for (int32_t k = 0; k < g.nz; ++k)
        for (int32_t j = 0; j < g.ny; ++j)
            for (int32_t i = 0; i < g.nx; ++i) s += diag_value(g, i, j, k);
    return s / double(g.m);
}

}  // namespace aijhip_poisson
