// poisson.hip — device-side assembly of the reference's operand (SURVEY §8f
// row 4): generateA + setRefPoint (/root/reference/src/helper.cpp:161-279)
// and generateRHS/generateExt (:78-157) written straight into HBM, one lane
// per row, bit-identical to the host producer in harness.cpp (same constants
// from poisson_grid.h, same stencil order, same sequential diagonal). At 600^3
// this replaces ~18 GB of host assembly plus its PCIe upload.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <string>
#include <vector>

#include "aijhip.h"
#include "aijhip_harness.h"
#include "aijhip_internal.h"
#include "poisson_grid.h"

namespace {

using aijhip_poisson::Grid;

struct DevGrid {
    int32_t nx, ny, nz, z0, z1;
    int64_t nxy;
    double vx, vy, vz;
};

// Entries before slab-local row (i, j, k): whole planes z0..k-1, whole lines
// 0..j-1 of plane k, cells 0..i-1 of line j. Each cell stores 1 + its in-domain
// neighbours; the counts separate over the three axes.
__device__ __forceinline__ int64_t row_offset(const DevGrid &g, int32_t i, int32_t j, int32_t k) {
    const int64_t X = 2 * (int64_t)(g.nx - 1) * g.ny, Y = 2 * (int64_t)(g.ny - 1) * g.nx;
    const int64_t np = k - g.z0;
    const int64_t zlow = np - ((g.z0 == 0 && np > 0) ? 1 : 0);            // planes kk > 0
    const int64_t zhigh = max((int64_t)0, (int64_t)min(k, g.nz - 1) - g.z0);  // planes kk < nz-1
    int64_t off = np * (g.nxy + X + Y) + g.nxy * (zlow + zhigh);
    if (k >= g.z1) return off;
    const int32_t zc = (k > 0) + (k < g.nz - 1);
    off += (int64_t)j * g.nx * (1 + zc) + (int64_t)g.nx * (max(j - 1, 0) + min(j, g.ny - 1)) +
           2 * (int64_t)j * (g.nx - 1);
    const int32_t yc = (j > 0) + (j < g.ny - 1);
    off += (int64_t)i * (1 + zc + yc) + max(i - 1, 0) + min(i, g.nx - 1);
    return off;
}

// harness.cpp diag_value / helper.cpp:229-233: 0, minus each in-domain
// neighbour's coefficient in stencil order.
__device__ __forceinline__ double diag_value(const DevGrid &g, int32_t i, int32_t j, int32_t k) {
    double d = 0.0;
    if (i > 0) d -= g.vx;
    if (i < g.nx - 1) d -= g.vx;
    if (j > 0) d -= g.vy;
    if (j < g.ny - 1) d -= g.vy;
    if (k > 0) d -= g.vz;
    if (k < g.nz - 1) d -= g.vz;
    return d;
}

__global__ void k_poisson_fill(DevGrid g, int64_t mloc, int32_t *__restrict__ ai, int32_t *__restrict__ aj,
                               double *__restrict__ aa) {
    const int64_t l = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (l > mloc) return;
    if (l == mloc) {
        ai[mloc] = (int32_t)row_offset(g, 0, 0, g.z1);
        return;
    }
    const int32_t i = (int32_t)(l % g.nx), j = (int32_t)((l / g.nx) % g.ny), k = g.z0 + (int32_t)(l / g.nxy);
    int64_t p = row_offset(g, i, j, k);
    ai[l] = (int32_t)p;
    const int64_t r = i + (int64_t)g.nx * (j + (int64_t)g.ny * k);
    // SeqAIJ's sorted row: k-1, j-1, i-1, c, i+1, j+1, k+1 (harness.cpp)
    if (k > 0) { aj[p] = (int32_t)(r - g.nxy); aa[p++] = g.vz; }
    if (j > 0) { aj[p] = (int32_t)(r - g.nx); aa[p++] = g.vy; }
    if (i > 0) { aj[p] = (int32_t)(r - 1); aa[p++] = g.vx; }
    aj[p] = (int32_t)r; aa[p++] = diag_value(g, i, j, k);
    if (i < g.nx - 1) { aj[p] = (int32_t)(r + 1); aa[p++] = g.vx; }
    if (j < g.ny - 1) { aj[p] = (int32_t)(r + g.nx); aa[p++] = g.vy; }
    if (k < g.nz - 1) { aj[p] = (int32_t)(r + g.nxy); aa[p++] = g.vz; }
}

// setRefPoint on the assembled slab (harness.cpp order): column 0 zeroed in
// rows 1, nx, nx*ny when local, then row 0 = scale on its diagonal, 0 elsewhere.
__global__ void k_poisson_ref_point(DevGrid g, int64_t m, int64_t row0, int64_t mloc, const int32_t *ai,
                                    const int32_t *aj, double *aa, double sc) {
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    const int64_t cand[3] = {1, (int64_t)g.nx, g.nxy};
    for (int q = 0; q < 3; ++q) {
        const int64_t c = cand[q], l = c - row0;
        if (c >= m || l < 0 || l >= mloc) continue;
        for (int32_t e = ai[l]; e < ai[l + 1]; ++e)
            if (aj[e] == 0) aa[e] = 0.0;
    }
    if (row0 == 0 && mloc > 0)
        for (int32_t e = ai[0]; e < ai[1]; ++e) aa[e] = (aj[e] == 0) ? sc : 0.0;
}

__global__ void k_poisson_vectors(DevGrid g, int64_t mloc, const double *__restrict__ cx,
                                  const double *__restrict__ cy, const double *__restrict__ cz, double *rhs,
                                  double *exact) {
    const int64_t l = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (l >= mloc) return;
    const int32_t i = (int32_t)(l % g.nx), j = (int32_t)((l / g.nx) % g.ny), k = g.z0 + (int32_t)(l / g.nxy);
    // helper.cpp:107-110 and :148-151, left to right as in harness.cpp
    if (rhs) rhs[l] = -3.0 * 2.0 * 1.0 * M_PI * 2.0 * 1.0 * M_PI * cx[i] * cy[j] * cz[k];
    if (exact) exact[l] = cx[i] * cy[j] * cz[k];
}

// setRefPoint's right-hand-side update (MatZeroRowsColumns with x = exact).
__global__ void k_poisson_rhs_ref(DevGrid g, int64_t m, int64_t row0, int64_t mloc, double ex0, double sc,
                                  double *rhs) {
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    const int64_t cand[3] = {1, (int64_t)g.nx, g.nxy};
    const double coef[3] = {g.vx, g.vy, g.vz};
    const int32_t ext[3] = {g.nx, g.ny, g.nz};
    for (int q = 0; q < 3; ++q) {
        const int64_t c = cand[q];
        if (c >= m || c - row0 < 0 || c - row0 >= mloc || ext[q] < 2) continue;
        rhs[c - row0] -= coef[q] * ex0;
    }
    if (row0 == 0 && mloc > 0) rhs[0] = sc * ex0;
}

DevGrid dev_grid(const Grid &g, int32_t z0, int32_t z1) {
    return DevGrid{g.nx, g.ny, g.nz, z0, z1, g.nxy, g.vx, g.vy, g.vz};
}

int herr(hipError_t e, const char *what) {
    aijhip::set_error(std::string(what) + ": " + hipGetErrorString(e));
    return AIJHIP_ERR_HIP;
}

}  // namespace

extern "C" {

int aijhip_poisson_fill_device(int32_t nx, int32_t ny, int32_t nz, int32_t z0, int32_t z1, int ref_point,
                               int32_t *d_ai, int32_t *d_aj, double *d_aa, double *scale, void *stream) {
    Grid g;
    if (!d_ai || aijhip_poisson::make_grid(nx, ny, nz, z0, z1, &g) || (z1 > z0 && (!d_aj || !d_aa))) {
        aijhip::set_error("poisson_fill_device: bad grid or NULL array");
        return AIJHIP_ERR_ARG;
    }
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const int64_t mloc = (int64_t)(z1 - z0) * g.nxy, row0 = (int64_t)z0 * g.nxy;
    const DevGrid dg = dev_grid(g, z0, z1);
    hipLaunchKernelGGL(k_poisson_fill, dim3((unsigned)((mloc + 1 + 255) / 256)), dim3(256), 0, s, dg, mloc, d_ai,
                       d_aj, d_aa);
    double sc = 0.0;
    if (ref_point) {
        sc = aijhip_poisson::ref_scale(g);
        hipLaunchKernelGGL(k_poisson_ref_point, dim3(1), dim3(64), 0, s, dg, g.m, row0, mloc, d_ai, d_aj, d_aa,
                           sc);
    }
    if (scale) *scale = sc;
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? AIJHIP_OK : herr(e, "poisson_fill_device launch");
}

int aijhip_poisson_vectors_device(int32_t nx, int32_t ny, int32_t nz, int32_t z0, int32_t z1, int ref_point,
                                  double *d_rhs, double *d_exact, void *stream) {
    Grid g;
    if (aijhip_poisson::make_grid(nx, ny, nz, z0, z1, &g)) {
        aijhip::set_error("poisson_vectors_device: bad grid");
        return AIJHIP_ERR_ARG;
    }
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const int64_t mloc = (int64_t)(z1 - z0) * g.nxy, row0 = (int64_t)z0 * g.nxy;
    // the cosine factors are host libm values (as in harness.cpp), uploaded
    const double dx = aijhip_poisson::kL / nx, dy = aijhip_poisson::kL / ny, dz = aijhip_poisson::kL / nz;
    std::vector<double> c((size_t)nx + ny + nz);
    for (int32_t i = 0; i < nx; ++i) c[i] = aijhip_poisson::cfac(i, dx);
    for (int32_t j = 0; j < ny; ++j) c[(size_t)nx + j] = aijhip_poisson::cfac(j, dy);
    for (int32_t k = 0; k < nz; ++k) c[(size_t)nx + ny + k] = aijhip_poisson::cfac(k, dz);
    double *d_c = nullptr;
    hipError_t e = hipMalloc(&d_c, sizeof(double) * c.size());
    if (e != hipSuccess) return herr(e, "poisson_vectors_device alloc");
    e = hipMemcpyAsync(d_c, c.data(), sizeof(double) * c.size(), hipMemcpyHostToDevice, s);
    const DevGrid dg = dev_grid(g, z0, z1);
    if (e == hipSuccess && mloc > 0) {
        hipLaunchKernelGGL(k_poisson_vectors, dim3((unsigned)((mloc + 255) / 256)), dim3(256), 0, s, dg, mloc, d_c,
                           d_c + nx, d_c + nx + ny, d_rhs, d_exact);
        if (ref_point && d_rhs)
            hipLaunchKernelGGL(k_poisson_rhs_ref, dim3(1), dim3(64), 0, s, dg, g.m, row0, mloc,
                               c[0] * c[(size_t)nx] * c[(size_t)nx + ny], aijhip_poisson::ref_scale(g), d_rhs);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipStreamSynchronize(s);  // the tables are freed below
    hipFree(d_c);
    return e == hipSuccess ? AIJHIP_OK : herr(e, "poisson_vectors_device");
}

int aijhip_mat_create_poisson(int device, int32_t nx, int32_t ny, int32_t nz, int32_t z0, int32_t z1, int ref_point,
                              double *scale, aijhip_mat_t *out) {
    if (!out) {
        aijhip::set_error("out is NULL");
        return AIJHIP_ERR_ARG;
    }
    *out = nullptr;
    int64_t nnz = 0;
    int rc = aijhip_poisson_nnz(nx, ny, nz, z0, z1, &nnz);
    if (rc) {
        aijhip::set_error("mat_create_poisson: bad grid");
        return rc;
    }
    if (nnz > INT32_MAX) {
        aijhip::set_error("mat_create_poisson: slab nnz exceeds the int32 PetscInt range");
        return AIJHIP_ERR_ARG;
    }
    if (aijhip::visible_devices() <= 0) {
        aijhip::set_error("no HIP device visible");
        return AIJHIP_ERR_NODEVICE;
    }
    int prev = -1;
    hipGetDevice(&prev);
    hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) return herr(e, "set device");
    const int64_t mloc = (int64_t)(z1 - z0) * nx * (int64_t)ny;
    const int64_t ncols = (int64_t)nx * ny * nz;
    int32_t *ai = nullptr, *aj = nullptr;
    double *aa = nullptr;
    if ((e = hipMalloc(&ai, sizeof(int32_t) * (size_t)(mloc + 1))) != hipSuccess ||
        (e = hipMalloc(&aj, sizeof(int32_t) * (size_t)std::max<int64_t>(nnz, 1))) != hipSuccess ||
        (e = hipMalloc(&aa, sizeof(double) * (size_t)std::max<int64_t>(nnz, 1))) != hipSuccess) {
        rc = herr(e, "mat_create_poisson alloc");
    } else {
        rc = aijhip_poisson_fill_device(nx, ny, nz, z0, z1, ref_point, ai, aj, aa, scale, nullptr);
        if (!rc && (e = hipDeviceSynchronize()) != hipSuccess) rc = herr(e, "poisson assembly");
        if (!rc) rc = aijhip_mat_create_from_device(device, (int32_t)mloc, (int32_t)ncols, nnz, ai, aj, aa, out);
    }
    hipFree(ai);
    hipFree(aj);
    hipFree(aa);
    if (prev >= 0) hipSetDevice(prev);
    return rc;
}

}  // extern "C"
