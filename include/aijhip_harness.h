/*
 * aijhip_harness.h — host-side operand producers for the SpMV path.
 *
 * Not the hot path: these restate the reference's problem set-up so that the
 * benchmark and the tests feed the SpMV the same matrix PETSc would.
 *   Poisson 7-point operand  <- generateA, /root/reference/src/helper.cpp:161-246
 *   reference-point fix      <- setRefPoint, helper.cpp:250-279
 *   RHS / exact solution     <- generateRHS :78-116, generateExt :120-157
 *   row-block split          <- PETSc MPIAIJ diagonal / off-diagonal blocks
 *                               (MatSetUpMultiply_MPIAIJ [ext]) for the
 *                               DMDA z-slab partition (helper.cpp:31-36)
 * plus a seeded skewed CSR standing in for SuiteSparse Flan_1565, which is not
 * available offline.
 *
 * Rows are generated for a z-slab [z0, z1) of an nx*ny*nz grid in natural
 * ordering r = i + nx*(j + ny*k); column indices are GLOBAL. With z0 = 0,
 * z1 = nz this is the whole 1-rank matrix.
 */
#ifndef AIJHIP_HARNESS_H
#define AIJHIP_HARNESS_H

#include <stdint.h>

#include "aijhip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Number of stored entries of slab rows [z0, z1): 7 per row minus one per
 * out-of-domain neighbour (nnz of the full grid is 7N^3 - 6N^2 at nx=ny=nz=N). */
int aijhip_poisson_nnz(int32_t nx, int32_t ny, int32_t nz, int32_t z0, int32_t z1,
                       int64_t *nnz);

/* Fill ai[mloc+1] (local offsets), aj[nnz] (global columns, ascending within a
 * row), aa[nnz]. ref_point != 0 applies setRefPoint's MatZeroRowsColumns on
 * global row/column 0 (explicit zeros kept) and returns its scale. */
int aijhip_poisson_fill(int32_t nx, int32_t ny, int32_t nz, int32_t z0, int32_t z1,
                        int ref_point, int32_t *ai, int32_t *aj, double *aa,
                        double *scale);

/* rhs (generateRHS, then setRefPoint's rhs update) and exact (generateExt)
 * for slab rows; either pointer may be NULL. */
int aijhip_poisson_vectors(int32_t nx, int32_t ny, int32_t nz, int32_t z0, int32_t z1,
                           int ref_point, double *rhs, double *exact);

/* Counter-based uniform [-1, 1): x[i] = f(seed, offset + i) (splitmix64). */
void aijhip_splitmix_uniform(int64_t n, uint64_t seed, int64_t offset, double *x);

/* Seeded skewed CSR (Flan_1565 stand-in, square m x m): per-row lengths are
 * uniform in [24, 81] (Flan's range) except a heavy tail of hub rows with
 * 1e3..2e5 entries; columns are sorted and unique. Pass ai/aj/aa = NULL to
 * get nnz only. */
int aijhip_skewed_csr(int32_t m, uint64_t seed, int64_t *nnz, int32_t *ai, int32_t *aj,
                      double *aa);

/* Seeded FEM-structured CSR (the other Flan_1565 stand-in: Flan is a 3-D
 * hexahedral mesh with 3 dofs per node): nodes on an nx x ny x nz grid in
 * natural order, `dofs` unknowns per node numbered node*dofs + d, and every
 * row coupling all dofs of the (up to) 27 neighbouring nodes, columns sorted;
 * values uniform [-1, 1) from (seed, entry index). Interior rows hold
 * 27*dofs entries. Pass ai/aj/aa = NULL to get nnz only. */
int aijhip_fem_hex_csr(int32_t nx, int32_t ny, int32_t nz, int32_t dofs, uint64_t seed,
                       int64_t *nnz, int32_t *ai, int32_t *aj, double *aa);

/* Split local rows into PETSc MPIAIJ blocks: columns in [col_lo, col_hi) go to
 * the diagonal block (renumbered c - col_lo); the others to the off-diagonal
 * block, renumbered by position in garray (the sorted unique off-block global
 * columns). Call once with d_ai == NULL to get sizes (nz_d, nz_o, n_garray),
 * then again with arrays of those sizes. Entry order within a row is kept. */
int aijhip_split_rows(int32_t m, const int32_t *ai, const int32_t *aj, const double *aa,
                      int32_t col_lo, int32_t col_hi, int64_t *nz_d, int64_t *nz_o,
                      int32_t *n_garray, int32_t *d_ai, int32_t *d_aj, double *d_aa,
                      int32_t *o_ai, int32_t *o_aj, double *o_aa, int32_t *garray);

/* ---- Device-side producers: the same operand and vectors
 * written straight into device memory, bit-identical to the host producers
 * above. Arrays are device pointers sized as for aijhip_poisson_fill /
 * _vectors; `stream` is a hipStream_t (NULL = default stream); the calls are
 * asynchronous on it except where noted. */

/* Device generateA + setRefPoint into d_ai[mloc+1], d_aj[nnz], d_aa[nnz]
 * (nnz from aijhip_poisson_nnz); *scale as aijhip_poisson_fill. */
int aijhip_poisson_fill_device(int32_t nx, int32_t ny, int32_t nz, int32_t z0, int32_t z1,
                               int ref_point, int32_t *d_ai, int32_t *d_aj, double *d_aa,
                               double *scale, void *stream);

/* Device generateRHS / generateExt (+ setRefPoint's rhs update); either
 * pointer may be NULL. Returns after the work on `stream` is done. */
int aijhip_poisson_vectors_device(int32_t nx, int32_t ny, int32_t nz, int32_t z0, int32_t z1,
                                  int ref_point, double *d_rhs, double *d_exact, void *stream);

/* Assemble the slab operator on `device` and return it as a SeqAIJ handle
 * (aijhip_mat_create_from_device on the assembled arrays): no host CSR, no
 * PCIe upload of the matrix. Columns are global (n = nx*ny*nz). */
int aijhip_mat_create_poisson(int device, int32_t nx, int32_t ny, int32_t nz, int32_t z0,
                              int32_t z1, int ref_point, double *scale, aijhip_mat_t *out);

#ifdef __cplusplus
}
#endif

#endif /* AIJHIP_HARNESS_H */
