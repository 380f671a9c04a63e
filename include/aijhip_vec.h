/*
 * aijhip_vec.h — device vector operations of the Krylov path (PETSc Vec on
 * the device; SURVEY.md §8b: "a Vec type is needed too, or the PCIe x/y
 * traffic dominates", and §8e: CG's dots all-reduced across ranks).
 *
 * These are the building blocks a caller that owns the outer Krylov loop
 * needs — e.g. the row-partitioned CG (petsc-openacc_amd/ksp.py KSPCGMPI,
 * one process per GPU, dots combined with an RCCL all-reduce) — with the
 * same arithmetic as the fused kernels inside aijhip_ksp:
 *   VecAYPX                      aijhip_vec_aypx
 *   VecDot                       aijhip_vec_dot       (local part)
 *   VecAXPY x2 + PCApply_Jacobi  aijhip_vec_cg_update (+ local z.z, z.r, r.r)
 *   PCApply_Jacobi               aijhip_vec_jacobi    (+ local z.z, z.r, r.r)
 *   PCSetUp_Jacobi               aijhip_mat_jacobi_inverse
 * Reductions are summed in a fixed order (deterministic) into DEVICE
 * doubles, so they can be handed to a collective without a host round trip.
 * Every call is asynchronous on `stream` (a hipStream_t; NULL = default).
 */
#ifndef AIJHIP_VEC_H
#define AIJHIP_VEC_H

#include <stdint.h>

#include "aijhip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* y = x + beta * y (VecAYPX: the product first, then the add). */
int aijhip_vec_aypx(int64_t n, double beta, const double *x, double *y, void *stream);

/* d_result[0] = x . y over the n local entries. */
int aijhip_vec_dot(int64_t n, const double *x, const double *y, double *d_result, void *stream);

/* x = x + alpha p; r = r + (-alpha) w; z = dinv * r (dinv NULL: z = r);
 * d_result[0..2] = z.z, z.r, r.r. z may alias w (read before written). */
int aijhip_vec_cg_update(int64_t n, double alpha, double *x, const double *p, double *r,
                         const double *w, double *z, const double *dinv, double *d_result,
                         void *stream);

/* z = dinv * r (dinv NULL: z = r); d_result[0..2] = z.z, z.r, r.r. */
int aijhip_vec_jacobi(int64_t n, const double *r, const double *dinv, double *z, double *d_result,
                      void *stream);

/* Diagnostic: reads d_buf[0 .. n & ~1) once with 16-B loads by 512-lane
 * workgroups streaming contiguous tiles — the achievable HBM read rate the
 * SpMV's roofline fraction is read against (bench.py
 * roofline.ceiling_flat_read). mode 0: the fastest shape measured
 * (non-temporal loads, two per lane, tools/read_sweep.hip); mode 1: the
 * STREAM kernel's own shape (plain loads, four per lane). d_buf 16-B
 * aligned. */
int aijhip_read_probe(const double *d_buf, int64_t n, int mode, void *stream);

/* Diagnostic: one wave on `stream` that finishes `us` microseconds after it
 * starts (the device's constant-rate wall clock; 0 <= us <= 1e6). Queued
 * ahead of timed launches it keeps the device busy while the host enqueues
 * them, so HIP events around them time device work only, not host launch
 * overhead (bench.py halo_forms, tools/halo_probe.py). */
int aijhip_delay_probe(double us, void *stream);

/* PCSetUp_Jacobi on A's rows: d_dinv[i] = 1 / (first stored a_ii, 0 -> 1). */
int aijhip_mat_jacobi_inverse(aijhip_mat_t A, double *d_dinv, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* AIJHIP_VEC_H */
