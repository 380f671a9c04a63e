/*
 * aijhip_ksp.h — device-resident Krylov solve around the MI355X SpMV
 * (the caller of MatMult_SeqAIJ in the reference,
 * /root/reference/src/main_ksp.cpp:92-103 with
 * /root/reference/configs/PETSc_SolverOptions_GAMG.info:1-4).
 *
 * Mirrors PETSc 3.7.6's KSPSolve_CG [ext] (src/ksp/ksp/impls/cg/cg.c) and
 * KSPConvergedDefault [ext] (src/ksp/ksp/interface/iterativ.c): preconditioned
 * CG with the preconditioned residual norm by default, the same breakdown
 * checks (beta = 0, indefinite PC, indefinite matrix) and the same reason
 * codes. Vectors are device arrays; all scalar work (alpha, beta, the
 * convergence test) runs on the device, so iterations are launched without a
 * host round trip. Dot products are reduced in a fixed order (deterministic
 * run to run) but not in BLAS ddot's order, so results match PETSc to
 * rounding, not bit for bit.
 */
#ifndef AIJHIP_KSP_H
#define AIJHIP_KSP_H

#include <stdint.h>

#include "aijhip.h"
#include "aijhip_gamg.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct aijhip_ksp *aijhip_ksp_t;

/* PCType: PCNONE, PCJACOBI (= bjacobi + jacobi sub-PC on one rank,
 * PETSc_SolverOptions_GAMG.info:16-21), PCGAMG (agg, one V-cycle per
 * application: Richardson(1) + Jacobi smoothing down and up on every level,
 * preonly + Jacobi on the coarsest — PETSc_SolverOptions_GAMG.info:6-21;
 * hierarchy from include/aijhip_gamg.h). */
enum {
    AIJHIP_PC_NONE = 0,
    AIJHIP_PC_JACOBI = 1,
    AIJHIP_PC_GAMG = 2,         /* PCGAMG; on a distributed operator (aijhip_kspmpi,
                                   more than one rank) the hierarchy spans the
                                   ranks, as PETSc's agg GAMG does             */
    AIJHIP_PC_BJACOBI_GAMG = 3  /* distributed operator only: -pc_type bjacobi
                                   -sub_pc_type gamg (one hierarchy per rank's
                                   diagonal block, no coupling)               */
};

/* KSPNormType values as in PETSc. */
enum {
    AIJHIP_KSP_NORM_NONE = 0,
    AIJHIP_KSP_NORM_PRECONDITIONED = 1,
    AIJHIP_KSP_NORM_UNPRECONDITIONED = 2,
    AIJHIP_KSP_NORM_NATURAL = 3
};

/* KSPConvergedReason values as in PETSc 3.7. */
enum {
    AIJHIP_KSP_CONVERGED_ITERATING = 0,
    AIJHIP_KSP_CONVERGED_RTOL = 2,
    AIJHIP_KSP_CONVERGED_ATOL = 3,
    AIJHIP_KSP_DIVERGED_ITS = -3,
    AIJHIP_KSP_DIVERGED_DTOL = -4,
    AIJHIP_KSP_DIVERGED_INDEFINITE_PC = -8,
    AIJHIP_KSP_DIVERGED_NANORINF = -9,
    AIJHIP_KSP_DIVERGED_INDEFINITE_MAT = -10
};

/* KSPCreate + KSPSetOperators(A, A) + KSPSetType(KSPCG). A must be square;
 * the handle borrows A (A must outlive it). Defaults as PETSc: rtol 1e-5,
 * atol 1e-50, dtol 1e5, max_it 10000, PC Jacobi, preconditioned norm,
 * zero initial guess. */
int aijhip_ksp_create(aijhip_mat_t A, aijhip_ksp_t *ksp);
int aijhip_ksp_set_tolerances(aijhip_ksp_t ksp, double rtol, double abstol, double dtol,
                              int32_t max_it);
int aijhip_ksp_set_pc_type(aijhip_ksp_t ksp, int pc_type);
int aijhip_ksp_set_norm_type(aijhip_ksp_t ksp, int norm_type);
int aijhip_ksp_set_initial_guess_nonzero(aijhip_ksp_t ksp, int flg);
/* KSPSetUp: PC set-up (inverse diagonal) and work vectors. Called by solve
 * if needed; call it explicitly to time set-up apart from the solve. */
int aijhip_ksp_set_up(aijhip_ksp_t ksp);
/* KSPSolve: b, x device fp64[m]; x is overwritten (zeroed first unless the
 * initial guess is nonzero). Returns once the solve has finished. */
int aijhip_ksp_solve(aijhip_ksp_t ksp, const double *b, double *x, void *stream);
/* KSPSolve with HOST vectors b, x (fp64[m]; x is also read when the initial
 * guess is nonzero): b goes up and x comes down once per solve, the whole
 * solve runs on the device — the solve-level offload an unchanged PETSc
 * caller with host Vecs reaches through a registered KSP type
 * (petsc-openacc_amd/petsc/aijhip_ksp_petsc.c), instead of two PCIe copies per
 * MatMult. Synchronous. */
int aijhip_ksp_solve_host(aijhip_ksp_t ksp, const double *b, double *x);
int aijhip_ksp_get_iteration_number(aijhip_ksp_t ksp, int32_t *its);
int aijhip_ksp_get_residual_norm(aijhip_ksp_t ksp, double *rnorm);
int aijhip_ksp_get_converged_reason(aijhip_ksp_t ksp, int *reason);
/* KSPGetResidualHistory: copies min(na, its + 1) norms; *n = that count. */
int aijhip_ksp_get_residual_history(aijhip_ksp_t ksp, double *hist, int32_t na, int32_t *n);
/* Fused kernels used per iteration (1 = SpMV with the p.Ap dot in its
 * epilogue), for reporting. */
int aijhip_ksp_get_fused(aijhip_ksp_t ksp, int *fused);
/* Host synchronisations made by the last solve: the polls of the device stop
 * flag (one per batch of 8 iterations, AIJHIP_KSP_POLL overrides) plus the
 * final read. */
int aijhip_ksp_get_host_syncs(aijhip_ksp_t ksp, int32_t *n);
/* Compulsory HBM bytes one CG iteration of the set-up solver moves (the
 * roofline of the solve): every SpMV at its plan's layout bytes
 * (aijhip_info_t.mult_layout_bytes: matrix, x once, y once) plus the vector
 * passes' reads and writes — CG's p = z + b p (with the deferred x += a p),
 * the r update, and for GAMG per level the Jacobi pass, the residual and
 * post-smoothing SpMVs with their b / D^-1 reads, MatRestrict (P^T),
 * MatInterpolateAdd (P, reading the level's x) and the coarse Jacobi. The
 * per-part split: *spmv_bytes of the total are matrix launches, *level0 of
 * the total belong to the finest level (its SpMVs and vectors). Valid after
 * set-up; the first iteration moves a little less. */
int aijhip_ksp_get_iteration_bytes(aijhip_ksp_t ksp, int64_t *bytes, int64_t *spmv_bytes, int64_t *level0);
/* GAMG options (before set-up); NULL = PETSc defaults
 * (aijhip_gamg_params_default). */
int aijhip_ksp_set_gamg_params(aijhip_ksp_t ksp, const aijhip_gamg_params_t *p);
/* Multigrid levels of the set-up PC (1 for non-GAMG): rows and operator nnz
 * per level (finest first; up to cap entries), and the host set-up time. */
int aijhip_ksp_get_pc_levels(aijhip_ksp_t ksp, int32_t *nlevels, int32_t *rows, int64_t *nnz,
                             int32_t cap, double *setup_seconds);

/* Copy out GAMG level l's operator (which = 'A') or interpolation to level
 * l+1 ('P') from the device (PCMGGetSmoother / PCGetInterpolations
 * introspection): sizes into m, n, nnz; with ai == NULL only the sizes. */
int aijhip_ksp_get_pc_level(aijhip_ksp_t ksp, int32_t l, char which, int32_t *m, int32_t *n,
                            int64_t *nnz, int32_t *ai, int32_t *aj, double *aa);
/* How the GAMG set-up built each coarsening l -> l+1 (up to cap entries,
 * one per level but the coarsest): path[l] = 1 on the device
 * (aijhip_gamg build_device), 0 on the host builder; product_cols[l] = the
 * widest accumulator the device Galerkin products needed (0 = the wavefront
 * form, else 32 / 64 / 128 / 256 LDS columns per row; -1 on the host).
 * *host_fallback = 1 when a level the device would have built went to the
 * host because a product row exceeded 256 distinct columns. */
int aijhip_ksp_get_gamg_setup_path(aijhip_ksp_t ksp, int32_t cap, int32_t *path, int32_t *product_cols,
                                   int32_t *host_fallback);
int aijhip_ksp_destroy(aijhip_ksp_t ksp);

#ifdef __cplusplus
}
#endif

#endif /* AIJHIP_KSP_H */
