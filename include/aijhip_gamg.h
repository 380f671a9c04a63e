/*
 * aijhip_gamg.h — smoothed-aggregation multigrid hierarchy (the PCGAMG the
 * reference configures: /root/reference/configs/PETSc_SolverOptions_GAMG.info
 * :6-21, -pc_gamg_type agg -pc_gamg_agg_nsmooths 1 -pc_gamg_threshold 0.0;
 * SURVEY.md §8f row 3).
 *
 * The hierarchy is built on the host ("setup can stay on the
 * host") by the same steps as PETSc 3.7's PCSetUp_GAMG with the agg type
 * [ext]: strength graph |a_ij| > threshold*sqrt(|a_ii a_jj|), i != j;
 * aggregation; tentative prolongator from the near-null space (constant
 * vector on the finest level; the QR factors carry it down); one Jacobi
 * smoothing step P = (I - 1.4/emax D^-1 A) P0 (PCGAMGOptProlongator_AGG's
 * alpha = -1.4/emax); Galerkin coarse operator Pt A P. Aggregation:
 * PETSc 3.7's own agg coarsening restated (coarsen 1, the default since
 * round 5: a maximal independent set of the squared graph in a hashed random
 * order, aggregates smoothed — agg.c PCGAMGCoarsen_AGG / smoothAggs, mis.c;
 * PETSc's random stream is not reproduced) or a deterministic greedy pass in
 * natural order (coarsen 0, the default through round 4), with emax from
 * CG's Lanczos tridiagonal as PCGAMGOptProlongator_AGG does (eig_ksp 1, the
 * default) or a power iteration (eig_ksp 0). GAMG iteration parity with
 * PETSc is unpinned either way (PETSc is absent). The distributed set-up
 * (PCGAMG across ranks) takes the same parameters, its MIS on each rank's
 * diagonal block.
 * The solve-phase V-cycle runs on the device inside aijhip_ksp
 * (AIJHIP_PC_GAMG), whose set-up builds the large levels on the device
 * (device_min_rows) with results identical to aijhip_gamg_build_host.
 */
#ifndef AIJHIP_GAMG_H
#define AIJHIP_GAMG_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct aijhip_gamg_params {
    double threshold;        /* -pc_gamg_threshold (0.0)                     */
    int32_t coarse_eq_limit; /* -pc_gamg_coarse_eq_limit (50)                */
    int32_t max_levels;      /* -pc_mg_levels (10)                           */
    int32_t nsmooths;        /* -pc_gamg_agg_nsmooths (1)                    */
    double smooth_scale;     /* 1.4 in alpha = -smooth_scale / emax          */
    int32_t eig_its;         /* iterations of the emax(D^-1 A) estimate (10) */
    int32_t threads;         /* host threads for set-up (0 = OpenMP default) */
    int32_t device_min_rows; /* KSP set-up: levels with at least this many rows
                              * (or 25 x as many entries) are built on the
                              * device (strength graph, emax, aggregation,
                              * smoothing, Galerkin product); smaller ones on
                              * the host.
                              * 0 = every level on the device, INT32_MAX = all
                              * on the host. Same hierarchy either way.     */
    /* ABI 3: */
    int32_t coarsen;         /* 1 (default): PETSc 3.7 agg's MIS (see above);
                              * 0: greedy aggregation (natural order)       */
    int32_t square_graph;    /* -pc_gamg_square_graph (1): coarsen 1 squares
                              * the graph on this many levels from the finest */
    int32_t eig_ksp;         /* emax(D^-1 A): 1 (default) CG's Lanczos estimate,
                              * PETSc's; 0 power iteration                   */
    int32_t pad0;
} aijhip_gamg_params_t;

typedef struct aijhip_gamg_host *aijhip_gamg_host_t;

int aijhip_gamg_params_default(aijhip_gamg_params_t *p);

/* Build the hierarchy for the square CSR operator (host arrays). Level 0 is
 * the input operator; level l+1 = Pt_l A_l P_l. */
int aijhip_gamg_build_host(int32_t m, const int32_t *ai, const int32_t *aj, const double *aa,
                           const aijhip_gamg_params_t *p, aijhip_gamg_host_t *out);
int aijhip_gamg_host_num_levels(aijhip_gamg_host_t h, int32_t *nlevels);
/* Sizes of level l: rows, nnz of A_l; for l < nlevels-1 also nnz of P_l
 * (rows m_l, columns m_{l+1}) and the emax estimate used to smooth it. */
int aijhip_gamg_host_level_info(aijhip_gamg_host_t h, int32_t l, int32_t *m, int64_t *nnz_a,
                                int64_t *nnz_p, double *emax);
/* Copy out level l's operator (l >= 1), interpolation P_l, aggregates of
 * level l's rows (agg[i] = coarse row), into caller arrays sized by
 * level_info. */
int aijhip_gamg_host_get_A(aijhip_gamg_host_t h, int32_t l, int32_t *ai, int32_t *aj, double *aa);
int aijhip_gamg_host_get_P(aijhip_gamg_host_t h, int32_t l, int32_t *ai, int32_t *aj, double *aa);
int aijhip_gamg_host_get_aggregates(aijhip_gamg_host_t h, int32_t l, int32_t *agg);
/* Borrow level l's operator (which = 'A', l >= 1) or interpolation
 * (which = 'P', l < nlevels-1) in place: the pointers stay valid until
 * aijhip_gamg_host_destroy (no copy; the device set-up uploads from them). */
int aijhip_gamg_host_view(aijhip_gamg_host_t h, int32_t l, char which, const int32_t **ai, const int32_t **aj,
                          const double **aa);
int aijhip_gamg_host_destroy(aijhip_gamg_host_t h);

#ifdef __cplusplus
}
#endif

#endif /* AIJHIP_GAMG_H */
