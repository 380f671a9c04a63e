/*
 * aijhip_ksp_petsc.c — PETSc 3.7 KSP type "cghip": the whole KSPSolve of
 * main_ksp.cpp:92-103 (CG with the reference's PC) on the MI355X through
 * include/aijhip_ksp.h, for a caller whose Vecs stay on the host.
 *
 * NOT COMPILED IN THIS IMAGE (no PETSc here or on the GPU box); built into
 * libaijhip_petsc.so beside aijhip_petsc.c when PETSC_DIR is set. The entry
 * point it calls, aijhip_ksp_solve_host, is exercised through the same C ABI
 * by tests/test_ksp.py::test_gpu_solve_host_vectors_equals_device_solve.
 *
 * Why: with the Mat adapter alone every MatMult of an unchanged caller moves
 * x up and y down over PCIe (the reference's step-2 cost, 432 MB per 300^3
 * MatMult, SURVEY §7 "Host-resident Vecs kill it"). Selecting this type in
 * the options file (`-ksp_type cghip` beside configs/PETSc_SolverOptions_
 * GAMG.info's other lines) moves b up and x down once per solve instead; the
 * CG iteration, the PC (gamg / jacobi / none with PETSc's option names) and
 * the convergence test run on the device (aijhip_ksp.h). main_ksp.cpp reads
 * its, reason, rnorm and the history back through the usual KSP getters.
 * Any other operator or PC falls back to PETSc's own KSPCG, run as an inner
 * KSP on the caller's operators and PC (this KSP never changes its own type,
 * so nothing it owns is freed under a running solve). While the device path
 * is active ksp->pc is a PCNONE stand-in (KSPCGHIPStandIn): KSPGetPC /
 * PCView then show the stand-in, and the caller's PC is reachable again after
 * a fall-back or KSPDestroy.
 *
 * STATUS: not yet working code until it is compiled and run against PETSc
 * 3.7 — the PETSc-facing half is written to the 3.7 headers but has never
 * been built.
 */
#include <petsc/private/kspimpl.h>
#include <petsc/private/pcimpl.h>

#include "aijhip.h"
#include "aijhip_gamg.h"
#include "aijhip_ksp.h"

/* aijhip_petsc.c: the device handle of a seqaij(hip) matrix, brought up to
 * date with the host values; NULL for any other matrix. */
PETSC_EXTERN PetscErrorCode AIJHIPGetHandle(Mat A, aijhip_mat_t *h);

typedef struct {
  aijhip_ksp_t     k;
  aijhip_mat_t     h;       /* the handle k was set up on */
  PetscObjectState state;   /* the operator's state at that set-up */
  int              pc;
  PC               user_pc; /* the caller's PC while ksp->pc is a PCNONE stand-in */
  KSP              inner;   /* PETSc's KSPCG on the caller's PC: the fall-back */
  PetscBool        fallback;
} KSP_CGHIP;

static PetscErrorCode KSPCGHIPFree(KSP_CGHIP *c)
{
  PetscFunctionBegin;
  if (c->k) aijhip_ksp_destroy(c->k);
  c->k = NULL;
  c->h = NULL;
  PetscFunctionReturn(0);
}

/* The caller's PC: the one KSPGetPC handed out, even while ksp->pc is the
 * stand-in. */
static PC KSPCGHIPUserPC(KSP ksp)
{
  KSP_CGHIP *c = (KSP_CGHIP*)ksp->data;
  return c->user_pc ? c->user_pc : ksp->pc;
}

/* The reference's PCs, by PETSc type name; -1: not offered on the device. */
static PetscErrorCode KSPCGHIPPCType(KSP ksp, int *pc)
{
  PC             upc = KSPCGHIPUserPC(ksp);
  PetscBool      is;
  PetscErrorCode ierr;

  PetscFunctionBegin;
  *pc = -1;
  ierr = PetscObjectTypeCompare((PetscObject)upc, PCGAMG, &is);CHKERRQ(ierr);
  if (is) { *pc = AIJHIP_PC_GAMG; PetscFunctionReturn(0); }
  ierr = PetscObjectTypeCompare((PetscObject)upc, PCJACOBI, &is);CHKERRQ(ierr);
  if (is) { *pc = AIJHIP_PC_JACOBI; PetscFunctionReturn(0); }
  ierr = PetscObjectTypeCompare((PetscObject)upc, PCNONE, &is);CHKERRQ(ierr);
  if (is) *pc = AIJHIP_PC_NONE;
  PetscFunctionReturn(0);
}

/* Device path: KSPSetUp calls PCSetUp(ksp->pc) after ops->setup, which for
 * PCGAMG would build PETSc's host hierarchy beside the device one (inside
 * main_ksp.cpp's timed "create solver"). Put a PCNONE stand-in in ksp->pc and
 * keep the caller's PC (its type and options are what the device KSP reads). */
static PetscErrorCode KSPCGHIPStandIn(KSP ksp)
{
  KSP_CGHIP      *c = (KSP_CGHIP*)ksp->data;
  PC             none;
  Mat            Amat, Pmat;
  PetscErrorCode ierr;

  PetscFunctionBegin;
  if (c->user_pc) PetscFunctionReturn(0);
  ierr = PetscObjectReference((PetscObject)ksp->pc);CHKERRQ(ierr);
  c->user_pc = ksp->pc;
  ierr = PCGetOperators(c->user_pc, &Amat, &Pmat);CHKERRQ(ierr);
  ierr = PCCreate(PetscObjectComm((PetscObject)ksp), &none);CHKERRQ(ierr);
  ierr = PCSetType(none, PCNONE);CHKERRQ(ierr);
  ierr = PCSetOperators(none, Amat, Pmat);CHKERRQ(ierr);
  ierr = KSPSetPC(ksp, none);CHKERRQ(ierr); /* references none, releases the caller's (held above) */
  ierr = PCDestroy(&none);CHKERRQ(ierr);
  PetscFunctionReturn(0);
}

/* Give the caller's PC back to ksp->pc (the fall-back runs PETSc's CG on it).
 * A KSPSetOperators made after the stand-in went in reached the stand-in
 * (ksp->pc), not the caller's PC: those operators move to the caller's PC
 * here, so the fall-back and any later KSPGetPC see the current system. */
static PetscErrorCode KSPCGHIPRestorePC(KSP ksp)
{
  KSP_CGHIP      *c = (KSP_CGHIP*)ksp->data;
  Mat            Amat = NULL, Pmat = NULL;
  PetscBool      has = PETSC_FALSE;
  PetscErrorCode ierr;

  PetscFunctionBegin;
  if (!c->user_pc) PetscFunctionReturn(0);
  ierr = PCGetOperatorsSet(ksp->pc, &has, NULL);CHKERRQ(ierr);
  if (has) { /* held across KSPSetPC, which frees the stand-in and its references */
    ierr = PCGetOperators(ksp->pc, &Amat, &Pmat);CHKERRQ(ierr);
    ierr = PetscObjectReference((PetscObject)Amat);CHKERRQ(ierr);
    ierr = PetscObjectReference((PetscObject)Pmat);CHKERRQ(ierr);
  }
  ierr = KSPSetPC(ksp, c->user_pc);CHKERRQ(ierr);
  if (has) {
    ierr = PCSetOperators(c->user_pc, Amat, Pmat);CHKERRQ(ierr);
    ierr = MatDestroy(&Amat);CHKERRQ(ierr);
    ierr = MatDestroy(&Pmat);CHKERRQ(ierr);
  }
  ierr = PCDestroy(&c->user_pc);CHKERRQ(ierr); /* drops the reference taken by KSPCGHIPStandIn */
  PetscFunctionReturn(0);
}

/* PETSc's own CG for what the device path does not cover: an inner KSPCG on
 * the caller's operators and PC, with this KSP's tolerances and norm. This
 * KSP keeps its type (no KSPSetType from inside its own set-up or solve). */
static PetscErrorCode KSPCGHIPFallBack(KSP ksp)
{
  KSP_CGHIP      *c = (KSP_CGHIP*)ksp->data;
  Mat            Amat, Pmat;
  PetscErrorCode ierr;

  PetscFunctionBegin;
  ierr = PetscInfo(ksp, "cghip: operator or PC not on the device; using KSPCG\n");CHKERRQ(ierr);
  ierr = KSPCGHIPFree(c);CHKERRQ(ierr);
  ierr = KSPCGHIPRestorePC(ksp);CHKERRQ(ierr); /* (carries the current operators to the caller's PC) */
  if (!c->inner) {
    ierr = KSPCreate(PetscObjectComm((PetscObject)ksp), &c->inner);CHKERRQ(ierr);
    ierr = KSPSetType(c->inner, KSPCG);CHKERRQ(ierr);
  }
  ierr = KSPGetOperators(ksp, &Amat, &Pmat);CHKERRQ(ierr);
  ierr = KSPSetOperators(c->inner, Amat, Pmat);CHKERRQ(ierr);
  ierr = KSPSetPC(c->inner, ksp->pc);CHKERRQ(ierr);
  ierr = KSPSetTolerances(c->inner, ksp->rtol, ksp->abstol, ksp->divtol, ksp->max_it);CHKERRQ(ierr);
  ierr = KSPSetNormType(c->inner, ksp->normtype);CHKERRQ(ierr);
  ierr = KSPSetInitialGuessNonzero(c->inner, ksp->guess_zero ? PETSC_FALSE : PETSC_TRUE);CHKERRQ(ierr);
  ierr = KSPSetUp(c->inner);CHKERRQ(ierr);
  c->fallback = PETSC_TRUE;
  PetscFunctionReturn(0);
}

/* KSPSetUp (PCSetUp_GAMG included, timed by main_ksp.cpp as "create
 * solver"): the device KSP on the operator's handle with the options file's
 * PC settings. */
static PetscErrorCode KSPSetUp_CGHIP(KSP ksp)
{
  KSP_CGHIP            *c = (KSP_CGHIP*)ksp->data;
  Mat                  A;
  aijhip_mat_t         h = NULL;
  PetscObjectState     state;
  aijhip_gamg_params_t gp;
  PetscInt             iv;
  PetscReal            rv;
  PetscBool            set;
  int                  pc, nt, rc;
  PetscErrorCode       ierr;

  PetscFunctionBegin;
  ierr = KSPGetOperators(ksp, &A, NULL);CHKERRQ(ierr);
  ierr = AIJHIPGetHandle(A, &h);CHKERRQ(ierr);
  ierr = KSPCGHIPPCType(ksp, &pc);CHKERRQ(ierr);
  if (!h || pc < 0) {
    ierr = KSPCGHIPFallBack(ksp);CHKERRQ(ierr);
    PetscFunctionReturn(0);
  }
  c->fallback = PETSC_FALSE;
  ierr = KSPCGHIPStandIn(ksp);CHKERRQ(ierr);
  ierr = PetscObjectStateGet((PetscObject)A, &state);CHKERRQ(ierr);
  if (c->k && c->h == h && c->state == state && c->pc == pc) PetscFunctionReturn(0);
  ierr = KSPCGHIPFree(c);CHKERRQ(ierr);
  rc = aijhip_ksp_create(h, &c->k);
  if (!rc) rc = aijhip_ksp_set_pc_type(c->k, pc);
  if (!rc && pc == AIJHIP_PC_GAMG) {
    aijhip_gamg_params_default(&gp);
    ierr = PetscOptionsGetReal(NULL, NULL, "-pc_gamg_threshold", &rv, &set);CHKERRQ(ierr);
    if (set) gp.threshold = (double)rv;
    ierr = PetscOptionsGetInt(NULL, NULL, "-pc_gamg_agg_nsmooths", &iv, &set);CHKERRQ(ierr);
    if (set) gp.nsmooths = (int32_t)iv;
    ierr = PetscOptionsGetInt(NULL, NULL, "-pc_gamg_coarse_eq_limit", &iv, &set);CHKERRQ(ierr);
    if (set) gp.coarse_eq_limit = (int32_t)iv;
    ierr = PetscOptionsGetInt(NULL, NULL, "-pc_mg_levels", &iv, &set);CHKERRQ(ierr);
    if (set) gp.max_levels = (int32_t)iv;
    ierr = PetscOptionsGetInt(NULL, NULL, "-pc_gamg_square_graph", &iv, &set);CHKERRQ(ierr);
    if (set) gp.square_graph = (int32_t)iv;
    /* this library's extensions (0: the greedy aggregation / power-iteration emax) */
    ierr = PetscOptionsGetInt(NULL, NULL, "-aijhip_gamg_coarsen", &iv, &set);CHKERRQ(ierr);
    if (set) gp.coarsen = (int32_t)iv;
    ierr = PetscOptionsGetInt(NULL, NULL, "-aijhip_gamg_eig_ksp", &iv, &set);CHKERRQ(ierr);
    if (set) gp.eig_ksp = (int32_t)iv;
    rc = aijhip_ksp_set_gamg_params(c->k, &gp);
  }
  switch (ksp->normtype) {
    case KSP_NORM_NONE:            nt = AIJHIP_KSP_NORM_NONE; break;
    case KSP_NORM_UNPRECONDITIONED: nt = AIJHIP_KSP_NORM_UNPRECONDITIONED; break;
    case KSP_NORM_NATURAL:         nt = AIJHIP_KSP_NORM_NATURAL; break;
    default:                       nt = AIJHIP_KSP_NORM_PRECONDITIONED; break;
  }
  if (!rc) rc = aijhip_ksp_set_norm_type(c->k, nt);
  if (!rc) rc = aijhip_ksp_set_tolerances(c->k, ksp->rtol, ksp->abstol, ksp->divtol, (int32_t)ksp->max_it);
  if (!rc) rc = aijhip_ksp_set_up(c->k);
  if (rc) SETERRQ1(PetscObjectComm((PetscObject)ksp), PETSC_ERR_LIB, "aijhip: %s", aijhip_last_error());
  c->h = h;
  c->state = state;
  c->pc = pc;
  PetscFunctionReturn(0);
}

/* KSPSolve: b up, the whole CG on the device, x down (aijhip_ksp_solve_host);
 * then its, rnorm, reason and the residual history as KSPSolve_CG leaves
 * them, and the monitors replayed from the history. */
static PetscErrorCode KSPSolve_CGHIP(KSP ksp)
{
  KSP_CGHIP         *c = (KSP_CGHIP*)ksp->data;
  const PetscScalar *b;
  PetscScalar       *x;
  int32_t           its, n = 0, i;
  double            rnorm, *hist = NULL;
  int               reason, rc;
  PetscErrorCode    ierr;

  PetscFunctionBegin;
  /* values changed since the set-up (KSPSolve does not call ops->setup
   * again for that): refresh the device KSP, or fall back */
  ierr = KSPSetUp_CGHIP(ksp);CHKERRQ(ierr);
  if (c->fallback) {
    ierr = KSPSetTolerances(c->inner, ksp->rtol, ksp->abstol, ksp->divtol, ksp->max_it);CHKERRQ(ierr);
    ierr = KSPSetInitialGuessNonzero(c->inner, ksp->guess_zero ? PETSC_FALSE : PETSC_TRUE);CHKERRQ(ierr);
    ierr = KSPSolve(c->inner, ksp->vec_rhs, ksp->vec_sol);CHKERRQ(ierr);
    ierr = KSPGetIterationNumber(c->inner, &ksp->its);CHKERRQ(ierr);
    ierr = KSPGetResidualNorm(c->inner, &ksp->rnorm);CHKERRQ(ierr);
    ierr = KSPGetConvergedReason(c->inner, &ksp->reason);CHKERRQ(ierr);
    PetscFunctionReturn(0);
  }
  rc = aijhip_ksp_set_tolerances(c->k, ksp->rtol, ksp->abstol, ksp->divtol, (int32_t)ksp->max_it);
  if (!rc) rc = aijhip_ksp_set_initial_guess_nonzero(c->k, ksp->guess_zero ? 0 : 1);
  if (rc) SETERRQ1(PetscObjectComm((PetscObject)ksp), PETSC_ERR_LIB, "aijhip: %s", aijhip_last_error());
  ierr = VecGetArrayRead(ksp->vec_rhs, &b);CHKERRQ(ierr);
  ierr = VecGetArray(ksp->vec_sol, &x);CHKERRQ(ierr);
  rc = aijhip_ksp_solve_host(c->k, b, x);
  ierr = VecRestoreArrayRead(ksp->vec_rhs, &b);CHKERRQ(ierr);
  ierr = VecRestoreArray(ksp->vec_sol, &x);CHKERRQ(ierr);
  if (rc) SETERRQ1(PetscObjectComm((PetscObject)ksp), PETSC_ERR_LIB, "aijhip: %s", aijhip_last_error());
  aijhip_ksp_get_iteration_number(c->k, &its);
  aijhip_ksp_get_residual_norm(c->k, &rnorm);
  aijhip_ksp_get_converged_reason(c->k, &reason); /* PETSc's KSPConvergedReason values */
  ksp->its    = its;
  ksp->rnorm  = rnorm;
  ksp->reason = (KSPConvergedReason)reason;
  ierr = PetscMalloc1(its + 2, &hist);CHKERRQ(ierr);
  aijhip_ksp_get_residual_history(c->k, hist, its + 2, &n);
  for (i = 0; i < n; ++i) {
    ierr = KSPLogResidualHistory(ksp, hist[i]);CHKERRQ(ierr);
    ierr = KSPMonitor(ksp, i, hist[i]);CHKERRQ(ierr);
  }
  ierr = PetscFree(hist);CHKERRQ(ierr);
  PetscFunctionReturn(0);
}

static PetscErrorCode KSPDestroy_CGHIP(KSP ksp)
{
  PetscErrorCode ierr;

  PetscFunctionBegin;
  ierr = KSPCGHIPFree((KSP_CGHIP*)ksp->data);CHKERRQ(ierr);
  ierr = KSPCGHIPRestorePC(ksp);CHKERRQ(ierr);
  ierr = KSPDestroy(&((KSP_CGHIP*)ksp->data)->inner);CHKERRQ(ierr);
  ierr = KSPDestroyDefault(ksp);CHKERRQ(ierr);
  PetscFunctionReturn(0);
}

PETSC_EXTERN PetscErrorCode KSPCreate_CGHIP(KSP ksp)
{
  KSP_CGHIP      *c;
  PetscErrorCode ierr;

  PetscFunctionBegin;
  ierr = PetscNewLog(ksp, &c);CHKERRQ(ierr);
  ksp->data = (void*)c;
  /* KSPCG's norms and sides (left preconditioning only) */
  ierr = KSPSetSupportedNorm(ksp, KSP_NORM_PRECONDITIONED, PC_LEFT, 3);CHKERRQ(ierr);
  ierr = KSPSetSupportedNorm(ksp, KSP_NORM_UNPRECONDITIONED, PC_LEFT, 2);CHKERRQ(ierr);
  ierr = KSPSetSupportedNorm(ksp, KSP_NORM_NATURAL, PC_LEFT, 2);CHKERRQ(ierr);
  ierr = KSPSetSupportedNorm(ksp, KSP_NORM_NONE, PC_LEFT, 1);CHKERRQ(ierr);
  ksp->ops->setup          = KSPSetUp_CGHIP;
  ksp->ops->solve          = KSPSolve_CGHIP;
  ksp->ops->destroy        = KSPDestroy_CGHIP;
  ksp->ops->setfromoptions = NULL;
  ksp->ops->buildsolution  = KSPBuildSolutionDefault;
  ksp->ops->buildresidual  = KSPBuildResidualDefault;
  PetscFunctionReturn(0);
}
