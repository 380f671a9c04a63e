/*
 * aijhip_petsc.c — PETSc 3.7 adapter: SeqAIJ matrices whose MatMult runs on
 * the MI355X through libaijhip.so (include/aijhip.h).
 *
 * NOT COMPILED IN THIS IMAGE: there is no PETSc here or on the GPU box
 * (SURVEY.md §8c). `make -C petsc-openacc_amd/petsc` builds it against a
 * PETSc source tree when PETSC_DIR/PETSC_ARCH are set. The logic it wraps —
 * create / update_values / assembly_end / mult_host / destroy — is what the
 * tests exercise through the same C ABI.
 *
 * What the reference does: scripts/petsc.sh:81-89 cuts
 * MatMult_SeqAIJ, MatAssemblyEnd_SeqAIJ and MatDestroy_SeqAIJ out of aij.c
 * and Makefile:153-158 links OpenACC-patched copies ahead of libpetsc.a.
 * Two ways to put this library in their place:
 *
 *  (1) Registered type (default build). AIJHIPRegister() adds the type
 *      "seqaijhip" and, with replace = PETSC_TRUE, also re-registers the
 *      "seqaij" constructor, so every SeqAIJ matrix PETSc creates — the
 *      DMCreateMatrix operand that helper.cpp:39 forces to MATAIJ, the
 *      diagonal block of an MPIAIJ, GAMG's Galerkin operators — gets the
 *      device MatMult while keeping the type name "seqaij" that GAMG and
 *      MPIAIJ compare against. With a shared PETSc the options file line
 *      `-dll_append <path>/libaijhip_petsc.so` runs the registration
 *      (PetscDLLibraryRegister_aijhip_petsc below), so main_ksp.cpp and
 *      configs/PETSc_SolverOptions_GAMG.info are used unchanged.
 *  (2) Link-time override (-DAIJHIP_PETSC_OVERRIDE), for the reference's
 *      static build: defines the three cut-out symbols. MatAssemblyEnd_SeqAIJ
 *      and MatDestroy_SeqAIJ wrap PETSc's original bodies, which
 *      scripts/petsc.sh:81-86 has already extracted to src/original/*.c
 *      (included here under a renamed symbol, not copied); MatMult_SeqAIJ
 *      is replaced outright.
 *
 * Vectors: PETSc 3.7 Vecs are host arrays, so MatMult has the reference's
 * step-2 semantics (matrix resident on the device, x in and y out over PCIe
 * per call: aijhip_mat_mult_host, which pipelines the two copies with the
 * product the way steps 3/4 do). MatMultAdd (MatMult_MPIAIJ's off-diagonal
 * product, PCMG's interpolation) and MatMultTranspose (PCMG's restriction),
 * which the reference leaves on the CPU, run on the device too when the
 * matrix has at least -aijhip_transfer_min_nz entries (default 262144:
 * below that PETSc's own loop beats a PCIe round trip); smaller ones keep
 * PETSc's SeqAIJ (or Inode) bodies. A device Vec type is what removes the
 * PCIe traffic; the KSP type "cghip"
 * (aijhip_ksp_petsc.c, registered below) removes it for the reference's
 * solver by running the whole KSPSolve on the device.
 */
#include <petsc/private/matimpl.h>
#include <petscksp.h>
#include <../src/mat/impls/aij/seq/aij.h>

#include "aijhip.h"

typedef struct {
  aijhip_mat_t     h;
  PetscObjectState nonzerostate; /* A->nonzerostate at the last upload */
  PetscObjectState state;        /* object state at the last upload: values
                                    changed without an assembly (MatScale,
                                    MatShift, MatDuplicate, ...) raise it */
  PetscBool        stale;        /* set by the assembly hook: the next product
                                    re-uploads and records the state it sees */
  /* PETSc's CPU bodies the assembly left in the ops table (SeqAIJ or Inode),
     for matrices below the transfer threshold */
  PetscErrorCode (*cpu_multadd)(Mat, Vec, Vec, Vec);
  PetscErrorCode (*cpu_multtranspose)(Mat, Vec, Vec);
} Mat_AIJHIP;

static PetscInt transfer_min_nz = -1; /* -aijhip_transfer_min_nz, read once */

static PetscErrorCode AIJHIPTransferMinNz(PetscInt *out)
{
  PetscErrorCode ierr;

  PetscFunctionBegin;
  if (transfer_min_nz < 0) {
    transfer_min_nz = 262144;
    ierr = PetscOptionsGetInt(NULL, NULL, "-aijhip_transfer_min_nz", &transfer_min_nz, NULL);CHKERRQ(ierr);
  }
  *out = transfer_min_nz;
  PetscFunctionReturn(0);
}

static PetscErrorCode AIJHIPDevice(Mat A, int *dev)
{
  PetscMPIInt    rank;
  int            count = 0;
  PetscErrorCode ierr;

  PetscFunctionBegin;
  ierr = MPI_Comm_rank(PETSC_COMM_WORLD, &rank);CHKERRQ(ierr);
  if (aijhip_device_count(&count) || count < 1) SETERRQ1(PetscObjectComm((PetscObject)A), PETSC_ERR_LIB, "aijhip: %s", aijhip_last_error());
  *dev = (int)(rank % count); /* ranks of a node share its GPUs round-robin */
  PetscFunctionReturn(0);
}

/* The device copy brought up to date (step2 MatAssemblyEnd patch:17-44, done
 * at the first product after the assembly as step 2's MatMult copyin does,
 * step2 MatMult patch:19-21): first use creates; same nonzero structure ->
 * new values only; changed structure -> drop and re-upload. The state
 * recorded is the one read here, at product time, so it is exact whatever
 * PETSc raised after the assembly hook returned (the public MatAssemblyEnd
 * raises it once more; an internal direct call does not). */
static PetscErrorCode AIJHIPUpload(Mat A)
{
  Mat_SeqAIJ     *a = (Mat_SeqAIJ*)A->data;
  Mat_AIJHIP     *d = (Mat_AIJHIP*)A->spptr;
  int            dev, rc;
  PetscErrorCode ierr;

  PetscFunctionBegin;
  if (!d) {
    ierr = PetscNew(&d);CHKERRQ(ierr);
    A->spptr = d;
  }
  if (!d->h) {
    ierr = AIJHIPDevice(A, &dev);CHKERRQ(ierr);
    rc = aijhip_mat_create(dev, (int32_t)A->rmap->n, (int32_t)A->cmap->n, (int64_t)a->nz, a->i, a->j, a->a, &d->h);
  } else if (d->nonzerostate == A->nonzerostate) {
    rc = aijhip_mat_update_values(d->h, a->a);
  } else {
    rc = aijhip_mat_assembly_end(d->h, (int64_t)a->nz, a->i, a->j, a->a);
  }
  if (rc) SETERRQ1(PetscObjectComm((PetscObject)A), PETSC_ERR_LIB, "aijhip: %s", aijhip_last_error());
  d->nonzerostate = A->nonzerostate;
  ierr = PetscObjectStateGet((PetscObject)A, &d->state);CHKERRQ(ierr);
  d->stale = PETSC_FALSE;
  PetscFunctionReturn(0);
}

/* The assembly hook's device half: a final assembly makes the device copy
 * stale (flush assembly does nothing, step2 MatAssemblyEnd patch:15). */
static PetscErrorCode AIJHIPMarkStale(Mat A, MatAssemblyType mode)
{
  Mat_AIJHIP     *d = (Mat_AIJHIP*)A->spptr;
  PetscErrorCode ierr;

  PetscFunctionBegin;
  if (mode == MAT_FLUSH_ASSEMBLY) PetscFunctionReturn(0);
  if (!d) {
    ierr = PetscNew(&d);CHKERRQ(ierr);
    A->spptr = d;
  }
  d->stale = PETSC_TRUE;
  PetscFunctionReturn(0);
}

static PetscErrorCode AIJHIPFree(Mat A)
{
  Mat_AIJHIP     *d = (Mat_AIJHIP*)A->spptr;
  PetscErrorCode ierr;

  PetscFunctionBegin;
  if (d) {
    if (d->h) aijhip_mat_destroy(d->h);
    ierr = PetscFree(d);CHKERRQ(ierr);
    A->spptr = NULL;
  }
  PetscFunctionReturn(0);
}

static PetscErrorCode AIJHIPCurrent(Mat, Mat_AIJHIP**);

/* y = A x with the device-resident matrix; x and y are host arrays. */
static PetscErrorCode AIJHIPMult(Mat A, Vec xx, Vec yy)
{
  Mat_SeqAIJ        *a = (Mat_SeqAIJ*)A->data;
  Mat_AIJHIP        *d = (Mat_AIJHIP*)A->spptr;
  const PetscScalar *x;
  PetscScalar       *y;
  PetscErrorCode    ierr;

  PetscFunctionBegin;
  ierr = AIJHIPCurrent(A, &d);CHKERRQ(ierr); /* never uploaded, or host values changed since */
  ierr = VecGetArrayRead(xx, &x);CHKERRQ(ierr);
  ierr = VecGetArray(yy, &y);CHKERRQ(ierr);
  if (aijhip_mat_mult_host(d->h, x, y)) SETERRQ1(PetscObjectComm((PetscObject)A), PETSC_ERR_LIB, "aijhip: %s", aijhip_last_error());
  ierr = VecRestoreArrayRead(xx, &x);CHKERRQ(ierr);
  ierr = VecRestoreArray(yy, &y);CHKERRQ(ierr);
  ierr = PetscLogFlops(2.0*a->nz - a->nonzerorowcnt);CHKERRQ(ierr); /* step2 MatMult patch:47 */
  PetscFunctionReturn(0);
}

/* Bring the device copy up to date before a product (first use, or host
 * values changed since the last upload). */
static PetscErrorCode AIJHIPCurrent(Mat A, Mat_AIJHIP **out)
{
  Mat_AIJHIP       *d = (Mat_AIJHIP*)A->spptr;
  PetscObjectState state;
  PetscErrorCode   ierr;

  PetscFunctionBegin;
  ierr = PetscObjectStateGet((PetscObject)A, &state);CHKERRQ(ierr);
  if (!d || !d->h || d->stale || d->state != state) {
    if (!A->assembled) SETERRQ(PetscObjectComm((PetscObject)A), PETSC_ERR_ARG_WRONGSTATE, "aijhip: product with an unassembled matrix");
    ierr = AIJHIPUpload(A);CHKERRQ(ierr);
  }
  *out = (Mat_AIJHIP*)A->spptr;
  PetscFunctionReturn(0);
}

/* The device handle of A brought up to date (aijhip_ksp_petsc.c's KSP type
 * solves on it); NULL when A is not a matrix of this adapter. */
PETSC_EXTERN PetscErrorCode AIJHIPGetHandle(Mat A, aijhip_mat_t *h)
{
  Mat_AIJHIP     *d;
  PetscErrorCode ierr;

  PetscFunctionBegin;
  *h = NULL;
  if (A->ops->mult != AIJHIPMult) PetscFunctionReturn(0);
  ierr = AIJHIPCurrent(A, &d);CHKERRQ(ierr);
  *h = d->h;
  PetscFunctionReturn(0);
}

/* zz = yy + A xx (MatMultAdd_SeqAIJ: each row sum starts from yy[i]). */
static PetscErrorCode AIJHIPMultAdd(Mat A, Vec xx, Vec yy, Vec zz)
{
  Mat_SeqAIJ        *a = (Mat_SeqAIJ*)A->data;
  Mat_AIJHIP        *d = (Mat_AIJHIP*)A->spptr;
  const PetscScalar *x, *y;
  PetscScalar       *z;
  PetscInt          min_nz;
  PetscErrorCode    ierr;

  PetscFunctionBegin;
  ierr = AIJHIPTransferMinNz(&min_nz);CHKERRQ(ierr);
  if (a->nz < min_nz && d && d->cpu_multadd) {
    ierr = (*d->cpu_multadd)(A, xx, yy, zz);CHKERRQ(ierr);
    PetscFunctionReturn(0);
  }
  ierr = AIJHIPCurrent(A, &d);CHKERRQ(ierr);
  ierr = VecGetArrayRead(xx, &x);CHKERRQ(ierr);
  if (yy == zz) {
    ierr = VecGetArray(zz, &z);CHKERRQ(ierr);
    y = z;
  } else {
    ierr = VecGetArrayRead(yy, &y);CHKERRQ(ierr);
    ierr = VecGetArray(zz, &z);CHKERRQ(ierr);
  }
  if (aijhip_mat_mult_add_host(d->h, x, y, z)) SETERRQ1(PetscObjectComm((PetscObject)A), PETSC_ERR_LIB, "aijhip: %s", aijhip_last_error());
  ierr = VecRestoreArrayRead(xx, &x);CHKERRQ(ierr);
  if (yy != zz) {
    ierr = VecRestoreArrayRead(yy, &y);CHKERRQ(ierr);
  }
  ierr = VecRestoreArray(zz, &z);CHKERRQ(ierr);
  ierr = PetscLogFlops(2.0*a->nz);CHKERRQ(ierr);
  PetscFunctionReturn(0);
}

/* yy = A^T xx (MatMultTranspose_SeqAIJ's scatter order, kept by the device
 * transpose). */
static PetscErrorCode AIJHIPMultTranspose(Mat A, Vec xx, Vec yy)
{
  Mat_SeqAIJ        *a = (Mat_SeqAIJ*)A->data;
  Mat_AIJHIP        *d = (Mat_AIJHIP*)A->spptr;
  const PetscScalar *x;
  PetscScalar       *y;
  PetscInt          min_nz;
  PetscErrorCode    ierr;

  PetscFunctionBegin;
  ierr = AIJHIPTransferMinNz(&min_nz);CHKERRQ(ierr);
  if (a->nz < min_nz && d && d->cpu_multtranspose) {
    ierr = (*d->cpu_multtranspose)(A, xx, yy);CHKERRQ(ierr);
    PetscFunctionReturn(0);
  }
  ierr = AIJHIPCurrent(A, &d);CHKERRQ(ierr);
  ierr = VecGetArrayRead(xx, &x);CHKERRQ(ierr);
  ierr = VecGetArray(yy, &y);CHKERRQ(ierr);
  if (aijhip_mat_mult_transpose_host(d->h, x, y)) SETERRQ1(PetscObjectComm((PetscObject)A), PETSC_ERR_LIB, "aijhip: %s", aijhip_last_error());
  ierr = VecRestoreArrayRead(xx, &x);CHKERRQ(ierr);
  ierr = VecRestoreArray(yy, &y);CHKERRQ(ierr);
  ierr = PetscLogFlops(2.0*a->nz);CHKERRQ(ierr);
  PetscFunctionReturn(0);
}

/* After PETSc's assembly: remember the CPU multadd / multtranspose it
 * installed (the Inode check may pick its own), then point the ops table at
 * the device forms. */
static PetscErrorCode AIJHIPInstallOps(Mat A)
{
  Mat_AIJHIP *d = (Mat_AIJHIP*)A->spptr;

  PetscFunctionBegin;
  if (A->ops->multadd != AIJHIPMultAdd) d->cpu_multadd = A->ops->multadd;
  if (A->ops->multtranspose != AIJHIPMultTranspose) d->cpu_multtranspose = A->ops->multtranspose;
  A->ops->multadd       = AIJHIPMultAdd;
  A->ops->multtranspose = AIJHIPMultTranspose;
  PetscFunctionReturn(0);
}

#if !defined(AIJHIP_PETSC_OVERRIDE)
/* ---------------------------------------------------------------- (1) */
/* PETSc's own SeqAIJ operations, taken from the ops table MatCreate_SeqAIJ
 * fills (the symbols are PETSC_INTERN in shared builds). */
static PetscErrorCode (*seqaij_assemblyend)(Mat, MatAssemblyType) = NULL;
static PetscErrorCode (*seqaij_destroy)(Mat) = NULL;

static PetscErrorCode MatAssemblyEnd_SeqAIJHIP(Mat A, MatAssemblyType mode)
{
  PetscErrorCode ierr;

  PetscFunctionBegin;
  ierr = (*seqaij_assemblyend)(A, mode);CHKERRQ(ierr); /* compaction, compressed rows, inodes */
  /* MatAssemblyEnd_SeqAIJ_Inode [ext] points ops->mult at MatMult_SeqAIJ_Inode
   * when it finds identical-pattern rows (multi-dof FEM operators such as
   * Flan_1565): take MatMult back, or such matrices would multiply on the CPU */
  A->ops->mult = AIJHIPMult;
  ierr = AIJHIPMarkStale(A, mode);CHKERRQ(ierr);
  if (mode == MAT_FINAL_ASSEMBLY) {
    ierr = AIJHIPInstallOps(A);CHKERRQ(ierr);
  }
  PetscFunctionReturn(0);
}

static PetscErrorCode MatDestroy_SeqAIJHIP(Mat A)
{
  PetscErrorCode ierr;

  PetscFunctionBegin;
  ierr = AIJHIPFree(A);CHKERRQ(ierr); /* device copy first (step2 MatDestroy patch:27-34) */
  ierr = (*seqaij_destroy)(A);CHKERRQ(ierr);
  PetscFunctionReturn(0);
}

static PetscBool type_name_seqaij = PETSC_FALSE;

PETSC_EXTERN PetscErrorCode MatCreate_SeqAIJHIP(Mat A)
{
  PetscErrorCode ierr;

  PetscFunctionBegin;
  ierr = MatCreate_SeqAIJ(A);CHKERRQ(ierr);
  if (!seqaij_assemblyend) {
    seqaij_assemblyend = A->ops->assemblyend;
    seqaij_destroy     = A->ops->destroy;
  }
  A->ops->assemblyend = MatAssemblyEnd_SeqAIJHIP;
  A->ops->destroy     = MatDestroy_SeqAIJHIP;
  A->ops->mult        = AIJHIPMult;
  if (!type_name_seqaij) {
    ierr = PetscObjectChangeTypeName((PetscObject)A, "seqaijhip");CHKERRQ(ierr);
  }
  PetscFunctionReturn(0);
}

/* replace = PETSC_TRUE: every "seqaij" matrix uses the device MatMult and
 * keeps its type name (the reference's link-time patch reaches every SeqAIJ
 * the same way). */
PETSC_EXTERN PetscErrorCode KSPCreate_CGHIP(KSP); /* aijhip_ksp_petsc.c */

PETSC_EXTERN PetscErrorCode AIJHIPRegister(PetscBool replace)
{
  PetscErrorCode ierr;

  PetscFunctionBegin;
  ierr = MatRegister("seqaijhip", MatCreate_SeqAIJHIP);CHKERRQ(ierr);
  /* -ksp_type cghip: the whole KSPSolve on the device (host Vecs cross PCIe
     once per solve, not per MatMult) */
  ierr = KSPRegister("cghip", KSPCreate_CGHIP);CHKERRQ(ierr);
  if (replace) {
    type_name_seqaij = PETSC_TRUE;
    ierr = MatRegister(MATSEQAIJ, MatCreate_SeqAIJHIP);CHKERRQ(ierr);
  }
  PetscFunctionReturn(0);
}

/* PETSc calls this when the library is loaded with -dll_append. */
PETSC_EXTERN PetscErrorCode PetscDLLibraryRegister_aijhip_petsc(void)
{
  PetscErrorCode ierr;
  PetscBool      replace = PETSC_TRUE;

  PetscFunctionBegin;
  ierr = PetscOptionsGetBool(NULL, NULL, "-aijhip_replace_seqaij", &replace, NULL);CHKERRQ(ierr);
  ierr = AIJHIPRegister(replace);CHKERRQ(ierr);
  PetscFunctionReturn(0);
}

#else
/* ---------------------------------------------------------------- (2) */
/* The originals scripts/petsc.sh extracted (reference build tree). */
#define MatAssemblyEnd_SeqAIJ MatAssemblyEnd_SeqAIJ_Original
#include "original/MatAssemblyEnd_SeqAIJ.c"
#undef MatAssemblyEnd_SeqAIJ
#define MatDestroy_SeqAIJ MatDestroy_SeqAIJ_Original
#include "original/MatDestroy_SeqAIJ.c"
#undef MatDestroy_SeqAIJ

PetscErrorCode MatMult_SeqAIJ(Mat, Vec, Vec);

PetscErrorCode MatAssemblyEnd_SeqAIJ(Mat A, MatAssemblyType mode)
{
  PetscErrorCode ierr;

  PetscFunctionBegin;
  ierr = MatAssemblyEnd_SeqAIJ_Original(A, mode);CHKERRQ(ierr);
  A->ops->mult = MatMult_SeqAIJ; /* the inode check may have installed MatMult_SeqAIJ_Inode */
  ierr = AIJHIPMarkStale(A, mode);CHKERRQ(ierr);
  if (mode == MAT_FINAL_ASSEMBLY) { /* MatMultAdd_SeqAIJ / MatMultTranspose_SeqAIJ stay in aij.o: only the ops table changes */
    ierr = AIJHIPInstallOps(A);CHKERRQ(ierr);
  }
  PetscFunctionReturn(0);
}

PetscErrorCode MatDestroy_SeqAIJ(Mat A)
{
  PetscErrorCode ierr;

  PetscFunctionBegin;
  ierr = AIJHIPFree(A);CHKERRQ(ierr);
  ierr = MatDestroy_SeqAIJ_Original(A);CHKERRQ(ierr);
  PetscFunctionReturn(0);
}

PetscErrorCode MatMult_SeqAIJ(Mat A, Vec xx, Vec yy)
{
  return AIJHIPMult(A, xx, yy);
}
#endif
