/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of PETSc 3.7.6's sequential AIJ (CSR) kernels, the hot path
 * that olcf/PETSC-OpenACC offloads. Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this file's library, and only as the
 * checker / the timed CPU baseline — never as the product path.
 *
 * Parity status: PINNED ONLY BY RESTATEMENT. The reference holds no golden
 * vectors for MatMult_SeqAIJ and PETSc itself (which holds the original loop,
 * aij.c:1277-1335 [ext], cut out by /root/reference/scripts/petsc.sh:85-86) is
 * not in this image, so the reference cannot be built here.
 * This restatement is cross-checked bit for bit against an independent numpy
 * restatement (oracle/seqaij.py) and against the committed fixtures in
 * tests/golden/ generated from it. "parity unpinned" w.r.t. a reference run.
 *
 * Arithmetic contract (what the GPU path must reproduce):
 *   - rows in index order; within a row, products in storage (ascending
 *     column) order;                              step1 patch:22-31
 *   - sum starts at 0.0 (MatMult) or at z[i] (MatMultAdd);
 *   - each product aa[k]*x[aj[k]] is rounded to fp64, then added (no FMA
 *     contraction: build with -ffp-contract=off).
 */
#include <stdint.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* MatMult_SeqAIJ: y = A*x, overwrite.
 * Follows /root/reference/src/openacc-step1/MatMult_SeqAIJ.patch:22-31
 * (the original loop visible as context in step2 patch:30-40):
 *   n = ii[i+1]-ii[i]; aj = a->j+ii[i]; aa = a->a+ii[i]; sum = 0.0;
 *   PetscSparseDensePlusDot(sum,x,aa,aj,n); y[i] = sum;
 * PetscSparseDensePlusDot [ext] expands to `for (k<n) sum += aa[k]*x[aj[k]]`. */
void oracle_matmult_seqaij(int32_t m, const int32_t *ai, const int32_t *aj,
                           const double *aa, const double *x, double *y)
{
    for (int32_t i = 0; i < m; i++) {
        const int32_t n = ai[i + 1] - ai[i];
        const int32_t *cj = aj + ai[i];
        const double *ca = aa + ai[i];
        double sum = 0.0;
        for (int32_t k = 0; k < n; k++) sum += ca[k] * x[cj[k]];
        y[i] = sum;
    }
}

/* MatMultAdd_SeqAIJ [ext, aij.c in PETSc 3.7.6]: w = z + A*x.
 * Same loop with `sum = z[i]` as the starting value; PETSc logs 2*nz flops. */
void oracle_matmultadd_seqaij(int32_t m, const int32_t *ai, const int32_t *aj,
                              const double *aa, const double *x,
                              const double *z, double *w)
{
    for (int32_t i = 0; i < m; i++) {
        const int32_t n = ai[i + 1] - ai[i];
        const int32_t *cj = aj + ai[i];
        const double *ca = aa + ai[i];
        double sum = z[i];
        for (int32_t k = 0; k < n; k++) sum += ca[k] * x[cj[k]];
        w[i] = sum;
    }
}

/* MatMultTranspose_SeqAIJ [ext]: y = A^T x. PETSc zeroes y, then for each row
 * i scatters alpha = x[i] into y[aj[k]] += aa[k]*alpha in row order. */
void oracle_matmulttranspose_seqaij(int32_t m, int32_t ncols, const int32_t *ai,
                                    const int32_t *aj, const double *aa,
                                    const double *x, double *y)
{
    memset(y, 0, sizeof(double) * (size_t)ncols);
    for (int32_t i = 0; i < m; i++) {
        const double alpha = x[i];
        for (int32_t k = ai[i]; k < ai[i + 1]; k++) y[aj[k]] += aa[k] * alpha;
    }
}

/* Row-block parallel variant of oracle_matmult_seqaij for the all-cores CPU
 * baseline (the analogue of the reference's 16-rank node run,
 * /root/reference/runs/single-node-scaling.pbs:56-67). Each row is still
 * summed sequentially, so results are bitwise identical to the 1-core loop. */
void oracle_matmult_seqaij_omp(int32_t m, const int32_t *ai, const int32_t *aj,
                               const double *aa, const double *x, double *y)
{
#pragma omp parallel for schedule(static)
    for (int32_t i = 0; i < m; i++) {
        const int32_t n = ai[i + 1] - ai[i];
        const int32_t *cj = aj + ai[i];
        const double *ca = aa + ai[i];
        double sum = 0.0;
        for (int32_t k = 0; k < n; k++) sum += ca[k] * x[cj[k]];
        y[i] = sum;
    }
}

int oracle_omp_threads(void)
{
    int t = 1;
#ifdef _OPENMP
#pragma omp parallel
    {
#pragma omp single
        t = omp_get_num_threads();
    }
#endif
    return t;
}
