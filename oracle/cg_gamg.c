/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (bench.py's cpu_baseline leg and tests/).
 *
 * Host CG + GAMG solve on all host cores: the reference's CPU configuration
 * (/root/reference/src/main_ksp.cpp:92-106 with
 * /root/reference/configs/PETSc_SolverOptions_GAMG.info:1-21, timed on
 * 1-16 ranks by /root/reference/runs/single-node-scaling.pbs:56-67) restated
 * in C with OpenMP row blocks, over a hierarchy handed in by the caller (the
 * library's host builder, include/aijhip_gamg.h). Numerically it is the
 * restatement of oracle/ksp_cg.py (KSPSolve_CG [ext] + KSPConvergedDefault)
 * preconditioned by oracle/gamg.py's V-cycle (PCMG multiplicative,
 * Richardson(1) + Jacobi down and up, P^T restriction, P interpolation,
 * preonly + Jacobi on the coarsest); rows are summed sequentially in storage
 * order as MatMult_SeqAIJ (step1 patch:22-31), dots are OpenMP reductions.
 *
 * Parity unpinned w.r.t. PETSc (absent). Used as the measured CPU baseline
 * ("port") beside the device solve, never as the product path.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef struct {
    int32_t m;                      /* rows of A_l                            */
    const int32_t *ai, *aj;         /* A_l (m x m)                            */
    const double *aa;
    const int32_t *pi, *pj;         /* P_l (m x m_{l+1}); NULL on the coarsest */
    const double *pa;
} oracle_level_t;

typedef struct {
    int32_t m, mc;
    int32_t *ti, *tj;               /* P^T (mc x m), rows in ascending fine order */
    double *ta;
    double *dinv, *b, *x, *r;
} lvl_t;

static double first_diag_inv(const oracle_level_t *L, int32_t i)
{
    double d = 0.0;
    for (int32_t k = L->ai[i]; k < L->ai[i + 1]; k++)
        if (L->aj[k] == i) { d = L->aa[k]; break; }
    if (d == 0.0) d = 1.0;
    return 1.0 / d;
}

/* P^T by counting sort on the column: each column's entries keep ascending
 * fine-row order, PETSc's MatMultTranspose scatter order. */
static int transpose(const oracle_level_t *L, int32_t mc, lvl_t *T)
{
    const int32_t m = L->m;
    const int64_t nz = L->pi[m];
    T->ti = calloc((size_t)mc + 1, sizeof(int32_t));
    T->tj = malloc(sizeof(int32_t) * (size_t)(nz > 0 ? nz : 1));
    T->ta = malloc(sizeof(double) * (size_t)(nz > 0 ? nz : 1));
    int32_t *pos = malloc(sizeof(int32_t) * ((size_t)mc + 1));
    if (!T->ti || !T->tj || !T->ta || !pos) { free(pos); return 1; }
    for (int64_t k = 0; k < nz; k++) T->ti[L->pj[k] + 1]++;
    for (int32_t c = 0; c < mc; c++) T->ti[c + 1] += T->ti[c];
    memcpy(pos, T->ti, sizeof(int32_t) * ((size_t)mc + 1));
    for (int32_t i = 0; i < m; i++)
        for (int32_t k = L->pi[i]; k < L->pi[i + 1]; k++) {
            const int32_t c = L->pj[k];
            T->tj[pos[c]] = i;
            T->ta[pos[c]++] = L->pa[k];
        }
    free(pos);
    return 0;
}

/* y = M v, rows in parallel, each row sequential */
static void spmv(int32_t m, const int32_t *ai, const int32_t *aj, const double *aa, const double *v, double *y)
{
#pragma omp parallel for schedule(static)
    for (int32_t i = 0; i < m; i++) {
        double s = 0.0;
        for (int32_t k = ai[i]; k < ai[i + 1]; k++) s += aa[k] * v[aj[k]];
        y[i] = s;
    }
}

static double dot(int32_t n, const double *a, const double *b)
{
    double s = 0.0;
#pragma omp parallel for schedule(static) reduction(+ : s)
    for (int32_t i = 0; i < n; i++) s += a[i] * b[i];
    return s;
}

/* PCApply_MG: one V-cycle, z = B r */
static void vcycle(int nl, const oracle_level_t *L, lvl_t *V, const double *r0, double *z0)
{
    for (int l = 0; l < nl; l++) {
        lvl_t *v = &V[l];
        const double *b = l == 0 ? r0 : v->b;
        double *x = l == 0 ? z0 : v->x;
        const oracle_level_t *A = &L[l];
        /* smoothd (Richardson(1)+Jacobi from x = 0): x = D^-1 b */
#pragma omp parallel for schedule(static)
        for (int32_t i = 0; i < v->m; i++) x[i] = v->dinv[i] * b[i];
        if (l == nl - 1) break;  /* coarse: preonly + Jacobi */
        /* r = b - A x */
#pragma omp parallel for schedule(static)
        for (int32_t i = 0; i < v->m; i++) {
            double s = 0.0;
            for (int32_t k = A->ai[i]; k < A->ai[i + 1]; k++) s += A->aa[k] * x[A->aj[k]];
            v->r[i] = b[i] + (-1.0) * s;
        }
        /* MatRestrict: b_{l+1} = P^T r */
        spmv(v->mc, v->ti, v->tj, v->ta, v->r, V[l + 1].b);
    }
    for (int l = nl - 2; l >= 0; l--) {
        lvl_t *v = &V[l];
        const double *b = l == 0 ? r0 : v->b;
        double *x = l == 0 ? z0 : v->x;
        const double *xc = V[l + 1].x;
        const oracle_level_t *A = &L[l];
        /* MatInterpolateAdd: t = x + P x_c (t in r) */
#pragma omp parallel for schedule(static)
        for (int32_t i = 0; i < v->m; i++) {
            double s = x[i];
            for (int32_t k = A->pi[i]; k < A->pi[i + 1]; k++) s += A->pa[k] * xc[A->pj[k]];
            v->r[i] = s;
        }
        /* smoothu: x = t + D^-1 (b - A t) */
#pragma omp parallel for schedule(static)
        for (int32_t i = 0; i < v->m; i++) {
            double s = 0.0;
            for (int32_t k = A->ai[i]; k < A->ai[i + 1]; k++) s += A->aa[k] * v->r[A->aj[k]];
            x[i] = v->r[i] + 1.0 * (v->dinv[i] * (b[i] + (-1.0) * s));
        }
    }
}

/* KSPSolve_CG with the GAMG V-cycle as PC, from x = 0, preconditioned norm.
 * Returns the KSPConvergedReason; *its, *rnorm, hist[0..its] as PETSc.
 * threads <= 0: OpenMP's default. *setup_s: the P^T / Jacobi / work-vector
 * set-up time of this call (the hierarchy itself is the caller's). */
int oracle_cg_gamg(int nl, const oracle_level_t *L, const double *b, double *x, double rtol, double atol,
                   int32_t max_it, int threads, int32_t *its_out, double *rnorm_out, double *hist,
                   double *setup_s)
{
#ifdef _OPENMP
    const int threads0 = omp_get_max_threads();  /* restored on return: the ICV is process-wide */
    if (threads > 0) omp_set_num_threads(threads);
    double t0 = omp_get_wtime();
#endif
    lvl_t *V = calloc((size_t)nl, sizeof(lvl_t));
    const int32_t m = L[0].m;
    double *r = malloc(sizeof(double) * (size_t)m), *z = malloc(sizeof(double) * (size_t)m);
    double *p = malloc(sizeof(double) * (size_t)m), *w = malloc(sizeof(double) * (size_t)m);
    int reason = 0, fail = !V || !r || !z || !p || !w;
    for (int l = 0; l < nl && !fail; l++) {
        lvl_t *v = &V[l];
        v->m = L[l].m;
        v->mc = l + 1 < nl ? L[l + 1].m : 0;
        const size_t vb = sizeof(double) * (size_t)(v->m > 0 ? v->m : 1);
        v->dinv = malloc(vb); v->b = malloc(vb); v->x = malloc(vb); v->r = malloc(vb);
        if (!v->dinv || !v->b || !v->x || !v->r) { fail = 1; break; }
#pragma omp parallel for schedule(static)
        for (int32_t i = 0; i < v->m; i++) v->dinv[i] = first_diag_inv(&L[l], i);
        if (l + 1 < nl && transpose(&L[l], v->mc, v)) fail = 1;
    }
#ifdef _OPENMP
    if (setup_s) *setup_s = omp_get_wtime() - t0;
#else
    if (setup_s) *setup_s = 0.0;
#endif
    int32_t its = 0;
    double dp = 0.0;
    if (!fail) {
        const oracle_level_t *A = &L[0];
        memset(x, 0, sizeof(double) * (size_t)m);
        memcpy(r, b, sizeof(double) * (size_t)m);
        vcycle(nl, L, V, r, z);
        dp = sqrt(dot(m, z, z));
        hist[0] = dp;
        const double ttol = fmax(rtol * dp, atol), rnorm0 = dp;
        if (isnan(dp) || isinf(dp)) reason = -9;
        else if (dp <= ttol) reason = dp < atol ? 3 : 2;
        double beta = dot(m, z, r), betaold = 0.0, dpi = 0.0, dpiold;
        for (int32_t i = 0; !reason && i < max_it; i++) {
            its = i + 1;
            if (beta == 0.0) { reason = 3; break; }
            if (i > 0 && beta * betaold < 0.0) { reason = -8; break; }
            const double bb = i == 0 ? 0.0 : beta / betaold;
#pragma omp parallel for schedule(static)
            for (int32_t k = 0; k < m; k++) p[k] = i == 0 ? z[k] : z[k] + bb * p[k];
            spmv(m, A->ai, A->aj, A->aa, p, w);
            dpiold = dpi;
            dpi = dot(m, p, w);
            betaold = beta;
            if (dpi == 0.0 || (i > 0 && dpi * dpiold <= 0.0)) { reason = -10; break; }
            const double a = beta / dpi;
#pragma omp parallel for schedule(static)
            for (int32_t k = 0; k < m; k++) {
                x[k] = x[k] + a * p[k];
                r[k] = r[k] + (-a) * w[k];
            }
            vcycle(nl, L, V, r, z);
            dp = sqrt(dot(m, z, z));
            hist[i + 1] = dp;
            if (isnan(dp) || isinf(dp)) reason = -9;
            else if (dp <= ttol) reason = dp < atol ? 3 : 2;
            else if (dp >= 1e5 * rnorm0) reason = -4;
            if (reason) break;
            beta = dot(m, z, r);
        }
        if (!reason) reason = -3;
    }
    for (int l = 0; V && l < nl; l++) {
        free(V[l].ti); free(V[l].tj); free(V[l].ta);
        free(V[l].dinv); free(V[l].b); free(V[l].x); free(V[l].r);
    }
    free(V); free(r); free(z); free(p); free(w);
    if (its_out) *its_out = its;
    if (rnorm_out) *rnorm_out = dp;
#ifdef _OPENMP
    omp_set_num_threads(threads0);
#endif
    return fail ? 0 : reason;
}
