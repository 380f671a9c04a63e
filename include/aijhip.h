/*
 * aijhip.h — C ABI of the MI355X (gfx950) sequential-AIJ (CSR) SpMV.
 *
 * This is the drop-in boundary for the hot path olcf/PETSC-OpenACC offloads:
 * PETSc 3.7.6's MatMult_SeqAIJ plus the two residency hooks the reference
 * patches in beside it. The reference replaces three PETSc-internal C symbols
 * at link time (/root/reference/scripts/petsc.sh:81-89 cuts them out of aij.c,
 * /root/reference/Makefile:31,153-158 links the patched objects ahead of
 * libpetsc.a). Those symbols take PETSc types (Mat, Vec); this ABI takes plain
 * pointers and sizes instead, so a PETSc adapter — or any
 * C / ctypes / FFI caller — binds it without PETSc, CUDA-compat or torch
 * headers.
 *
 * Mapping (reference entry point -> this ABI):
 *   MatAssemblyEnd_SeqAIJ hook, src/openacc-step2/MatAssemblyEnd_SeqAIJ.patch:17-44
 *     first upload           -> aijhip_mat_create
 *     values changed          -> aijhip_mat_update_values
 *     structure changed       -> aijhip_mat_assembly_end
 *   MatMult_SeqAIJ, src/openacc-step{1..4}/MatMult_SeqAIJ.patch
 *     device-resident x, y    -> aijhip_mat_mult          (y = A x)
 *     host x, y (step-2 form) -> aijhip_mat_mult_host     (copy x in, y out)
 *   MatMultAdd_SeqAIJ [ext; left on the CPU by the reference, SURVEY §8f row 2]
 *                             -> aijhip_mat_mult_add      (w = z + A x)
 *   MatMultTranspose_SeqAIJ [ext; SURVEY §8f row 2]
 *                             -> aijhip_mat_mult_transpose (y = A^T x)
 *   MatDestroy_SeqAIJ hook, src/openacc-step2/MatDestroy_SeqAIJ.patch:18-34
 *                             -> aijhip_mat_destroy
 *
 * Types follow the reference's PETSc build: PetscInt is int32 (no
 * --with-64-bit-indices in scripts/petsc-release.sh:3-67), PetscScalar is
 * real fp64 (petsc-release.sh:6,62). Offsets into aj/aa are int32 as in PETSc;
 * all device address arithmetic is 64-bit.
 *
 * Error convention: every function returns 0 on success or a positive
 * AIJHIP_ERR_* code (PetscErrorCode is an int, 0 on success; CHKERRQ-style
 * propagation, step1 patch:16). Nothing throws across the ABI.
 * aijhip_last_error() returns a message for the calling thread's last error.
 *
 * Threading: one handle = one device, one host thread at a time (PETSc 3.7
 * objects are not thread-safe). Calls that take a `stream`
 * (a hipStream_t passed as void*, NULL = the legacy default stream) are
 * asynchronous with respect to the host; the ..._host variant synchronises.
 * A handle's launches must not be in flight on two streams at once: the
 * fork / join events of its side stream (AIJHIP_OPT_LONG_OVERLAP) are the
 * handle's own, so a second caller stream would wait on the first's fork.
 */
#ifndef AIJHIP_H
#define AIJHIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: aijhip_info_t gained mult_layout_bytes and lost the fields of the
 * withdrawn A/B-only options; their option values and kernel 4 are reserved
 * and return AIJHIP_ERR_ARG (measured slower, profiles/README.md).
 * 3: aijhip_gamg_params_t gained coarsen / square_graph / eig_ksp (PETSc
 * 3.7's MIS coarsening and CG emax estimate as options).
 * 4: aijhip_info_t gained hw_queues (the side streams' automatic choice
 * follows it); aijhip_mpi.h gained aijhip_mpiaij_get_overlap and the
 * automatic value -1 of aijhip_mpiaij_set_overlap.
 * 5: AIJHIP_OPT_ROW_TEMPLATES and AIJHIP_OPT_VALUE_CODES; aijhip_info_t's
 * former reserved0 is row_templates, and it gained value_codes (+ a
 * reserved word). */
#define AIJHIP_ABI_VERSION 5

enum {
    AIJHIP_OK = 0,
    AIJHIP_ERR_ARG = 1,      /* bad size, null pointer, malformed CSR        */
    AIJHIP_ERR_ALLOC = 2,    /* device or host allocation failed             */
    AIJHIP_ERR_HIP = 3,      /* a HIP runtime call failed                    */
    AIJHIP_ERR_NODEVICE = 4, /* no usable gfx950 device                      */
    AIJHIP_ERR_STATE = 5     /* call not valid in the handle's current state */
};

/* SpMV kernel families. AUTO picks by row-length
 * statistics at assembly time. */
enum {
    AIJHIP_KERNEL_AUTO = 0,
    AIJHIP_KERNEL_STREAM = 1, /* adaptive row blocks, products staged in LDS,
                                 sequential per-row sum: bit-exact vs PETSc */
    AIJHIP_KERNEL_SCALAR = 2, /* one lane per row (the reference's
                                 `gang vector(32)` shape, step1 patch:19-21) */
    AIJHIP_KERNEL_VECTOR = 3, /* 2..64 lanes per row, __shfl tree reduction
                                 (64 = wavefront per row)                    */
    /* 4: reserved (the explicit merge-path kernel, withdrawn in ABI 2;
       aijhip_mat_set_kernel returns AIJHIP_ERR_ARG) */
};

typedef struct aijhip_mat *aijhip_mat_t;

typedef struct aijhip_info {
    int32_t m;               /* rows                                         */
    int32_t n;               /* columns (length of x)                        */
    int64_t nz;              /* stored entries, explicit zeros included      */
    int32_t nonzerorowcnt;   /* rows with >= 1 stored entry (PETSc a->nonzerorowcnt) */
    int32_t max_row_nz;
    int32_t compressed_row;  /* 1 if the compressed-row form is used (PETSc
                                MatCheckCompressedRow, ratio 0.6)            */
    int32_t kernel;          /* AIJHIP_KERNEL_* actually used by mult        */
    int32_t vector_lanes;    /* lanes per row of the VECTOR kernel           */
    int32_t n_blocks;        /* STREAM row blocks                            */
    int32_t n_long_rows;     /* rows split across workgroups                 */
    int32_t device;
    int64_t device_bytes;    /* device memory owned by the handle            */
    double mult_flops;       /* PETSc-logged flops per MatMult: 2nz - nonzerorowcnt
                                (step2 MatMult patch:47)                     */
    int64_t mult_bytes;      /* algorithmic bytes per MatMult:
                                12 nz + 4 (m+1) + 8 n + 8 m     */
    int32_t stream_geometry; /* AIJHIP_OPT_* values in effect                */
    int32_t nt_loads;
    int32_t stream_threads;  /* lanes / entries / rows per STREAM block      */
    int32_t stream_nnz_cap;
    int32_t stream_rows;
    int32_t exact;           /* AIJHIP_OPT_EXACT in effect                   */
    int32_t gather_sorted;   /* MatMult reads the gather-ordered copy of the
                                row blocks (AIJHIP_OPT_GATHER_SORT): 1 with
                                32-bit columns, 2 with 16-bit block-relative
                                columns (every block spans < 2^16); 0 off   */
    int32_t column_codes;    /* MatMult reads 16-bit column codes instead of
                                aj (AIJHIP_OPT_COLUMN_CODES): the row blocks
                                whose columns the codes cover (10 bytes per
                                entry instead of 12); 0 off                  */
    int32_t row_patterns;    /* MatMult reads a pattern id per row instead of
                                aj (AIJHIP_OPT_ROW_PATTERNS): the number of
                                distinct column - row offset lists (with
                                row_templates: of distinct rows, offsets and
                                values); 0 off                               */
    int32_t long_overlap;    /* 1 when the long rows' segments and the wide
                                blocks run on a side stream beside the row
                                blocks (AIJHIP_OPT_LONG_OVERLAP), else 0
                                (fills the former padding word, layout
                                unchanged)                                    */
    int64_t mult_layout_bytes; /* compulsory bytes one MatMult of the plan in
                                effect moves: mult_bytes for CSR (aj read);
                                less where the plan reads column codes (10 B
                                per coded entry) or row patterns (8 B per
                                entry + 1 B per row + the offset table);
                                more for the 32-bit gather-ordered copy
                                (14 B per entry). x and the matrix read once,
                                y written once (ABI 2)                        */
    int32_t hw_queues;       /* hardware queues HIP maps the process's streams
                                onto (GPU_MAX_HW_QUEUES, 4 when unset). With
                                fewer than 8 the automatic choices keep every
                                launch on the caller's stream: long rows after
                                the row blocks (AIJHIP_OPT_LONG_OVERLAP -1,
                                exact mode too), the MPIAIJ exchange in order
                                (aijhip_mpiaij_set_overlap -1) — a side
                                stream would share the compute stream's queue
                                and run behind it (ABI 4)                     */
    int32_t row_templates;   /* 1 when the row patterns carry the values too
                                (AIJHIP_OPT_ROW_TEMPLATES): aa is not read
                                by MatMult, else 0 (ABI 5; the former
                                reserved word)                               */
    int32_t value_codes;     /* the dictionary's size when MatMult reads a
                                16-bit value code per entry instead of aa
                                (AIJHIP_OPT_VALUE_CODES), else 0 (ABI 5)     */
    int32_t reserved1;
} aijhip_info_t;

/* Library / device. */
int aijhip_abi_version(void);
const char *aijhip_last_error(void);
int aijhip_device_count(int *count);

/* Create a device-resident copy of a host CSR matrix (ai[m+1], aj[nz],
 * aa[nz]) on `device`. Columns must lie in [0, n) and ai must be monotone
 * with ai[0] == 0 and ai[m] == nz; columns need not be sorted (the sum order
 * is storage order, as in PETSc). The handle owns its device buffers; the
 * host arrays are only read during the call. */
int aijhip_mat_create(int device, int32_t m, int32_t n, int64_t nz,
                      const int32_t *ai, const int32_t *aj, const double *aa,
                      aijhip_mat_t *out);

/* Same, from arrays already on `device` (e.g. a device-side assembly). The
 * arrays are copied; the caller keeps ownership of its pointers. */
int aijhip_mat_create_from_device(int device, int32_t m, int32_t n, int64_t nz,
                                  const int32_t *d_ai, const int32_t *d_aj,
                                  const double *d_aa, aijhip_mat_t *out);

/* Choose the SpMV kernel family (AIJHIP_KERNEL_*); lanes is used by VECTOR
 * (0 = pick from the mean row length). Re-plans on the device. */
int aijhip_mat_set_kernel(aijhip_mat_t A, int kernel, int lanes);

/* Speed-only knobs of the STREAM kernel; results are identical for every
 * setting. Re-plans on the device. */
enum {
    /* Values 2, 4, 5, 7, 11, 15 and 16 (and kernel 4) are reserved:
     * A/B-only variants withdrawn (measured slower; profiles/README.md); setting
     * them returns AIJHIP_ERR_ARG. */
    AIJHIP_OPT_STREAM_GEOMETRY = 1, /* 0..9: lanes / LDS entries / rows per block
                                       (DESIGN.md §5); -1 (default):
                                       6 for short rows, 1 for long rows    */
    AIJHIP_OPT_NT_LOADS = 3,        /* -1 (default): non-temporal for long rows
                                       with scattered gathers (the geometry-1
                                       operands), plain otherwise; 0 plain;
                                       1 non-temporal aa/aj loads            */
    AIJHIP_OPT_EXACT = 6,           /* 1: every row of the row blocks summed
                                       sequentially in PETSc's order. Default
                                       0: row blocks whose mean row length
                                       exceeds 128 (and rows of more than
                                       1024 entries, which get a block of
                                       their own) use 2..64 lanes per row
                                       (reordered sum, within the fp64
                                       bound); shorter rows (7-pt Poisson,
                                       FEM rows) are bit-exact either way.
                                       Rows longer than a block's entry cap
                                       are split into segments either way
                                       (deterministic, not PETSc's order)   */
    AIJHIP_OPT_LONG_XCD = 8,        /* 1 (default): segments of long rows are
                                       launched so that XCD q (slot % 8)
                                       reduces those whose columns lie in the
                                       q-th eighth of x (its L2 then holds the
                                       x range of their scattered gathers);
                                       0: segment order. Same results        */
    AIJHIP_OPT_HOST_PIPELINE = 10,  /* aijhip_mat_mult_host: -1 (default) x
                                       uploads in ~983,040-row chunks while
                                       the row blocks whose columns have
                                       arrived multiply and their y chunks
                                       download (step3/step4 analogue); k > 0:
                                       chunks of >= k rows; 0: the serial
                                       step-2 form. Same results              */
    AIJHIP_OPT_LONG_OVERLAP = 9,    /* operands with long rows: 0 the
                                       segments and the wide blocks after the
                                       row blocks; 1 on a side stream beside
                                       them (plain MatMult / MatMultAdd;
                                       forked from and joined to the caller's
                                       stream by events); -1 (default): 0,
                                       or 1 with AIJHIP_OPT_EXACT when the
                                       process has >= 8 hardware queues
                                       (aijhip_info_t.hw_queues). Same
                                       results                              */
    AIJHIP_OPT_GATHER_SORT = 12,    /* MatMult / MatMultAdd from a copy of the
                                       row blocks with each block's entries
                                       sorted by column and their positions
                                       in the block: x is gathered in column
                                       order, the products are summed in the
                                       rows' storage order (the same bits).
                                       1 on, 0 off, -1 (default): on for
                                       operands with scattered gathers (long
                                       rows, > 0.25 distinct x lines per
                                       entry); costs a second copy of the
                                       entries plus 2 bytes each            */
    AIJHIP_OPT_COLUMN_CODES = 13,   /* MatMult / MatMultAdd / the CG and V-cycle
                                       epilogues read a 16-bit code per entry
                                       instead of aj: (row in block << b) |
                                       index into the block's dictionary of
                                       column - row offsets (a stencil has a
                                       handful per block), aa unchanged, the
                                       same sums. 1 on, 0 off, -1 (default):
                                       tried first at geometry 6 (gather
                                       order off) and kept where the row
                                       blocks' offsets fit (>= 90 % of the
                                       entries), else the automatic layout
                                       without them; costs 2 bytes per entry
                                       of device memory                      */
    AIJHIP_OPT_ROW_PATTERNS = 14,   /* short-row operands whose rows follow at
                                       most 256 distinct column - row offset
                                       lists (stencils): no per-entry column
                                       at all — a pattern id per row (1 byte),
                                       the lists staged in LDS, x gathered by
                                       one lane per row; aa unchanged, the same
                                       sums. 1 on, 0 off, -1 (default): tried
                                       first where the mean row is at most 16
                                       entries; costs 1 byte per row          */
    AIJHIP_OPT_ROW_TEMPLATES = 17,  /* with row patterns: when the operand's rows
                                       are at most 256 distinct (offsets,
                                       values) lists — a constant-coefficient
                                       stencil — the table holds the values
                                       too and MatMult reads neither aj nor
                                       aa: the row's id, x and y (the values
                                       are the same bits, summed in the same
                                       order: the same results). 1 on, 0 off,
                                       -1 (default): tried before the plain
                                       row patterns. aijhip_mat_update_values
                                       re-plans (new values may not fit)     */
    AIJHIP_OPT_VALUE_CODES = 18     /* a 16-bit index per entry into a
                                       dictionary of the operator's distinct
                                       values (at most 512) in aa's place:
                                       6 bytes per entry with aj or the packed
                                       gather-ordered columns instead of 12;
                                       the same bits. 1 on (where it fits),
                                       0 off, -1 (default): on for the
                                       set-up's own operators (GAMG's finest
                                       P and P^T), off for a caller's handle.
                                       aijhip_mat_update_values re-plans     */
};
int aijhip_mat_set_option(aijhip_mat_t A, int option, int value);

/* New values, same nonzero structure (host aa[nz]): the re-upload half of
 * MatAssemblyEnd_SeqAIJ's hook (step2 MatAssemblyEnd patch:42-44). */
int aijhip_mat_update_values(aijhip_mat_t A, const double *aa);

/* New structure and values (MAT_FINAL_ASSEMBLY after compaction): drops the
 * device copy and re-uploads everything (step2 MatAssemblyEnd patch:21-29,
 * :42-44). Sizes m and n are kept. */
int aijhip_mat_assembly_end(aijhip_mat_t A, int64_t nz, const int32_t *ai,
                            const int32_t *aj, const double *aa);

/* y = A x (overwrite). x: device fp64[n], y: device fp64[m]; x and y must not
 * alias (PETSc requires distinct Vecs). Enqueued on `stream`. */
int aijhip_mat_mult(aijhip_mat_t A, const double *x, double *y, void *stream);

/* w = z + A x. z may alias w (PETSc's yy == zz case); x must not alias w. */
int aijhip_mat_mult_add(aijhip_mat_t A, const double *x, const double *z,
                        double *w, void *stream);

/* y = A^T x. x: device fp64[m], y: device fp64[n]. Uses a transposed copy
 * built on first call (kept until the structure changes). */
int aijhip_mat_mult_transpose(aijhip_mat_t A, const double *x, double *y,
                              void *stream);

/* Step-2 semantics with host vectors: x (host fp64[n]) is copied in, y
 * (host fp64[m]) copied out; returns after y is on the host. The copies are
 * pipelined with the product (AIJHIP_OPT_HOST_PIPELINE, the reference's
 * step3/step4: src/openacc-step4/MatMult_SeqAIJ.patch:51-91): host arrays
 * that are already pinned (hipHostMalloc / hipHostRegister) are DMA'd
 * directly; pageable ones are copied straight from and to the caller's arrays
 * as well (the runtime's pageable path measured faster than staging through
 * pinned slots): x chunks upload on one stream, y chunks download on another,
 * issued from a second host thread. */
int aijhip_mat_mult_host(aijhip_mat_t A, const double *x, double *y);

/* w = z + A x with host vectors (MatMultAdd_SeqAIJ, aij.c [ext]: the
 * off-diagonal product of MatMult_MPIAIJ and PCMG's interpolation reach it);
 * each row sum starts from z[i], as PETSc's does. z may alias w; x must not.
 * The reference leaves this on the CPU; the PETSc adapter
 * routes it here for matrices above a size threshold. */
int aijhip_mat_mult_add_host(aijhip_mat_t A, const double *x, const double *z,
                             double *w);

/* y = A^T x with host vectors (MatMultTranspose_SeqAIJ [ext]: PCMG's
 * restriction). Same transposed copy and scatter order as
 * aijhip_mat_mult_transpose; the copies are pipelined as for mult_host. */
int aijhip_mat_mult_transpose_host(aijhip_mat_t A, const double *x, double *y);

int aijhip_mat_get_info(aijhip_mat_t A, aijhip_info_t *info);

/* Borrow the handle's device CSR (read-only; valid until the next
 * assembly_end / destroy). The analogue of PETSc's device-array getters for
 * GPU Mat types; aj and aa carry a 2-entry zero pad past nz. */
int aijhip_mat_get_device_csr(aijhip_mat_t A, const int32_t **ai, const int32_t **aj,
                              const double **aa);

/* Free every device buffer of the handle (MatDestroy_SeqAIJ hook,
 * step2 MatDestroy patch:18-34). NULL is a no-op. */
int aijhip_mat_destroy(aijhip_mat_t A);

#ifdef __cplusplus
}
#endif

#endif /* AIJHIP_H */
