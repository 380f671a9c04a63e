// aijhip_internal.h — handle layout and kernel launchers shared by the
// SpMV translation units. Not part of the ABI (include/aijhip.h is).
#pragma once

#include <hip/hip_runtime.h>
#include <rocprofiler-sdk-roctx/roctx.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "aijhip.h"
#include "aijhip_ksp.h"
#include "host_alloc.h"

namespace aijhip {

// roctx range for the PETSc-level phases (MatAssemblyEnd, KSPSetUp,
// KSPSolve, the GAMG set-up levels): shown by `rocprofv3 --marker-trace`,
// a no-op call when no tool is attached.
struct Range {
    explicit Range(const char *name) { roctxRangePushA(name); }
    ~Range() { roctxRangePop(); }
    Range(const Range &) = delete;
    Range &operator=(const Range &) = delete;
};

// STREAM kernel geometries: `threads` lanes per row
// block, up to `nnz_cap` products staged in LDS (8 B each) and up to
// `rows` rows (rows / threads rows per lane in the reduction phase).
struct StreamGeom {
    int threads, nnz_cap, rows;
};
// Caps of the form 2*threads*ITERS - 2 leave exactly one pair slot for the
// 16-B alignment of the block start, so no load iteration is wasted
// (a fully idle 5th iteration cost 6 % at 300^3: profiles/r01/style.jsonl).
constexpr StreamGeom kStreamGeoms[] = {
    {256, 2048, 256},    // 0: 4 waves, 16 KiB LDS
    {512, 4096, 512},    // 1: 8 waves, 32 KiB
    {256, 4096, 512},    // 2: 4 waves, 32 KiB, 2 rows per lane
    {128, 1024, 128},    // 3: 2 waves, 8 KiB
    {1024, 8192, 1024},  // 4: 16 waves, 64 KiB
    {256, 1024, 256},    // 5: 4 waves, 8 KiB
    {512, 4094, 512},    // 6: 8 waves, 4 pair-iterations (measured best)
    {1024, 8190, 1024},  // 7: 16 waves, 4 pair-iterations
    {256, 2046, 256},    // 8: 4 waves, 4 pair-iterations
    {512, 2046, 512},    // 9: 8 waves, 2 pair-iterations, 16 KiB
};
// (Round 4's geometries of 6 and 8 pair-iterations, sized for the withdrawn
// LDS x tiles, were removed in round 5; the 2-pair geometry is now 9.)
constexpr int kNumStreamGeoms = sizeof(kStreamGeoms) / sizeof(kStreamGeoms[0]);
constexpr int kMaxStreamNnzCap = 8192;
// A row longer than the geometry's nnz_cap leaves the STREAM blocks and is split into
// segments of at most kLongSegNnz entries, each summed by one workgroup.
constexpr int kLongSegNnz = 4096;
// 512 lanes x 4 pairs in flight = one 4096-entry segment per round
constexpr int kLongThreads = 512;

// One STREAM row block: rows [row0, row0+nrows) of the row list, entries
// [k0, k0+nk) of aj/aa.
struct BlockDesc {
    int32_t row0, nrows, k0, nk;
};

// One segment of a long row: entries [k0, k0+nk), partial sum -> partials[seg].
struct LongSeg {
    int32_t k0, nk;
};

// A long row: output row `orow`, segments [seg0, seg0+nseg).
struct LongRow {
    int32_t orow, seg0, nseg, pad;
};

// Row list the kernels walk: nr rows with offsets rai[0..nr] into aj/aa and
// (compressed-row form only) output row ids ridx[0..nr-1].
struct RowList {
    int32_t nr;
    const int32_t *rai;
    const int32_t *ridx;  // nullptr = identity
};

// Speed-only knobs (aijhip_mat_set_option); they never change results.
// Defaults are the fastest measured on MI355X (profiles/README.md): geometry 6 for
// short rows and for long rows whose gathers run along x lines, geometry 1 for
// scattered long rows; plain loads except for those (non-temporal); hardware
// round-robin block placement. The A/B-only variants measured slower
// (XCD-contiguous placement, the persistent pipelined grid, clamped loads,
// register row groups, a side stream for the long rows, LDS x tiles, long
// rows by x column window) were withdrawn in ABI 2; profiles/r01-r04 keep
// their records.
struct Tuning {
    int geom = -1;       // index into kStreamGeoms; -1 = by row length and gather locality (6 or 1)
    int nt = -1;         // matrix loads: -1 by gather locality (non-temporal for scattered long rows),
                         // 0 plain, 1 non-temporal
    bool exact = false;    // always sum rows sequentially (PETSc order), even long ones
    bool long_xcd = true;  // long-row segments placed on the XCD that owns their column range
    int overlap = -1;      // MatMult / MatMultAdd with wide blocks or long rows: those launches on a
                           // side stream concurrent with the row blocks (1), or after them (0; -1
                           // auto = 0 since round 5, 1 with exact). Skewed stand-in r04: 299.0 vs 310.5 us
                           // (profiles/r04/s2/); round 5, rows > 1024 in blocks of their own, the
                           // same box interleaved: side 315.1, serial 310.2 us (profiles/r05/ac/)
    int host_chunk = -1;   // host-vector MatMult: -1 pipelined in ~1M-row chunks, 0 serial (step-2 form),
                           // k > 0 pipelined in chunks of >= k rows
    int gsort = -1;        // gather-ordered copy of the row blocks (MatMult / MatMultAdd and the
                           // fused V-cycle launches): -1 auto (long rows; a caller's handle only
                           // in the packed form), 0 off, 1 on
    int codes = -1;        // 16-bit column codes instead of aj (Plan::d_code): -1 auto (where the
                           // blocks' offset dictionaries fit and gsort is off), 0 off, 1 on
    int patterns = -1;     // row patterns instead of aj (Plan::d_pid): -1 auto (short rows whose
                           // offset lists are few), 0 off, 1 on
    int templates = -1;    // with row patterns, the values in the table too (Plan::d_pval; a
                           // constant-coefficient stencil): -1 auto (tried first), 0 off, 1 on
    int vcodes = -1;       // 16-bit value codes instead of aa (Plan::d_vcode): -1 auto (the set-up's own
                           // operators, where <= kVDictMax distinct values), 0 off, 1 on
};

// Column codes (Tuning::codes): entry k of a row block starting at row0 is
// coded as (r << b) | i, r = its row - row0, i = the index of aj[k] - row in
// the block's sorted dictionary of distinct column - row offsets. b is a
// function of the block's row count only (the rows need 16 - b bits), capped
// so the dictionary fits kCodeDictMax LDS entries: 512-row blocks get 7 bits
// (128 offsets; a 7-point stencil has 7), 50-row blocks of FEM rows 9
// (512; a block of the FEM stand-in has ~135).
constexpr int kCodeDictMax = 512;
// Row patterns (Tuning::patterns): at most 256 distinct column - row offset
// lists per operand, their table (a start | length word per pattern, then
// the offsets) at most kPatTableMax words, staged in LDS by every block.
constexpr int kPatTableMax = 1024;
// Value codes (Tuning::vcodes): at most kVDictMax distinct values, staged in
// LDS by every block (4 KiB)
constexpr int kVDictMax = 512;
constexpr int kPatMax = 256;
__host__ __device__ inline int code_index_bits(int nrows) {
    int rb = 0;
    while (rb < 16 && (1 << rb) < nrows) ++rb;
    return 16 - rb < 9 ? 16 - rb : 9;
}

struct HostPipe;  // host-vector MatMult pipeline state (host_pipe.cpp)

// STREAM blocks whose mean row length exceeds this use several lanes per row
// in the reduction phase (reordered sum) unless Tuning::exact is set. Measured
// (tools/rowlen_sweep.py, profiles/r01/rowlen_sweep.jsonl): one lane per row
// is as fast or faster up to ~100 entries per row, several lanes win from
// ~200 (row length 384: 346 vs 619 us).
constexpr int kSplitMinMean = 128;
// One-lane-per-row blocks whose mean row length exceeds this read their LDS
// products eight at a time ahead of the sequential adds (row_sum_seq; same
// order, same bits). Measured (profiles/r01/rowsum/): FEM-structured stand-in
// 310 -> 280 us at geometry 6, skewed stand-in 429 -> 405 us at geometry 1.
constexpr int kBatchMinMean = 16;
// A row longer than this (and within the block cap) gets a row block of its
// own, so it is summed by 64 lanes (reordered; exact = 1 keeps one lane and
// PETSc's order) instead of one lane's dependent chain holding its block of
// short rows: the skewed stand-in's 40 rows of 1e3-4e3 scattered entries
// made its wide blocks a 29 us launch (round 5, profiles/r05/x).
constexpr int kIsolateRowNnz = 1024;
// Automatic geometry for long rows (mean > 16): above this many distinct x
// lines per entry the gathers count as scattered (geometry 1), below it they
// run along lines (geometry 6). Measured: 7-pt 0.73, GAMG coarse operators
// 0.51-0.68, skewed stand-in 0.40, FEM-structured stand-in 0.17.
constexpr double kScatteredLinesPerEntry = 0.25;
struct Plan {
    int kernel = AIJHIP_KERNEL_STREAM;
    int lanes = 0;
    Tuning tune;
    // STREAM
    BlockDesc *d_blocks = nullptr;
    int32_t n_blocks = 0;
    LongSeg *d_segs = nullptr;
    int32_t n_segs = 0;
    LongRow *d_longs = nullptr;
    int32_t n_longs = 0;
    double *d_partials = nullptr;
    // launch slot -> segment (nullptr = identity): slot s runs on XCD s % 8
    // under round-robin placement, and is given a segment whose columns lie in
    // the s % 8-th eighth of x, so each XCD's L2 holds the x range its
    // scattered gathers hit (speed only; partials and their order unchanged)
    int32_t *d_segperm = nullptr;
    // Tuning::overlap: the side stream the wide blocks and the long rows'
    // segments run on, forked from / joined to the caller's by two events
    hipStream_t side = nullptr;
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    // Tuning::gsort: each row block's entries sorted by column (columns,
    // values) and their positions in the block (the products' LDS slots)
    int32_t *d_saj = nullptr;
    double *d_saa = nullptr;
    uint16_t *d_sslot = nullptr;
    // ... or, when the blocks' columns span < 2^20 (kPackedColBits), one
    // 32-bit word per entry in d_sidx: the column relative to the block's
    // first (d_sbase) in the low 20 bits, the product slot (< 4096: block
    // caps <= 4096 entries) in the high 12 (d_saj / d_sslot then freed):
    // 12 bytes per entry with aa. (Round 5 packed 16-bit columns and 16-bit
    // slots per entry pair: the same bytes, but blocks spanning 2^16 columns
    // and more — the GAMG level-1 operator's and P^T's — fell back to the
    // 32-bit sorted columns, 14 bytes per entry.)
    uint32_t *d_sidx = nullptr;
    int32_t *d_sbase = nullptr;
    // ... and when only some blocks are that narrow (a wide row within the
    // block cap: the skewed stand-in's shorter hub rows), the narrow blocks
    // in d_nblocks (d_sbase follows their order) and the others in
    // d_wblocks, launched from the original arrays
    BlockDesc *d_nblocks = nullptr, *d_wblocks = nullptr;
    int32_t n_nblocks = 0, n_wblocks = 0;
    int64_t nz_wide = 0;  // entries of the d_wblocks (read from aj / aa)
    // Tuning::codes: one 16-bit code per entry (nz + 2, pairs read as one
    // 4-B word) and d_cmeta = per coded block {dictionary start, size} then
    // the dictionaries; the coded blocks are d_blocks, or d_nblocks with the
    // others in d_wblocks (launched from aj) when some do not fit
    uint16_t *d_code = nullptr;
    int32_t *d_cmeta = nullptr;
    int64_t n_cmeta = 0;  // int32 words of d_cmeta (per-block meta + dictionaries)
    // Tuning::patterns: a pattern id per row and the pattern table (start |
    // length << 16 per pattern, then the offsets); geometry 6, full rows
    uint8_t *d_pid = nullptr;
    int32_t *d_ptab = nullptr;
    int32_t n_ptab = 0, n_pat = 0;
    int32_t pat_dmax = 0;    // largest |column - row| offset in the table (the stencil's plane distance)
    int32_t pat_maxlen = 0;  // longest pattern (entries)
    bool tmpl_diag = false;  // every pattern has the offset 0 (the diagonal)
    // Tuning::templates: the values of each pattern's entries, indexed like
    // the offsets in d_ptab (n_ptab doubles; the first n_pat unused): MatMult
    // reads neither aj nor aa
    double *d_pval = nullptr;
    BlockDesc *d_tblocks = nullptr;  // the blocks in the template launch's order, k0 = the block's index
    // Tuning::vcodes: a 16-bit index per entry into d_vdict (n_vdict values),
    // in aa's order (d_vcode) and, with the packed gather-ordered copy, in
    // its order (d_svcode); nz + 2 each
    uint16_t *d_vcode = nullptr, *d_svcode = nullptr;
    double *d_vdict = nullptr;
    int32_t n_vdict = 0;
    int64_t bytes = 0;  // device bytes held by the plan
    HostPipe *hpipe = nullptr;  // built on the first host-vector MatMult
};

}  // namespace aijhip

struct aijhip_mat {
    int device = 0;
    // changes whenever the device arrays or the plan are rebuilt (a fresh
    // value of a process-wide counter): a set-up KSP on this handle re-plans
    // its fused launches when it moved (ksp.hip)
    uint64_t plan_gen = 0;
    // changes whenever the values change (aijhip_mat_update_values, and
    // every plan_gen change): a set-up KSP redoes its PC set-up (Jacobi's
    // D^-1, the GAMG hierarchy) when it moved, as PETSc's PCSetUp does when
    // the operator's state changed
    uint64_t values_gen = 0;
    int n_cu = 256;  // compute units of the device
    int32_t m = 0, n = 0;
    int64_t nz = 0;
    int32_t nonzerorowcnt = 0;
    int32_t max_row_nz = 0;
    bool compressed = false;
    int32_t *d_ai = nullptr;
    int32_t *d_aj = nullptr;   // nz + 2 entries: the tail pad keeps 16-B loads in bounds
    double *d_aa = nullptr;    // nz + 2 entries
    int32_t n_crow = 0;        // compressed-row form (PETSc a->compressedrow)
    int32_t *d_cai = nullptr;
    int32_t *d_ridx = nullptr;
    aijhip::HostVec<int32_t> h_rai;  // host copy of the row-list offsets (planning)
    aijhip::Plan plan;
    int requested_kernel = AIJHIP_KERNEL_AUTO;
    int requested_lanes = 0;
    aijhip::Tuning requested_tune;
    // a set-up's own operator (GAMG levels, P, Pᵀ: adopt_device_csr): long
    // rows keep the gather-ordered copy when its packed form does not fit
    bool setup_op = false;
    // host-vector staging for aijhip_mat_mult_host (allocated on first use)
    double *d_xstage = nullptr, *d_ystage = nullptr;
    hipStream_t host_stream = nullptr;
    // lazily built A^T (for aijhip_mat_mult_transpose)
    aijhip_mat *transpose = nullptr;
    int64_t device_bytes = 0;
};

namespace aijhip {

// Launchers (aijhip_kernels.hip). All enqueue on `s` and return the launch's
// hipError_t.
hipError_t launch_stream(const aijhip_mat &A, const double *x, const double *z,
                         double *y, bool add, hipStream_t s, double *dpart = nullptr,
                         const int *stop = nullptr);
// CG fusion: y = A x with the per-block partials of x . y in dpart[0..n_blocks)
// (deterministic); every block returns at once when *stop != 0. Only for
// square full-row STREAM plans without long rows.
bool stream_dot_fusable(const aijhip_mat &A);
hipError_t launch_stream_dot(const aijhip_mat &A, const double *x, double *y, double *dpart,
                             const int *stop, hipStream_t s);
// Fused V-cycle smoothing SpMVs on a STREAM plan (same conditions as
// stream_dot_fusable): the pre-smoothing residual r = b - A x, and one
// Richardson+Jacobi step x = t + D^-1 (b - A t) (x != t) with optional
// z.z / z.b partials (2 x n_blocks) for CG on the finest level.
bool stream_mg_fusable(const aijhip_mat &A);
// y = D^-1 A x in PETSc's row order (exact), for the GAMG set-up.
hipError_t launch_dinv_mult(const aijhip_mat &A, const double *dinv, const double *x, double *y, hipStream_t s);
// y = A x in PETSc's row order on a STREAM plan (exact; the GAMG set-up's CG estimate).
hipError_t launch_mult_exact(const aijhip_mat &A, const double *x, double *y, hipStream_t s);
// r = b - A x on a STREAM plan (residual in the SpMV epilogue).
hipError_t launch_mg_resid(const aijhip_mat &A, const double *x, const double *b, double *r, hipStream_t s,
                           bool nt, const int *stop = nullptr);
hipError_t launch_mg_post(const aijhip_mat &A, const double *t, const double *b, const double *dinv, double *x,
                          double *dpart, hipStream_t s, bool nt, const int *stop = nullptr,
                          const double *tdinv = nullptr);
// Dispatch y = A x (or w = z + A x) through the handle's plan. stop: a device
// flag (CG's `done`); STREAM row blocks return at once once it is set.
hipError_t launch_mult(const aijhip_mat &A, const double *x, const double *z, double *y,
                       bool add, hipStream_t s, const int *stop = nullptr);
hipError_t launch_scalar(const aijhip_mat &A, const double *x, const double *z,
                         double *y, bool add, hipStream_t s);
hipError_t launch_vector(const aijhip_mat &A, const double *x, const double *z,
                         double *y, bool add, hipStream_t s);
// Transpose (stable by row): builds At's device CSR (n x m). Returns arrays
// allocated with hipMalloc; caller owns them.
hipError_t build_transpose(const aijhip_mat &A, int32_t **d_tai, int32_t **d_taj,
                           double **d_taa, hipStream_t s);

RowList row_list(const aijhip_mat &A);
// Per long-row segment: the column of its middle entry (synchronous).
hipError_t segment_mid_columns(const aijhip_mat &A, const LongSeg *d_segs, int32_t n_segs, int32_t *h_out);
// Per STREAM block: min column and span (max - min + 1) of its entries.
hipError_t block_column_ranges(const aijhip_mat &A, const BlockDesc *d_blocks, int32_t n_blocks, int2 *d_out);
// The gather-ordered copy of the plan's row blocks (Plan::d_saj/d_saa/
// d_sslot, allocated by the caller); values_only: the values again, in the
// order already built.
hipError_t build_gather_order(const aijhip_mat &A, const Plan &P, bool values_only);
// Per block: first sorted column and the span of its columns (after build_gather_order).
hipError_t gather_order_spans(const Plan &P, int32_t *d_base, int32_t *d_span);
// The 16-bit packed form of the sorted columns and slots of blocks
// d_blk[0, nblk) (d_base: their first columns, in that order).
hipError_t pack_gather_order(const Plan &P, const BlockDesc *d_blk, int32_t nblk, const int32_t *d_base,
                             uint32_t *d_sidx);
constexpr int kPackedColBits = 20;  // the packed gather-ordered form: 20-bit columns, 12-bit slots
constexpr int kPackedMaxCap = 1 << (32 - kPackedColBits);  // slots < 4096: block caps up to 4096 entries
// Column codes: pass 0 counts each block's distinct column - row offsets
// into d_cnt[0, nblk); pass 1 (d_cmeta laid out by the caller) writes the
// dictionaries and the codes of blocks d_blk[0, nblk).
// Row patterns: when the operand's rows follow at most kPatMax distinct
// column - row offset lists (64-bit hashes, verified entry by entry) whose
// table fits kPatTableMax words, allocates and fills P.d_pid / P.d_ptab and
// sets *ok; otherwise leaves them null. values: the lists are (offset, value)
// pairs (the value bits hashed and verified too) and P.d_pval is filled.
hipError_t build_row_patterns(const aijhip_mat &A, Plan &P, bool *ok, bool values);
// Value codes: when aa holds at most kVDictMax distinct values (bit
// patterns), fills P.d_vdict (sorted by bits) and P.d_vcode (and
// P.d_svcode from P.d_saa when the packed gather-ordered copy exists) and
// sets *ok; otherwise leaves them null.
hipError_t build_value_codes(const aijhip_mat &A, Plan &P, bool *ok);
hipError_t column_code_counts(const aijhip_mat &A, const BlockDesc *d_blk, int32_t nblk, int32_t *d_cnt);
hipError_t column_code_write(const aijhip_mat &A, const BlockDesc *d_blk, int32_t nblk, int32_t *d_cmeta,
                             uint16_t *d_code);
// Distinct 128-B x lines per entry over a row sample (at most 65536 rows):
// ~0.7 for the 7-point stencil, ~0.17 for a 3-dof hexahedral FEM operator.
hipError_t gather_lines_per_entry(const aijhip_mat &A, double *out);
// A handle that takes ownership of device CSR arrays made inside the library
// (aj / aa allocated with nz + 2 entries; trusted: no column check, no copy).
// Tuning and kernel choice copied from `like` when given. The arrays are
// freed on failure.
int adopt_device_csr(int device, int32_t m, int32_t n, int64_t nz, int32_t *d_ai, int32_t *d_aj, double *d_aa,
                     const aijhip_mat *like, aijhip_mat **out);
// Install A^T (device arrays, adopted) as A's transpose handle.
int attach_transpose(aijhip_mat *A, int32_t *tai, int32_t *taj, double *taa);
// Number of device column indices outside [0, n) (synchronous).
hipError_t count_bad_columns(const int32_t *d_aj, int64_t nz, int32_t n, int64_t *bad);

// y = A x over the STREAM row blocks [b0, b0 + nb) only (default speed
// knobs; full-row, no long rows).
hipError_t launch_stream_blocks(const aijhip_mat &A, int32_t b0, int32_t nb, const double *x, double *y,
                                hipStream_t s);
// Host-vector MatMult (aijhip_mat_mult_host), host_pipe.cpp: x uploaded in
// chunks while the row blocks whose columns have arrived multiply and their y
// chunks download (step-3/4 analogue). Returns an AIJHIP_* code.
int host_pipe_mult(aijhip_mat *A, const double *x, double *y);
void host_pipe_free(HostPipe *p);

// The V-cycle of a set-up GAMG KSP (ksp.hip) as a preconditioner of another
// solver (the distributed CG's block-Jacobi sub-PC, ksp_mpi.hip): x = B b on
// `s`. When the finest post-smoothing carried the z.z / z.b partials, *dots
// points at them (2 x *nbz doubles), else NULL.
hipError_t ksp_pc_vcycle(aijhip_ksp *K, const double *b, double *x, hipStream_t s, const double **dots,
                         int *nbz, const int *stop = nullptr);

// A fresh value for aijhip_mat::plan_gen.
uint64_t next_plan_gen();

// Flags of the library's cross-stream fork / join events (the MPIAIJ halo,
// the long-row side stream): hipEventDisableTiming plus the release scope
// AIJHIP_EVENT_FENCE selects at creation — "system" (HIP's default),
// "device" (hipEventReleaseToDevice) or "none" (hipEventDisableSystemFence).
// Both ends of every such edge are on one device.
unsigned sync_event_flags();
// The hardware queues HIP maps this process's streams onto: GPU_MAX_HW_QUEUES
// as HIP reads it at initialisation, 4 (HIP's default) when unset. Streams
// are dealt to the queues round-robin in creation order, so with fewer than
// kOverlapMinQueues the library's second streams (the MPIAIJ exchange, the
// long rows' side stream) share a queue with the compute stream beside
// torch's and RCCL's, and their "concurrent" work runs behind it (measured,
// profiles/r05/e/: the halo's empty fork / join 29.5 us at 4 queues vs 13.5
// at 8; the skewed stand-in's side stream 344 us, slower than serial, at 4).
int hw_queues();
constexpr int kOverlapMinQueues = 8;

// Compulsory bytes one MatMult under A's plan moves (aijhip_info_t.mult_layout_bytes).
int64_t mult_layout_bytes(const aijhip_mat &A);

// Sets the calling thread's aijhip_last_error() message.
void set_error(const std::string &msg);
int visible_devices();  // hipGetDeviceCount, cached
std::string no_device_reason();  // the error text when visible_devices() is 0

}  // namespace aijhip
