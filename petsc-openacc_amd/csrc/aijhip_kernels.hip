// aijhip_kernels.hip — gfx950 CSR SpMV kernels (y = A x, w = z + A x).
//
// Replaces the PGI-generated OpenACC kernels of
// /root/reference/src/openacc-step{1..4}/MatMult_SeqAIJ.patch. The arithmetic
// contract is the PETSc row loop (step1 patch:22-31): per row, products
// aa[k]*x[aj[k]] rounded to fp64 and added in storage order starting at 0.0
// (or z[i] for MatMultAdd). The build uses -ffp-contract=off so no product is
// fused into an add.
//
//  STREAM  (default) — CSR-stream row blocks: a 256-lane workgroup streams the
//          contiguous aa/aj range of up to 256 rows / 2048 entries with
//          16-byte loads, gathers x, stages the products in LDS, then each
//          lane sums one row sequentially. Every global access of the matrix
//          is a full-width coalesced load and every lane is busy in the
//          streaming phase, independent of row length; the per-row order is
//          PETSc's, so results are bit-identical to the CPU loop.
//  SCALAR  — one lane per row: the reference's kernel shape (`gang vector(32)`
//          with a sequential inner dot, step1 patch:19-31). Bit-exact, but
//          its loads are strided by the row length (kept as a baseline).
//  VECTOR  — L = 2..64 lanes per row (64 = one wavefront per row), strided
//          loads, __shfl_xor tree reduction. For long uniform rows.
//  (MERGE, an explicit merge-path kernel, was withdrawn in ABI 2: the STREAM
//  planner already cuts the merge list of rows and entries into balanced
//  blocks, and the kernel measured 1.6x slower on its own stress operand.)
//
// Rows longer than a block's entry cap leave the STREAM blocks and are split
// into kLongSegNnz-entry segments, each reduced by one workgroup (placed on
// the XCD whose eighth of x its columns fall in), then summed in segment
// order by a finishing kernel (deterministic, not bit-identical).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "aijhip_internal.h"

namespace aijhip {
namespace {

// Row blocks run in launch order; the hardware deals them round-robin over
// the 8 XCDs (MI355X_MICROARCH §Workgroup dispatch). XCD-contiguous and
// chunked remaps of that order were measured 1-10 % slower at 300^3 (DESIGN
// §5; withdrawn in ABI 2): the cross-XCD x re-reads they remove are served by
// the Infinity Cache.
typedef double f64x2 __attribute__((ext_vector_type(2)));
typedef int i32x2 __attribute__((ext_vector_type(2)));

// Matrix entries are read exactly once per SpMV: with NT the loads carry the
// non-temporal hint so the stream does not evict the reused x window from L2.
template <bool NT, typename T>
__device__ __forceinline__ T ld_stream(const T *p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}

// Loads and gathers are predicated on `k < k1`: lanes past the block issue no
// request (branch-free clamped loads measured slower, tools/ablate_style.py).
// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS ops,
// not for its outstanding global loads (__syncthreads() would add
// s_waitcnt vmcnt(0) and drain the prefetch; cdna_hip_programming.md §8).
// The "memory" clobber keeps the compiler from moving LDS accesses across it.
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Block-wide fp64 sum in a fixed order (wave __shfl_down tree, then the
// waves' sums in wave order): deterministic run to run. LDS-only barriers:
// the row results just stored to global memory need not have landed.
template <int T>
__device__ __forceinline__ double block_sum(double v, double *scratch) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
    const int t = threadIdx.x;
    lds_barrier();  // scratch may still be read by the caller's previous phase
    if ((t & 63) == 0) scratch[t >> 6] = v;
    lds_barrier();
    double s = 0.0;
    if (t == 0) {
#pragma unroll
        for (int w = 0; w < T / 64; ++w) s += scratch[w];
    }
    return s;  // valid in thread 0
}

// Row results are written once and not re-read by this launch: stored with the
// non-temporal hint (`global_store … nt`). Measured on the 300^3 operand
// (tools/ablate_buf.py, profiles/r01/ablate_buf{1,2}*.jsonl): 472 -> 450 us and
// 491 -> 462 us on two boxes; the sc0/sc1 policy variants with nt tie, plain or
// sc0/sc1-only stores do not gain.
__device__ __forceinline__ void st_stream(double *p, double v) { __builtin_nontemporal_store(v, p); }

// What a STREAM launch gathers and writes. The row sum s_i = sum a_ij g(j)
// is formed in PETSc's order (or the deterministic multi-lane order); `seed`
// starts it (MatMultAdd's z_i), `put` stores the row's result and adds to
// the block's dot partials d[0..kDots). `row` loads the row's other operands
// (Row) so that a launch can issue them before the gathers (the row-template
// kernel: with no matrix stream, a load issued after the sum is one more
// latency per block) and put(o, v, d, row) takes them; put(o, v, d) loads
// them itself, after the sum (the STREAM kernels' form).
template <bool ADD>
struct OpMult {  // y = A x (+ z); optional x . y partials (CG's p . w)
    static constexpr int kDots = 1;
    static constexpr bool kSeeded = ADD;
    static constexpr bool kTmplDiag = false;
    static constexpr bool kXoFromSlot = false;
    const double *x, *z;
    double *y;
    bool dot;
    struct Row {
        double xo;
    };
    __device__ double gx(int32_t j) const { return x[j]; }
    __device__ double seed(int o) const { return ADD ? z[o] : 0.0; }
    __device__ Row row(int o) const { return {dot ? x[o] : 0.0}; }
    __device__ void put(int o, double v, double *d, const Row &w) const {
        st_stream(y + o, v);
        if (dot) d[0] += w.xo * v;
    }
    __device__ void put(int o, double v, double *d) const {
        st_stream(y + o, v);
        if (dot) d[0] += x[o] * v;
    }
};

// OpMult with the dot decided at compile time, for the pipelined template
// launch: OpMult::row's load behind the runtime `dot` is a load behind a
// branch, and the loop's waits then count for the path without it (one
// load more waited for on the other)
// (XS: the dot's x[o] taken from the row's gathered diagonal, every template
// having one — Plan::tmpl_diag — so the stage carries no load of its own)
template <bool ADD, bool DOT, bool XS = false>
struct OpMultT : OpMult<ADD> {
    using Row = typename OpMult<ADD>::Row;
    static constexpr bool kXoFromSlot = DOT && XS;
    __device__ Row row(int o) const { return {DOT && !XS ? this->x[o] : 0.0}; }
    __device__ void set_diag(Row &w, double xd) const { w.xo = xd; }
    __device__ void put(int o, double v, double *d, const Row &w) const {
        st_stream(this->y + o, v);
        if (DOT) d[0] += w.xo * v;
    }
};

// MatResidual with the SpMV: r_i = b_i + (-1) (A x)_i (SpMV + k_resid, same
// roundings) — the second half of the pre-smoothing, after x = D^-1 b was
// written by a vector pass.
template <bool NT>
struct OpMgResid {
    static constexpr int kDots = 0;
    static constexpr bool kSeeded = false;
    static constexpr bool kTmplDiag = false;
    static constexpr bool kXoFromSlot = false;
    const double *x, *b;
    double *r;
    struct Row {
        double bo;
    };
    __device__ double gx(int32_t j) const { return x[j]; }
    __device__ double seed(int) const { return 0.0; }
    __device__ Row row(int o) const { return {b[o]}; }
    __device__ void put(int o, double v, double *, const Row &w) const {
        const double ro = w.bo + (-1.0) * v;
        if constexpr (NT) st_stream(r + o, ro);
        else r[o] = ro;
    }
    __device__ void put(int o, double v, double *) const {
        const double ro = b[o] + (-1.0) * v;
        if constexpr (NT) st_stream(r + o, ro);
        else r[o] = ro;
    }
};

// V-cycle post-smoothing, one Richardson step with Jacobi from the guess t
// (SpMV + k_richardson): x_i = t_i + 1.0 (dinv_i (b_i + (-1) (A t)_i)); x
// must not alias t. With dot, the finest level also yields CG's z.z and z.b
// partials (z = x, b = CG's residual). TD (row templates): D^-1 of row o is
// tdinv[pid[o]], the template's (the same bits as dinv[o]).
template <bool NT, bool TD = false, bool XS = false>
struct OpMgPost {
    static constexpr int kDots = 2;
    static constexpr bool kSeeded = false;
    static constexpr bool kTmplDiag = TD;  // the pipelined template launch stages tdinv in LDS (row_td)
    // XS (with TD, the pipelined template launch only): t[o] taken from the
    // row's gathered diagonal slot (set_diag) instead of a load of its own
    static constexpr bool kXoFromSlot = XS;
    const double *t, *b, *dinv;
    double *x;
    bool dot;
    const uint8_t *pid = nullptr;
    const double *tdinv = nullptr;
    struct Row {
        double to, bo, dio;
    };
    __device__ double di(int o) const { return TD ? tdinv[pid[o]] : dinv[o]; }
    __device__ double gx(int32_t j) const { return t[j]; }
    __device__ double seed(int) const { return 0.0; }
    __device__ Row row(int o) const { return {t[o], b[o], di(o)}; }
    __device__ Row row_td(int o, double td) const { return {XS ? 0.0 : t[o], b[o], td}; }  // td = tdinv[pid[o]]
    __device__ void set_diag(Row &w, double td) const { w.to = td; }
    __device__ void put(int o, double v, double *d, const Row &w) const {
        const double xo = w.to + 1.0 * (w.dio * (w.bo + (-1.0) * v));
        if constexpr (NT) st_stream(x + o, xo);
        else x[o] = xo;
        if (dot) {
            d[0] += xo * xo;
            d[1] += xo * w.bo;
        }
    }
    __device__ void put(int o, double v, double *d) const {
        const double bo = b[o];
        const double xo = t[o] + 1.0 * (di(o) * (bo + (-1.0) * v));
        if constexpr (NT) st_stream(x + o, xo);
        else x[o] = xo;
        if (dot) {
            d[0] += xo * xo;
            d[1] += xo * bo;
        }
    }
};

// y = D^-1 A x (the GAMG set-up's power iteration, gamg_setup.cpp dinv_apply).
struct OpDinvMult {
    static constexpr int kDots = 0;
    static constexpr bool kSeeded = false;
    static constexpr bool kTmplDiag = false;
    static constexpr bool kXoFromSlot = false;
    const double *x, *dinv;
    double *y;
    struct Row {
        double dio;
    };
    __device__ double gx(int32_t j) const { return x[j]; }
    __device__ double seed(int) const { return 0.0; }
    __device__ Row row(int o) const { return {dinv[o]}; }
    __device__ void put(int o, double v, double *, const Row &w) const { st_stream(y + o, w.dio * v); }
    __device__ void put(int o, double v, double *) const { st_stream(y + o, dinv[o] * v); }
};

// s + p[0] + p[1] + ... + p[n-1], added left to right (PETSc's order). The LDS
// reads go out eight (then four) at a time ahead of their adds, so a lane's chain waits on
// one read latency per eight entries instead of one per entry (FEM rows of
// 50-100 entries are otherwise a serial LDS-latency chain on few lanes).
// Software-pipelined (round 5): the next eight are read before this eight's
// adds, so the chain waits on one LDS latency per row instead of one per
// batch (rows of 45-99 entries: 6-12 batches). Same order, same bits.
__device__ __forceinline__ double row_sum_seq(const double *p, int32_t n, double s) {
    int32_t k = 0;
    if (n >= 8) {
        double v[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = p[i];
        for (k = 8; k + 8 <= n; k += 8) {
            double w[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) w[i] = p[k + i];
#pragma unroll
            for (int i = 0; i < 8; ++i) s += v[i];
#pragma unroll
            for (int i = 0; i < 8; ++i) v[i] = w[i];
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) s += v[i];
    }
    if (k + 4 <= n) {
        double v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = p[k + i];
#pragma unroll
        for (int i = 0; i < 4; ++i) s += v[i];
        k += 4;
    }
    for (; k < n; ++k) s += p[k];
    return s;
}

// One STREAM row block b of blk[0, nblk) by the T lanes of the calling
// workgroup; prod (CAP doubles) and cdict (kCodeDictMax ints, column codes
// only) are the workgroup's LDS.
// NTMODE bit 0: non-temporal matrix loads (scattered long-row operands).
template <int T, int CAP, int RPT, bool CROW, int NTMODE, class Op>
__device__ __forceinline__ void stream_block(
    const int b, const BlockDesc *__restrict__ blk, int nblk, int exact,
    const int32_t *__restrict__ rai, const int32_t *__restrict__ ridx, const int32_t *__restrict__ aj,
    const double *__restrict__ aa, const Op &op, double *dpart, const int *stop, const uint16_t *__restrict__ sslot,
    const int32_t *__restrict__ sbase, double *prod, int32_t *cdict, const double *__restrict__ vdict, int nvd,
    double *vlds) {
    constexpr bool NT = (NTMODE & 1) != 0;
    // bit 3: gather-ordered blocks (Plan::d_saj/d_saa): aj/aa hold each
    // block's entries sorted by column, sslot their positions in the block,
    // where the products go; the row sums below read them in storage order
    constexpr bool SORTED = (NTMODE & 8) != 0;
    // bit 4: the same with each entry's column (relative to the block's
    // first, sbase[b]; 20 bits) and slot (12 bits) packed in one word in
    // aj's place (k_pack_gather_order): one 8-B load per pair as in CSR, 12
    // bytes per entry like the original arrays
    constexpr bool S16 = (NTMODE & 16) != 0;
    // bit 5: column codes (Plan::d_code, full-row lists only): aj holds one
    // 16-bit code per entry, (row - row0) << b | index into the block's
    // dictionary of column - row offsets; sbase holds per block {dictionary
    // start, size} and then the dictionaries. 10 bytes per entry instead of
    // 12; the products, their slots and the sums are the plain kernel's
    constexpr bool CODES = (NTMODE & 32) != 0;
    static_assert(!(CODES && (S16 || SORTED || CROW)), "column codes: plain full-row form only");
    // bit 6: phase 1 without branches: every lane loads its pairs (lanes past
    // the block re-read the block's last pair) and gathers them, so the
    // compiler issues all aj loads, then all aa loads, then all gathers, each
    // group waiting only for what it needs. The predicated form compiles the
    // per-pair `if`s to branches, and at each join the gathers wait for every
    // earlier load, their own predecessors included (vmcnt(0) per pair: four
    // gather round trips per lane instead of one).
    constexpr bool BF = (NTMODE & 64) != 0;
    static_assert(!(BF && SORTED), "branch-free phase 1: plain, coded and 16-bit gather-ordered forms");
    // bit 7: value codes (Plan::d_vcode, set-up operators with few distinct
    // values, e.g. GAMG's finest P and P^T): `aa` holds a 16-bit index per
    // entry (in the array's order, sorted or not) into the dictionary vdict
    // (nvd <= kVDictMax values, staged in LDS; decoded after the gathers are
    // issued): 6 bytes per entry read instead of 12 with aj or the packed
    // columns; the products are the same bits
    constexpr bool VC = (NTMODE & 128) != 0;
    static_assert(!VC || (!CODES && !SORTED && (BF || !S16)),
                  "value codes: the plain (predicated or branch-free) or 16-bit gather-ordered forms");
    constexpr int ITERS = (CAP + 1 + 2 * T - 1) / (2 * T);
    constexpr int DPT = CODES ? (kCodeDictMax + T - 1) / T : 1;  // dictionary entries per lane
    const BlockDesc d = blk[b];
    int32_t nd = 0, dbase = 0;
    if constexpr (CODES) {
        dbase = sbase[2 * b];
        nd = sbase[2 * b + 1];
    }
    // CG launched past convergence: no work. The test also reads the
    // descriptor (d.nk is never negative), so both scalar loads are issued
    // before one wait instead of the descriptor load waiting for the branch.
    if ((stop ? *stop : 0) != 0 || d.nk < 0) return;
    const int t = threadIdx.x;
    const int64_t k0 = d.k0, k1 = (int64_t)d.k0 + d.nk;
    // the block's offset dictionary, loaded ahead of the stream (to LDS below)
    int32_t dval[DPT];
    if constexpr (CODES && BF) {  // unconditional (clamped) loads: no branch ahead of the stream's waits
#pragma unroll
        for (int i = 0; i < DPT; ++i) dval[i] = sbase[nd > 0 ? dbase + min(t + i * T, nd - 1) : 0];
    } else if constexpr (CODES) {
#pragma unroll
        for (int i = 0; i < DPT; ++i)
            if (t + i * T < nd) dval[i] = sbase[dbase + t + i * T];
    }

    constexpr int VPT = VC ? (kVDictMax + T - 1) / T : 1;  // dictionary values per lane
    double vval[VPT];
    if constexpr (VC) {
#pragma unroll
        for (int i = 0; i < VPT; ++i) vval[i] = vdict[min(t + i * T, nvd - 1)];
    }

    // Row extents and MatMultAdd seeds first: they overlap the stream below.
    int32_t rs[RPT], re[RPT], orow[RPT];
    double sum[RPT];
#pragma unroll
    for (int q = 0; q < RPT; ++q) {
        const int r = d.row0 + min(t + q * T, d.nrows - 1);
        rs[q] = rai[r];
        re[q] = rai[r + 1];
        orow[q] = CROW ? ridx[r] : r;
        sum[q] = op.seed(orow[q]);
    }

    // Phase 1: coalesced 16-B loads of aa and 8-B loads of aj from an even
    // (16-B aligned) start; the arrays carry a 2-entry tail pad.
    const int64_t kb = k0 & ~int64_t(1);
    f64x2 av[ITERS];
    i32x2 cv[ITERS];
    f64x2 xv[ITERS];
    uint32_t vw[VC ? ITERS : 1] = {};  // value codes: a pair's two 16-bit indices
    if constexpr (BF) {
        uint32_t cw[CODES ? ITERS : 1];  // a pair's two codes
        const int64_t kl = (k1 - 1) & ~int64_t(1);  // the last pair start (>= kb when nk > 0)
        if (d.nk > 0) {  // (block-uniform)
#pragma unroll
            for (int it = 0; it < ITERS; ++it) {
                const int64_t k = min(kb + 2 * (int64_t)(t + it * T), kl);
                if constexpr (CODES) cw[it] = ld_stream<NT>(reinterpret_cast<const uint32_t *>(aj) + (k >> 1));
                else cv[it] = ld_stream<NT>(reinterpret_cast<const i32x2 *>(aj + k));
            }
            if constexpr (VC) {  // decoded just before the products (the gathers go out first)
#pragma unroll
                for (int it = 0; it < ITERS; ++it)
                    vw[it] = ld_stream<NT>(reinterpret_cast<const uint32_t *>(aa) +
                                           (min(kb + 2 * (int64_t)(t + it * T), kl) >> 1));
            } else {
#pragma unroll
                for (int it = 0; it < ITERS; ++it)
                    av[it] = ld_stream<NT>(
                        reinterpret_cast<const f64x2 *>(aa + min(kb + 2 * (int64_t)(t + it * T), kl)));
            }
        }
        if constexpr (CODES) {
#pragma unroll
            for (int i = 0; i < DPT; ++i)
                if (t + i * T < nd) cdict[t + i * T] = dval[i];
            lds_barrier();
            if (d.nk > 0) {
                const int ib = code_index_bits(d.nrows);
                const uint32_t im = (1u << ib) - 1u;
                const int e0 = (int)(k0 - kb), ne = (int)(k1 - kb), el = (int)(kl - kb);
#pragma unroll
                for (int it = 0; it < ITERS; ++it) {
                    const int e = min(2 * (t + it * T), el);  // the pair this lane loaded
                    const uint32_t lo = cw[it] & 0xffffu, hi = cw[it] >> 16;
                    int32_t c0 = d.row0 + (int32_t)(lo >> ib) + cdict[lo & im];
                    int32_t c1 = d.row0 + (int32_t)(hi >> ib) + cdict[hi & im];
                    if (e < e0) c0 = c1;
                    if (e + 1 >= ne) c1 = c0;
                    xv[it].x = op.gx(c0);
                    xv[it].y = op.gx(c1);
                }
            }
        }
    } else {
        uint32_t cw[CODES ? ITERS : 1];  // a pair's two codes
#pragma unroll
        for (int it = 0; it < ITERS; ++it) {
            const int64_t k = kb + 2 * (int64_t)(t + it * T);
            if (k < k1) {
                if constexpr (VC) vw[it] = ld_stream<NT>(reinterpret_cast<const uint32_t *>(aa) + (k >> 1));
                else av[it] = ld_stream<NT>(reinterpret_cast<const f64x2 *>(aa + k));
                if constexpr (CODES)
                    cw[it] = ld_stream<NT>(reinterpret_cast<const uint32_t *>(aj) + (k >> 1));
                else
                    cv[it] = ld_stream<NT>(reinterpret_cast<const i32x2 *>(aj + k));
            }
        }
        if constexpr (CODES) {
#pragma unroll
            for (int i = 0; i < DPT; ++i)
                if (t + i * T < nd) cdict[t + i * T] = dval[i];
            lds_barrier();
            // decoded and gathered pair by pair (one pair's columns live at a
            // time: decoding all first took 70 VGPRs, 7 waves/SIMD)
            const int ib = code_index_bits(d.nrows);
            const uint32_t im = (1u << ib) - 1u;
            const int e0 = (int)(k0 - kb), ne = (int)(k1 - kb);  // the block's entries relative to kb
#pragma unroll
            for (int it = 0; it < ITERS; ++it) {
                const int e = 2 * (t + it * T);
                if (e < ne) {
                    const uint32_t lo = cw[it] & 0xffffu, hi = cw[it] >> 16;
                    int32_t c0 = d.row0 + (int32_t)(lo >> ib) + cdict[lo & im];
                    int32_t c1 = d.row0 + (int32_t)(hi >> ib) + cdict[hi & im];
                    // a pair straddling a block edge carries the neighbour's
                    // code: that half gathers this half's column (never stored)
                    if (e < e0) c0 = c1;
                    if (e + 1 >= ne) c1 = c0;
                    xv[it].x = op.gx(c0);
                    xv[it].y = op.gx(c1);
                }
            }
        }
    }
    uint32_t sv[(SORTED || S16) ? ITERS : 1];  // the pairs' product slots (two 16-bit positions)
    if constexpr (S16) {  // unpack: .x, .y = the pair's words (column | slot << 20)
        // A pair straddling a block edge carries the neighbour's word,
        // relative to the neighbour's first column: that half is gathered
        // (never stored) at this block's first column instead, which exists.
        const int32_t base = sbase[b];
        constexpr uint32_t cm = (1u << kPackedColBits) - 1u;
#pragma unroll
        for (int it = 0; it < ITERS; ++it) {
            const int64_t k = kb + 2 * (int64_t)(t + it * T);
            const uint32_t w0 = (uint32_t)cv[it].x, w1 = (uint32_t)cv[it].y;
            sv[it] = (w0 >> kPackedColBits) | ((w1 >> kPackedColBits) << 16);
            cv[it].x = base + (k >= k0 && k < k1 ? (int32_t)(w0 & cm) : 0);
            cv[it].y = base + (k + 1 < k1 ? (int32_t)(w1 & cm) : 0);
        }
    }
    if constexpr (SORTED) {
#pragma unroll
        for (int it = 0; it < ITERS; ++it) {
            const int64_t k = kb + 2 * (int64_t)(t + it * T);
            if (k < k1) sv[it] = *reinterpret_cast<const uint32_t *>(sslot + k);
        }
    }
    if constexpr (BF && !CODES) {  // every pair gathered (the clamped ones re-gather the last pair's columns)
        if (d.nk > 0) {
#pragma unroll
            for (int it = 0; it < ITERS; ++it) {
                xv[it].x = op.gx(cv[it].x);
                xv[it].y = op.gx(cv[it].y);
            }
        }
    } else if constexpr (!CODES && !BF) {  // (the coded form gathered with the decode above)
#pragma unroll
        for (int it = 0; it < ITERS; ++it) {
            const int64_t k = kb + 2 * (int64_t)(t + it * T);
            if (k < k1) {
                xv[it].x = op.gx(cv[it].x);
                xv[it].y = op.gx(cv[it].y);
            }
        }
    }
    if constexpr (VC) {
#pragma unroll
        for (int i = 0; i < VPT; ++i)
            if (t + i * T < nvd) vlds[t + i * T] = vval[i];
        lds_barrier();
#pragma unroll
        for (int it = 0; it < ITERS; ++it) {
            av[it].x = vlds[vw[it] & 0xffffu];
            av[it].y = vlds[vw[it] >> 16];
        }
    }
    // products into LDS; only the stores are predicated
#pragma unroll
    for (int it = 0; it < ITERS; ++it) {
        const int64_t k = kb + 2 * (int64_t)(t + it * T);
        if (k < k1) {
            const int s0 = (SORTED || S16) ? (int)(sv[it] & 0xffffu) : (int)(k - k0);
            const int s1 = (SORTED || S16) ? (int)(sv[it] >> 16) : (int)(k + 1 - k0);
            if (k >= k0) prod[s0] = av[it].x * xv[it].x;
            if (k + 1 < k1) prod[s1] = av[it].y * xv[it].y;
        }
    }
    __syncthreads();

    // Phase 2. Short rows (block mean <= kSplitMinMean entries): one lane per
    // row, PETSc's sequential order (bit-exact). Long rows: L lanes per row
    // (strided partial sums + __shfl_xor tree; reordered, deterministic), so
    // a block of few long rows does not leave most lanes idle on a serial
    // LDS chain. `exact` forces the sequential form everywhere.
    double dv[Op::kDots > 0 ? Op::kDots : 1] = {};
    const int nr = d.nrows;
    int L = 1;
    if (RPT == 1 && !exact && d.nk > kSplitMinMean * nr) {
        const int cap = min(64, T / max(nr, 1));
        while (L * 2 <= cap) L *= 2;
    }
    if (L == 1) {
        // batched LDS reads only where rows are long enough to use them (a
        // block-uniform branch): the 7-point rows keep the plain loop, which
        // measured 1-2 % faster for them
        const bool batch = d.nk > kBatchMinMean * nr;
#pragma unroll
        for (int q = 0; q < RPT; ++q) {
            if (t + q * T < nr) {
                double s = sum[q];
                if (batch) {
                    s = row_sum_seq(prod + (rs[q] - k0), re[q] - rs[q], s);
                } else {
                    for (int32_t k = rs[q]; k < re[q]; ++k) s += prod[k - k0];
                }
                op.put(orow[q], s, dv);
            }
        }
    } else {
        const int g = t / L, j = t - g * L;
        const bool own = g < nr;
        const int r = d.row0 + min(g, nr - 1);
        const int32_t grs = rai[r], gre = rai[r + 1];
        double s = 0.0;
        if (own)
            for (int32_t k = grs + j; k < gre; k += L) s += prod[k - k0];
        for (int off = L >> 1; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
        if (own && j == 0) {
            const int o = CROW ? ridx[r] : r;
            op.put(o, Op::kSeeded ? op.seed(o) + s : s, dv);
        }
    }
    // Optional fused epilogue (grid-uniform branch): the block's dot
    // partials, written to dpart[q * nblk + b] for a fixed-order final sum.
    if (Op::kDots > 0 && dpart) {
#pragma unroll
        for (int q = 0; q < (Op::kDots > 0 ? Op::kDots : 1); ++q) {
            const double v = block_sum<T>(dv[q], prod);
            if (t == 0) dpart[(int64_t)q * nblk + b] = v;
        }
    }
}

template <int T, int CAP, int RPT, bool CROW, int NTMODE, class Op>
__global__ __launch_bounds__(T) void k_spmv_stream(
    const BlockDesc *__restrict__ blk, int nblk, int exact,
    const int32_t *__restrict__ rai, const int32_t *__restrict__ ridx, const int32_t *__restrict__ aj,
    const double *__restrict__ aa, Op op, double *dpart, const int *stop, const uint16_t *__restrict__ sslot,
    const int32_t *__restrict__ sbase, const double *__restrict__ vdict = nullptr, int nvd = 0) {
    __shared__ double prod[CAP];
    __shared__ int32_t cdict[(NTMODE & 32) ? kCodeDictMax : 1];
    __shared__ double vlds[(NTMODE & 128) ? kVDictMax : 1];
    stream_block<T, CAP, RPT, CROW, NTMODE, Op>((int)blockIdx.x, blk, nblk, exact, rai, ridx, aj, aa, op, dpart, stop,
                                                sslot, sbase, prod, cdict, vdict, nvd, vlds);
}

// Row patterns (Tuning::patterns; short-row operands whose rows follow a
// few column - row offset lists: stencils): the STREAM row blocks, but the
// columns are not stored per entry. Each row has a pattern id (1 byte), the
// pattern table (offsets in storage order) is staged in LDS per block, and
// the matrix stream is aa alone, staged in LDS by coalesced 16-B loads.
// Phase 2 takes one lane per row: column = row + offset, x gathered by the
// row's lane (neighbouring lanes gather neighbouring x for a stencil), and
// s += aa * x in storage order from s = seed — the arithmetic and order of
// the STREAM kernel's phase 1 + phase 2, so the result is bit-identical.
// ptab: [0, npat) = start | len << 16 of each pattern's offsets, then the
// offsets; ntab entries in all (<= kPatTableMax). The row starts come from
// ai (a scan of the patterns' lengths, branch-free 8-slot gathers, x[r +- 1]
// from the neighbouring lanes, one 16-B LDS write per pair and XCD-chunked
// block placement were all measured slower: profiles/README.md, profiles/r03/patterns/).
template <int T, int CAP, class Op>
__global__ __launch_bounds__(T) void k_spmv_pattern(const BlockDesc *__restrict__ blk, const int32_t *__restrict__ rai,
                                                    const uint8_t *__restrict__ pid, const int32_t *__restrict__ ptab,
                                                    int ntab, int npat, const double *__restrict__ aa, Op op,
                                                    double *dpart, const int *stop) {
    constexpr int ITERS = (CAP + 1 + 2 * T - 1) / (2 * T);
    constexpr int TPT = (kPatTableMax + T - 1) / T;
    __shared__ double av[CAP];
    __shared__ int32_t tab[kPatTableMax];
    const int b = (int)blockIdx.x;
    const BlockDesc d = blk[b];
    if ((stop ? *stop : 0) != 0 || d.nk < 0) return;
    const int t = threadIdx.x;
    const int64_t k0 = d.k0, k1 = (int64_t)d.k0 + d.nk;
    int32_t tv[TPT];
#pragma unroll
    for (int i = 0; i < TPT; ++i)
        if (t + i * T < ntab) tv[i] = ptab[t + i * T];
    const bool own = t < d.nrows;
    const int r = d.row0 + min(t, d.nrows - 1);
    const int p = min((int)pid[r], npat - 1);
    const int32_t rs = rai[r], n = rai[r + 1] - rs;
    const double seed = op.seed(r);
    // the block's values: 16-B loads from an even start (2-entry tail pad)
    const int64_t kb = k0 & ~int64_t(1);
    f64x2 a2[ITERS];
#pragma unroll
    for (int it = 0; it < ITERS; ++it) {
        const int64_t k = kb + 2 * (int64_t)(t + it * T);
        if (k < k1) a2[it] = *reinterpret_cast<const f64x2 *>(aa + k);
    }
#pragma unroll
    for (int i = 0; i < TPT; ++i)
        if (t + i * T < ntab) tab[t + i * T] = tv[i];
#pragma unroll
    for (int it = 0; it < ITERS; ++it) {
        const int64_t k = kb + 2 * (int64_t)(t + it * T);
        if (k < k1) {
            if (k >= k0) av[k - k0] = a2[it].x;
            if (k + 1 < k1) av[k + 1 - k0] = a2[it].y;
        }
    }
    __syncthreads();
    double dv[Op::kDots > 0 ? Op::kDots : 1] = {};
    const int32_t pm = tab[p];
    if (own) {
        const int32_t *off = tab + (pm & 0xffff);
        const double *ar = av + (rs - k0);
        double s = seed;
        for (int32_t j0 = 0; j0 < n; j0 += 8) {
            double xv[8];
#pragma unroll
            for (int j = 0; j < 8; ++j)
                if (j0 + j < n) xv[j] = op.gx(r + off[j0 + j]);
#pragma unroll
            for (int j = 0; j < 8; ++j)
                if (j0 + j < n) s += ar[j0 + j] * xv[j];
        }
        op.put(r, s, dv);
    }
    if (Op::kDots > 0 && dpart) {
#pragma unroll
        for (int q = 0; q < (Op::kDots > 0 ? Op::kDots : 1); ++q) {
            const double v = block_sum<T>(dv[q], av);
            if (t == 0) dpart[(int64_t)q * gridDim.x + b] = v;
        }
    }
}

// Row templates (Tuning::templates; the row patterns of a constant-
// coefficient stencil, values included): the table holds each template's
// offsets and values (pval indexed like the offsets), staged in LDS once per
// workgroup, and the launch streams only the 1-byte ids, x and y — neither
// aj nor aa. One lane per row: s = seed, then s += value * x[r + offset] in
// the row's storage order, the products and sums of k_spmv_pattern on the
// same bits (the values are the row's own, verified bit for bit at plan
// time). With no matrix stream a block's work is three dependent latencies
// (descriptor, ids, gathers), so the workgroups are persistent: each takes
// the row blocks b = first, first + step, ... with the next block's ids and
// the one after's descriptor loaded while the current block gathers. xcd:
// XCD q (workgroup g % 8) takes the q-th eighth of the blocks, so the x
// planes a block gathers are in its own L2. dpart: one partial per block, as
// the STREAM launches write them.
template <int T, int R, class Op>
__global__ __launch_bounds__(T) void k_spmv_template(const BlockDesc *__restrict__ blk, int nblk, int xcd,
                                                     const uint8_t *__restrict__ pid, const int32_t *__restrict__ ptab,
                                                     const double *__restrict__ pval, int ntab, int npat, Op op,
                                                     double *dpart, const int *stop) {
    constexpr int TPT = (kPatTableMax + T - 1) / T;
    __shared__ int32_t tab[kPatTableMax];
    __shared__ double val[kPatTableMax];
    __shared__ double red[R * T / 64];
    if ((stop ? *stop : 0) != 0) return;
    const int t = threadIdx.x, G = (int)gridDim.x, g = (int)blockIdx.x;
    int first = g, step = G, last = nblk;
    if (xcd && G >= 8 && (G & 7) == 0) {
        const int q = g & 7;
        first = (int)((int64_t)nblk * q / 8) + (g >> 3);
        step = G >> 3;
        last = (int)((int64_t)nblk * (q + 1) / 8);
    }
    if (first >= last) return;
#pragma unroll
    for (int i = 0; i < TPT; ++i)
        if (t + i * T < ntab) {
            tab[t + i * T] = ptab[t + i * T];
            val[t + i * T] = pval[t + i * T];
        }
    // lane t takes rows t, t + T, ... (R of them) of each block
    BlockDesc d = blk[first], dn = d;
    if (first + step < last) dn = blk[first + step];
    int p[R];
#pragma unroll
    for (int u = 0; u < R; ++u) p[u] = pid[d.row0 + min(t + u * T, d.nrows - 1)];
    __syncthreads();
    for (int b = first; b < last; b += step) {
        int pn[R] = {};
        BlockDesc dnn = dn;
        if (b + step < last) {
#pragma unroll
            for (int u = 0; u < R; ++u) pn[u] = pid[dn.row0 + min(t + u * T, dn.nrows - 1)];
        }
        if (b + 2 * step < last) dnn = blk[b + 2 * step];
        if (d.nk >= 0) {
            double dv[R][Op::kDots > 0 ? Op::kDots : 1] = {};
            int r[R], st[R], n[R];
            double s[R];
            typename Op::Row rw[R];
            int nmax = 0;
#pragma unroll
            for (int u = 0; u < R; ++u) {
                const bool own = t + u * T < d.nrows;
                r[u] = d.row0 + min(t + u * T, d.nrows - 1);
                const int32_t pm = tab[min(p[u], npat - 1)];
                st[u] = pm & 0xffff;
                n[u] = own ? pm >> 16 : 0;
                nmax = max(nmax, n[u]);
                s[u] = op.seed(r[u]);
                rw[u] = op.row(r[u]);  // issued with the gathers (r is a valid row for every lane)
            }
            for (int32_t j0 = 0; j0 < nmax; j0 += 8) {
                double xv[R][8];
#pragma unroll
                for (int u = 0; u < R; ++u)
#pragma unroll
                    for (int j = 0; j < 8; ++j)
                        if (j0 + j < n[u]) xv[u][j] = op.gx(r[u] + tab[st[u] + j0 + j]);
#pragma unroll
                for (int u = 0; u < R; ++u)
#pragma unroll
                    for (int j = 0; j < 8; ++j)
                        if (j0 + j < n[u]) s[u] += val[st[u] + j0 + j] * xv[u][j];
            }
#pragma unroll
            for (int u = 0; u < R; ++u)
                if (t + u * T < d.nrows) op.put(r[u], s[u], dv[u], rw[u]);
            if (Op::kDots > 0 && dpart) {
                // block_sum<R * T> of the rows in block order: each wave's 64
                // rows by the same shuffle tree, then the R * T / 64 wave sums
                // in row order (the bits of a one-row-per-lane launch)
#pragma unroll
                for (int q = 0; q < (Op::kDots > 0 ? Op::kDots : 1); ++q) {
                    lds_barrier();
#pragma unroll
                    for (int u = 0; u < R; ++u) {
                        double v = dv[u][q];
#pragma unroll
                        for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
                        if ((t & 63) == 0) red[u * (T / 64) + (t >> 6)] = v;
                    }
                    lds_barrier();
                    if (t == 0) {
                        double v = 0.0;
#pragma unroll
                        for (int w = 0; w < R * T / 64; ++w) v += red[w];
                        dpart[(int64_t)q * nblk + b] = v;
                    }
                }
            }
        }
        d = dn;
        dn = dnn;
#pragma unroll
        for (int u = 0; u < R; ++u) p[u] = pn[u];
    }
}

// The same launch software-pipelined across a workgroup's blocks (one lane
// per row; templates of at most kTmplFast entries): while block i is summed,
// block i+1's gathers and row operands and block i+2's ids are in flight.
// Two fixed register sets (A, B) take the blocks in turn — a register copy of
// a load in flight would wait for it — each block's ids are loaded before the
// previous block's gathers, and nothing that loads or stores is behind a
// branch (a path-dependent count of loads in flight makes the compiler wait
// for all of them): past the last block the descriptors repeat the last one
// (its loads are issued again and not used), a lane past a block's rows
// loads the block's last row, and a workgroup with an odd number of blocks
// sums its last block twice, so the loop body has no branch for the compiler
// to sink a prefetch into. Only the stores are per lane (exec-masked): a lane
// stores only its own row of a live block — the waves of a workgroup do not
// run in step, so a duplicate's store could land after another wave already
// stored that row and an in-place MatMultAdd (z = y) read it as its seed. The templates' offsets and values sit in LDS 16-B
// aligned and zero-padded to kTmplFast (an unused slot gathers x[r] and is
// not summed). The sum is s = seed, s += value * x in storage order.
constexpr int kTmplFast = 8;
typedef int32_t i32x4 __attribute__((ext_vector_type(4)));
// F: the gather slots a row takes (7 where every template has at most 7
// entries — the 7-point operand: one load and two registers per stage fewer
// — else kTmplFast)
template <class Op, int F>
struct TmplStage {
    int r, n, p;
    double s;
    typename Op::Row rw;
    double xv[F];
};
template <class Op, int F>
__device__ __forceinline__ void tmpl_issue(const Op &op, const BlockDesc &d, int pid, int npat, const int32_t *tab,
                                           const int32_t *off8, const double *tdl, TmplStage<Op, F> &g) {
    g.r = d.row0 + min((int)threadIdx.x, d.nrows - 1);
    g.p = min(pid, npat - 1);
    const i32x4 o0 = *reinterpret_cast<const i32x4 *>(off8 + g.p * kTmplFast);
    const i32x4 o1 = *reinterpret_cast<const i32x4 *>(off8 + g.p * kTmplFast + 4);
    g.n = tab[g.p] >> 16;
    g.s = op.seed(g.r);
    // D^-1 per template from LDS (Op::kTmplDiag): tdinv[pid[r]] from global
    // memory would wait for the id's load, and so for every load before it
    if constexpr (Op::kTmplDiag) g.rw = op.row_td(g.r, tdl[g.p]);
    else g.rw = op.row(g.r);
    g.xv[0] = op.gx(g.r + o0.x);
    g.xv[1] = op.gx(g.r + o0.y);
    g.xv[2] = op.gx(g.r + o0.z);
    g.xv[3] = op.gx(g.r + o0.w);
    g.xv[4] = op.gx(g.r + o1.x);
    g.xv[5] = op.gx(g.r + o1.y);
    g.xv[6] = op.gx(g.r + o1.z);
    if constexpr (F > 7) g.xv[7] = op.gx(g.r + o1.w);
}
template <int T, class Op, int F>
__device__ __forceinline__ void tmpl_finish(const Op &op, const BlockDesc &d, int live, const TmplStage<Op, F> &g,
                                            const double *val8, const int32_t *dsl, double *red, double *dpart,
                                            int nblk) {
    const int t = threadIdx.x;
    const bool own = t < live;
    const f64x2 *v8 = reinterpret_cast<const f64x2 *>(val8 + g.p * kTmplFast);
    const f64x2 v0 = v8[0], v1 = v8[1], v2 = v8[2], v3 = v8[3];
    const double vv[kTmplFast] = {v0.x, v0.y, v1.x, v1.y, v2.x, v2.y, v3.x, v3.y};
    double s = g.s;
#pragma unroll
    for (int j = 0; j < F; ++j)
        if (j < g.n) s += vv[j] * g.xv[j];
    double dd[Op::kDots > 0 ? Op::kDots : 1] = {};
    typename Op::Row rw = g.rw;
    if constexpr (Op::kXoFromSlot) {  // x[r] = the gathered x of the template's diagonal slot
        const int ds = dsl[g.p];
        double xo = g.xv[0];
#pragma unroll
        for (int j = 1; j < F; ++j) xo = ds == j ? g.xv[j] : xo;
        op.set_diag(rw, xo);
    }
    if (own) op.put(g.r, s, dd, rw);
    if (Op::kDots > 0 && dpart) {
#pragma unroll
        for (int q = 0; q < (Op::kDots > 0 ? Op::kDots : 1); ++q) {
            const double v = block_sum<T>(own ? dd[q] : 0.0, red);
            if (t == 0 && live > 0) dpart[(int64_t)q * nblk + d.k0] = v;
        }
    }
}
template <int T, int F, class Op>
__global__ __launch_bounds__(T) void k_spmv_template_pipe(const BlockDesc *__restrict__ blk, int nblk,
                                                          const uint8_t *__restrict__ pid,
                                                          const int32_t *__restrict__ ptab,
                                                          const double *__restrict__ pval, int ntab, int npat, Op op,
                                                          double *dpart, const int *stop) {
    constexpr int FPT = (kPatMax * kTmplFast + T - 1) / T;
    __shared__ int32_t tab[kPatMax];
    __shared__ __attribute__((aligned(16))) int32_t off8[kPatMax * kTmplFast];
    __shared__ __attribute__((aligned(16))) double val8[kPatMax * kTmplFast];
    __shared__ double tdl[Op::kTmplDiag ? kPatMax : 1];
    __shared__ int32_t dsl[Op::kXoFromSlot ? kPatMax : 1];  // each template's diagonal slot
    __shared__ double red[T / 64];
    if ((stop ? *stop : 0) != 0) return;
    const int t = threadIdx.x, G = (int)gridDim.x, g = (int)blockIdx.x;
    int first = g, step = G, last = nblk;
    if (G >= 8 && (G & 7) == 0) {  // XCD q = g % 8 takes the q-th eighth of the blocks
        const int q = g & 7;
        first = (int)((int64_t)nblk * q / 8) + (g >> 3);
        step = G >> 3;
        last = (int)((int64_t)nblk * (q + 1) / 8);
    }
    if (first >= last) return;
    const int lastb = first + (last - 1 - first) / step * step;  // this workgroup's last block
    if (t < npat) tab[t] = ptab[t];
    if constexpr (Op::kTmplDiag) {
        if (t < npat) tdl[t] = op.tdinv[t];
    }
    if constexpr (Op::kXoFromSlot) {
        if (t < npat) {
            const int32_t pm = ptab[t], st = pm & 0xffff, n = pm >> 16;
            int j0 = 0;
            for (int j = n - 1; j >= 0; --j)
                if (ptab[st + j] == 0) j0 = j;
            dsl[t] = j0;
        }
    }
#pragma unroll
    for (int i = 0; i < FPT; ++i) {
        const int e = t + i * T, pp = e / kTmplFast, j = e % kTmplFast;
        if (pp < npat) {
            const int32_t pm = ptab[pp], st = pm & 0xffff, n = pm >> 16;
            off8[e] = j < n ? ptab[st + j] : 0;
            val8[e] = j < n ? pval[st + j] : 0.0;
        }
    }
    auto lane_row = [&](const BlockDesc &dd) { return dd.row0 + min(t, dd.nrows - 1); };
    BlockDesc d0 = blk[first], d1 = blk[min(first + step, lastb)], d2 = blk[min(first + 2 * step, lastb)];
    int pa = pid[lane_row(d0)];
    int pb = pid[lane_row(d1)];
    __syncthreads();
    TmplStage<Op, F> A, B;
    tmpl_issue(op, d0, pa, npat, tab, off8, tdl, A);
    for (int b = first; b <= lastb; b += 2 * step) {
        // block b (A); b + step's gathers into B; b + 2 step's ids
        pa = pid[lane_row(d2)];
        tmpl_issue(op, d1, pb, npat, tab, off8, tdl, B);
        const BlockDesc d3 = blk[min(b + 3 * step, lastb)];
        __builtin_amdgcn_sched_barrier(0);  // B's loads issue before A's sums wait
        tmpl_finish<T, Op, F>(op, d0, d0.nrows, A, val8, dsl, red, dpart, nblk);
        // block b + step (B; past lastb: lastb again, loaded and summed but
        // not stored); b + 2 step's gathers into A; b + 3 step's ids
        pb = pid[lane_row(d3)];
        tmpl_issue(op, d2, pa, npat, tab, off8, tdl, A);
        const BlockDesc d4 = blk[min(b + 4 * step, lastb)];
        __builtin_amdgcn_sched_barrier(0);
        tmpl_finish<T, Op, F>(op, d1, b + step <= lastb ? d1.nrows : 0, B, val8, dsl, red, dpart, nblk);
        d0 = d2;
        d1 = d3;
        d2 = d4;
    }
}

// Row-template launch shapes. The pipelined kernel (templates of at most
// kTmplFast entries) against the one below (2 rows per lane, no pipeline;
// its fallback for longer templates), per launch inside the 300^3 CG + GAMG
// solve (tools/runs/tmpl_ab.sh, profiles/r06/w; us): V-cycle post-smoothing
// with CG's two dots 301 vs 476, residual 209 vs 237, CG's SpMV + dot 242 vs
// 224; solve 0.1375 vs 0.1492 s (row patterns, aa read: 0.164 s). The one
// below, plain MatMult in tools/ab_opts.py (profiles/r06/o, p): 2 rows per
// lane 134 vs 142 us (1 row) and 160 (4 rows); 32 waves per CU 134 vs 142
// (16); the XCD chunks 134 vs 143 (g % 8 interleaved); row patterns 342.
// (A block's x[row0 - halo, row0 + nrows + halo) staged in LDS by coalesced
// loads, the offsets within the halo read from it and only the neighbour
// planes gathered — 3 window loads + 2 gathers a row for 7 gathers — was
// bit-identical but slower for the plain MatMult, 169.4 / 170.0 vs 139.1 /
// 141.1 us, and equal inside CG, 1841 / 1832 vs 1836 / 1828 it/s, in
// alternating processes, profiles/r06/wa: the per-entry gathers are not what
// bounds this kernel; withdrawn.)
constexpr int kTmplRows = 2;
constexpr int kTmplThreads = kStreamGeoms[6].threads / kTmplRows;
constexpr int kTmplWavesPerCu = 32;
inline int template_grid(const aijhip_mat &A, int32_t nblk) {
    int g = (int)std::min<int64_t>(nblk, (int64_t)A.n_cu * (kTmplWavesPerCu * 64 / kTmplThreads));
    if (g >= 8) g &= ~7;
    return g;
}
// (forcing 8 waves per SIMD, __launch_bounds__(512, 8), spills a few words
// in most epilogues and ran slower: CG + Jacobi 1637-1644 vs 1832-1839 it/s,
// solve 0.137 vs 0.125 s, profiles/r06/w8)
template <int TP, int F, class Op>
static void launch_template_pipe(const aijhip_mat &A, const Op &op, double *dpart, hipStream_t s, const int *stop) {
    const Plan &P = A.plan;
    static const int per_cu = [] {
        int n = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_spmv_template_pipe<TP, F, Op>, TP, 0) != hipSuccess ||
            n < 1)
            n = 1;
        return n;
    }();
    int g = (int)std::min<int64_t>(P.n_blocks, (int64_t)A.n_cu * per_cu);
    if (g >= 8) g &= ~7;
    hipLaunchKernelGGL((k_spmv_template_pipe<TP, F, Op>), dim3(g), dim3(TP), 0, s, P.d_tblocks, P.n_blocks, P.d_pid,
                       P.d_ptab, P.d_pval, P.n_ptab, P.n_pat, op, dpart, stop);
}
template <class Op>
static void launch_template(const aijhip_mat &A, const Op &op, double *dpart, hipStream_t s, const int *stop) {
    const Plan &P = A.plan;
    static_assert(kStreamGeoms[6].rows == kTmplThreads * kTmplRows, "a block's rows = the lanes x kTmplRows");
    if (P.pat_maxlen <= kTmplFast) {
        // persistent: as many workgroups as fit on the device at once (the
        // kernel's registers decide), a multiple of 8 for the XCD chunks
        constexpr int TP = kStreamGeoms[6].threads;
        if (P.pat_maxlen <= 7) launch_template_pipe<TP, 7>(A, op, dpart, s, stop);
        else launch_template_pipe<TP, kTmplFast>(A, op, dpart, s, stop);
        return;
    }
    hipLaunchKernelGGL((k_spmv_template<kTmplThreads, kTmplRows, Op>), dim3(template_grid(A, P.n_blocks)),
                       dim3(kTmplThreads), 0, s, P.d_blocks, P.n_blocks, 1, P.d_pid, P.d_ptab, P.d_pval, P.n_ptab,
                       P.n_pat, op, dpart, stop);
}
// MatMult / MatMultAdd: the dot as a compile-time choice (OpMultT)
template <bool ADD>
static void launch_template(const aijhip_mat &A, const OpMult<ADD> &op, double *dpart, hipStream_t s,
                            const int *stop) {
    const Plan &P = A.plan;
    if (op.dot && P.tmpl_diag && P.pat_maxlen <= kTmplFast) launch_template(A, OpMultT<ADD, true, true>{op}, dpart, s, stop);
    else if (op.dot) launch_template(A, OpMultT<ADD, true>{op}, dpart, s, stop);
    else launch_template(A, OpMultT<ADD, false>{op}, dpart, s, stop);
}

// Segments of long rows: tree-reduced partial sums. (Round 5: lane t taking
// entries k0 + t + 512u instead, so that one gather instruction reads 64
// consecutive entries, measured 43.7 vs 44.9 us — the second gather of a
// pair already hits L1; not kept.) A lane takes 16-B pairs
// (aa as f64x2, aj as i32x2 from an even start, as the STREAM blocks do) at
// pair stride kLongThreads and keeps U pairs in flight: a 4096-entry segment
// is 2048 pairs (512 lanes x 4), so every load and gather of the segment is
// issued before the first product is needed (the previous form, 8 scalar entries per round,
// waited on two dependent latencies per round: 2.66 TB/s). The
// lane's U partial sums are combined u = 0..U-1, then the wave tree, then the
// waves in order: a fixed order.
// The body, for the first kLongThreads lanes of the calling workgroup (any
// further lanes only pass the barrier). red: >= kLongThreads / 64 LDS doubles.
__device__ __forceinline__ void long_segment(const int32_t id, const LongSeg *__restrict__ seg,
                                             const int32_t *__restrict__ aj, const double *__restrict__ aa,
                                             const double *__restrict__ x, double *__restrict__ partials,
                                             double *red) {
    constexpr int U = kLongSegNnz / (2 * kLongThreads);  // pairs in flight per lane
    static_assert(U >= 1, "a round of pairs must fit a segment");
    const LongSeg s = seg[id];
    const int t = threadIdx.x;
    double acc[U] = {};
    const int64_t k0 = s.k0, k1 = (int64_t)s.k0 + s.nk, kb = k0 & ~int64_t(1);
    const int64_t kl = (k1 - 1) & ~int64_t(1);        // the segment's last pair (nk >= 1)
    const int64_t kend = t < kLongThreads ? k1 : kb;  // lanes past kLongThreads take no pairs
    // Straight-line rounds: every pair slot loads (past the segment: its last
    // pair again) and gathers, and the sums take only the segment's entries
    // (selects). Predicated loads compiled to branches, and each gather
    // then waited for all earlier loads: U x 2 dependent scattered round
    // trips per round instead of one (the hub rows' 47 us in r03-r04).
    for (int64_t k = kb + 2 * t; k < kend; k += (int64_t)2 * U * kLongThreads) {
        f64x2 a[U];
        i32x2 c[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            c[u] = __builtin_nontemporal_load(
                reinterpret_cast<const i32x2 *>(aj + min(k + (int64_t)2 * u * kLongThreads, kl)));
#pragma unroll
        for (int u = 0; u < U; ++u)
            a[u] = __builtin_nontemporal_load(
                reinterpret_cast<const f64x2 *>(aa + min(k + (int64_t)2 * u * kLongThreads, kl)));
        double x0[U], x1[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            x0[u] = x[c[u].x];
            x1[u] = x[c[u].y];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t kk = k + (int64_t)2 * u * kLongThreads;
            const double s0 = acc[u] + a[u].x * x0[u];
            acc[u] = (kk < k1 && kk >= k0) ? s0 : acc[u];
            const double s1 = acc[u] + a[u].y * x1[u];
            acc[u] = (kk + 1 < k1) ? s1 : acc[u];
        }
    }
    double v = acc[0];
#pragma unroll
    for (int u = 1; u < U; ++u) v += acc[u];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
    if ((t & 63) == 0 && t < kLongThreads) red[t >> 6] = v;
    __syncthreads();
    if (t == 0) {
        double r = red[0];
#pragma unroll
        for (int w = 1; w < kLongThreads / 64; ++w) r += red[w];
        partials[id] = r;
    }
}

__global__ __launch_bounds__(kLongThreads) void k_long_partial(
    const LongSeg *__restrict__ seg, const int32_t *__restrict__ aj,
    const double *__restrict__ aa, const double *__restrict__ x,
    double *__restrict__ partials, const int32_t *__restrict__ perm) {
    __shared__ double red[kLongThreads / 64];
    long_segment(perm ? perm[blockIdx.x] : (int32_t)blockIdx.x, seg, aj, aa, x, partials, red);
}

// One wavefront per long row: the lanes load 64 partials at once and the sum
// runs through them in segment order by broadcast (a lane-per-row loop waited
// on one dependent load per segment: 9 us for the stand-in's 119 hub rows).
template <bool ADD>
__global__ __launch_bounds__(64) void k_long_finish(const LongRow *__restrict__ lr, int nl,
                                                    const double *__restrict__ partials, const double *z,
                                                    double *y) {
    const int i = blockIdx.x;
    if (i >= nl) return;
    const LongRow r = lr[i];
    const int t = threadIdx.x;
    double s = ADD ? z[r.orow] : 0.0;
    for (int q0 = 0; q0 < r.nseg; q0 += 64) {
        const int nq = min(64, r.nseg - q0);
        const double v = t < nq ? partials[r.seg0 + q0 + t] : 0.0;
        for (int q = 0; q < nq; ++q) s += __shfl(v, q, 64);
    }
    if (t == 0) y[r.orow] = s;
}

template <bool ADD, bool CROW>
__global__ __launch_bounds__(256) void k_spmv_scalar(
    int nr, const int32_t *__restrict__ rai, const int32_t *__restrict__ ridx,
    const int32_t *__restrict__ aj, const double *__restrict__ aa,
    const double *__restrict__ x, const double *z, double *y) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nr) return;
    const int orow = CROW ? ridx[i] : i;
    double s = ADD ? z[orow] : 0.0;
    const int32_t k1 = rai[i + 1];
    for (int32_t k = rai[i]; k < k1; ++k) s += aa[k] * x[aj[k]];
    y[orow] = s;
}

template <int L, bool ADD, bool CROW>
__global__ __launch_bounds__(256) void k_spmv_vector(
    int nr, const int32_t *__restrict__ rai, const int32_t *__restrict__ ridx,
    const int32_t *__restrict__ aj, const double *__restrict__ aa,
    const double *__restrict__ x, const double *z, double *y) {
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t row = gid / L;
    const int lane = threadIdx.x & (L - 1);
    if (row >= nr) return;  // uniform across the L lanes of a row group
    double acc = 0.0;
    const int32_t k1 = rai[row + 1];
    for (int32_t k = rai[row] + lane; k < k1; k += L) acc += aa[k] * x[aj[k]];
#pragma unroll
    for (int off = L / 2; off > 0; off >>= 1) acc += __shfl_xor(acc, off, L);
    if (lane == 0) {
        const int orow = CROW ? ridx[row] : (int)row;
        y[orow] = ADD ? z[orow] + acc : acc;
    }
}

// ------------------------------------------------------------ transpose
__global__ void k_expand_rows(int m, const int32_t *__restrict__ ai, int32_t *rows) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    for (int32_t k = ai[i]; k < ai[i + 1]; ++k) rows[k] = i;
}

__global__ void k_iota(int64_t n, int32_t *v) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) v[i] = (int32_t)i;
}

__global__ void k_gather_transpose(int64_t nz, const int32_t *__restrict__ perm,
                                   const int32_t *__restrict__ rows,
                                   const double *__restrict__ aa, int32_t *taj,
                                   double *taa) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= nz) return;
    const int32_t k = perm[p];
    taj[p] = rows[k];
    taa[p] = aa[k];
}

// tai[c] = first position of column c in the sorted key list (lower bound).
__global__ void k_col_offsets(int n, int64_t nz, const int32_t *__restrict__ keys,
                              int32_t *tai) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c > n) return;
    int64_t lo = 0, hi = nz;
    while (lo < hi) {
        const int64_t p = (lo + hi) >> 1;
        if (keys[p] < c) lo = p + 1;
        else hi = p;
    }
    tai[c] = (int32_t)lo;
}

inline unsigned grid_for(int64_t n, int threads) {
    return (unsigned)((n + threads - 1) / threads);
}

}  // namespace

namespace {
__global__ void k_count_bad_columns(const int32_t *__restrict__ aj, int64_t nz, int32_t n,
                                    unsigned long long *bad) {
    unsigned long long c = 0;
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < nz; k += (int64_t)gridDim.x * blockDim.x)
        c += (uint32_t)aj[k] >= (uint32_t)n;
    if (c) atomicAdd(bad, c);
}
}  // namespace

hipError_t count_bad_columns(const int32_t *d_aj, int64_t nz, int32_t n, int64_t *bad) {
    unsigned long long *d = nullptr, h = 0;
    hipError_t e = hipMalloc(&d, sizeof(*d));
    if (e != hipSuccess) return e;
    if ((e = hipMemset(d, 0, sizeof(*d))) == hipSuccess) {
        hipLaunchKernelGGL(k_count_bad_columns, dim3(4096), dim3(256), 0, nullptr, d_aj, nz, n, d);
        if ((e = hipGetLastError()) == hipSuccess)
            e = hipMemcpy(&h, d, sizeof(h), hipMemcpyDeviceToHost);
    }
    hipFree(d);
    *bad = (int64_t)h;
    return e;
}

namespace {
// per block: min column and span of its entries (one workgroup per block)
__global__ __launch_bounds__(256) void k_block_xrange(const BlockDesc *__restrict__ blk,
                                                      const int32_t *__restrict__ aj, int2 *out) {
    __shared__ int lo_s[4], hi_s[4];
    const BlockDesc d = blk[blockIdx.x];
    int lo = INT32_MAX, hi = -1;
    for (int64_t k = d.k0 + threadIdx.x; k < (int64_t)d.k0 + d.nk; k += 256) {
        lo = min(lo, aj[k]);
        hi = max(hi, aj[k]);
    }
    for (int off = 32; off > 0; off >>= 1) {
        lo = min(lo, __shfl_down(lo, off, 64));
        hi = max(hi, __shfl_down(hi, off, 64));
    }
    if ((threadIdx.x & 63) == 0) {
        lo_s[threadIdx.x >> 6] = lo;
        hi_s[threadIdx.x >> 6] = hi;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < 4; ++w) {
            lo = min(lo, lo_s[w]);
            hi = max(hi, hi_s[w]);
        }
        out[blockIdx.x] = hi < 0 ? make_int2(0, 0) : make_int2(lo, hi - lo + 1);
    }
}
}  // namespace

// Gather-ordered row blocks (Tuning::gsort): one workgroup sorts its
// block's entries by column (ties by position: the keys are unique) and
// writes the sorted columns, the values in that order and each entry's
// position in the block. x is then gathered in column order — a wave's 64
// lanes read a few x lines instead of one per scattered node — while the
// products land at their storage positions, so the row sums (and their bits)
// are the unsorted kernel's.
// The sort: bitonic over N keys, lane t holding keys [tE, tE + E) in
// registers; the stages whose partner lies in another lane go through LDS
// (one barrier each), the last log2(E) stages of every merge stay in
// registers (round 5: the set-up's long-row operators are sorted by default,
// and the LDS-only form — 256 lanes, every stage through LDS — took 17 ms of
// the 300³ GAMG set-up).
template <int E>
__device__ __forceinline__ void bitonic_lane_stage(unsigned long long (&v)[E], int base, int k, int j) {
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const int pe = e ^ j;
        if (pe > e) {
            const bool up = ((base + e) & k) == 0;
            const unsigned long long a = v[e], b = v[pe];
            if ((a > b) == up) {
                v[e] = b;
                v[pe] = a;
            }
        }
    }
}

template <int N, int TB>
__global__ __launch_bounds__(TB) void k_block_gather_order(const BlockDesc *__restrict__ blk,
                                                           const int32_t *__restrict__ aj,
                                                           const double *__restrict__ aa, int32_t *saj,
                                                           double *saa, uint16_t *sslot) {
    constexpr int E = N / TB;
    static_assert(E >= 2 && (E & (E - 1)) == 0 && N <= 65536, "keys per lane: a power of two; 16-bit slots");
    __shared__ unsigned long long key[N];
    const BlockDesc d = blk[blockIdx.x];
    const int t = threadIdx.x, base = t * E;
    unsigned long long v[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const int i = base + e;
        v[e] = i < d.nk ? ((unsigned long long)(uint32_t)aj[(int64_t)d.k0 + i] << 16) | (unsigned)i : ~0ull;
    }
#pragma unroll
    for (int k = 2; k <= E; k <<= 1)
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) bitonic_lane_stage<E>(v, base, k, j);
    for (int k = 2 * E; k <= N; k <<= 1) {
#pragma unroll
        for (int e = 0; e < E; ++e) key[base + e] = v[e];
        __syncthreads();
        for (int j = k >> 1; j >= E; j >>= 1) {
#pragma unroll
            for (int q = 0; q < E / 2; ++q) {
                const int p = t + q * TB;  // pair p: i has bit j clear, its partner i | j
                const int i = ((p & ~(j - 1)) << 1) | (p & (j - 1)), ixj = i | j;
                const unsigned long long a = key[i], b = key[ixj];
                if ((a > b) == ((i & k) == 0)) {
                    key[i] = b;
                    key[ixj] = a;
                }
            }
            __syncthreads();
        }
#pragma unroll
        for (int e = 0; e < E; ++e) v[e] = key[base + e];
#pragma unroll
        for (int j = E >> 1; j > 0; j >>= 1) bitonic_lane_stage<E>(v, base, k, j);
        __syncthreads();  // every lane's reads done before the next merge's writes
    }
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const int i = base + e;
        if (i < d.nk) {
            const int slot = (int)(v[e] & 0xffffu);
            const int64_t k = (int64_t)d.k0 + i;
            saj[k] = (int32_t)(v[e] >> 16);
            sslot[k] = (uint16_t)slot;
            saa[k] = aa[(int64_t)d.k0 + slot];
        }
    }
}

// The block's column span after the sort: (first column, last - first)
__global__ void k_block_col_span(const BlockDesc *__restrict__ blk, int32_t nblk, const int32_t *__restrict__ saj,
                                 int32_t *base, int32_t *span) {
    const int32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nblk) return;
    const BlockDesc d = blk[b];
    const int32_t lo = d.nk > 0 ? saj[d.k0] : 0, hi = d.nk > 0 ? saj[(int64_t)d.k0 + d.nk - 1] : 0;
    base[b] = lo;
    span[b] = hi - lo;
}

// packed form: entry k -> sidx[k] = (column - the block's first) | slot <<
// kPackedColBits (aj's layout: a pair shared by two blocks gets one word
// from each)
__global__ __launch_bounds__(256) void k_pack_gather_order(const BlockDesc *__restrict__ blk,
                                                           const int32_t *__restrict__ saj,
                                                           const uint16_t *__restrict__ sslot,
                                                           const int32_t *__restrict__ base, uint32_t *sidx) {
    const BlockDesc d = blk[blockIdx.x];
    const int32_t b0 = base[blockIdx.x];
    for (int i = threadIdx.x; i < d.nk; i += 256) {
        const int64_t k = (int64_t)d.k0 + i;
        sidx[k] = (uint32_t)(saj[k] - b0) | ((uint32_t)sslot[k] << kPackedColBits);
    }
}

// Column codes (Tuning::codes), one workgroup per row block: the offsets
// aj[k] - row of its entries (a lane per row) are sorted (bitonic over the
// next power of two) and made unique by wave 0 (ballot compaction). Pass 0
// stores the number of distinct offsets; pass 1 stores the dictionary at
// cmeta[cmeta[2b]] and each entry's code (row - row0) << b | rank, the rank
// found by binary search. A block whose count exceeds 2^b is never passed
// to pass 1 (the host splits it off).
template <int N>
__global__ __launch_bounds__(256) void k_block_codes(const BlockDesc *__restrict__ blk,
                                                     const int32_t *__restrict__ rai,
                                                     const int32_t *__restrict__ aj, int32_t *cnt, int32_t *cmeta,
                                                     uint16_t *code) {
    __shared__ int32_t key[N];
    __shared__ int32_t uq[kCodeDictMax];
    __shared__ int32_t s_nd;
    const BlockDesc d = blk[blockIdx.x];
    const int t = threadIdx.x;
    int n2 = 2;
    while (n2 < d.nk) n2 <<= 1;
    for (int r = t; r < d.nrows; r += 256) {
        const int32_t row = d.row0 + r;
        for (int32_t k = rai[row]; k < rai[row + 1]; ++k) key[k - d.k0] = aj[k] - row;
    }
    for (int i = d.nk + t; i < n2; i += 256) key[i] = INT32_MAX;
    __syncthreads();
    for (int k = 2; k <= n2; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = t; i < n2; i += 256) {
                const int ixj = i ^ j;
                if (ixj > i) {
                    const int32_t a = key[i], c = key[ixj];
                    if ((a > c) == ((i & k) == 0)) {
                        key[i] = c;
                        key[ixj] = a;
                    }
                }
            }
            __syncthreads();
        }
    if (t < 64) {
        int n = 0;
        for (int i0 = 0; i0 < d.nk; i0 += 64) {
            const int i = i0 + t;
            const bool f = i < d.nk && (i == 0 || key[i] != key[i - 1]);
            const unsigned long long m = __ballot(f);
            const int pos = n + __popcll(m & ((1ull << t) - 1ull));
            if (f && pos < kCodeDictMax) uq[pos] = key[i];
            n += __popcll(m);
        }
        if (t == 0) s_nd = n;
    }
    __syncthreads();
    const int nd = s_nd;
    if (cmeta == nullptr) {
        if (t == 0) cnt[blockIdx.x] = nd;
        return;
    }
    const int32_t base = cmeta[2 * blockIdx.x];
    for (int i = t; i < nd; i += 256) cmeta[base + i] = uq[i];
    const int ib = code_index_bits(d.nrows);
    for (int r = t; r < d.nrows; r += 256) {
        const int32_t row = d.row0 + r;
        for (int32_t k = rai[row]; k < rai[row + 1]; ++k) {
            const int32_t off = aj[k] - row;
            int lo = 0, hi = nd - 1;
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (uq[mid] < off) lo = mid + 1;
                else hi = mid;
            }
            code[k] = (uint16_t)(((uint32_t)r << ib) | (uint32_t)lo);
        }
    }
}

// The sorted values again after new values (aijhip_mat_update_values)
__global__ __launch_bounds__(256) void k_gather_order_values(const BlockDesc *__restrict__ blk,
                                                             const uint16_t *__restrict__ sslot,
                                                             const double *__restrict__ aa, double *saa) {
    const BlockDesc d = blk[blockIdx.x];
    for (int i = threadIdx.x; i < d.nk; i += 256) {
        const int64_t k = (int64_t)d.k0 + i;
        saa[k] = aa[(int64_t)d.k0 + sslot[k]];
    }
}

hipError_t build_gather_order(const aijhip_mat &A, const Plan &P, bool values_only) {
    if (P.n_blocks == 0) return hipSuccess;
    if (values_only) {
        hipLaunchKernelGGL(k_gather_order_values, dim3(P.n_blocks), dim3(256), 0, nullptr, P.d_blocks, P.d_sslot,
                           A.d_aa, P.d_saa);
        return hipGetLastError();
    }
    const int cap = kStreamGeoms[P.tune.geom].nnz_cap;
#define AIJHIP_GO(NN)                                                                                       \
    hipLaunchKernelGGL((k_block_gather_order<NN, 512>), dim3(P.n_blocks), dim3(512), 0, nullptr, P.d_blocks, \
                       A.d_aj, A.d_aa, P.d_saj, P.d_saa, P.d_sslot)
    if (cap <= 1024) AIJHIP_GO(1024);
    else if (cap <= 2048) AIJHIP_GO(2048);
    else if (cap <= 4096) AIJHIP_GO(4096);
    else AIJHIP_GO(8192);
#undef AIJHIP_GO
    return hipGetLastError();
}

hipError_t gather_order_spans(const Plan &P, int32_t *d_base, int32_t *d_span) {
    if (P.n_blocks == 0) return hipSuccess;
    hipLaunchKernelGGL(k_block_col_span, dim3(grid_for(P.n_blocks, 256)), dim3(256), 0, nullptr, P.d_blocks,
                       P.n_blocks, P.d_saj, d_base, d_span);
    return hipGetLastError();
}

hipError_t pack_gather_order(const Plan &P, const BlockDesc *d_blk, int32_t nblk, const int32_t *d_base,
                             uint32_t *d_sidx) {
    if (nblk == 0) return hipSuccess;
    hipLaunchKernelGGL(k_pack_gather_order, dim3(nblk), dim3(256), 0, nullptr, d_blk, P.d_saj, P.d_sslot, d_base,
                       d_sidx);
    return hipGetLastError();
}

// ---- row patterns (Tuning::patterns) -----------------------------------
__device__ __forceinline__ unsigned long long pat_mix(unsigned long long h) {
    h ^= h >> 30;
    h *= 0xbf58476d1ce4e5b9ull;
    h ^= h >> 27;
    h *= 0x94d049bb133111ebull;
    return h ^ (h >> 31);
}

// 64-bit hash of each row's length and column - row offsets (never 0); with
// aa (row templates) the value bits of each entry too
__global__ __launch_bounds__(256) void k_pat_hash(int32_t m, const int32_t *__restrict__ ai,
                                                  const int32_t *__restrict__ aj, const double *__restrict__ aa,
                                                  unsigned long long *hash) {
    const int32_t r = blockIdx.x * 256 + threadIdx.x;
    if (r >= m) return;
    const int32_t k0 = ai[r], k1 = ai[r + 1];
    unsigned long long h = pat_mix(0x9e3779b97f4a7c15ull + (unsigned long long)(k1 - k0));
    for (int32_t k = k0; k < k1; ++k) {
        h = pat_mix(h ^ (unsigned long long)(uint32_t)(aj[k] - r));
        if (aa) h = pat_mix(h ^ (unsigned long long)__double_as_longlong(aa[k]));
    }
    hash[r] = h | 1ull;
}

// Distinct hashes into an open-addressing table of `ts` slots (a power of
// two): a lane whose wave neighbour holds the same hash leaves the insert to
// it, and a slot already holding the hash is read before any CAS, so the
// ~all-interior rows of a stencil cost one atomic per new pattern. Every
// successful insert is counted (counts[0]); once more than kPatMax distinct
// hashes are in, the operand cannot use row patterns: the inserting lane
// raises `overflow` and every lane that sees it leaves, so a large
// unstructured operand costs ~kPatMax inserts, not m walks of a full table
// (ADVICE r03).
constexpr int kPatTableSlots = 4096;
__global__ __launch_bounds__(256) void k_pat_insert(int32_t m, const unsigned long long *__restrict__ hash,
                                                    unsigned long long *table, int *overflow, int *count) {
    const int32_t r = blockIdx.x * 256 + threadIdx.x;
    const unsigned long long h = r < m ? hash[r] : 0ull;
    const unsigned long long hp = __shfl_up(h, 1, 64);
    if (r >= m || ((threadIdx.x & 63) != 0 && hp == h)) return;
    if (__atomic_load_n(overflow, __ATOMIC_RELAXED)) return;
    unsigned int slot = (unsigned int)(h >> 20) & (kPatTableSlots - 1);
    for (int probe = 0; probe < kPatTableSlots; ++probe) {
        const unsigned long long cur = __atomic_load_n(table + slot, __ATOMIC_RELAXED);
        if (cur == h) return;
        if (cur == 0ull) {
            const unsigned long long prev = atomicCAS(table + slot, 0ull, h);
            if (prev == h) return;
            if (prev == 0ull) {
                if (atomicAdd(count, 1) >= kPatMax) atomicExch(overflow, 1);
                return;
            }
        }
        if ((probe & 15) == 15 && __atomic_load_n(overflow, __ATOMIC_RELAXED)) return;
        slot = (slot + 1) & (kPatTableSlots - 1);
    }
    atomicExch(overflow, 1);
}

// Pattern id of each row (binary search in the sorted distinct hashes) and
// each pattern's first row
__global__ __launch_bounds__(256) void k_pat_assign(int32_t m, const unsigned long long *__restrict__ hash,
                                                    const unsigned long long *__restrict__ sorted, int npat,
                                                    uint8_t *pid, int32_t *rep) {
    const int32_t r = blockIdx.x * 256 + threadIdx.x;
    if (r >= m) return;
    const unsigned long long h = hash[r];
    int lo = 0, hi = npat - 1;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (sorted[mid] < h) lo = mid + 1;
        else hi = mid;
    }
    pid[r] = (uint8_t)lo;
    if (__atomic_load_n(rep + lo, __ATOMIC_RELAXED) > r) atomicMin(rep + lo, r);
}

// The offsets (and with aa the values) of each pattern's first row (at most
// kPatTableMax per row)
__global__ void k_pat_rows(int npat, const int32_t *__restrict__ rep, const int32_t *__restrict__ ai,
                           const int32_t *__restrict__ aj, const double *__restrict__ aa, int32_t *len, int32_t *off,
                           double *val) {
    const int p = blockIdx.x;
    const int32_t r = rep[p], k0 = ai[r], n = ai[r + 1] - k0;
    if (threadIdx.x == 0) len[p] = n;
    for (int j = threadIdx.x; j < n && j < kPatTableMax; j += blockDim.x) {
        off[p * kPatTableMax + j] = aj[k0 + j] - r;
        if (aa) val[p * kPatTableMax + j] = aa[k0 + j];
    }
}

// Rows whose entries differ from their pattern's (a hash collision); with
// pval the value bits are compared too
__global__ __launch_bounds__(256) void k_pat_verify(int32_t m, const int32_t *__restrict__ ai,
                                                    const int32_t *__restrict__ aj, const double *__restrict__ aa,
                                                    const uint8_t *__restrict__ pid, const int32_t *__restrict__ ptab,
                                                    const double *__restrict__ pval, int *bad) {
    const int32_t r = blockIdx.x * 256 + threadIdx.x;
    if (r >= m) return;
    const int32_t pm = ptab[pid[r]], st = pm & 0xffff, len = pm >> 16;
    const int32_t k0 = ai[r], n = ai[r + 1] - k0;
    bool ok = n == len;
    for (int32_t j = 0; ok && j < n; ++j)
        ok = aj[k0 + j] - r == ptab[st + j] &&
             (!pval || __double_as_longlong(aa[k0 + j]) == __double_as_longlong(pval[st + j]));
    if (!ok) atomicAdd(bad, 1);
}

hipError_t build_row_patterns(const aijhip_mat &A, Plan &P, bool *ok, bool values) {
    *ok = false;
    const int32_t m = A.m;
    if (m <= 0 || A.compressed) return hipSuccess;
    const int g = (int)((m + 255) / 256);
    unsigned long long *d_hash = nullptr, *d_table = nullptr, *d_sorted = nullptr;
    int *d_flag = nullptr;
    int32_t *d_rep = nullptr, *d_len = nullptr, *d_off = nullptr;
    double *d_val = nullptr;
    const double *vaa = values ? A.d_aa : nullptr;
    hipError_t e;
    auto done = [&](hipError_t r) {
        hipFree(d_hash); hipFree(d_table); hipFree(d_sorted); hipFree(d_flag);
        hipFree(d_rep); hipFree(d_len); hipFree(d_off); hipFree(d_val);
        return r;
    };
    if ((e = hipMalloc(&d_hash, sizeof(unsigned long long) * (size_t)m)) != hipSuccess ||
        (e = hipMalloc(&d_table, sizeof(unsigned long long) * kPatTableSlots)) != hipSuccess ||
        (e = hipMalloc(&d_flag, sizeof(int) * 3)) != hipSuccess ||
        (e = hipMemset(d_table, 0, sizeof(unsigned long long) * kPatTableSlots)) != hipSuccess ||
        (e = hipMemset(d_flag, 0, sizeof(int) * 3)) != hipSuccess)
        return done(e);
    hipLaunchKernelGGL(k_pat_hash, dim3(g), dim3(256), 0, nullptr, m, A.d_ai, A.d_aj, vaa, d_hash);
    hipLaunchKernelGGL(k_pat_insert, dim3(g), dim3(256), 0, nullptr, m, d_hash, d_table, d_flag, d_flag + 2);
    std::vector<unsigned long long> table(kPatTableSlots);
    int flag[2] = {0, 0};
    if ((e = hipGetLastError()) != hipSuccess ||
        (e = hipMemcpy(table.data(), d_table, sizeof(unsigned long long) * table.size(), hipMemcpyDeviceToHost)) !=
            hipSuccess ||
        (e = hipMemcpy(flag, d_flag, sizeof(int), hipMemcpyDeviceToHost)) != hipSuccess)
        return done(e);
    std::vector<unsigned long long> hs;
    for (unsigned long long h : table)
        if (h) hs.push_back(h);
    if (flag[0] || hs.empty() || (int)hs.size() > kPatMax) return done(hipSuccess);
    std::sort(hs.begin(), hs.end());  // pattern ids in hash order: the same ids run to run
    const int npat = (int)hs.size();
    std::vector<int32_t> rep_init(npat, INT32_MAX);
    if ((e = hipMalloc(&d_sorted, sizeof(unsigned long long) * npat)) != hipSuccess ||
        (e = hipMalloc(&d_rep, sizeof(int32_t) * npat)) != hipSuccess ||
        (e = hipMalloc(&d_len, sizeof(int32_t) * npat)) != hipSuccess ||
        (e = hipMalloc(&d_off, sizeof(int32_t) * (size_t)npat * kPatTableMax)) != hipSuccess ||
        (values && (e = hipMalloc(&d_val, sizeof(double) * (size_t)npat * kPatTableMax)) != hipSuccess) ||
        (e = hipMalloc(&P.d_pid, (size_t)m + 256)) != hipSuccess ||
        (e = hipMemcpy(d_sorted, hs.data(), sizeof(unsigned long long) * npat, hipMemcpyHostToDevice)) !=
            hipSuccess ||
        (e = hipMemcpy(d_rep, rep_init.data(), sizeof(int32_t) * npat, hipMemcpyHostToDevice)) != hipSuccess)
        return done(e);
    hipLaunchKernelGGL(k_pat_assign, dim3(g), dim3(256), 0, nullptr, m, d_hash, d_sorted, npat, P.d_pid, d_rep);
    hipLaunchKernelGGL(k_pat_rows, dim3(npat), dim3(64), 0, nullptr, npat, d_rep, A.d_ai, A.d_aj, vaa, d_len, d_off,
                       d_val);
    std::vector<int32_t> len(npat);
    if ((e = hipGetLastError()) != hipSuccess ||
        (e = hipMemcpy(len.data(), d_len, sizeof(int32_t) * npat, hipMemcpyDeviceToHost)) != hipSuccess)
        return done(e);
    std::vector<int32_t> tab(npat);
    int64_t total = npat;
    for (int p = 0; p < npat; ++p) total += len[p];
    if (total > kPatTableMax) {
        hipFree(P.d_pid);
        P.d_pid = nullptr;
        return done(hipSuccess);
    }
    std::vector<int32_t> off((size_t)npat * kPatTableMax);
    std::vector<double> val(values ? off.size() : 0);
    if ((e = hipMemcpy(off.data(), d_off, sizeof(int32_t) * off.size(), hipMemcpyDeviceToHost)) != hipSuccess ||
        (values && (e = hipMemcpy(val.data(), d_val, sizeof(double) * val.size(), hipMemcpyDeviceToHost)) !=
                       hipSuccess))
        return done(e);
    int32_t dmax = 0;
    std::vector<double> tval(values ? npat : 0, 0.0);
    for (int p = 0; p < npat; ++p) {
        tab[p] = (int32_t)tab.size() | (len[p] << 16);
        for (int j = 0; j < len[p]; ++j) {
            const int32_t o = off[(size_t)p * kPatTableMax + j];
            tab.push_back(o);
            if (values) tval.push_back(val[(size_t)p * kPatTableMax + j]);
            dmax = std::max(dmax, o < 0 ? -o : o);
        }
    }
    P.pat_dmax = dmax;
    P.pat_maxlen = *std::max_element(len.begin(), len.end());
    P.tmpl_diag = true;  // every pattern has the offset 0
    for (int p = 0; p < npat; ++p) {
        bool has = false;
        for (int j = 0; j < len[p]; ++j) has = has || off[(size_t)p * kPatTableMax + j] == 0;
        P.tmpl_diag = P.tmpl_diag && has;
    }
    auto drop = [&]() {
        hipFree(P.d_pid);
        hipFree(P.d_ptab);
        hipFree(P.d_pval);
        P.d_pid = nullptr;
        P.d_ptab = nullptr;
        P.d_pval = nullptr;
    };
    if ((e = hipMalloc(&P.d_ptab, sizeof(int32_t) * tab.size())) != hipSuccess ||
        (e = hipMemcpy(P.d_ptab, tab.data(), sizeof(int32_t) * tab.size(), hipMemcpyHostToDevice)) != hipSuccess ||
        (values && ((e = hipMalloc(&P.d_pval, sizeof(double) * tval.size())) != hipSuccess ||
                    (e = hipMemcpy(P.d_pval, tval.data(), sizeof(double) * tval.size(), hipMemcpyHostToDevice)) !=
                        hipSuccess))) {
        drop();
        return done(e);
    }
    hipLaunchKernelGGL(k_pat_verify, dim3(g), dim3(256), 0, nullptr, m, A.d_ai, A.d_aj, A.d_aa, P.d_pid, P.d_ptab,
                       P.d_pval, d_flag + 1);
    if ((e = hipGetLastError()) != hipSuccess ||
        (e = hipMemcpy(flag, d_flag, sizeof(int) * 2, hipMemcpyDeviceToHost)) != hipSuccess) {
        drop();
        return done(e);
    }
    if (flag[1] != 0) {  // a collision: keep aj (and aa)
        drop();
        return done(hipSuccess);
    }
    P.n_ptab = (int32_t)tab.size();
    P.n_pat = npat;
    P.bytes += (int64_t)m + 256 + 4 * (int64_t)tab.size() + (values ? 8 * (int64_t)tval.size() : 0);
    *ok = true;
    return done(hipSuccess);
}

// ---- value codes (Tuning::vcodes) ---------------------------------------
// The distinct value bit patterns of aa into an open-addressing table of
// kVTableSlots keys (key = bits ^ kVKeyXor; 0 = empty), read before any CAS
// as k_pat_insert does; more than kVDictMax distinct raises `overflow`
// (and every lane then leaves: a matrix of many values costs ~kVDictMax
// inserts). A value whose key would be 0 raises it too.
constexpr int kVTableSlots = 4096;
constexpr unsigned long long kVKeyXor = 0x7ff4dead5a5a1234ull;
__device__ __forceinline__ unsigned int vslot(unsigned long long key) {
    return (unsigned int)(pat_mix(key) >> 20) & (kVTableSlots - 1);
}
__global__ __launch_bounds__(256) void k_vhash_insert(int64_t n, int64_t stride, const double *__restrict__ aa,
                                                      unsigned long long *table, int *flags) {
    const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const unsigned long long key =
        k < n ? ((unsigned long long)__double_as_longlong(aa[k * stride]) ^ kVKeyXor) : 0ull;
    const unsigned long long kp = __shfl_up(key, 1, 64);
    if (k >= n || ((threadIdx.x & 63) != 0 && kp == key)) return;
    if (key == 0ull) {
        atomicExch(flags, 1);
        return;
    }
    if (__atomic_load_n(flags, __ATOMIC_RELAXED)) return;
    unsigned int slot = vslot(key);
    for (int probe = 0; probe < kVTableSlots; ++probe) {
        const unsigned long long cur = __atomic_load_n(table + slot, __ATOMIC_RELAXED);
        if (cur == key) return;
        if (cur == 0ull) {
            const unsigned long long prev = atomicCAS(table + slot, 0ull, key);
            if (prev == key) return;
            if (prev == 0ull) {
                if (atomicAdd(flags + 1, 1) >= kVDictMax) atomicExch(flags, 1);
                return;
            }
        }
        if (__atomic_load_n(flags, __ATOMIC_RELAXED)) return;
        slot = (slot + 1) & (kVTableSlots - 1);
    }
    atomicExch(flags, 1);
}
// Each entry's code: its key's slot, then the slot's dictionary index
__global__ __launch_bounds__(256) void k_vcode_fill(int64_t n, const double *__restrict__ aa,
                                                    const unsigned long long *__restrict__ table,
                                                    const uint16_t *__restrict__ map, uint16_t *code, int *miss) {
    const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (k >= n) return;
    const unsigned long long key = (unsigned long long)__double_as_longlong(aa[k]) ^ kVKeyXor;
    unsigned int slot = vslot(key);
    for (int probe = 0; probe < kVTableSlots; ++probe) {
        if (table[slot] == key) {
            code[k] = map[slot];
            return;
        }
        slot = (slot + 1) & (kVTableSlots - 1);
    }
    atomicExch(miss, 1);
}

hipError_t build_value_codes(const aijhip_mat &A, Plan &P, bool *ok) {
    *ok = false;
    const int64_t nz = A.nz;
    if (nz <= 0) return hipSuccess;
    unsigned long long *d_table = nullptr;
    int *d_flags = nullptr;
    uint16_t *d_map = nullptr;
    hipError_t e;
    auto done = [&](hipError_t r) {
        hipFree(d_table); hipFree(d_flags); hipFree(d_map);
        return r;
    };
    auto drop = [&]() {
        hipFree(P.d_vcode); hipFree(P.d_svcode); hipFree(P.d_vdict);
        P.d_vcode = P.d_svcode = nullptr;
        P.d_vdict = nullptr;
        P.n_vdict = 0;
    };
    const unsigned g = (unsigned)((nz + 255) / 256);
    if ((e = hipMalloc(&d_table, sizeof(unsigned long long) * kVTableSlots)) != hipSuccess ||
        (e = hipMalloc(&d_flags, sizeof(int) * 3)) != hipSuccess ||
        (e = hipMemset(d_table, 0, sizeof(unsigned long long) * kVTableSlots)) != hipSuccess ||
        (e = hipMemset(d_flags, 0, sizeof(int) * 3)) != hipSuccess)
        return done(e);
    int flags[3] = {0, 0, 0};
    // a strided sample of 4096 entries first: an operator of many values (a
    // Galerkin product) is turned away by it after ~kVDictMax inserts (the
    // full pass's lanes would all insert before the overflow is seen: 7.7 ms
    // for a 1 M-entry operator, r06/vd)
    if (nz > (int64_t)1 << 14) {
        const int64_t ns = (int64_t)1 << 12, stride = nz / ns;
        hipLaunchKernelGGL(k_vhash_insert, dim3((unsigned)(ns / 256)), dim3(256), 0, nullptr, ns, stride, A.d_aa,
                           d_table, d_flags);
        if ((e = hipGetLastError()) != hipSuccess ||
            (e = hipMemcpy(flags, d_flags, sizeof(int) * 2, hipMemcpyDeviceToHost)) != hipSuccess)
            return done(e);
        if (flags[0]) return done(hipSuccess);
    }
    hipLaunchKernelGGL(k_vhash_insert, dim3(g), dim3(256), 0, nullptr, nz, (int64_t)1, A.d_aa, d_table, d_flags);
    std::vector<unsigned long long> table(kVTableSlots);
    if ((e = hipGetLastError()) != hipSuccess ||
        (e = hipMemcpy(flags, d_flags, sizeof(int) * 2, hipMemcpyDeviceToHost)) != hipSuccess)
        return done(e);
    if (flags[0] || flags[1] <= 0 || flags[1] > kVDictMax) return done(hipSuccess);
    if ((e = hipMemcpy(table.data(), d_table, sizeof(unsigned long long) * kVTableSlots, hipMemcpyDeviceToHost)) !=
        hipSuccess)
        return done(e);
    std::vector<unsigned long long> bits;  // the distinct values' bits, ascending: the same codes run to run
    for (unsigned long long k : table)
        if (k) bits.push_back(k ^ kVKeyXor);
    std::sort(bits.begin(), bits.end());
    std::vector<uint16_t> map(kVTableSlots, 0);
    std::vector<double> dict(bits.size());
    for (size_t i = 0; i < bits.size(); ++i) std::memcpy(&dict[i], &bits[i], sizeof(double));
    for (int sl = 0; sl < kVTableSlots; ++sl)
        if (table[sl])
            map[sl] = (uint16_t)(std::lower_bound(bits.begin(), bits.end(), table[sl] ^ kVKeyXor) - bits.begin());
    const size_t ncode = (size_t)nz + 2;
    if ((e = hipMalloc(&d_map, sizeof(uint16_t) * kVTableSlots)) != hipSuccess ||
        (e = hipMemcpy(d_map, map.data(), sizeof(uint16_t) * kVTableSlots, hipMemcpyHostToDevice)) != hipSuccess ||
        (e = hipMalloc(&P.d_vdict, sizeof(double) * dict.size())) != hipSuccess ||
        (e = hipMemcpy(P.d_vdict, dict.data(), sizeof(double) * dict.size(), hipMemcpyHostToDevice)) != hipSuccess ||
        // the packed gather-ordered launches read the sorted copy's codes
        // only; the plain blocks the original order's
        (!P.d_saa && ((e = hipMalloc(&P.d_vcode, sizeof(uint16_t) * ncode)) != hipSuccess ||
                      (e = hipMemset(P.d_vcode, 0, sizeof(uint16_t) * ncode)) != hipSuccess)) ||
        (P.d_saa && ((e = hipMalloc(&P.d_svcode, sizeof(uint16_t) * ncode)) != hipSuccess ||
                     (e = hipMemset(P.d_svcode, 0, sizeof(uint16_t) * ncode)) != hipSuccess))) {
        drop();
        return done(e);
    }
    if (!P.d_saa)
        hipLaunchKernelGGL(k_vcode_fill, dim3(g), dim3(256), 0, nullptr, nz, A.d_aa, d_table, d_map, P.d_vcode,
                           d_flags + 2);
    else
        hipLaunchKernelGGL(k_vcode_fill, dim3(g), dim3(256), 0, nullptr, nz, P.d_saa, d_table, d_map, P.d_svcode,
                           d_flags + 2);
    if ((e = hipGetLastError()) != hipSuccess ||
        (e = hipMemcpy(flags + 2, d_flags + 2, sizeof(int), hipMemcpyDeviceToHost)) != hipSuccess) {
        drop();
        return done(e);
    }
    if (flags[2]) {  // (cannot happen: every value was inserted)
        drop();
        return done(hipSuccess);
    }
    P.n_vdict = (int32_t)dict.size();
    P.bytes += (int64_t)(2 * ncode + 8 * dict.size());
    *ok = true;
    return done(hipSuccess);
}

template <bool WRITE>
static hipError_t launch_block_codes(const aijhip_mat &A, const BlockDesc *d_blk, int32_t nblk, int32_t *d_cnt,
                                     int32_t *d_cmeta, uint16_t *d_code, int cap) {
    if (nblk <= 0) return hipSuccess;
    int32_t *meta = WRITE ? d_cmeta : nullptr;
#define AIJHIP_BC(NN) \
    hipLaunchKernelGGL(k_block_codes<NN>, dim3(nblk), dim3(256), 0, nullptr, d_blk, A.d_ai, A.d_aj, d_cnt, meta, d_code)
    if (cap <= 1024) AIJHIP_BC(1024);
    else if (cap <= 2048) AIJHIP_BC(2048);
    else if (cap <= 4096) AIJHIP_BC(4096);
    else AIJHIP_BC(8192);
#undef AIJHIP_BC
    return hipGetLastError();
}

hipError_t column_code_counts(const aijhip_mat &A, const BlockDesc *d_blk, int32_t nblk, int32_t *d_cnt) {
    return launch_block_codes<false>(A, d_blk, nblk, d_cnt, nullptr, nullptr,
                                     kStreamGeoms[A.plan.tune.geom].nnz_cap);
}

hipError_t column_code_write(const aijhip_mat &A, const BlockDesc *d_blk, int32_t nblk, int32_t *d_cmeta,
                             uint16_t *d_code) {
    return launch_block_codes<true>(A, d_blk, nblk, nullptr, d_cmeta, d_code, kStreamGeoms[A.plan.tune.geom].nnz_cap);
}

hipError_t block_column_ranges(const aijhip_mat &A, const BlockDesc *d_blocks, int32_t n_blocks, int2 *d_out) {
    if (n_blocks <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_block_xrange, dim3(n_blocks), dim3(256), 0, nullptr, d_blocks, A.d_aj, d_out);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? hipDeviceSynchronize() : e;
}

// Gather locality of a row sample: distinct 16-column (128-B) x lines per
// entry, counted along each sampled row (columns are sorted within a row)
// over its first kRowLinesWalk entries: a lane that walked a whole 2e5-entry
// hub row serially made this planning kernel 30x the SpMV (12.4 ms).
constexpr int32_t kRowLinesWalk = 512;
__global__ __launch_bounds__(256) void k_row_lines(const int32_t *__restrict__ rai, int32_t nr, int32_t stride,
                                                   const int32_t *__restrict__ aj, unsigned long long *out) {
    const int64_t r = ((int64_t)blockIdx.x * 256 + threadIdx.x) * stride;
    long long ent = 0, lines = 0;
    if (r < nr) {
        const int32_t k0 = rai[r], k1 = min(rai[r + 1], rai[r] + kRowLinesWalk);
        int32_t prev = -1;
        for (int32_t k = k0; k < k1; ++k) {
            const int32_t l = aj[k] >> 4;
            lines += (l != prev);
            prev = l;
        }
        ent = k1 - k0;
    }
    for (int off = 32; off > 0; off >>= 1) {
        ent += __shfl_down(ent, off, 64);
        lines += __shfl_down(lines, off, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(out, (unsigned long long)ent);
        atomicAdd(out + 1, (unsigned long long)lines);
    }
}

hipError_t gather_lines_per_entry(const aijhip_mat &A, double *out) {
    *out = 0.0;
    const int32_t nr = A.h_rai.empty() ? 0 : (int32_t)A.h_rai.size() - 1;
    if (nr <= 0 || A.nz <= 0) return hipSuccess;
    const int32_t stride = std::max<int32_t>(1, nr / 65536);
    const int32_t nsamp = (int32_t)(((int64_t)nr + stride - 1) / stride);
    unsigned long long *d_cnt = nullptr, h_cnt[2] = {0, 0};
    hipError_t e = hipMalloc(&d_cnt, sizeof(h_cnt));
    if (e != hipSuccess) return e;
    if ((e = hipMemset(d_cnt, 0, sizeof(h_cnt))) == hipSuccess) {
        hipLaunchKernelGGL(k_row_lines, dim3(grid_for(nsamp, 256)), dim3(256), 0, nullptr,
                           A.compressed ? A.d_cai : A.d_ai, nr, stride, A.d_aj, d_cnt);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpy(h_cnt, d_cnt, sizeof(h_cnt), hipMemcpyDeviceToHost);
    hipFree(d_cnt);
    if (e == hipSuccess && h_cnt[0] > 0) *out = (double)h_cnt[1] / (double)h_cnt[0];
    return e;
}

__global__ __launch_bounds__(256) void k_seg_midcol(const LongSeg *__restrict__ seg, int32_t ns,
                                                    const int32_t *__restrict__ aj, int32_t *out) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= ns) return;
    const LongSeg s = seg[i];
    out[i] = s.nk > 0 ? aj[(int64_t)s.k0 + s.nk / 2] : 0;
}

hipError_t segment_mid_columns(const aijhip_mat &A, const LongSeg *d_segs, int32_t n_segs, int32_t *h_out) {
    if (n_segs <= 0) return hipSuccess;
    int32_t *d_out = nullptr;
    hipError_t e = hipMalloc(&d_out, sizeof(int32_t) * (size_t)n_segs);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_seg_midcol, dim3(grid_for(n_segs, 256)), dim3(256), 0, nullptr, d_segs, n_segs, A.d_aj,
                       d_out);
    e = hipGetLastError();
    if (e == hipSuccess) e = hipMemcpy(h_out, d_out, sizeof(int32_t) * (size_t)n_segs, hipMemcpyDeviceToHost);
    hipFree(d_out);
    return e;
}

RowList row_list(const aijhip_mat &A) {
    if (A.compressed) return RowList{A.n_crow, A.d_cai, A.d_ridx};
    return RowList{A.m, A.d_ai, nullptr};
}

// Compressed-row form: rows outside the list are 0 (MatMult) or z (MatMultAdd).
static hipError_t compressed_prologue(const aijhip_mat &A, const double *z, double *y,
                                      bool add, hipStream_t s) {
    if (!A.compressed) return hipSuccess;
    if (!add) return hipMemsetAsync(y, 0, sizeof(double) * (size_t)A.m, s);
    if (z != y) return hipMemcpyAsync(y, z, sizeof(double) * (size_t)A.m, hipMemcpyDeviceToDevice, s);
    return hipSuccess;
}

// The wide blocks (few long rows of scattered columns each, split from the
// narrow ones) on the branch-free phase 1 with non-temporal matrix loads:
// with the predicated form each lane's eight scattered gathers waited on one
// another (vmcnt(0) per pair), and a launch of a few dozen such blocks is
// one block's latency — 29 us of the skewed stand-in's serial 331 us
// (round 5, profiles/r05/x)
constexpr int kWideMode = 64 | 1;

template <int T, int CAP, int RPT>
static void stream_dispatch(const aijhip_mat &A, const Plan &P, const RowList &L, const double *x,
                            const double *z, double *y, bool add, hipStream_t s, double *dpart,
                            const int *stop, hipStream_t sw) {  // sw: the wide blocks' stream
    constexpr bool kGeom6 = T == kStreamGeoms[6].threads && CAP == kStreamGeoms[6].nnz_cap && RPT == 1;
#define AIJHIP_SL(ADD, CROW, NT)                                                                             \
    hipLaunchKernelGGL((k_spmv_stream<T, CAP, RPT, CROW, NT, OpMult<ADD>>), dim3(P.n_blocks), dim3(T), 0, s, \
                       P.d_blocks, P.n_blocks, (int)P.tune.exact, L.rai, L.ridx, A.d_aj, A.d_aa,             \
                       OpMult<ADD>{x, z, y, dpart != nullptr}, dpart, stop, nullptr, nullptr);       \
    return
    // Row patterns (Plan::d_pid; geometry 6, full-row lists, short rows)
    if constexpr (kGeom6) {
        if (P.d_pid && !L.ridx) {
#define AIJHIP_PT(ADD)                                                                                        \
    if (P.d_pval)                                                                                             \
        launch_template(A, OpMult<ADD>{x, z, y, dpart != nullptr}, dpart, s, stop);                           \
    else                                                                                                      \
        hipLaunchKernelGGL((k_spmv_pattern<T, CAP, OpMult<ADD>>), dim3(P.n_blocks), dim3(T), 0, s, P.d_blocks, \
                           L.rai, P.d_pid, P.d_ptab, P.n_ptab, P.n_pat, A.d_aa,                                 \
                           OpMult<ADD>{x, z, y, dpart != nullptr}, dpart, stop);                                \
    return
            if (add) { AIJHIP_PT(true); }
            AIJHIP_PT(false);
#undef AIJHIP_PT
        }
    }
    // Column codes (Plan::d_code; geometry 6, full-row lists): MatMult,
    // MatMultAdd and the CG's fused dot; with a coded / uncoded split the dot's
    // partials would come from two launches, so that case takes aj
    if constexpr (kGeom6) {
        if (P.d_code && !L.ridx && (P.n_wblocks == 0 || !dpart)) {
            const BlockDesc *cb = P.n_wblocks ? P.d_nblocks : P.d_blocks;
            const int32_t nc = P.n_wblocks ? P.n_nblocks : P.n_blocks;
#define AIJHIP_SC(ADD, NTM)                                                                                       \
    if (nc > 0)                                                                                                   \
        hipLaunchKernelGGL((k_spmv_stream<T, CAP, RPT, false, NTM, OpMult<ADD>>), dim3(nc), dim3(T), 0, s, cb, nc, \
                           (int)P.tune.exact, L.rai, nullptr, reinterpret_cast<const int32_t *>(P.d_code), A.d_aa, \
                           OpMult<ADD>{x, z, y, dpart != nullptr}, dpart, stop, nullptr, P.d_cmeta);     \
    if (P.n_wblocks > 0)                                                                                          \
        hipLaunchKernelGGL((k_spmv_stream<T, CAP, RPT, false, kWideMode, OpMult<ADD>>), dim3(P.n_wblocks), dim3(T), 0, sw, \
                           P.d_wblocks, P.n_wblocks, (int)P.tune.exact, L.rai, nullptr, A.d_aj, A.d_aa,           \
                           OpMult<ADD>{x, z, y, false}, nullptr, stop, nullptr, nullptr);                \
    return
            // branch-free phase 1 (bit 64): FEM stand-in 229.7 vs 253.5 us
            // predicated (profiles/r04/s1/bf_fem.jsonl)
            if (add) {
                if (P.tune.nt == 1) { AIJHIP_SC(true, 97); }
                AIJHIP_SC(true, 96);
            }
            if (P.tune.nt == 1) { AIJHIP_SC(false, 97); }
            AIJHIP_SC(false, 96);
#undef AIJHIP_SC
        }
    }
    // Gather-ordered blocks (Plan::d_sslot): the sorted copy, every variant
    // (MatMult / MatMultAdd, full or compressed rows, dot epilogue)
    // (with the narrow / wide split, the dot epilogue's partials would come
    // from two launches: the CG's fused product takes the original arrays)
    if (P.d_sidx && (P.n_wblocks == 0 || !dpart)) {  // packed columns and slots, a word per entry
        const BlockDesc *nb = P.n_wblocks ? P.d_nblocks : P.d_blocks;
        const int32_t nn = P.n_wblocks ? P.n_nblocks : P.n_blocks;
#define AIJHIP_SS(ADD, CROW, NTM)                                                                              \
    if (nn > 0)                                                                                                \
        hipLaunchKernelGGL((k_spmv_stream<T, CAP, RPT, CROW, NTM, OpMult<ADD>>), dim3(nn), dim3(T), 0, s, nb, nn, \
                           (int)P.tune.exact, L.rai, L.ridx, reinterpret_cast<const int32_t *>(P.d_sidx), P.d_saa, \
                           OpMult<ADD>{x, z, y, dpart != nullptr}, dpart, stop, nullptr, P.d_sbase);  \
    if (P.n_wblocks > 0)                                                                                       \
        hipLaunchKernelGGL((k_spmv_stream<T, CAP, RPT, CROW, kWideMode, OpMult<ADD>>), dim3(P.n_wblocks), dim3(T), 0, sw, \
                           P.d_wblocks, P.n_wblocks, (int)P.tune.exact, L.rai, L.ridx, A.d_aj, A.d_aa,         \
                           OpMult<ADD>{x, z, y, false}, nullptr, stop, nullptr, nullptr);             \
    return
        // value codes (bit 128: 16-bit indices into the dictionary for aa)
        if constexpr (kGeom6) {
            if (P.d_svcode && !L.ridx) {
#define AIJHIP_SV(ADD)                                                                                         \
    if (nn > 0)                                                                                                \
        hipLaunchKernelGGL((k_spmv_stream<T, CAP, RPT, false, 208, OpMult<ADD>>), dim3(nn), dim3(T), 0, s, nb, nn, \
                           (int)P.tune.exact, L.rai, nullptr, reinterpret_cast<const int32_t *>(P.d_sidx),      \
                           reinterpret_cast<const double *>(P.d_svcode), OpMult<ADD>{x, z, y, dpart != nullptr}, \
                           dpart, stop, nullptr, P.d_sbase, P.d_vdict, P.n_vdict);                             \
    if (P.n_wblocks > 0)                                                                                       \
        hipLaunchKernelGGL((k_spmv_stream<T, CAP, RPT, false, kWideMode, OpMult<ADD>>), dim3(P.n_wblocks), dim3(T), 0, \
                           sw, P.d_wblocks, P.n_wblocks, (int)P.tune.exact, L.rai, nullptr, A.d_aj, A.d_aa,     \
                           OpMult<ADD>{x, z, y, false}, nullptr, stop, nullptr, nullptr);                      \
    return
                if (add) { AIJHIP_SV(true); }
                AIJHIP_SV(false);
#undef AIJHIP_SV
            }
        }
        // branch-free phase 1 (bit 64): skewed stand-in 331.9 vs 340.2 us
        // predicated (profiles/r04/s1/bf_skewed.jsonl)
        if (add && L.ridx) { AIJHIP_SS(true, true, 80); }
        if (add) { AIJHIP_SS(true, false, 80); }
        if (L.ridx) { AIJHIP_SS(false, true, 80); }
        AIJHIP_SS(false, false, 80);
#undef AIJHIP_SS
    }
    if (P.d_sidx) {  // split plan, fused dot: the original arrays in one launch
        if (L.ridx) { AIJHIP_SL(false, true, 0); }
        AIJHIP_SL(false, false, 0);
    }
    if (P.d_sslot) {
#define AIJHIP_SS(ADD, CROW)                                                                                \
    hipLaunchKernelGGL((k_spmv_stream<T, CAP, RPT, CROW, 8, OpMult<ADD>>), dim3(P.n_blocks), dim3(T), 0, s, \
                       P.d_blocks, P.n_blocks, (int)P.tune.exact, L.rai, L.ridx, P.d_saj, P.d_saa,          \
                       OpMult<ADD>{x, z, y, dpart != nullptr}, dpart, stop, P.d_sslot, nullptr);   \
    return
        if (add && L.ridx) { AIJHIP_SS(true, true); }
        if (add) { AIJHIP_SS(true, false); }
        if (L.ridx) { AIJHIP_SS(false, true); }
        AIJHIP_SS(false, false);
#undef AIJHIP_SS
    }
    // (the plain aj blocks keep the predicated phase 1: branch-free measured
    // 505.9 vs 492.8 us at 300^3, profiles/r04/s1/bf_poisson.jsonl — for the
    // 7-point rows the clamped lanes' extra loads and gathers cost more than
    // the serialised gathers, which hit L1/L2; round 5's straight-line form
    // through range-checked buffer loads, whose ISA waits vmcnt(7..4) — one
    // round trip for all eight gathers — measured 483.1 vs 469.8 us too,
    // profiles/r05/b/ab_buf.jsonl: the gathers' serialisation is not what
    // bounds this kernel)
    // (two blocks in flight per workgroup — a persistent grid loading block
    // b + grid's aj / aa while block b gathers, sums and stores, with
    // alternating register sets and unconditional LDS stores so that no wait
    // drains the prefetch — measured 540-630 us vs 469 us at 300^3, bit-exact:
    // at 87 VGPRs it holds 4-5 waves per SIMD against 8, and the hardware's
    // four resident workgroups per CU overlap each other's phases better,
    // profiles/r05/l/ab_pipe.jsonl; withdrawn, option 16 reserved)
    // value codes on the plain blocks: the predicated phase 1 with 16-bit
    // indices into the dictionary for aa (bit 128)
    if constexpr (kGeom6) {
        if (P.d_vcode && !P.d_sslot && !L.ridx && P.n_wblocks == 0) {
#define AIJHIP_PV(ADD)                                                                                     \
    hipLaunchKernelGGL((k_spmv_stream<T, CAP, RPT, false, 128, OpMult<ADD>>), dim3(P.n_blocks), dim3(T), 0, s, \
                       P.d_blocks, P.n_blocks, (int)P.tune.exact, L.rai, nullptr, A.d_aj,                  \
                       reinterpret_cast<const double *>(P.d_vcode), OpMult<ADD>{x, z, y, dpart != nullptr}, \
                       dpart, stop, nullptr, nullptr, P.d_vdict, P.n_vdict);                               \
    return
            if (add) { AIJHIP_PV(true); }
            AIJHIP_PV(false);
#undef AIJHIP_PV
        }
    }
    // non-temporal matrix loads: the plain full-row MatMult / MatMultAdd
    // (the compressed-row form, MPIAIJ's off-diagonal blocks, keeps plain loads)
    if (P.tune.nt == 1 && !L.ridx) {
        if (add) { AIJHIP_SL(true, false, 1); }
        AIJHIP_SL(false, false, 1);
    }
    if (add && L.ridx) { AIJHIP_SL(true, true, 0); }
    if (add) { AIJHIP_SL(true, false, 0); }
    if (L.ridx) { AIJHIP_SL(false, true, 0); }
    AIJHIP_SL(false, false, 0);
#undef AIJHIP_SL
}

#define AIJHIP_GEOM(G) kStreamGeoms[G].threads, kStreamGeoms[G].nnz_cap, \
                       kStreamGeoms[G].rows / kStreamGeoms[G].threads

bool stream_dot_fusable(const aijhip_mat &A) {
    const Plan &P = A.plan;
    return P.kernel == AIJHIP_KERNEL_STREAM && !A.compressed && P.n_longs == 0 && A.m == A.n;
}

hipError_t launch_stream_dot(const aijhip_mat &A, const double *x, double *y, double *dpart,
                             const int *stop, hipStream_t s) {
    if (!stream_dot_fusable(A)) return hipErrorInvalidValue;
    return launch_stream(A, x, nullptr, y, false, s, dpart, stop);
}

bool stream_mg_fusable(const aijhip_mat &A) { return stream_dot_fusable(A); }

template <class Op>
static hipError_t launch_stream_op(const aijhip_mat &A, const Op &op, double *dpart, hipStream_t s,
                                   int exact = -1, const int *stop = nullptr) {
    if (!stream_mg_fusable(A)) return hipErrorInvalidValue;
    const Plan &P = A.plan;
    if (P.n_blocks == 0) return hipSuccess;
    const int ex = exact < 0 ? (int)P.tune.exact : exact;
    if (P.d_pid && P.d_pval) {  // row templates (planned at geometry 6)
        if (P.tune.geom != 6) return hipErrorInvalidValue;
        launch_template(A, op, dpart, s, stop);
        return hipGetLastError();
    }
    if (P.d_pid) {  // row patterns (planned at geometry 6)
        if (P.tune.geom != 6) return hipErrorInvalidValue;
        hipLaunchKernelGGL((k_spmv_pattern<kStreamGeoms[6].threads, kStreamGeoms[6].nnz_cap, Op>), dim3(P.n_blocks),
                           dim3(kStreamGeoms[6].threads), 0, s, P.d_blocks, A.d_ai, P.d_pid, P.d_ptab, P.n_ptab,
                           P.n_pat, A.d_aa, op, dpart, stop);
        return hipGetLastError();
    }
    if (P.d_code && P.n_wblocks == 0 && P.tune.geom == 6) {  // column codes (the planner builds them at geometry 6)
        hipLaunchKernelGGL((k_spmv_stream<AIJHIP_GEOM(6), false, 96, Op>), dim3(P.n_blocks),
                           dim3(kStreamGeoms[6].threads), 0, s, P.d_blocks, P.n_blocks, ex, A.d_ai, nullptr,
                           reinterpret_cast<const int32_t *>(P.d_code), A.d_aa, op, dpart, stop, nullptr,
                           P.d_cmeta);
        return hipGetLastError();
    }
    // gather-ordered blocks: the products land in their storage slots, so the
    // fused epilogues see the same sums as from aj / aa
    if (P.d_sidx && P.n_wblocks == 0 && P.tune.geom == 6) {  // packed columns (planned at geometry 6)
        hipLaunchKernelGGL((k_spmv_stream<AIJHIP_GEOM(6), false, 80, Op>), dim3(P.n_blocks),
                           dim3(kStreamGeoms[6].threads), 0, s, P.d_blocks, P.n_blocks, ex, A.d_ai, nullptr,
                           reinterpret_cast<const int32_t *>(P.d_sidx), P.d_saa, op, dpart, stop, nullptr,
                           P.d_sbase);
        return hipGetLastError();
    }
    if (P.d_sslot && P.d_saj && P.tune.geom == 6) {  // 32-bit sorted columns
        hipLaunchKernelGGL((k_spmv_stream<AIJHIP_GEOM(6), false, 8, Op>), dim3(P.n_blocks),
                           dim3(kStreamGeoms[6].threads), 0, s, P.d_blocks, P.n_blocks, ex, A.d_ai, nullptr,
                           P.d_saj, P.d_saa, op, dpart, stop, P.d_sslot, nullptr);
        return hipGetLastError();
    }
    static_assert(kNumStreamGeoms == 10, "update the geometry dispatch");
#define AIJHIP_OG(G)                                                                                          \
    case G:                                                                                                      \
        hipLaunchKernelGGL((k_spmv_stream<AIJHIP_GEOM(G), false, 0, Op>), dim3(P.n_blocks),                      \
                           dim3(kStreamGeoms[G].threads), 0, s, P.d_blocks, P.n_blocks, ex, A.d_ai, nullptr, A.d_aj, \
                           A.d_aa, op, dpart, stop, nullptr, nullptr);                                  \
        break
    switch (P.tune.geom) {
        AIJHIP_OG(0); AIJHIP_OG(1); AIJHIP_OG(2); AIJHIP_OG(3); AIJHIP_OG(4);
        AIJHIP_OG(5); AIJHIP_OG(6); AIJHIP_OG(7); AIJHIP_OG(8); AIJHIP_OG(9);
        default: return hipErrorInvalidValue;
    }
#undef AIJHIP_OG
    return hipGetLastError();
}

hipError_t launch_stream_blocks(const aijhip_mat &A, int32_t b0, int32_t nb, const double *x, double *y,
                                hipStream_t s) {
    const Plan &P = A.plan;
    if (P.kernel != AIJHIP_KERNEL_STREAM || A.compressed || P.n_longs > 0 || b0 < 0 || b0 + nb > P.n_blocks)
        return hipErrorInvalidValue;
    if (nb <= 0) return hipSuccess;
    static_assert(kNumStreamGeoms == 10, "update the geometry dispatch");
#define AIJHIP_BG(G)                                                                                             \
    case G:                                                                                                      \
        hipLaunchKernelGGL((k_spmv_stream<AIJHIP_GEOM(G), false, 0, OpMult<false>>), dim3(nb),                   \
                           dim3(kStreamGeoms[G].threads), 0, s, P.d_blocks + b0, nb, (int)P.tune.exact, A.d_ai,  \
                           nullptr, A.d_aj, A.d_aa, OpMult<false>{x, nullptr, y, false}, nullptr, nullptr,      \
                           nullptr, nullptr);                                                                    \
        break
    switch (P.tune.geom) {
        AIJHIP_BG(0); AIJHIP_BG(1); AIJHIP_BG(2); AIJHIP_BG(3); AIJHIP_BG(4);
        AIJHIP_BG(5); AIJHIP_BG(6); AIJHIP_BG(7); AIJHIP_BG(8); AIJHIP_BG(9);
        default: return hipErrorInvalidValue;
    }
#undef AIJHIP_BG
    return hipGetLastError();
}

hipError_t launch_mg_resid(const aijhip_mat &A, const double *x, const double *b, double *r, hipStream_t s,
                           bool nt, const int *stop) {
    if (nt) return launch_stream_op(A, OpMgResid<true>{x, b, r}, nullptr, s, -1, stop);
    return launch_stream_op(A, OpMgResid<false>{x, b, r}, nullptr, s, -1, stop);
}

hipError_t launch_mg_post(const aijhip_mat &A, const double *t, const double *b, const double *dinv, double *x,
                          double *dpart, hipStream_t s, bool nt, const int *stop, const double *tdinv) {
    if (tdinv && A.plan.d_pid && A.plan.d_pval) {  // row templates: D^-1 per template
        if (A.plan.tmpl_diag && A.plan.pat_maxlen <= kTmplFast)  // the pipelined launch: t[r] from the diagonal slot
            return launch_stream_op(A, OpMgPost<true, true, true>{t, b, dinv, x, dpart != nullptr, A.plan.d_pid, tdinv},
                                    dpart, s, -1, stop);
        return launch_stream_op(A, OpMgPost<true, true>{t, b, dinv, x, dpart != nullptr, A.plan.d_pid, tdinv}, dpart,
                                s, -1, stop);
    }
    if (nt) return launch_stream_op(A, OpMgPost<true>{t, b, dinv, x, dpart != nullptr}, dpart, s, -1, stop);
    return launch_stream_op(A, OpMgPost<false>{t, b, dinv, x, dpart != nullptr}, dpart, s, -1, stop);
}

hipError_t launch_dinv_mult(const aijhip_mat &A, const double *dinv, const double *x, double *y, hipStream_t s) {
    return launch_stream_op(A, OpDinvMult{x, dinv, y}, nullptr, s, 1);  // PETSc row order
}

hipError_t launch_mult_exact(const aijhip_mat &A, const double *x, double *y, hipStream_t s) {
    return launch_stream_op(A, OpMult<false>{x, nullptr, y, false}, nullptr, s, 1);  // PETSc row order
}

hipError_t launch_stream(const aijhip_mat &A, const double *x, const double *z, double *y,
                         bool add, hipStream_t s, double *dpart, const int *stop) {
    hipError_t e = compressed_prologue(A, z, y, add, s);
    if (e != hipSuccess) return e;
    const RowList L = row_list(A);
    const Plan &P = A.plan;
    // Tuning::overlap: the long rows' segments and the wide blocks (the
    // latency-bound launches) on the side stream, forked from s before any of
    // them and joined back after; the row blocks on s meanwhile. Every launch
    // writes its own rows of y, so the order between them is free. The fork /
    // join events live in the plan: a handle is used by one host thread at a
    // time (include/aijhip.h, "Threading"), as PETSc's Mat is.
    const bool ovl = P.tune.overlap > 0 && P.side && !L.ridx && !dpart && !stop &&
                     (P.n_wblocks > 0 || P.n_longs > 0);
    hipStream_t sw = s;
    if (ovl) {
        if ((e = hipEventRecord(P.ev_fork, s)) != hipSuccess || (e = hipStreamWaitEvent(P.side, P.ev_fork, 0)) !=
                                                                      hipSuccess)
            return e;
        sw = P.side;
    }
    // long rows: segment partials, then their ordered sums
    if (P.n_longs > 0) {
        hipLaunchKernelGGL(k_long_partial, dim3(P.n_segs), dim3(kLongThreads), 0, sw, P.d_segs, A.d_aj, A.d_aa, x,
                           P.d_partials, P.d_segperm);
        if (add) hipLaunchKernelGGL(k_long_finish<true>, dim3(P.n_longs), dim3(64), 0, sw, P.d_longs, P.n_longs,
                                    P.d_partials, z, y);
        else hipLaunchKernelGGL(k_long_finish<false>, dim3(P.n_longs), dim3(64), 0, sw, P.d_longs, P.n_longs,
                                P.d_partials, z, y);
        e = hipGetLastError();
    }
    // Every geometry is dispatched explicitly: the kernel's LDS size must be
    // the one the plan's row blocks were cut for.
    static_assert(kNumStreamGeoms == 10, "update the geometry dispatch");
    if (e == hipSuccess && P.n_blocks > 0) {
#define AIJHIP_SG(G) case G: stream_dispatch<AIJHIP_GEOM(G)>(A, P, L, x, z, y, add, s, dpart, stop, sw); break
        switch (P.tune.geom) {
            AIJHIP_SG(0); AIJHIP_SG(1); AIJHIP_SG(2); AIJHIP_SG(3); AIJHIP_SG(4);
            AIJHIP_SG(5); AIJHIP_SG(6); AIJHIP_SG(7); AIJHIP_SG(8); AIJHIP_SG(9);
            default: e = hipErrorInvalidValue; break;
        }
#undef AIJHIP_SG
        if (e == hipSuccess) e = hipGetLastError();
    }
    // the join is recorded even after a failed launch, so the caller's stream
    // never runs ahead of side-stream work that was already queued
    if (ovl) {
        const hipError_t j = hipEventRecord(P.ev_join, P.side);
        const hipError_t w = j == hipSuccess ? hipStreamWaitEvent(s, P.ev_join, 0) : j;
        if (e == hipSuccess) e = w;
    }
    return e;
}

hipError_t launch_scalar(const aijhip_mat &A, const double *x, const double *z, double *y,
                         bool add, hipStream_t s) {
    hipError_t e = compressed_prologue(A, z, y, add, s);
    if (e != hipSuccess) return e;
    const RowList L = row_list(A);
    if (L.nr == 0) return hipSuccess;
    const dim3 g(grid_for(L.nr, 256)), b(256);
#define AIJHIP_SCALAR(ADD, CROW) \
    hipLaunchKernelGGL((k_spmv_scalar<ADD, CROW>), g, b, 0, s, L.nr, L.rai, L.ridx, A.d_aj, A.d_aa, x, z, y)
    if (add) { if (L.ridx) AIJHIP_SCALAR(true, true); else AIJHIP_SCALAR(true, false); }
    else { if (L.ridx) AIJHIP_SCALAR(false, true); else AIJHIP_SCALAR(false, false); }
#undef AIJHIP_SCALAR
    return hipGetLastError();
}

template <int LN>
static void vector_dispatch(const aijhip_mat &A, const RowList &L, const double *x,
                            const double *z, double *y, bool add, hipStream_t s) {
    const dim3 g(grid_for((int64_t)L.nr * LN, 256)), b(256);
    if (add) {
        if (L.ridx) hipLaunchKernelGGL((k_spmv_vector<LN, true, true>), g, b, 0, s, L.nr, L.rai, L.ridx, A.d_aj, A.d_aa, x, z, y);
        else hipLaunchKernelGGL((k_spmv_vector<LN, true, false>), g, b, 0, s, L.nr, L.rai, L.ridx, A.d_aj, A.d_aa, x, z, y);
    } else {
        if (L.ridx) hipLaunchKernelGGL((k_spmv_vector<LN, false, true>), g, b, 0, s, L.nr, L.rai, L.ridx, A.d_aj, A.d_aa, x, z, y);
        else hipLaunchKernelGGL((k_spmv_vector<LN, false, false>), g, b, 0, s, L.nr, L.rai, L.ridx, A.d_aj, A.d_aa, x, z, y);
    }
}

hipError_t launch_vector(const aijhip_mat &A, const double *x, const double *z, double *y,
                         bool add, hipStream_t s) {
    hipError_t e = compressed_prologue(A, z, y, add, s);
    if (e != hipSuccess) return e;
    const RowList L = row_list(A);
    if (L.nr == 0) return hipSuccess;
    switch (A.plan.lanes) {
        case 2: vector_dispatch<2>(A, L, x, z, y, add, s); break;
        case 4: vector_dispatch<4>(A, L, x, z, y, add, s); break;
        case 8: vector_dispatch<8>(A, L, x, z, y, add, s); break;
        case 16: vector_dispatch<16>(A, L, x, z, y, add, s); break;
        case 32: vector_dispatch<32>(A, L, x, z, y, add, s); break;
        default: vector_dispatch<64>(A, L, x, z, y, add, s); break;
    }
    return hipGetLastError();
}

hipError_t launch_mult(const aijhip_mat &A, const double *x, const double *z, double *y,
                       bool add, hipStream_t s, const int *stop) {
    switch (A.plan.kernel) {
        // the stop flag reaches the STREAM row blocks (the long-row, SCALAR
        // and VECTOR kernels ignore it: they recompute the same values)
        case AIJHIP_KERNEL_STREAM: return launch_stream(A, x, z, y, add, s, nullptr, stop);
        case AIJHIP_KERNEL_SCALAR: return launch_scalar(A, x, z, y, add, s);
        case AIJHIP_KERNEL_VECTOR: return launch_vector(A, x, z, y, add, s);
        default: return hipErrorInvalidValue;
    }
}

hipError_t build_transpose(const aijhip_mat &A, int32_t **d_tai, int32_t **d_taj,
                           double **d_taa, hipStream_t s) {
    const int64_t nz = A.nz;
    int32_t *rows = nullptr, *keys_out = nullptr, *perm_in = nullptr, *perm_out = nullptr;
    void *tmp = nullptr;
    size_t tmp_bytes = 0;
    hipError_t e = hipSuccess;
    *d_tai = nullptr; *d_taj = nullptr; *d_taa = nullptr;
    const size_t nzb = sizeof(int32_t) * (size_t)(nz > 0 ? nz : 1);
#define AIJHIP_TRY(call) do { if ((e = (call)) != hipSuccess) goto done; } while (0)
    AIJHIP_TRY(hipMalloc(d_tai, sizeof(int32_t) * ((size_t)A.n + 1)));
    AIJHIP_TRY(hipMalloc(d_taj, sizeof(int32_t) * (size_t)(nz + 2)));
    AIJHIP_TRY(hipMalloc(d_taa, sizeof(double) * (size_t)(nz + 2)));
    AIJHIP_TRY(hipMemsetAsync(*d_taj, 0, sizeof(int32_t) * (size_t)(nz + 2), s));
    AIJHIP_TRY(hipMemsetAsync(*d_taa, 0, sizeof(double) * (size_t)(nz + 2), s));
    if (nz > 0) {
        AIJHIP_TRY(hipMalloc(&rows, nzb));
        AIJHIP_TRY(hipMalloc(&keys_out, nzb));
        AIJHIP_TRY(hipMalloc(&perm_in, nzb));
        AIJHIP_TRY(hipMalloc(&perm_out, nzb));
        hipLaunchKernelGGL(k_expand_rows, dim3(grid_for(A.m, 256)), dim3(256), 0, s, A.m, A.d_ai, rows);
        hipLaunchKernelGGL(k_iota, dim3(grid_for(nz, 256)), dim3(256), 0, s, nz, perm_in);
        // Stable LSD radix sort by column keeps each column's entries in
        // ascending row order: exactly the order PETSc's MatMultTranspose
        // scatters them, so a row-sequential sum over A^T reproduces it.
        // (only the bits a column index can have: 22 for 3.27 M columns,
        // three 8-bit passes instead of four)
        int bits = 1;
        while (bits < 32 && (int64_t(1) << bits) < (int64_t)A.n) ++bits;
        AIJHIP_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, A.d_aj, keys_out, perm_in,
                                                      perm_out, (int)nz, 0, bits, s));
        AIJHIP_TRY(hipMalloc(&tmp, tmp_bytes));
        AIJHIP_TRY(hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, A.d_aj, keys_out, perm_in,
                                                      perm_out, (int)nz, 0, bits, s));
        hipLaunchKernelGGL(k_gather_transpose, dim3(grid_for(nz, 256)), dim3(256), 0, s, nz,
                           perm_out, rows, A.d_aa, *d_taj, *d_taa);
        hipLaunchKernelGGL(k_col_offsets, dim3(grid_for((int64_t)A.n + 1, 256)), dim3(256), 0, s,
                           A.n, nz, keys_out, *d_tai);
    } else {
        AIJHIP_TRY(hipMemsetAsync(*d_tai, 0, sizeof(int32_t) * ((size_t)A.n + 1), s));
    }
    AIJHIP_TRY(hipGetLastError());
    AIJHIP_TRY(hipStreamSynchronize(s));
done:
#undef AIJHIP_TRY
    hipFree(rows); hipFree(keys_out); hipFree(perm_in); hipFree(perm_out); hipFree(tmp);
    if (e != hipSuccess) {
        hipFree(*d_tai); hipFree(*d_taj); hipFree(*d_taa);
        *d_tai = nullptr; *d_taj = nullptr; *d_taa = nullptr;
    }
    return e;
}

}  // namespace aijhip
