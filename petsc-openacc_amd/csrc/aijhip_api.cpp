// aijhip_api.cpp — the extern "C" boundary (include/aijhip.h): device
// residency of the CSR matrix, row-block planning and kernel dispatch.
//
// Residency lifecycle, as the reference's patched hooks define it:
//   create / assembly_end  <- MatAssemblyEnd_SeqAIJ hook
//                             (src/openacc-step2/MatAssemblyEnd_SeqAIJ.patch:17-44)
//   destroy                <- MatDestroy_SeqAIJ hook
//                             (src/openacc-step2/MatDestroy_SeqAIJ.patch:18-34)
// Unlike the OpenACC present table (acc_is_present, MatAssemblyEnd patch:21-23)
// the handle owns its device buffers explicitly: no reference counting, no
// implicit copies on MatMult (the step-2 `enter data copyin` per call,
// step2 MatMult patch:19-21, becomes a one-off upload here).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <tuple>
#include <atomic>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "aijhip_internal.h"

using aijhip::BlockDesc;
using aijhip::LongRow;
using aijhip::LongSeg;

namespace {

thread_local std::string g_err;
// row lists at least this long are planned on several host threads
constexpr int32_t kParallelPlanRows = 1 << 20;

int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}

int hipfail(hipError_t e, const char *what) {
    g_err = std::string(what) + ": " + hipGetErrorString(e);
    return (e == hipErrorNoDevice || e == hipErrorInvalidDevice) ? AIJHIP_ERR_NODEVICE
                                                                 : AIJHIP_ERR_HIP;
}

// Sets the handle's device for the duration of a call, restoring the
// caller's current device afterwards (torch keeps its own notion of it).
struct DeviceGuard {
    int prev = -1;
    hipError_t err = hipSuccess;
    explicit DeviceGuard(int dev) {
        err = hipGetDevice(&prev);
        if (err == hipSuccess && prev != dev) err = hipSetDevice(dev);
        else if (err == hipSuccess) prev = -1;
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

template <typename T>
hipError_t dmalloc(T **p, size_t count, int64_t *acct) {
    *p = nullptr;
    const size_t bytes = sizeof(T) * (count > 0 ? count : 1);
    hipError_t e = hipMalloc(reinterpret_cast<void **>(p), bytes);
    if (e == hipSuccess && acct) *acct += (int64_t)bytes;
    return e;
}

void free_plan(aijhip::Plan &P) {
    hipFree(P.d_blocks);
    hipFree(P.d_segs);
    hipFree(P.d_longs);
    hipFree(P.d_partials);
    hipFree(P.d_segperm);
    hipFree(P.d_saj);
    hipFree(P.d_saa);
    hipFree(P.d_sslot);
    hipFree(P.d_sidx);
    hipFree(P.d_sbase);
    hipFree(P.d_nblocks);
    hipFree(P.d_wblocks);
    hipFree(P.d_code);
    hipFree(P.d_cmeta);
    hipFree(P.d_pid);
    hipFree(P.d_ptab);
    hipFree(P.d_pval);
    hipFree(P.d_tblocks);
    hipFree(P.d_vcode);
    hipFree(P.d_svcode);
    hipFree(P.d_vdict);
    if (P.side) hipStreamDestroy(P.side);
    if (P.ev_fork) hipEventDestroy(P.ev_fork);
    if (P.ev_join) hipEventDestroy(P.ev_join);
    aijhip::host_pipe_free(P.hpipe);
    P = aijhip::Plan();
}

void free_matrix(aijhip_mat *A) {
    A->plan_gen = A->values_gen = aijhip::next_plan_gen();
    free_plan(A->plan);
    hipFree(A->d_ai);
    hipFree(A->d_aj);
    hipFree(A->d_aa);
    hipFree(A->d_cai);
    hipFree(A->d_ridx);
    A->d_ai = A->d_aj = A->d_cai = A->d_ridx = nullptr;
    A->d_aa = nullptr;
    A->device_bytes = 0;
    A->h_rai.clear();
    A->h_rai.shrink_to_fit();
    if (A->transpose) {
        free_matrix(A->transpose);
        delete A->transpose;
        A->transpose = nullptr;
    }
}

int validate_csr(int32_t m, int32_t n, int64_t nz, const int32_t *ai, const int32_t *aj) {
    if (m < 0 || n < 0 || nz < 0) return fail(AIJHIP_ERR_ARG, "negative size");
    if (nz > INT32_MAX) return fail(AIJHIP_ERR_ARG, "nz exceeds the int32 PetscInt range");
    if (!ai) return fail(AIJHIP_ERR_ARG, "ai is NULL");
    if (ai[0] != 0) return fail(AIJHIP_ERR_ARG, "ai[0] != 0");
    for (int32_t i = 0; i < m; ++i)
        if (ai[i + 1] < ai[i]) return fail(AIJHIP_ERR_ARG, "ai is not monotone at row " + std::to_string(i));
    if (ai[m] != nz) return fail(AIJHIP_ERR_ARG, "ai[m] != nz");
    if (aj)  // host columns; device columns are checked by aijhip::count_bad_columns
        for (int64_t k = 0; k < nz; ++k)
            if ((uint32_t)aj[k] >= (uint32_t)n)
                return fail(AIJHIP_ERR_ARG, "column index out of range at entry " + std::to_string(k));
    return AIJHIP_OK;
}

int32_t isolate_row_nnz() {
    const char *v = std::getenv("AIJHIP_ISOLATE_ROW_NNZ");
    return v ? (int32_t)std::atoi(v) : aijhip::kIsolateRowNnz;
}

// CSR-stream row blocks over the handle's row list (h_rai): greedily pack
// consecutive rows while the block holds <= nnz_cap entries and <= rows rows
// of the chosen geometry. A longer row becomes a long row, split into
// segments of <= kLongSegNnz entries.
// Greedy row blocks of rows [r0, r1) of the row list (see plan_stream).
void plan_rows(const aijhip_mat *A, const aijhip::StreamGeom &G, const int32_t *h_ridx, int32_t r0, int32_t r1,
               std::vector<BlockDesc> &blocks, std::vector<LongSeg> &segs, std::vector<LongRow> &longs) {
    using namespace aijhip;
    const auto &rai = A->h_rai;
    // segment length: 1024-16384 measured within 3 % on the skewed stand-in
    // (profiles/r03/longseg/)
    constexpr int64_t seg_nnz = kLongSegNnz;
    // rows longer than this get a block of their own (kIsolateRowNnz;
    // AIJHIP_ISOLATE_ROW_NNZ overrides it for A/B runs, 0 = never)
    const int32_t isolate = isolate_row_nnz();
    int32_t r = r0;
    while (r < r1) {
        const int32_t len = rai[r + 1] - rai[r];
        if (len > G.nnz_cap) {
            LongRow lr{};
            lr.orow = h_ridx ? h_ridx[r] : r;
            lr.seg0 = (int32_t)segs.size();
            for (int64_t k = rai[r]; k < rai[r + 1]; k += seg_nnz) {
                const int64_t nk = std::min<int64_t>(seg_nnz, rai[r + 1] - k);
                segs.push_back(LongSeg{(int32_t)k, (int32_t)nk});
            }
            lr.nseg = (int32_t)segs.size() - lr.seg0;
            longs.push_back(lr);
            ++r;
            continue;
        }
        const int32_t start = r;
        int32_t nk = 0;
        while (r < r1 && r - start < G.rows) {
            const int32_t l = rai[r + 1] - rai[r];
            if (l > G.nnz_cap || nk + l > G.nnz_cap) break;
            if (isolate > 0 && l > isolate) {  // a block of its own (see kIsolateRowNnz)
                if (r == start) {
                    nk = l;
                    ++r;
                }
                break;
            }
            nk += l;
            ++r;
        }
        blocks.push_back(BlockDesc{start, r - start, rai[start], nk});
    }
}

int plan_stream(aijhip_mat *A) {
    using namespace aijhip;
    const auto &rai = A->h_rai;
    const int32_t nr = rai.empty() ? 0 : (int32_t)rai.size() - 1;
    std::vector<BlockDesc> blocks;
    std::vector<LongSeg> segs;
    std::vector<LongRow> longs;
    std::vector<int32_t> h_ridx;
    if (A->compressed && A->n_crow > 0) {
        h_ridx.resize(A->n_crow);
        hipError_t e = hipMemcpy(h_ridx.data(), A->d_ridx, sizeof(int32_t) * A->n_crow, hipMemcpyDeviceToHost);
        if (e != hipSuccess) return hipfail(e, "plan: read ridx");
    }
    const StreamGeom G = kStreamGeoms[A->plan.tune.geom];
    const int32_t *ridx = h_ridx.empty() ? nullptr : h_ridx.data();
    // Large operands are planned in row ranges on host threads (a block
    // boundary at each range start: speed-only, the sums do not change);
    // 27 M rows take ~30 ms on one thread.
    const int nt = nr >= kParallelPlanRows ? (int)std::min<unsigned>(16, std::max(1u, std::thread::hardware_concurrency()))
                                          : 1;
    if (nt <= 1) {
        blocks.reserve((size_t)nr / 64 + 8);
        plan_rows(A, G, ridx, 0, nr, blocks, segs, longs);
    } else {
        std::vector<std::vector<BlockDesc>> pb(nt);
        std::vector<std::vector<LongSeg>> ps(nt);
        std::vector<std::vector<LongRow>> pl(nt);
        std::vector<std::thread> th;
        for (int t = 0; t < nt; ++t)
            th.emplace_back([&, t] {
                const int32_t r0 = (int32_t)((int64_t)nr * t / nt), r1 = (int32_t)((int64_t)nr * (t + 1) / nt);
                pb[t].reserve((size_t)(r1 - r0) / 64 + 8);
                plan_rows(A, G, ridx, r0, r1, pb[t], ps[t], pl[t]);
            });
        for (auto &x : th) x.join();
        for (int t = 0; t < nt; ++t) {
            blocks.insert(blocks.end(), pb[t].begin(), pb[t].end());
            for (LongRow lr : pl[t]) {
                lr.seg0 += (int32_t)segs.size();
                longs.push_back(lr);
            }
            segs.insert(segs.end(), ps[t].begin(), ps[t].end());
        }
    }
    Plan &P = A->plan;
    P.n_blocks = (int32_t)blocks.size();
    P.n_segs = (int32_t)segs.size();
    P.n_longs = (int32_t)longs.size();
    hipError_t e;
    if ((e = dmalloc(&P.d_blocks, blocks.size(), &P.bytes)) != hipSuccess) return hipfail(e, "plan: alloc blocks");
    if (!blocks.empty() &&
        (e = hipMemcpy(P.d_blocks, blocks.data(), sizeof(BlockDesc) * blocks.size(), hipMemcpyHostToDevice)) != hipSuccess)
        return hipfail(e, "plan: upload blocks");
    // gather-ordered copy of the row blocks (Tuning::gsort): for the plain
    // MatMult / MatMultAdd launch
    if (P.tune.gsort > 0 && !blocks.empty()) {
        const size_t nzp = (size_t)A->nz + 2;
        if ((e = dmalloc(&P.d_saj, nzp, &P.bytes)) != hipSuccess || (e = dmalloc(&P.d_saa, nzp, &P.bytes)) != hipSuccess ||
            (e = dmalloc(&P.d_sslot, nzp, &P.bytes)) != hipSuccess ||
            (e = hipMemset(P.d_saj, 0, sizeof(int32_t) * nzp)) != hipSuccess ||
            (e = hipMemset(P.d_saa, 0, sizeof(double) * nzp)) != hipSuccess ||
            (e = hipMemset(P.d_sslot, 0, sizeof(uint16_t) * nzp)) != hipSuccess ||
            (e = aijhip::build_gather_order(*A, P, false)) != hipSuccess)
            return hipfail(e, "plan: gather-ordered blocks");
        // the packed form (20-bit columns and 12-bit slots, one word per
        // entry) when the blocks' columns span < 2^20 and their caps fit the
        // slots: it replaces the 32-bit sorted columns (12 B per entry, not 14)
        int32_t *d_base = nullptr, *d_span = nullptr;
        std::vector<int32_t> span((size_t)P.n_blocks);
        if ((e = dmalloc(&d_base, (size_t)P.n_blocks, nullptr)) != hipSuccess ||
            (e = dmalloc(&d_span, (size_t)P.n_blocks, nullptr)) != hipSuccess ||
            (e = aijhip::gather_order_spans(P, d_base, d_span)) != hipSuccess ||
            (e = hipMemcpy(span.data(), d_span, sizeof(int32_t) * span.size(), hipMemcpyDeviceToHost)) != hipSuccess) {
            hipFree(d_base);
            hipFree(d_span);
            return hipfail(e, "plan: gather-ordered spans");
        }
        hipFree(d_span);
        // blocks whose columns span < 2^20 take the packed form; when most
        // do, the others (a wide row within the block cap) are launched from
        // the original arrays
        constexpr int32_t kNarrowSpan = 1 << aijhip::kPackedColBits;
        const bool slots_fit = aijhip::kStreamGeoms[P.tune.geom].nnz_cap <= aijhip::kPackedMaxCap;
        int64_t narrow_nz = 0, nz_all = 0;
        for (size_t b = 0; b < blocks.size(); ++b) {
            nz_all += blocks[b].nk;
            if (span[b] < kNarrowSpan) narrow_nz += blocks[b].nk;
        }
        if (slots_fit && narrow_nz > 0 && 10 * narrow_nz >= 9 * nz_all) {
            std::vector<BlockDesc> nb, wb;
            std::vector<int32_t> nbase, base((size_t)P.n_blocks);
            if ((e = hipMemcpy(base.data(), d_base, sizeof(int32_t) * base.size(), hipMemcpyDeviceToHost)) != hipSuccess) {
                hipFree(d_base);
                return hipfail(e, "plan: gather-ordered spans");
            }
            for (size_t b = 0; b < blocks.size(); ++b) {
                if (span[b] < kNarrowSpan) {
                    nb.push_back(blocks[b]);
                    nbase.push_back(base[b]);
                } else {
                    wb.push_back(blocks[b]);
                }
            }
            hipFree(d_base);
            const size_t words = (size_t)A->nz + 4;
            if ((e = dmalloc(&P.d_sidx, words, &P.bytes)) != hipSuccess ||
                (e = hipMemset(P.d_sidx, 0, sizeof(uint32_t) * words)) != hipSuccess ||
                (e = dmalloc(&P.d_sbase, nbase.size(), &P.bytes)) != hipSuccess ||
                (e = hipMemcpy(P.d_sbase, nbase.data(), sizeof(int32_t) * nbase.size(), hipMemcpyHostToDevice)) !=
                    hipSuccess)
                return hipfail(e, "plan: gather-ordered packed form");
            if (!wb.empty()) {
                if ((e = dmalloc(&P.d_nblocks, nb.size(), &P.bytes)) != hipSuccess ||
                    (e = dmalloc(&P.d_wblocks, wb.size(), &P.bytes)) != hipSuccess ||
                    (e = hipMemcpy(P.d_nblocks, nb.data(), sizeof(BlockDesc) * nb.size(), hipMemcpyHostToDevice)) !=
                        hipSuccess ||
                    (e = hipMemcpy(P.d_wblocks, wb.data(), sizeof(BlockDesc) * wb.size(), hipMemcpyHostToDevice)) !=
                        hipSuccess)
                    return hipfail(e, "plan: gather-ordered block lists");
                P.n_nblocks = (int32_t)nb.size();
                P.n_wblocks = (int32_t)wb.size();
                for (const BlockDesc &d : wb) P.nz_wide += d.nk;
            }
            if ((e = aijhip::pack_gather_order(P, wb.empty() ? P.d_blocks : P.d_nblocks, (int32_t)nb.size(), P.d_sbase,
                                               P.d_sidx)) != hipSuccess ||
                (e = hipDeviceSynchronize()) != hipSuccess)
                return hipfail(e, "plan: gather-ordered packed form");
            hipFree(P.d_saj);  // (d_sslot stays: it re-orders new values, aijhip_mat_update_values)
            P.bytes -= (int64_t)sizeof(int32_t) * (int64_t)nzp;
            P.d_saj = nullptr;
        } else {
            hipFree(d_base);
        }
    }
    // row patterns (Tuning::patterns): a pattern id per row in aj's place
    // for short-row operands whose rows follow few offset lists (stencils);
    // geometry 6, plain full-row launches, no long rows
    const int32_t nrl = rai.empty() ? 0 : (int32_t)rai.size() - 1;
    if (P.tune.patterns > 0 && P.tune.geom == 6 && !blocks.empty() && longs.empty() && !A->compressed &&
        A->nz <= (int64_t)kBatchMinMean * nrl && P.d_sslot == nullptr) {
        // with the values first (row templates: neither aj nor aa read), then
        // the offsets alone
        bool ok = false;
        if (P.tune.templates != 0 && (e = aijhip::build_row_patterns(*A, P, &ok, true)) != hipSuccess)
            return hipfail(e, "plan: row templates");
        if (!ok && (e = aijhip::build_row_patterns(*A, P, &ok, false)) != hipSuccess)
            return hipfail(e, "plan: row patterns");
        if (ok && P.d_pval) {
            // the row templates' block order: a stencil's rows r and r +- D
            // (D = the largest offset, a plane) share x lines, so the blocks
            // go through the operand in column slabs of S rows of each plane,
            // plane after plane within a slab: the x lines a block gathers
            // from the planes either side are reused while they are still in
            // the XCD's L2. k0 of the copy = the block's own index (its dot
            // partial's slot; a template launch reads no entry range).
            // S <= 8192 rows (profiles/r06/v, w: the CG SpMV's fetched bytes
            // 0.62 GB in natural order, 0.60 / 0.52 / 0.44 GB at S = 16384 /
            // 32768 / 8192; the times within a few per cent — the launch is
            // bound by its gathers' latency, not its traffic)
            const int64_t D = P.pat_dmax, split = 8192;
            std::vector<int32_t> order(blocks.size());
            for (size_t b = 0; b < blocks.size(); ++b) order[b] = (int32_t)b;
            if (split > 0 && D > split) {
                const int64_t ns = (D + split - 1) / split, S = (D + ns - 1) / ns;
                auto key = [&](int32_t b) {
                    const int64_t r = blocks[b].row0;
                    return std::make_tuple((r % D) / S, r / D, r % D);
                };
                std::stable_sort(order.begin(), order.end(), [&](int32_t a, int32_t b) { return key(a) < key(b); });
            }
            std::vector<BlockDesc> tb(blocks.size());
            for (size_t i = 0; i < order.size(); ++i) {
                tb[i] = blocks[order[i]];
                tb[i].k0 = order[i];
            }
            if ((e = dmalloc(&P.d_tblocks, tb.size(), &P.bytes)) != hipSuccess ||
                (e = hipMemcpy(P.d_tblocks, tb.data(), sizeof(BlockDesc) * tb.size(), hipMemcpyHostToDevice)) !=
                    hipSuccess)
                return hipfail(e, "plan: template block order");
        }
    }
    P.tune.templates = P.d_pval != nullptr ? 1 : 0;
    // column codes (Tuning::codes): a 16-bit code per entry in aj's place
    // for the row blocks whose offset dictionaries fit (geometry 6, plain
    // full-row launches: not with the x tiles or the gather order); when
    // some do not fit, they are launched from aj
    if (P.tune.codes > 0 && P.tune.geom == 6 && !blocks.empty() && P.d_pid == nullptr && !A->compressed &&
        P.d_sslot == nullptr) {
        int32_t *d_cnt = nullptr;
        std::vector<int32_t> cnt(blocks.size());
        if ((e = dmalloc(&d_cnt, blocks.size(), nullptr)) != hipSuccess ||
            (e = aijhip::column_code_counts(*A, P.d_blocks, P.n_blocks, d_cnt)) != hipSuccess ||
            (e = hipMemcpy(cnt.data(), d_cnt, sizeof(int32_t) * cnt.size(), hipMemcpyDeviceToHost)) != hipSuccess) {
            hipFree(d_cnt);
            return hipfail(e, "plan: column code counts");
        }
        hipFree(d_cnt);
        int64_t fit_nz = 0, nz_all = 0, dict = 0;
        std::vector<char> fit(blocks.size());
        for (size_t b = 0; b < blocks.size(); ++b) {
            fit[b] = cnt[b] <= (1 << aijhip::code_index_bits(blocks[b].nrows));
            nz_all += blocks[b].nk;
            if (fit[b]) {
                fit_nz += blocks[b].nk;
                dict += cnt[b];
            }
        }
        if (fit_nz > 0 && 10 * fit_nz >= 9 * nz_all) {
            std::vector<BlockDesc> nb, wb;
            std::vector<int32_t> meta;
            for (size_t b = 0; b < blocks.size(); ++b) (fit[b] ? nb : wb).push_back(blocks[b]);
            meta.resize(2 * nb.size());
            int64_t pos = (int64_t)meta.size();
            for (size_t b = 0, j = 0; b < blocks.size(); ++b)
                if (fit[b]) {
                    meta[2 * j] = (int32_t)pos;
                    meta[2 * j + 1] = cnt[b];
                    pos += cnt[b];
                    ++j;
                }
            if (pos > INT32_MAX) return fail(AIJHIP_ERR_ARG, "plan: column code dictionaries too large");
            P.n_cmeta = pos;
            const size_t ncode = (size_t)A->nz + 2;
            if ((e = dmalloc(&P.d_cmeta, (size_t)pos, &P.bytes)) != hipSuccess ||
                (e = hipMemcpy(P.d_cmeta, meta.data(), sizeof(int32_t) * meta.size(), hipMemcpyHostToDevice)) !=
                    hipSuccess ||
                (e = dmalloc(&P.d_code, ncode, &P.bytes)) != hipSuccess ||
                (e = hipMemset(P.d_code, 0, sizeof(uint16_t) * ncode)) != hipSuccess)
                return hipfail(e, "plan: column codes");
            if (!wb.empty()) {
                if ((e = dmalloc(&P.d_nblocks, nb.size(), &P.bytes)) != hipSuccess ||
                    (e = dmalloc(&P.d_wblocks, wb.size(), &P.bytes)) != hipSuccess ||
                    (e = hipMemcpy(P.d_nblocks, nb.data(), sizeof(BlockDesc) * nb.size(), hipMemcpyHostToDevice)) !=
                        hipSuccess ||
                    (e = hipMemcpy(P.d_wblocks, wb.data(), sizeof(BlockDesc) * wb.size(), hipMemcpyHostToDevice)) !=
                        hipSuccess)
                    return hipfail(e, "plan: column code block lists");
                P.n_nblocks = (int32_t)nb.size();
                P.n_wblocks = (int32_t)wb.size();
                for (const BlockDesc &d : wb) P.nz_wide += d.nk;
            }
            if ((e = aijhip::column_code_write(*A, wb.empty() ? P.d_blocks : P.d_nblocks, (int32_t)nb.size(),
                                               P.d_cmeta, P.d_code)) != hipSuccess ||
                (e = hipDeviceSynchronize()) != hipSuccess)
                return hipfail(e, "plan: column codes");
        }
    }
    // value codes (Tuning::vcodes): a 16-bit index per entry into a
    // dictionary of aa's distinct values, in aa's place, for operators of at
    // most kVDictMax distinct values (GAMG's finest P and Pᵀ: ~370) read by
    // the plain or packed gather-ordered blocks: 6 bytes per entry instead of
    // 12, the same bits
    // (automatic for the set-up's operators; measured in the 300³ solve,
    // profiles/r06/ve, vg: the finest Pᵀ 199 vs 275 us per launch, the finest
    // P — plain blocks, predicated loads — 231 vs 277 us; solve 0.130 vs
    // 0.1415 s; the many-valued operators are turned away by a sample)
    const bool want_vc = P.tune.vcodes > 0 || (P.tune.vcodes < 0 && A->setup_op);
    if (want_vc && P.tune.geom == 6 && !blocks.empty() && longs.empty() && !A->compressed && !P.d_pid &&
        !P.d_code && (P.d_sslot == nullptr || P.d_sidx != nullptr) && P.n_wblocks == 0) {
        bool ok = false;
        if ((e = aijhip::build_value_codes(*A, P, &ok)) != hipSuccess) return hipfail(e, "plan: value codes");
    }
    P.tune.vcodes = (P.d_vcode || P.d_svcode) ? 1 : 0;
    if (!longs.empty()) {
        if ((e = dmalloc(&P.d_segs, segs.size(), &P.bytes)) != hipSuccess ||
            (e = dmalloc(&P.d_longs, longs.size(), &P.bytes)) != hipSuccess ||
            (e = dmalloc(&P.d_partials, segs.size(), &P.bytes)) != hipSuccess)
            return hipfail(e, "plan: alloc long rows");
        if ((e = hipMemcpy(P.d_segs, segs.data(), sizeof(LongSeg) * segs.size(), hipMemcpyHostToDevice)) != hipSuccess ||
            (e = hipMemcpy(P.d_longs, longs.data(), sizeof(LongRow) * longs.size(), hipMemcpyHostToDevice)) != hipSuccess)
            return hipfail(e, "plan: upload long rows");
        if (P.tune.long_xcd && segs.size() >= 16 && A->n >= 8) {
            // deal segments to launch slots so that slot s (XCD s % 8 under
            // round-robin placement) gets one whose middle column lies in the
            // (s % 8)-th eighth of x; an exhausted eighth takes from the fullest
            std::vector<int32_t> mid(segs.size());
            if ((e = aijhip::segment_mid_columns(*A, P.d_segs, P.n_segs, mid.data())) != hipSuccess)
                return hipfail(e, "plan: segment columns");
            std::vector<std::vector<int32_t>> part(8);
            for (int32_t i = 0; i < P.n_segs; ++i)
                part[std::min<int64_t>(7, (int64_t)mid[i] * 8 / A->n)].push_back(i);
            std::vector<size_t> head(8, 0);
            std::vector<int32_t> perm(segs.size());
            for (int32_t s = 0; s < P.n_segs; ++s) {
                int q = s & 7;
                if (head[q] == part[q].size()) {
                    size_t best = 0;
                    for (int c = 0; c < 8; ++c)
                        if (part[c].size() - head[c] > best) { best = part[c].size() - head[c]; q = c; }
                }
                perm[s] = part[q][head[q]++];
            }
            if ((e = dmalloc(&P.d_segperm, perm.size(), &P.bytes)) != hipSuccess ||
                (e = hipMemcpy(P.d_segperm, perm.data(), sizeof(int32_t) * perm.size(), hipMemcpyHostToDevice)) !=
                    hipSuccess)
                return hipfail(e, "plan: segment placement");
        }
    }
    // Tuning::overlap: a side stream and its two events for the wide blocks
    // and the long rows (created once per plan that has them)
    if (P.tune.overlap > 0 && (P.n_wblocks > 0 || P.n_longs > 0)) {
        if ((e = hipStreamCreateWithFlags(&P.side, hipStreamNonBlocking)) != hipSuccess ||
            (e = hipEventCreateWithFlags(&P.ev_fork, aijhip::sync_event_flags())) != hipSuccess ||
            (e = hipEventCreateWithFlags(&P.ev_join, aijhip::sync_event_flags())) != hipSuccess)
            return hipfail(e, "plan: side stream");
    }
    return AIJHIP_OK;
}

int plan_build(aijhip_mat *A) {
    A->plan_gen = A->values_gen = aijhip::next_plan_gen();
    free_plan(A->plan);
    aijhip::Plan &P = A->plan;
    int kernel = A->requested_kernel;
    if (kernel == AIJHIP_KERNEL_AUTO) kernel = AIJHIP_KERNEL_STREAM;
    P.kernel = kernel;
    P.tune = A->requested_tune;
    // long rows after the row blocks, except in exact mode, where the rows
    // of 1-4 K entries keep one lane's sequential sum and the side stream
    // hides that chain (round 5: skewed stand-in default 310.7 vs 315.2 us
    // side stream; exact 350.5 us after, profiles/r05/ad/)
    // (with fewer hardware queues than a side stream needs, after them too)
    if (P.tune.overlap < 0) P.tune.overlap = P.tune.exact && aijhip::hw_queues() >= aijhip::kOverlapMinQueues;
    const bool auto_sort = P.tune.gsort < 0 && !A->setup_op;  // (a set-up operator keeps the 32-bit form)
    const bool auto_codes = P.tune.codes < 0;
    const bool auto_patterns = P.tune.patterns < 0;
    bool scattered = false;
    if (P.tune.geom < 0 || P.tune.nt < 0 || P.tune.gsort < 0) {
        // measured: 512 x 4094-entry blocks (geometry 6, 8 waves/SIMD) for
        // short rows (7-pt Poisson, profiles/r01/tune04) and for long rows
        // whose gathers run along x lines (FEM-structured stand-in: 283 vs
        // 313 us); 512 x 4096 (geometry 1: 76 VGPRs, 6 waves/SIMD) for long
        // rows with scattered gathers (skewed stand-in 405 vs 449 us, GAMG's
        // coarse operators) — profiles/r01/rowsum/. Non-temporal matrix
        // loads for the scattered ones (skewed 398 vs 411 us; Poisson and the
        // FEM stand-in are neutral to slower: profiles/r02/ntlong/)
        const int32_t nr = A->h_rai.empty() ? 0 : (int32_t)A->h_rai.size() - 1;
        const bool long_rows = nr > 0 && A->nz > (int64_t)16 * nr;
        if (long_rows) {
            double lpe = 1.0;
            const hipError_t e = aijhip::gather_lines_per_entry(*A, &lpe);
            if (e != hipSuccess) return hipfail(e, "plan: gather locality");
            scattered = lpe > aijhip::kScatteredLinesPerEntry;
        }
        // Long rows on a caller's handle: the gather-ordered copy of the row
        // blocks (Tuning::gsort; x read in column order within a block, the
        // sums unchanged) at geometry 6, plain loads, when its packed form
        // fits (below) — measured: skewed stand-in 406 -> 325 us, its
        // ordinary rows 342 -> 256, the FEM-structured one 287 -> 271
        // (profiles/r03/gsort_*.jsonl); the 7-pt Poisson (short rows) stays
        // unsorted (sorted: 551 vs 492 us). The set-up's own operators (GAMG
        // levels, P, Pᵀ; aijhip_mat::setup_op) take it for long rows too and
        // keep the 32-bit sorted columns when the packed form does not fit.
        if (P.tune.gsort < 0) P.tune.gsort = long_rows ? 1 : 0;
        const bool sorted = P.tune.gsort > 0;
        if (P.tune.geom < 0) P.tune.geom = (scattered && !sorted) ? 1 : 6;
        if (P.tune.nt < 0) P.tune.nt = (scattered && !sorted) ? 1 : 0;
    }
    if (P.tune.codes < 0) P.tune.codes = 0;  // automatic: tried below (STREAM)
    if (P.tune.patterns < 0) P.tune.patterns = 0;
    switch (kernel) {
        case AIJHIP_KERNEL_STREAM: {
            // Automatic column codes: tried first on every full-row operand
            // the coded launch serves (geometry 6, gather order off, no other
            // layout knob); kept when the blocks' offset dictionaries fit
            // (>= 90 % of the entries), else the choice above without them.
            // Measured in one process (profiles/r03/codes/): 300^3 Poisson
            // 486.6 -> 433.8 us, FEM stand-in 267.4 (gather-ordered) ->
            // 263.4 us; the skewed stand-in's blocks never fit.
            // Row patterns are tried the same way, before the codes, for
            // short rows (a stencil: no per-entry column at all).
            const aijhip::Tuning &rq = A->requested_tune;
            if ((auto_codes || auto_patterns) && !A->compressed && rq.gsort <= 0 && (rq.geom < 0 || rq.geom == 6) &&
                rq.nt <= 1) {
                const aijhip::Tuning keep = P.tune;
                if (auto_codes) P.tune.codes = 1;
                if (auto_patterns) P.tune.patterns = 1;
                P.tune.gsort = 0;
                P.tune.geom = 6;
                if (rq.nt < 0) P.tune.nt = 0;
                const int rc = plan_stream(A);
                if (rc || P.d_code || P.d_pid) return rc;
                free_plan(A->plan);
                P.kernel = kernel;
                P.tune = keep;
            }
            int rc = plan_stream(A);
            if (!rc && auto_sort && P.tune.gsort > 0 && !P.d_sidx) {
                // automatic and the packed form did not fit (blocks spanning
                // 2^20 columns and more): the original layout, the geometry
                // and loads the gather locality picks without it
                const aijhip::Tuning req = A->requested_tune;
                free_plan(A->plan);
                P.kernel = kernel;
                P.tune = req;
                if (P.tune.overlap < 0)
                    P.tune.overlap = P.tune.exact && aijhip::hw_queues() >= aijhip::kOverlapMinQueues;
                P.tune.gsort = 0;
                if (P.tune.geom < 0) P.tune.geom = scattered ? 1 : 6;
                if (P.tune.nt < 0) P.tune.nt = scattered ? 1 : 0;
                if (P.tune.codes < 0) P.tune.codes = 0;
                if (P.tune.patterns < 0) P.tune.patterns = 0;
                rc = plan_stream(A);
            }
            return rc;
        }
        case AIJHIP_KERNEL_SCALAR:
            return AIJHIP_OK;
        case AIJHIP_KERNEL_VECTOR: {
            int lanes = A->requested_lanes;
            if (lanes == 0) {
                const int32_t nr = A->h_rai.empty() ? 0 : (int32_t)A->h_rai.size() - 1;
                const double mean = nr > 0 ? (double)A->nz / nr : 1.0;
                lanes = 2;
                while (lanes < 64 && lanes < mean) lanes <<= 1;
            }
            if (lanes != 2 && lanes != 4 && lanes != 8 && lanes != 16 && lanes != 32 && lanes != 64)
                return fail(AIJHIP_ERR_ARG, "VECTOR lanes must be a power of two in [2, 64]");
            P.lanes = lanes;
            return AIJHIP_OK;
        }
        default:
            return fail(AIJHIP_ERR_ARG, "unknown kernel " + std::to_string(kernel));
    }
}

// Uploads a validated CSR into A (sizes already set) and plans it. ai is on
// the host; aj/aa on the host, or on the device when dev_src (copied D2D).
// own_ai, when given, holds ai and is moved into the handle's host offsets.
// Structure statistics, PETSc's compressed-row form and the host row list,
// then the plan — from the host row offsets ai (adopted when own_ai holds
// them). The device CSR is already in place.
int structure_and_plan(aijhip_mat *A, const int32_t *ai, aijhip::HostVec<int32_t> *own_ai) {
    const int32_t m = A->m;
    const int64_t nz = A->nz;
    hipError_t e;
    // structure statistics (PETSc a->nonzerorowcnt, MatCheckCompressedRow);
    // row ranges on host threads for large operands, as the planning below
    int32_t nzrows = 0, maxlen = 0;
    {
        const int nt = m >= kParallelPlanRows
                           ? (int)std::min<unsigned>(16, std::max(1u, std::thread::hardware_concurrency()))
                           : 1;
        std::vector<int32_t> pz(nt, 0), pm(nt, 0);
        auto stats = [&](int t) {
            const int32_t r0 = (int32_t)((int64_t)m * t / nt), r1 = (int32_t)((int64_t)m * (t + 1) / nt);
            int32_t z = 0, x = 0;
            for (int32_t i = r0; i < r1; ++i) {
                const int32_t l = ai[i + 1] - ai[i];
                z += l > 0;
                x = std::max(x, l);
            }
            pz[t] = z;
            pm[t] = x;
        };
        if (nt <= 1) {
            stats(0);
        } else {
            std::vector<std::thread> th;
            for (int t = 0; t < nt; ++t) th.emplace_back(stats, t);
            for (auto &x : th) x.join();
        }
        for (int t = 0; t < nt; ++t) {
            nzrows += pz[t];
            maxlen = std::max(maxlen, pm[t]);
        }
    }
    A->nonzerorowcnt = nzrows;
    A->max_row_nz = maxlen;
    // PETSc uses the compressed-row form when at least 60% of the rows are
    // empty (MatCheckCompressedRow(..., ratio=0.6) in MatAssemblyEnd_SeqAIJ,
    // step2 MatAssemblyEnd patch context :35 [ext]).
    A->compressed = m > 0 && (1.0 - (double)nzrows / (double)m) >= 0.6;
    if (A->compressed) {
        aijhip::HostVec<int32_t> cai;
        std::vector<int32_t> ridx;
        cai.reserve((size_t)nzrows + 1);
        ridx.reserve((size_t)nzrows);
        for (int32_t i = 0; i < m; ++i)
            if (ai[i + 1] > ai[i]) { cai.push_back(ai[i]); ridx.push_back(i); }
        cai.push_back((int32_t)nz);
        A->n_crow = nzrows;
        if ((e = dmalloc(&A->d_cai, cai.size(), &A->device_bytes)) != hipSuccess ||
            (e = dmalloc(&A->d_ridx, ridx.size(), &A->device_bytes)) != hipSuccess)
            return hipfail(e, "alloc compressed rows");
        if ((e = hipMemcpy(A->d_cai, cai.data(), sizeof(int32_t) * cai.size(), hipMemcpyHostToDevice)) != hipSuccess ||
            (!ridx.empty() &&
             (e = hipMemcpy(A->d_ridx, ridx.data(), sizeof(int32_t) * ridx.size(), hipMemcpyHostToDevice)) != hipSuccess))
            return hipfail(e, "upload compressed rows");
        A->h_rai.swap(cai);
    } else {
        A->n_crow = 0;
        if (own_ai && own_ai->data() == ai) A->h_rai.swap(*own_ai);
        else A->h_rai.assign(ai, ai + (size_t)m + 1);
    }
    return plan_build(A);
}

int upload_and_plan(aijhip_mat *A, const int32_t *ai, const int32_t *aj, const double *aa, bool dev_src = false,
                    aijhip::HostVec<int32_t> *own_ai = nullptr) {
    const int32_t m = A->m;
    const int64_t nz = A->nz;
    hipError_t e;
    if ((e = dmalloc(&A->d_ai, (size_t)m + 1, &A->device_bytes)) != hipSuccess ||
        (e = dmalloc(&A->d_aj, (size_t)nz + 2, &A->device_bytes)) != hipSuccess ||
        (e = dmalloc(&A->d_aa, (size_t)nz + 2, &A->device_bytes)) != hipSuccess)
        return hipfail(e, "alloc CSR");
    if ((e = hipMemcpy(A->d_ai, ai, sizeof(int32_t) * ((size_t)m + 1), hipMemcpyHostToDevice)) != hipSuccess ||
        (e = hipMemset(A->d_aj + nz, 0, 2 * sizeof(int32_t))) != hipSuccess ||
        (e = hipMemset(A->d_aa + nz, 0, 2 * sizeof(double))) != hipSuccess)
        return hipfail(e, "upload ai");
    const hipMemcpyKind kind = dev_src ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
    if (nz > 0 &&
        ((e = hipMemcpy(A->d_aj, aj, sizeof(int32_t) * (size_t)nz, kind)) != hipSuccess ||
         (e = hipMemcpy(A->d_aa, aa, sizeof(double) * (size_t)nz, kind)) != hipSuccess))
        return hipfail(e, "upload aj/aa");
    return structure_and_plan(A, ai, own_ai);
}

int check_handle(aijhip_mat_t A) {
    if (!A) return fail(AIJHIP_ERR_ARG, "NULL handle");
    return AIJHIP_OK;
}

int mult_impl(aijhip_mat_t A, const double *x, const double *z, double *y, bool add, void *stream) {
    int rc = check_handle(A);
    if (rc) return rc;
    if (A->m == 0) return AIJHIP_OK;
    if (!y || (A->nz > 0 && !x) || (add && !z)) return fail(AIJHIP_ERR_ARG, "NULL vector");
    if (x == y) return fail(AIJHIP_ERR_ARG, "x and y alias (PETSc requires distinct Vecs)");
    DeviceGuard g(A->device);
    if (g.err != hipSuccess) return hipfail(g.err, "set device");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    hipError_t e;
    e = aijhip::launch_mult(*A, x, z, y, add, s);
    if (e != hipSuccess) return hipfail(e, "SpMV launch");
    return AIJHIP_OK;
}

int create_impl(int device, int32_t m, int32_t n, int64_t nz, const int32_t *ai,
                const int32_t *aj, const double *aa, aijhip_mat_t *out, bool dev_src = false,
                aijhip::HostVec<int32_t> *own_ai = nullptr) {
    if (!out) return fail(AIJHIP_ERR_ARG, "out is NULL");
    *out = nullptr;
    if (nz > 0 && !aj) return fail(AIJHIP_ERR_ARG, "aj is NULL");
    int rc = validate_csr(m, n, nz, ai, dev_src ? nullptr : aj);
    if (rc) return rc;
    if (nz > 0 && !aa) return fail(AIJHIP_ERR_ARG, "aa is NULL");
    const int count = aijhip::visible_devices();
    if (count <= 0) return fail(AIJHIP_ERR_NODEVICE, aijhip::no_device_reason());
    if (device < 0 || device >= count) return fail(AIJHIP_ERR_ARG, "device ordinal out of range");
    DeviceGuard g(device);
    if (g.err != hipSuccess) return hipfail(g.err, "set device");
    aijhip_mat *A = new (std::nothrow) aijhip_mat();
    if (!A) return fail(AIJHIP_ERR_ALLOC, "host allocation");
    A->device = device;
    A->m = m;
    A->n = n;
    A->nz = nz;
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && cus > 0)
        A->n_cu = cus;
    if (dev_src && nz > 0) {
        int64_t bad = 0;
        hipError_t e = aijhip::count_bad_columns(aj, nz, n, &bad);
        if (e != hipSuccess) rc = hipfail(e, "check device columns");
        else if (bad) rc = fail(AIJHIP_ERR_ARG, std::to_string(bad) + " column indices out of range");
    }
    if (!rc) rc = upload_and_plan(A, ai, aj, aa, dev_src, own_ai);
    if (rc) {
        free_matrix(A);
        delete A;
        return rc;
    }
    *out = A;
    return AIJHIP_OK;
}

}  // namespace

namespace aijhip {
void set_error(const std::string &msg) { g_err = msg; }

int hw_queues() {
    static const int q = [] {
        const char *v = std::getenv("GPU_MAX_HW_QUEUES");
        const int n = v ? std::atoi(v) : 0;
        return n > 0 ? n : 4;
    }();
    return q;
}

unsigned sync_event_flags() {
    const char *v = std::getenv("AIJHIP_EVENT_FENCE");
    unsigned f = hipEventDisableTiming;
    if (v && std::strcmp(v, "device") == 0) f |= hipEventReleaseToDevice;
    else if (v && std::strcmp(v, "none") == 0) f |= hipEventDisableSystemFence;
    return f;
}

uint64_t next_plan_gen() {
    static std::atomic<uint64_t> gen{0};
    return ++gen;
}

// hipGetDeviceCount costs milliseconds per call on this stack; the count of a
// process does not change, so it is asked once.
namespace {
hipError_t g_count_err = hipSuccess;  // why hipGetDeviceCount failed, if it did
}

int visible_devices() {
    static const int count = [] {
        int c = 0;
        g_count_err = hipGetDeviceCount(&c);
        return g_count_err == hipSuccess ? c : 0;
    }();
    return count;
}

std::string no_device_reason() {
    return g_count_err == hipSuccess ? std::string("no HIP device visible")
                                     : std::string("no HIP device visible (hipGetDeviceCount: ") +
                                           hipGetErrorString(g_count_err) + ")";
}

int adopt_device_csr(int device, int32_t m, int32_t n, int64_t nz, int32_t *d_ai, int32_t *d_aj, double *d_aa,
                     const aijhip_mat *like, aijhip_mat **out) {
    *out = nullptr;
    aijhip_mat *A = new (std::nothrow) aijhip_mat();
    if (!A) {
        hipFree(d_ai); hipFree(d_aj); hipFree(d_aa);
        return fail(AIJHIP_ERR_ALLOC, "host allocation");
    }
    A->device = device;
    A->m = m;
    A->n = n;
    A->nz = nz;
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && cus > 0)
        A->n_cu = cus;
    if (like) {
        A->requested_tune = like->requested_tune;
        A->requested_kernel =
            like->requested_kernel == AIJHIP_KERNEL_VECTOR ? AIJHIP_KERNEL_AUTO : like->requested_kernel;
    }
    A->d_ai = d_ai;
    A->d_aj = d_aj;
    A->d_aa = d_aa;
    A->device_bytes = 4 * ((int64_t)m + 1) + 12 * (nz + 2);
    A->setup_op = like ? like->setup_op : true;
    if (!like) {  // the set-up's own operators: no codes or patterns (plan time); the gather-ordered
        // copy for long rows, 32-bit columns where the packed form does not fit (GAMG's level 1
        // and Pᵀ) — round 5, 300³ CG + GAMG: solve 0.1652-0.1656 s vs 0.1783-0.1791 unsorted,
        // set-up 0.167 vs 0.156-0.162 s; sorting every operator 0.169-0.170 s (the finest P,
        // short rows, runs slower sorted); profiles/r05/as/, at/. AIJHIP_SETUP_GSORT
        // overrides (0 off, 1 every operator).
        const char *gs = std::getenv("AIJHIP_SETUP_GSORT");
        A->requested_tune.gsort = gs ? std::atoi(gs) : -1;
        const char *vc = std::getenv("AIJHIP_SETUP_VCODES");  // value codes: -1 (default) where they fit, 0 off
        A->requested_tune.vcodes = vc ? std::atoi(vc) : -1;
        A->requested_tune.codes = 0;
        A->requested_tune.patterns = 0;
    }
    aijhip::HostVec<int32_t> h_ai;
    int rc = AIJHIP_OK;
    hipError_t e = hipSuccess;
    try {
        h_ai.resize((size_t)m + 1);
    } catch (const std::bad_alloc &) {
        rc = fail(AIJHIP_ERR_ALLOC, "host row offsets");
    }
    if (!rc && ((e = hipMemsetAsync(d_aj + nz, 0, 2 * sizeof(int32_t), nullptr)) != hipSuccess ||
                (e = hipMemsetAsync(d_aa + nz, 0, 2 * sizeof(double), nullptr)) != hipSuccess ||
                (e = hipMemcpy(h_ai.data(), d_ai, sizeof(int32_t) * h_ai.size(), hipMemcpyDeviceToHost)) != hipSuccess))
        rc = hipfail(e, "read device row offsets");
    if (!rc) rc = structure_and_plan(A, h_ai.data(), &h_ai);
    if (rc) {
        free_matrix(A);
        delete A;
        return rc;
    }
    *out = A;
    return AIJHIP_OK;
}

// A^T as a handle owned by A (MatMultTranspose), adopting the transpose's
// device arrays (n+1 / nz+2 / nz+2).
int attach_transpose(aijhip_mat *A, int32_t *tai, int32_t *taj, double *taa) {
    aijhip_mat *T = nullptr;
    const int rc = adopt_device_csr(A->device, A->n, A->m, A->nz, tai, taj, taa, A, &T);
    if (rc) return rc;
    if (A->transpose) { free_matrix(A->transpose); delete A->transpose; }
    A->transpose = T;
    return AIJHIP_OK;
}
}  // namespace aijhip

namespace aijhip {
// Compulsory bytes of one MatMult under the plan in effect: the arrays the
// launched kernels stream (each read once), x read once, y written once —
// SURVEY §8d's count for the layout actually read. Block descriptors,
// dictionaries and pattern tables are included where the layout needs them.
int64_t mult_layout_bytes(const aijhip_mat &A) {
    const aijhip::Plan &P = A.plan;
    const int64_t m = A.m, n = A.n, nz = A.nz;
    const int64_t rows = A.compressed ? (4 * ((int64_t)A.n_crow + 1) + 4 * (int64_t)A.n_crow) : 4 * (m + 1);
    const int64_t vec = 8 * n + 8 * m;
    if (P.kernel != AIJHIP_KERNEL_STREAM) return 12 * nz + rows + vec;
    if (P.d_pid && P.d_pval)  // row templates: a template id per row, the table (offsets and values)
        return m + 12 * (int64_t)P.n_ptab + vec;
    if (P.d_pid)  // aa, ai, a pattern id per row and the offset table
        return 8 * nz + rows + m + 4 * (int64_t)P.n_ptab + vec;
    if (P.d_code)  // coded entries 10 B, blocks launched from aj 12 B, the dictionaries
        return 10 * (nz - P.nz_wide) + 12 * P.nz_wide + rows + vec + 4 * P.n_cmeta;
    if (P.d_sidx && P.d_svcode)  // packed columns and slots, value codes (6 B per entry), the dictionary
        return 6 * nz + rows + vec + 4 * (int64_t)P.n_blocks + 8 * (int64_t)P.n_vdict;
    if (P.d_vcode && !P.d_sslot)  // aj and value codes (6 B per entry), the dictionary
        return 6 * nz + rows + vec + 8 * (int64_t)P.n_vdict;
    if (P.d_sidx)  // packed columns and slots (4 B per entry), sorted values, block bases
        return 12 * nz + rows + vec + 4 * (int64_t)(P.n_blocks - P.n_wblocks);
    if (P.d_sslot)  // sorted 32-bit columns + sorted values + 16-bit slots
        return 14 * nz + rows + vec;
    return 12 * nz + rows + vec;
}
}  // namespace aijhip

extern "C" {

int aijhip_abi_version(void) { return AIJHIP_ABI_VERSION; }

const char *aijhip_last_error(void) { return g_err.c_str(); }

int aijhip_device_count(int *count) {
    if (!count) return fail(AIJHIP_ERR_ARG, "count is NULL");
    *count = 0;
    hipError_t e = hipGetDeviceCount(count);
    if (e != hipSuccess) {
        *count = 0;
        return hipfail(e, "hipGetDeviceCount");
    }
    return AIJHIP_OK;
}

int aijhip_mat_create(int device, int32_t m, int32_t n, int64_t nz, const int32_t *ai,
                      const int32_t *aj, const double *aa, aijhip_mat_t *out) {
    aijhip::Range range("MatAssemblyEnd_SeqAIJHIP");
    return create_impl(device, m, n, nz, ai, aj, aa, out);
}

int aijhip_mat_create_from_device(int device, int32_t m, int32_t n, int64_t nz,
                                  const int32_t *d_ai, const int32_t *d_aj,
                                  const double *d_aa, aijhip_mat_t *out) {
    aijhip::Range range("MatAssemblyEnd_SeqAIJHIP (device arrays)");
    if (!out) return fail(AIJHIP_ERR_ARG, "out is NULL");
    if (m < 0 || n < 0 || nz < 0 || !d_ai || (nz > 0 && (!d_aj || !d_aa)))
        return fail(AIJHIP_ERR_ARG, "bad size or NULL array");
    // Planning reads the row offsets on the host (m+1 ints); the columns are
    // range-checked on the device and aj/aa are copied device to device.
    aijhip::HostVec<int32_t> ai((size_t)m + 1);
    {
        DeviceGuard g(device);
        if (g.err != hipSuccess) return hipfail(g.err, "set device");
        hipError_t e = hipMemcpy(ai.data(), d_ai, sizeof(int32_t) * ai.size(), hipMemcpyDeviceToHost);
        if (e != hipSuccess) return hipfail(e, "read device row offsets");
    }
    return create_impl(device, m, n, nz, ai.data(), d_aj, d_aa, out, true, &ai);
}

int aijhip_mat_set_kernel(aijhip_mat_t A, int kernel, int lanes) {
    int rc = check_handle(A);
    if (rc) return rc;
    if (kernel == 4)  // reserved: the withdrawn MERGE kernel
        return fail(AIJHIP_ERR_ARG, "the MERGE kernel was withdrawn in ABI 2: STREAM's row blocks are the "
                                    "merge-path decomposition (DESIGN.md §4)");
    if (kernel < AIJHIP_KERNEL_AUTO || kernel > AIJHIP_KERNEL_VECTOR)
        return fail(AIJHIP_ERR_ARG, "unknown kernel " + std::to_string(kernel));
    DeviceGuard g(A->device);
    if (g.err != hipSuccess) return hipfail(g.err, "set device");
    hipError_t e = hipDeviceSynchronize();  // in-flight launches may read the old plan
    if (e != hipSuccess) return hipfail(e, "sync before re-plan");
    A->requested_kernel = kernel;
    A->requested_lanes = lanes;
    return plan_build(A);
}

int aijhip_mat_set_option(aijhip_mat_t A, int option, int value) {
    int rc = check_handle(A);
    if (rc) return rc;
    aijhip::Tuning t = A->requested_tune;
    switch (option) {
        case AIJHIP_OPT_STREAM_GEOMETRY:
            if (value < -1 || value >= aijhip::kNumStreamGeoms) return fail(AIJHIP_ERR_ARG, "bad geometry");
            t.geom = value;
            break;
        case 2: case 4: case 5: case 7: case 11: case 15: case 16:  // reserved (include/aijhip.h)
            return fail(AIJHIP_ERR_ARG, "option " + std::to_string(option) +
                                            " was withdrawn (measured slower; profiles/README.md)");
        case AIJHIP_OPT_NT_LOADS:
            if (value < -1 || value > 1) return fail(AIJHIP_ERR_ARG, "nt_loads: -1 (auto), 0, 1");
            t.nt = value;
            break;
        case AIJHIP_OPT_EXACT: t.exact = value != 0; break;
        case AIJHIP_OPT_LONG_XCD: t.long_xcd = value != 0; break;
        case AIJHIP_OPT_LONG_OVERLAP:
            if (value < -1 || value > 1) return fail(AIJHIP_ERR_ARG, "long_overlap: -1 auto (off; on with exact), 0 off, 1 side stream");
            t.overlap = value;
            break;
        case AIJHIP_OPT_HOST_PIPELINE:
            if (value < -1) return fail(AIJHIP_ERR_ARG, "host_pipeline: -1 auto, 0 serial, k > 0 chunk rows");
            t.host_chunk = value;
            break;
        case AIJHIP_OPT_GATHER_SORT:
            if (value < -1 || value > 1) return fail(AIJHIP_ERR_ARG, "gather_sort: -1 auto, 0 off, 1 on");
            t.gsort = value;
            break;
        case AIJHIP_OPT_COLUMN_CODES:
            if (value < -1 || value > 1) return fail(AIJHIP_ERR_ARG, "column_codes: -1 auto, 0 off, 1 on");
            t.codes = value;
            break;
        case AIJHIP_OPT_ROW_PATTERNS:
            if (value < -1 || value > 1) return fail(AIJHIP_ERR_ARG, "row_patterns: -1 auto, 0 off, 1 on");
            t.patterns = value;
            break;
        case AIJHIP_OPT_ROW_TEMPLATES:
            if (value < -1 || value > 1) return fail(AIJHIP_ERR_ARG, "row_templates: -1 auto, 0 off, 1 on");
            t.templates = value;
            break;
        case AIJHIP_OPT_VALUE_CODES:
            if (value < -1 || value > 1) return fail(AIJHIP_ERR_ARG, "value_codes: -1 auto, 0 off, 1 on");
            t.vcodes = value;
            break;
        default: return fail(AIJHIP_ERR_ARG, "unknown option " + std::to_string(option));
    }
    DeviceGuard g(A->device);
    if (g.err != hipSuccess) return hipfail(g.err, "set device");
    hipError_t e = hipDeviceSynchronize();  // in-flight launches may read the old plan
    if (e != hipSuccess) return hipfail(e, "sync before re-plan");
    A->requested_tune = t;
    return plan_build(A);
}

int aijhip_mat_update_values(aijhip_mat_t A, const double *aa) {
    int rc = check_handle(A);
    if (rc) return rc;
    if (A->nz > 0 && !aa) return fail(AIJHIP_ERR_ARG, "aa is NULL");
    DeviceGuard g(A->device);
    if (g.err != hipSuccess) return hipfail(g.err, "set device");
    hipError_t e = hipDeviceSynchronize();
    if (e == hipSuccess && A->nz > 0)
        e = hipMemcpy(A->d_aa, aa, sizeof(double) * (size_t)A->nz, hipMemcpyHostToDevice);
    if (e == hipSuccess && A->plan.d_sslot)  // the gather-ordered copy of the values
        e = aijhip::build_gather_order(*A, A->plan, true);
    if (e != hipSuccess) return hipfail(e, "update values");
    // templates / value codes hold the old values, and explicitly requested
    // ones may fit the new values: plan again
    if (A->plan.d_pval || A->plan.d_vcode || A->plan.d_svcode || A->requested_tune.vcodes > 0 ||
        A->requested_tune.templates > 0) {
        rc = plan_build(A);
        if (rc) return rc;
    }
    A->values_gen = aijhip::next_plan_gen();  // a set-up KSP redoes its PC set-up
    if (A->transpose) {  // A^T values are stale
        free_matrix(A->transpose);
        delete A->transpose;
        A->transpose = nullptr;
    }
    return AIJHIP_OK;
}

int aijhip_mat_assembly_end(aijhip_mat_t A, int64_t nz, const int32_t *ai, const int32_t *aj,
                            const double *aa) {
    aijhip::Range range("MatAssemblyEnd_SeqAIJHIP");
    int rc = check_handle(A);
    if (rc) return rc;
    aijhip_mat_t B = nullptr;
    rc = create_impl(A->device, A->m, A->n, nz, ai, aj, aa, &B);
    if (rc) return rc;
    B->requested_tune = A->requested_tune;
    rc = aijhip_mat_set_kernel(B, A->requested_kernel, A->requested_lanes);
    if (rc) {
        aijhip_mat_destroy(B);
        return rc;
    }
    {
        DeviceGuard g(A->device);
        (void)hipDeviceSynchronize();
        free_matrix(A);
        if (A->d_xstage) hipFree(A->d_xstage);
        if (A->d_ystage) hipFree(A->d_ystage);
        if (A->host_stream) hipStreamDestroy(A->host_stream);
    }
    *A = std::move(*B);
    B->transpose = nullptr;
    B->d_xstage = B->d_ystage = nullptr;
    B->host_stream = nullptr;
    B->plan = aijhip::Plan();
    delete B;
    return AIJHIP_OK;
}

int aijhip_mat_mult(aijhip_mat_t A, const double *x, double *y, void *stream) {
    return mult_impl(A, x, nullptr, y, false, stream);
}

int aijhip_mat_mult_add(aijhip_mat_t A, const double *x, const double *z, double *w,
                        void *stream) {
    if (A && x && x == w) return fail(AIJHIP_ERR_ARG, "x and w alias");
    return mult_impl(A, x, z, w, true, stream);
}

namespace {

// A^T, built on first use (kept until the structure changes).
int ensure_transpose(aijhip_mat *A) {
    if (!A->transpose) {
        DeviceGuard g(A->device);
        if (g.err != hipSuccess) return hipfail(g.err, "set device");
        int32_t *tai = nullptr, *taj = nullptr;
        double *taa = nullptr;
        hipError_t e = hipDeviceSynchronize();
        if (e == hipSuccess) e = aijhip::build_transpose(*A, &tai, &taj, &taa, nullptr);
        if (e != hipSuccess) return hipfail(e, "build transpose");
        return aijhip::attach_transpose(A, tai, taj, taa);
    }
    return AIJHIP_OK;
}

// The handle's host-vector staging buffers and stream (first use).
int ensure_host_staging(aijhip_mat *A) {
    hipError_t e = hipSuccess;
    if (!A->host_stream) e = hipStreamCreateWithFlags(&A->host_stream, hipStreamNonBlocking);
    if (e == hipSuccess && !A->d_xstage) e = dmalloc(&A->d_xstage, (size_t)A->n, &A->device_bytes);
    if (e == hipSuccess && !A->d_ystage) e = dmalloc(&A->d_ystage, (size_t)A->m, &A->device_bytes);
    return e == hipSuccess ? AIJHIP_OK : hipfail(e, "host staging");
}

}  // namespace

int aijhip_mat_mult_transpose(aijhip_mat_t A, const double *x, double *y, void *stream) {
    int rc = check_handle(A);
    if (rc) return rc;
    if (A->n == 0) return AIJHIP_OK;
    if ((rc = ensure_transpose(A))) return rc;
    return mult_impl(A->transpose, x, nullptr, y, false, stream);
}

int aijhip_mat_mult_host(aijhip_mat_t A, const double *x, double *y) {
    int rc = check_handle(A);
    if (rc) return rc;
    if (A->m == 0) return AIJHIP_OK;
    if (!y || (A->n > 0 && !x)) return fail(AIJHIP_ERR_ARG, "NULL vector");
    DeviceGuard g(A->device);
    if (g.err != hipSuccess) return hipfail(g.err, "set device");
    if ((rc = ensure_host_staging(A))) return rc;
    // step2 MatMult patch:24 (x H2D), :27-40 (kernel), :29 (y D2H), pipelined
    // as steps 3/4 overlap them (host_pipe.cpp)
    return aijhip::host_pipe_mult(A, x, y);
}

int aijhip_mat_mult_add_host(aijhip_mat_t A, const double *x, const double *z, double *w) {
    int rc = check_handle(A);
    if (rc) return rc;
    if (A->m == 0) return AIJHIP_OK;
    if (!z || !w || (A->n > 0 && !x)) return fail(AIJHIP_ERR_ARG, "NULL vector");
    if (x == w) return fail(AIJHIP_ERR_ARG, "x and w alias");
    DeviceGuard g(A->device);
    if (g.err != hipSuccess) return hipfail(g.err, "set device");
    if ((rc = ensure_host_staging(A))) return rc;
    // z goes up before w comes down, so z == w (PETSc's yy == zz) is fine;
    // the row sums start from z[i] in the kernel (MatMultAdd_SeqAIJ's order)
    hipStream_t s = A->host_stream;
    hipError_t e = hipSuccess;
    if (A->n > 0) e = hipMemcpyAsync(A->d_xstage, x, sizeof(double) * (size_t)A->n, hipMemcpyHostToDevice, s);
    if (e == hipSuccess)
        e = hipMemcpyAsync(A->d_ystage, z, sizeof(double) * (size_t)A->m, hipMemcpyHostToDevice, s);
    if (e != hipSuccess) return hipfail(e, "copy x, z in");
    if ((e = aijhip::launch_mult(*A, A->d_xstage, A->d_ystage, A->d_ystage, true, s)) != hipSuccess)
        return hipfail(e, "MatMultAdd launch");
    if ((e = hipMemcpyAsync(w, A->d_ystage, sizeof(double) * (size_t)A->m, hipMemcpyDeviceToHost, s)) !=
            hipSuccess ||
        (e = hipStreamSynchronize(s)) != hipSuccess)
        return hipfail(e, "copy w out");
    return AIJHIP_OK;
}

int aijhip_mat_mult_transpose_host(aijhip_mat_t A, const double *x, double *y) {
    int rc = check_handle(A);
    if (rc) return rc;
    if (A->n == 0) return AIJHIP_OK;
    if (!y || (A->m > 0 && !x)) return fail(AIJHIP_ERR_ARG, "NULL vector");
    {
        DeviceGuard g(A->device);
        if (g.err != hipSuccess) return hipfail(g.err, "set device");
        if ((rc = ensure_transpose(A))) return rc;
    }
    // A^T is a handle of its own: its MatMult with host vectors is the
    // pipelined one above
    return aijhip_mat_mult_host(A->transpose, x, y);
}

int aijhip_mat_get_info(aijhip_mat_t A, aijhip_info_t *info) {
    int rc = check_handle(A);
    if (rc) return rc;
    if (!info) return fail(AIJHIP_ERR_ARG, "info is NULL");
    std::memset(info, 0, sizeof(*info));
    info->m = A->m;
    info->n = A->n;
    info->nz = A->nz;
    info->nonzerorowcnt = A->nonzerorowcnt;
    info->max_row_nz = A->max_row_nz;
    info->compressed_row = A->compressed ? 1 : 0;
    info->kernel = A->plan.kernel;
    info->vector_lanes = A->plan.lanes;
    info->n_blocks = A->plan.n_blocks;
    info->n_long_rows = A->plan.n_longs;
    info->device = A->device;
    info->device_bytes = A->device_bytes + A->plan.bytes;
    info->mult_flops = 2.0 * (double)A->nz - (double)A->nonzerorowcnt;
    info->mult_bytes = 12 * A->nz + 4 * ((int64_t)A->m + 1) + 8 * (int64_t)A->n + 8 * (int64_t)A->m;
    info->stream_geometry = A->plan.tune.geom;
    info->nt_loads = A->plan.tune.nt;
    info->stream_threads = aijhip::kStreamGeoms[A->plan.tune.geom].threads;
    info->stream_nnz_cap = aijhip::kStreamGeoms[A->plan.tune.geom].nnz_cap;
    info->stream_rows = aijhip::kStreamGeoms[A->plan.tune.geom].rows;
    info->exact = A->plan.tune.exact ? 1 : 0;
    info->gather_sorted = A->plan.d_sidx != nullptr ? 2 : (A->plan.d_sslot != nullptr ? 1 : 0);
    info->column_codes = A->plan.d_code != nullptr ? 1 : 0;
    info->row_patterns = A->plan.d_pid != nullptr ? A->plan.n_pat : 0;
    info->long_overlap = A->plan.side != nullptr ? 1 : 0;
    info->mult_layout_bytes = aijhip::mult_layout_bytes(*A);
    info->hw_queues = aijhip::hw_queues();
    info->row_templates = A->plan.d_pval != nullptr ? 1 : 0;
    info->value_codes = (A->plan.d_vcode || A->plan.d_svcode) ? A->plan.n_vdict : 0;
    info->reserved1 = 0;
    return AIJHIP_OK;
}

int aijhip_mat_get_device_csr(aijhip_mat_t A, const int32_t **ai, const int32_t **aj,
                              const double **aa) {
    int rc = check_handle(A);
    if (rc) return rc;
    if (ai) *ai = A->d_ai;
    if (aj) *aj = A->d_aj;
    if (aa) *aa = A->d_aa;
    return AIJHIP_OK;
}

int aijhip_mat_destroy(aijhip_mat_t A) {
    if (!A) return AIJHIP_OK;
    {
        DeviceGuard g(A->device);
        (void)hipDeviceSynchronize();
        free_matrix(A);
        hipFree(A->d_xstage);
        hipFree(A->d_ystage);
        if (A->host_stream) hipStreamDestroy(A->host_stream);
    }
    delete A;
    return AIJHIP_OK;
}

}  // extern "C"
