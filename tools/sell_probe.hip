// sell_probe.hip — measurement tool (not product code): a sliced-ELLPACK
// (SELL-64, natural row order) copy of the 300^3 Poisson operand against the
// library's STREAM MatMult, same x, bit-compared.
//
// Layout: slice s = rows [64 s, 64 s + 64); its entries column-major (entry k
// of lane l at off[s] + 64 k + l), width = the slice's longest row. A
// wavefront owns a slice: for each k the 64 lanes load 64 consecutive values
// and columns (coalesced), and the gathers of one k touch the k-th neighbours
// of 64 consecutive rows (x[i - N^2], ..., x[i + N^2]: runs of consecutive
// addresses). Each row is still summed sequentially from 0.0 in storage
// order (PETSc's order), so the result must be bit-identical.
//
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -Iinclude -o tools/sell_probe tools/sell_probe.hip \
//         -Lpetsc-openacc_amd/lib -laijhip -Wl,-rpath,$PWD/petsc-openacc_amd/lib
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "aijhip.h"
#include "aijhip_harness.h"

#define CHECK(x)                                                                   \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));           \
            std::exit(1);                                                          \
        }                                                                          \
    } while (0)

__global__ void k_width(int m, const int32_t *ai, int32_t *wid) {
    const int s = blockIdx.x * 4 + (threadIdx.x >> 6), l = threadIdx.x & 63;
    const int r = s * 64 + l;
    int len = r < m ? ai[r + 1] - ai[r] : 0;
    for (int o = 32; o > 0; o >>= 1) len = max(len, __shfl_xor(len, o, 64));
    if (l == 0 && s * 64 < m) wid[s] = len * 64;
}

__global__ void k_fill(int m, const int32_t *ai, const int32_t *aj, const double *aa, const int64_t *off,
                       int32_t *sj, double *sa) {
    const int r = blockIdx.x * 256 + threadIdx.x;
    if (r >= m) return;
    const int s = r >> 6, l = r & 63;
    const int64_t o = off[s], w = (off[s + 1] - o) / 64;
    const int32_t k0 = ai[r], len = ai[r + 1] - k0;
    for (int k = 0; k < w; ++k) {
        sj[o + 64 * k + l] = k < len ? aj[k0 + k] : r;
        sa[o + 64 * k + l] = k < len ? aa[k0 + k] : 0.0;
    }
}

// one slice per wavefront, W = compile-time bound on the width
template <int W, bool NT, int SPW>
__global__ __launch_bounds__(256) void k_sell(int m, int nslices, const int32_t *__restrict__ ai,
                                              const int64_t *__restrict__ off, const int32_t *__restrict__ sj,
                                              const double *__restrict__ sa, const double *__restrict__ x,
                                              double *y) {
    const int l = threadIdx.x & 63;
    for (int q = 0; q < SPW; ++q) {
        const int s = (blockIdx.x * 4 + (threadIdx.x >> 6)) * SPW + q;
        if (s >= nslices) return;
        const int r = s * 64 + l;
        const bool on = r < m;
        const int len = on ? ai[r + 1] - ai[r] : 0;
        const int64_t o = off[s];
        const int w = (int)((off[s + 1] - o) >> 6);
        int32_t j[W];
        double a[W], xv[W];
#pragma unroll
        for (int k = 0; k < W; ++k)
            if (k < w && k < len) {
                if constexpr (NT) {
                    j[k] = __builtin_nontemporal_load(sj + o + 64 * k + l);
                    a[k] = __builtin_nontemporal_load(sa + o + 64 * k + l);
                } else {
                    j[k] = sj[o + 64 * k + l];
                    a[k] = sa[o + 64 * k + l];
                }
            }
#pragma unroll
        for (int k = 0; k < W; ++k)
            if (k < w && k < len) xv[k] = x[j[k]];
        double sum = 0.0;
#pragma unroll
        for (int k = 0; k < W; ++k)
            if (k < w && k < len) sum += a[k] * xv[k];
        if (on) __builtin_nontemporal_store(sum, y + r);
    }
}

template <class F>
float time_us(F launch, int reps) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    for (int i = 0; i < 3; ++i) launch();
    std::vector<float> t;
    for (int r = 0; r < reps; ++r) {
        CHECK(hipEventRecord(a));
        launch();
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, a, b));
        t.push_back(ms * 1e3f);
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

int main(int argc, char **argv) {
    const int N = argc > 1 ? std::atoi(argv[1]) : 300;
    aijhip_mat_t A = nullptr;
    double scale = 0;
    if (aijhip_mat_create_poisson(0, N, N, N, 0, N, 1, &scale, &A)) {
        std::fprintf(stderr, "create: %s\n", aijhip_last_error());
        return 1;
    }
    aijhip_info_t inf;
    aijhip_mat_get_info(A, &inf);
    const int m = inf.m;
    const int64_t nz = inf.nz;
    const int32_t *ai, *aj;
    const double *aa;
    aijhip_mat_get_device_csr(A, &ai, &aj, &aa);
    const int nsl = (m + 63) / 64;
    int32_t *wid;
    int64_t *off;
    CHECK(hipMalloc(&wid, sizeof(int32_t) * (nsl + 1)));
    CHECK(hipMalloc(&off, sizeof(int64_t) * (nsl + 1)));
    CHECK(hipMemset(wid, 0, sizeof(int32_t) * (nsl + 1)));
    hipLaunchKernelGGL(k_width, dim3((nsl + 3) / 4), dim3(256), 0, nullptr, m, ai, wid);
    size_t tb = 0;
    CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, wid, off, nsl + 1));
    void *tmp;
    CHECK(hipMalloc(&tmp, tb));
    CHECK(hipcub::DeviceScan::ExclusiveSum(tmp, tb, wid, off, nsl + 1));
    int64_t total = 0;
    CHECK(hipMemcpy(&total, off + nsl, sizeof(int64_t), hipMemcpyDeviceToHost));
    int32_t *sj;
    double *sa;
    CHECK(hipMalloc(&sj, sizeof(int32_t) * total));
    CHECK(hipMalloc(&sa, sizeof(double) * total));
    hipLaunchKernelGGL(k_fill, dim3((m + 255) / 256), dim3(256), 0, nullptr, m, ai, aj, aa, off, sj, sa);
    CHECK(hipDeviceSynchronize());
    double *x, *y0, *y1;
    CHECK(hipMalloc(&x, sizeof(double) * m));
    CHECK(hipMalloc(&y0, sizeof(double) * m));
    CHECK(hipMalloc(&y1, sizeof(double) * m));
    std::vector<double> hx(m);
    aijhip_splitmix_uniform(m, 42, 0, hx.data());
    CHECK(hipMemcpy(x, hx.data(), sizeof(double) * m, hipMemcpyHostToDevice));
    const double bytes = 12.0 * nz + 4.0 * (m + 1) + 16.0 * m;
    std::printf("{\"m\": %d, \"nz\": %lld, \"sell_entries\": %lld, \"pad\": %.4f}\n", m, (long long)nz,
                (long long)total, (double)total / nz);
    const float ts = time_us([&] { aijhip_mat_mult(A, x, y0, nullptr); }, 30);
    std::printf("{\"kernel\": \"STREAM (library)\", \"us\": %.2f, \"TBs\": %.3f}\n", ts, bytes / ts / 1e6);
    std::vector<double> h0(m), h1(m);
    CHECK(hipMemcpy(h0.data(), y0, sizeof(double) * m, hipMemcpyDeviceToHost));
    auto run = [&](const char *name, auto launch) {
        CHECK(hipMemset(y1, 0xff, sizeof(double) * m));
        const float t = time_us(launch, 30);
        CHECK(hipMemcpy(h1.data(), y1, sizeof(double) * m, hipMemcpyDeviceToHost));
        const bool same = std::memcmp(h0.data(), h1.data(), sizeof(double) * m) == 0;
        std::printf("{\"kernel\": \"%s\", \"us\": %.2f, \"TBs\": %.3f, \"bitwise\": %s}\n", name, t, bytes / t / 1e6,
                    same ? "true" : "false");
        std::fflush(stdout);
    };
#define SELL(W, NT, SPW)                                                                                         \
    run("SELL-64 W=" #W " nt=" #NT " slices/wave=" #SPW, [&] {                                                    \
        hipLaunchKernelGGL((k_sell<W, NT, SPW>), dim3((nsl + 4 * SPW - 1) / (4 * SPW)), dim3(256), 0, nullptr, m, \
                           nsl, ai, off, sj, sa, x, y1);                                                         \
    })
    SELL(8, false, 1); SELL(8, true, 1); SELL(8, false, 2); SELL(8, true, 2); SELL(8, false, 4); SELL(8, true, 4);
    SELL(7, false, 1); SELL(7, true, 1);
    aijhip_mat_destroy(A);
    return 0;
}
