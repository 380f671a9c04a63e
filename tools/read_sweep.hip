// read_sweep.hip — measurement tool (not product code): the HBM read rate
// MI355X delivers for the SpMV's byte count under different access shapes,
// to bound what the STREAM kernel (a 512-lane workgroup streaming a
// contiguous tile with four 16-B loads per lane) can reach.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/read_sweep tools/read_sweep.hip
//   tools/read_sweep [bytes]        one JSON line per shape
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                   \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));           \
            std::exit(1);                                                          \
        }                                                                          \
    } while (0)

template <int T>
__device__ double block_sum(double v) {
    __shared__ double s[T / 64];
    for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
    if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = v;
    __syncthreads();
    double t = 0.0;
    if (threadIdx.x == 0)
        for (int w = 0; w < T / 64; ++w) t += s[w];
    return t;
}

// one tile of T * U 16-B loads per workgroup (the STREAM shape)
template <int T, int U, bool NT>
__global__ __launch_bounds__(T) void k_tile(int64_t n2, const double2 *__restrict__ v, double *out) {
    const int64_t base = (int64_t)blockIdx.x * T * U + threadIdx.x;
    double2 r[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int64_t i = base + (int64_t)u * T;
        if (i < n2) {
            if constexpr (NT) {
                r[u].x = __builtin_nontemporal_load(&v[i].x);
                r[u].y = __builtin_nontemporal_load(&v[i].y);
            } else {
                r[u] = v[i];
            }
        } else {
            r[u] = make_double2(0.0, 0.0);
        }
    }
    double s = 0.0;
#pragma unroll
    for (int u = 0; u < U; ++u) s += r[u].x + r[u].y;
    s = block_sum<T>(s);
    if (threadIdx.x == 0) out[blockIdx.x & 4095] = s;
}

// the STREAM shape with the tile moved by LDS-DMA (global_load_lds_dwordx4:
// no VGPR destination), then read back from LDS; AUX 2 = non-temporal
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) const void glob_void;
template <int T, int U, int AUX>
__global__ __launch_bounds__(T) void k_tile_glds(int64_t n2, const double2 *__restrict__ v, double *out) {
    __shared__ double2 buf[T * U];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t base = (int64_t)blockIdx.x * T * U;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int64_t i = base + (int64_t)u * T + w * 64 + lane;
        const double2 *src = v + (i < n2 ? i : n2 - 1);
        __builtin_amdgcn_global_load_lds((glob_void *)src, (lds_void *)&buf[u * T + w * 64], 16, 0, AUX);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    double s = 0.0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const double2 r = buf[u * T + threadIdx.x];
        s += r.x + r.y;
    }
    s = block_sum<T>(s);
    if (threadIdx.x == 0) out[blockIdx.x & 4095] = s;
}

// persistent grid-stride, U loads in flight per lane
template <int T, int U>
__global__ __launch_bounds__(T) void k_stride(int64_t n2, const double2 *__restrict__ v, double *out) {
    const int64_t stride = (int64_t)gridDim.x * T;
    int64_t i = (int64_t)blockIdx.x * T + threadIdx.x;
    double s = 0.0;
    for (; i + (U - 1) * stride < n2; i += U * stride) {
        double2 r[U];
#pragma unroll
        for (int u = 0; u < U; ++u) r[u] = v[i + u * stride];
#pragma unroll
        for (int u = 0; u < U; ++u) s += r[u].x + r[u].y;
    }
    for (; i < n2; i += stride) s += v[i].x + v[i].y;
    s = block_sum<T>(s);
    if (threadIdx.x == 0) out[blockIdx.x & 4095] = s;
}

__global__ void k_fill(int64_t n2, double2 *v) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n2; i += (int64_t)gridDim.x * 256)
        v[i] = make_double2(1.0 + (double)(i % 977) * 1e-3, -2.0 + (double)(i % 1031) * 1e-4);
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
    CHECK(hipEventDestroy(a));
    CHECK(hipEventDestroy(b));
    return t[t.size() / 2];
}

int main(int argc, char **argv) {
    const int64_t bytes = argc > 1 ? std::atoll(argv[1]) : 2801520004LL;
    const int64_t n2 = bytes / 16;
    double2 *v = nullptr;
    double *out = nullptr;
    CHECK(hipMalloc(&v, sizeof(double2) * n2));
    CHECK(hipMalloc(&out, sizeof(double) * 4096));
    // non-zero, index-dependent contents (no all-zero lines)
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, nullptr, n2, v);
    CHECK(hipDeviceSynchronize());
    int cus = 256;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    auto report = [&](const char *name, float us) {
        std::printf("{\"shape\": \"%s\", \"us\": %.2f, \"TBs\": %.3f}\n", name, us, (double)bytes / us / 1e6);
        std::fflush(stdout);
    };
#define TILE(T, U, NT)                                                                                     \
    report("tile T=" #T " U=" #U " nt=" #NT, time_us([&] {                                                 \
               hipLaunchKernelGGL((k_tile<T, U, NT>), dim3((unsigned)((n2 + T * U - 1) / (T * U))), dim3(T), \
                                  0, nullptr, n2, v, out);                                                 \
           }, 20))
    TILE(256, 4, false); TILE(256, 8, false); TILE(256, 16, false); TILE(256, 2, true); TILE(256, 4, true);
    TILE(256, 8, true);
    TILE(512, 1, false); TILE(512, 2, false); TILE(512, 4, false); TILE(512, 8, false); TILE(512, 1, true);
    TILE(512, 2, true); TILE(512, 4, true); TILE(512, 8, true);
    TILE(1024, 1, true); TILE(1024, 2, false); TILE(1024, 4, false); TILE(1024, 8, false); TILE(1024, 2, true);
    TILE(1024, 4, true);
#define GLDS(T, U, AUX)                                                                                     \
    report("glds T=" #T " U=" #U " aux=" #AUX, time_us([&] {                                                \
               hipLaunchKernelGGL((k_tile_glds<T, U, AUX>), dim3((unsigned)((n2 + T * U - 1) / (T * U))), dim3(T), \
                                  0, nullptr, n2, v, out);                                                   \
           }, 20))
    GLDS(512, 2, 0); GLDS(512, 4, 0); GLDS(512, 2, 2); GLDS(512, 4, 2); GLDS(256, 4, 2); GLDS(256, 8, 2);
    GLDS(512, 8, 2); GLDS(1024, 2, 2);
#define STRIDE(T, U, W)                                                                                      \
    report("stride T=" #T " U=" #U " wg/CU=" #W, time_us([&] {                                              \
               hipLaunchKernelGGL((k_stride<T, U>), dim3(cus * W), dim3(T), 0, nullptr, n2, v, out);          \
           }, 20))
    STRIDE(256, 4, 8); STRIDE(256, 8, 8); STRIDE(512, 4, 4); STRIDE(512, 8, 4); STRIDE(1024, 4, 2);
    STRIDE(256, 8, 16); STRIDE(512, 8, 8);
    CHECK(hipFree(v));
    CHECK(hipFree(out));
    return 0;
}
