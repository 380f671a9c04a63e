// dscan.h — the few device-wide primitives the GAMG set-up needs (exclusive
// scan of counts, min / max of an int array), written out instead of taken
// from hipCUB: integer arithmetic, so any order gives the same result, and a
// set-up translation unit without rocPRIM's dispatch templates is a code
// object of a few hundred kB instead of 7 MB, which the runtime loads at the
// set-up's first kernel launch (32 ms measured on the MI355X at 300^3).
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

namespace aijhip_dscan {

constexpr int kScanThreads = 256;
constexpr int kScanItems = 8;  // elements per lane: 2048 per workgroup
constexpr int64_t kScanTile = (int64_t)kScanThreads * kScanItems;

// Exclusive scan of one tile per workgroup; the tile's total to sums[b].
template <class In, class Out>
__global__ __launch_bounds__(kScanThreads) void k_scan_tiles(int64_t n, const In *__restrict__ in, Out *out,
                                                             Out *sums) {
    __shared__ Out part[kScanThreads];
    const int64_t base = (int64_t)blockIdx.x * kScanTile + (int64_t)threadIdx.x * kScanItems;
    Out v[kScanItems];
    Out s = 0;
#pragma unroll
    for (int u = 0; u < kScanItems; ++u) {
        v[u] = base + u < n ? (Out)in[base + u] : (Out)0;
        s += v[u];
    }
    part[threadIdx.x] = s;
    __syncthreads();
    // Hillis-Steele over the 256 lane sums (inclusive), then shift
    for (int off = 1; off < kScanThreads; off <<= 1) {
        const Out add = threadIdx.x >= (unsigned)off ? part[threadIdx.x - off] : (Out)0;
        __syncthreads();
        part[threadIdx.x] += add;
        __syncthreads();
    }
    Out run = threadIdx.x ? part[threadIdx.x - 1] : (Out)0;
#pragma unroll
    for (int u = 0; u < kScanItems; ++u) {
        if (base + u < n) out[base + u] = run;
        run += v[u];
    }
    if (threadIdx.x == kScanThreads - 1 && sums) sums[blockIdx.x] = part[kScanThreads - 1];
}

template <class Out>
__global__ __launch_bounds__(kScanThreads) void k_scan_add(int64_t n, const Out *__restrict__ offs, Out *out) {
    const int64_t i = (int64_t)blockIdx.x * kScanThreads + threadIdx.x;
    if (i < n) out[i] += offs[i / kScanTile];
}

// out[i] = in[0] + ... + in[i-1] for i in [0, n) (out may alias in only
// when In == Out); tmp: scan_tmp_elems(n) elements of Out.
inline int64_t scan_tmp_elems(int64_t n) {
    int64_t t = 0;
    for (int64_t nb = (n + kScanTile - 1) / kScanTile; nb > 1; nb = (nb + kScanTile - 1) / kScanTile) t += 2 * nb;
    return std::max<int64_t>(t, 1);
}

template <class In, class Out>
hipError_t exclusive_scan(const In *in, Out *out, int64_t n, Out *tmp, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const int64_t nb = (n + kScanTile - 1) / kScanTile;
    if (nb == 1) {
        hipLaunchKernelGGL((k_scan_tiles<In, Out>), dim3(1), dim3(kScanThreads), 0, s, n, in, out, (Out *)nullptr);
        return hipGetLastError();
    }
    Out *sums = tmp, *offs = tmp + nb;
    hipLaunchKernelGGL((k_scan_tiles<In, Out>), dim3((unsigned)nb), dim3(kScanThreads), 0, s, n, in, out, sums);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if ((e = exclusive_scan<Out, Out>(sums, offs, nb, tmp + 2 * nb, s)) != hipSuccess) return e;
    hipLaunchKernelGGL((k_scan_add<Out>), dim3((unsigned)((n + kScanThreads - 1) / kScanThreads)),
                       dim3(kScanThreads), 0, s, n, offs, out);
    return hipGetLastError();
}

template <class T, bool MAX>
__global__ __launch_bounds__(256) void k_extreme(int64_t n, const T *__restrict__ in, T *res) {
    __shared__ T part[256];
    T v = MAX ? in[0] : in[0];
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
        v = MAX ? (in[i] > v ? in[i] : v) : (in[i] < v ? in[i] : v);
    part[threadIdx.x] = v;
    __syncthreads();
    for (int off = 128; off > 0; off >>= 1) {
        if (threadIdx.x < (unsigned)off) {
            const T o = part[threadIdx.x + off];
            part[threadIdx.x] = MAX ? (o > part[threadIdx.x] ? o : part[threadIdx.x])
                                    : (o < part[threadIdx.x] ? o : part[threadIdx.x]);
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        if (MAX) atomicMax(res, part[0]);
        else atomicMin(res, part[0]);
    }
}

template <class T, bool MAX>
__global__ void k_extreme_init(const T *__restrict__ in, T *res) {
    if (threadIdx.x == 0) *res = in[0];
}

// *res (device) = min or max of in[0..n), n >= 1 (T: int32_t or unsigned
// long long: the types the device atomics take)
template <class T, bool MAX>
hipError_t extreme(const T *in, int64_t n, T *res, int n_cu, hipStream_t s) {
    if (n <= 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL((k_extreme_init<T, MAX>), dim3(1), dim3(64), 0, s, in, res);
    const int64_t g = std::min<int64_t>((n + 255) / 256, (int64_t)std::max(n_cu, 1) * 8);
    hipLaunchKernelGGL((k_extreme<T, MAX>), dim3((unsigned)g), dim3(256), 0, s, n, in, res);
    return hipGetLastError();
}

}  // namespace aijhip_dscan
