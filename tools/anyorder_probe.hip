// Does hipExtAnyOrderLaunch let a kernel start before the previous kernel
// on the same stream has finished, on this device (gfx950)? hip_ext.h notes
// the flag is "not supported on AMD GFX9xx boards"; this measures it.
//   k_hold: one wave that runs `us` microseconds, stamping its end time;
//   k_mark: one wave that stamps its start time.
// Launched back to back on one stream: mark after hold's end = in order;
// mark before hold's end = the second kernel ran beside the first.
// Also times an empty cross-stream fork / join against none (device clock).
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cstdio>
#include <cstdlib>

__global__ void k_hold(unsigned long long ticks, unsigned long long *stamp) {
    const unsigned long long t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
    if (threadIdx.x == 0) stamp[0] = wall_clock64();
}

__global__ void k_mark(unsigned long long *stamp) {
    if (threadIdx.x == 0) stamp[1] = wall_clock64();
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("{\"error\": \"%s: %s\"}\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main() {
    int khz = 0;
    CK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0));
    unsigned long long *d = nullptr, h[2];
    CK(hipMalloc(&d, 2 * sizeof(unsigned long long)));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    const unsigned long long ticks = 100ull * khz / 1000;  // 100 us
    int ahead[2] = {0, 0};
    double lead_us[2] = {0, 0};
    for (int flag = 0; flag < 2; ++flag) {
        for (int rep = 0; rep < 5; ++rep) {
            CK(hipMemset(d, 0, 2 * sizeof(unsigned long long)));
            hipLaunchKernelGGL(k_hold, dim3(1), dim3(64), 0, s, ticks, d);
            hipExtLaunchKernelGGL(k_mark, dim3(1), dim3(64), 0, s, nullptr, nullptr, flag ? hipExtAnyOrderLaunch : 0, d);
            CK(hipGetLastError());
            CK(hipStreamSynchronize(s));
            CK(hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost));
            const double lead = ((double)h[0] - (double)h[1]) * 1000.0 / khz;  // hold end - mark start, us
            if (lead > 0) ++ahead[flag];
            lead_us[flag] += lead / 5;
        }
    }
    std::printf("{\"wall_clock_khz\": %d, \"in_order\": {\"mark_before_hold_end\": %d, \"mean_lead_us\": %.2f}, "
                "\"any_order\": {\"mark_before_hold_end\": %d, \"mean_lead_us\": %.2f}}\n",
                khz, ahead[0], lead_us[0], ahead[1], lead_us[1]);
    CK(hipFree(d));
    CK(hipStreamDestroy(s));
    return 0;
}
