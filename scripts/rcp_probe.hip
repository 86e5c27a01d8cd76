// scripts/rcp_probe.hip -- where pt_exactmath.h's rcp_rn (v_rcp_f32 + one FMA Newton step) equals
// IEEE 1.0f / x, over every f32 bit pattern (dev tool).  Mismatches are counted per class:
// denormal x, normal |x| < 2^-125, 2^-125 <= |x| <= 2^125 (the verified range), |x| > 2^125.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "../cpuperformanceraytracer_amd/csrc/pt_exactmath.h"

__global__ void k(unsigned long long* out)
{
    unsigned long long bad[4] = {0, 0, 0, 0}, n[4] = {0, 0, 0, 0};
    for (uint64_t u = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; u < (1ull << 32); u += (uint64_t)gridDim.x * blockDim.x) {
        const float x = __builtin_bit_cast(float, (uint32_t)u);
        const float ax = __builtin_fabsf(x);
        if (!(ax > 0.0f && ax <= 3.4028235e38f)) continue;   // zero, inf, nan
        const int c = ax < 0x1p-126f ? 0 : (ax < 0x1p-125f ? 1 : (ax <= 0x1p125f ? 2 : 3));
        ++n[c];
        const float want = 1.0f / x, got = pt::rcp_rn(x);
        if (__builtin_bit_cast(uint32_t, want) != __builtin_bit_cast(uint32_t, got)) ++bad[c];
    }
    for (int c = 0; c < 4; ++c) {
        atomicAdd(&out[c], n[c]);
        atomicAdd(&out[4 + c], bad[c]);
    }
}

int main()
{
    unsigned long long* d;
    (void)hipMalloc(&d, 8 * sizeof(unsigned long long));
    (void)hipMemset(d, 0, 8 * sizeof(unsigned long long));
    hipLaunchKernelGGL(k, dim3(8192), dim3(256), 0, 0, d);
    unsigned long long h[8];
    (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    const char* nm[4] = {"denormal", "normal < 2^-125", "[2^-125, 2^125]", "> 2^125"};
    for (int c = 0; c < 4; ++c) printf("%-18s checked=%llu mismatches=%llu\n", nm[c], h[c], h[4 + c]);
    return 0;
}
