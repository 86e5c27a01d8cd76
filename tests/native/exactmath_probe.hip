// tests/native/exactmath_probe.hip -- exhaustive / large-sample GPU check of csrc/pt_exactmath.h
// against the compiler's IEEE f32 division and square root (built with the product's parity flags:
// -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -fno-gpu-flush-denormals-to-zero).
//
//   rcp_rn(x)  == 1.0f / x   for EVERY f32 x with 2^-125 <= |x| <= 2^125           (2^32 inputs)
//   rcp_tiny_rn(x) == 1.0f / x for EVERY f32 x with |x| < 2^-125 (zeros, denormals)  (same pass)
//   sqrt_rn(x) == sqrtf(x)   for EVERY f32 x >= 2^-100 (finite)                       (2^31 inputs)
//   div_rn(a, b, rcp_rn(b)) == a / b  on N pseudo-random pairs per operand class (normal results)
//
// Prints one line "name checked=<n> mismatches=<m>" per check; exit status 1 on any mismatch.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include "../../cpuperformanceraytracer_amd/csrc/pt_exactmath.h"

struct Res {
    unsigned long long checked, bad;
    unsigned int ex_in[4], ex_in2[4], ex_got[4], ex_want[4];
};

__device__ void record(Res* r, uint32_t in, uint32_t in2, float got, float want)
{
    unsigned long long k = atomicAdd(&r->bad, 1ull);
    if (k < 4) {
        r->ex_in[k] = in;
        r->ex_in2[k] = in2;
        r->ex_got[k] = __builtin_bit_cast(uint32_t, got);
        r->ex_want[k] = __builtin_bit_cast(uint32_t, want);
    }
}

__global__ void k_rcp(Res* r)
{
    unsigned long long n = 0;
    for (uint64_t u = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; u < (1ull << 32);
         u += (uint64_t)gridDim.x * blockDim.x) {
        const float x = __builtin_bit_cast(float, (uint32_t)u);
        const float ax = __builtin_fabsf(x);
        if (ax < 0x1p-125f) {   // rcp_tiny_rn: zeros, denormals, the lowest normals
            ++n;
            const float want = 1.0f / x;
            const float got = pt::rcp_tiny_rn(x);
            if (__builtin_bit_cast(uint32_t, want) != __builtin_bit_cast(uint32_t, got)) record(r, (uint32_t)u, 1, got, want);
            continue;
        }
        if (!(ax >= 0x1p-125f && ax <= 0x1p125f)) continue;
        ++n;
        const float want = 1.0f / x;
        const float got = pt::rcp_rn(x);
        if (__builtin_bit_cast(uint32_t, want) != __builtin_bit_cast(uint32_t, got)) record(r, (uint32_t)u, 0, got, want);
    }
    atomicAdd(&r->checked, n);
}

__global__ void k_sqrt(Res* r)
{
    unsigned long long n = 0;
    for (uint64_t u = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; u < (1ull << 31);
         u += (uint64_t)gridDim.x * blockDim.x) {
        const float x = __builtin_bit_cast(float, (uint32_t)u);
        if (!(x >= 0x1p-100f && x <= 3.4028235e38f)) continue;
        ++n;
        const float want = __builtin_sqrtf(x);
        const float got = pt::sqrt_rn(x);
        if (__builtin_bit_cast(uint32_t, want) != __builtin_bit_cast(uint32_t, got)) record(r, (uint32_t)u, 0, got, want);
    }
    atomicAdd(&r->checked, n);
}

__device__ __forceinline__ uint32_t mix(uint64_t z)
{
    z += 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return (uint32_t)(z ^ (z >> 31));
}

// random f32 with biased exponent in [e0, e1], random mantissa and sign
__device__ __forceinline__ float rnd(uint32_t h, uint32_t h2, int e0, int e1)
{
    const uint32_t e = (uint32_t)(e0 + (int)(h2 % (uint32_t)(e1 - e0 + 1)));
    return __builtin_bit_cast(float, (h & 0x807fffffu) | (e << 23));
}

__global__ void k_div(Res* r, uint64_t npairs, int cls)
{
    unsigned long long n = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < npairs; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t h0 = mix(i * 4 + 0), h1 = mix(i * 4 + 1), h2 = mix(i * 4 + 2), h3 = mix(i * 4 + 3);
        float a, b;
        if (cls == 0) {          // path-tracer shape: |b| in [2^-4, 1], |a| in [2^-20, 2^7]
            b = rnd(h0, h1, 127 - 4, 127);
            a = rnd(h2, h3, 127 - 20, 127 + 7);
        } else if (cls == 1) {   // wide: exponents over +-60
            b = rnd(h0, h1, 127 - 60, 127 + 60);
            a = rnd(h2, h3, 127 - 60, 127 + 60);
        } else {                 // mantissa edge cases: all-ones / all-zeros significands
            b = __builtin_bit_cast(float, (h0 & 0x80000000u) | ((uint32_t)(127 - 3 + (h1 % 7)) << 23) |
                                              ((h1 & 8) ? 0x7fffffu : (h0 & 0xffu)));
            a = rnd(h2, h3, 127 - 30, 127 + 30);
        }
        const float want = a / b;
        const float aw = __builtin_fabsf(want);
        if (!(aw >= 0x1p-120f && aw <= 0x1p120f)) continue;
        ++n;
        const float got = pt::div_rn(a, b, pt::rcp_rn(b));
        if (__builtin_bit_cast(uint32_t, want) != __builtin_bit_cast(uint32_t, got))
            record(r, __builtin_bit_cast(uint32_t, a), __builtin_bit_cast(uint32_t, b), got, want);
    }
    atomicAdd(&r->checked, n);
}

static int report(const char* name, Res* d)
{
    Res h;
    (void)hipDeviceSynchronize();
    (void)hipMemcpy(&h, d, sizeof(h), hipMemcpyDeviceToHost);
    printf("%s checked=%llu mismatches=%llu\n", name, h.checked, h.bad);
    for (unsigned k = 0; k < 4 && k < h.bad; ++k)
        printf("  in=%08x in2=%08x got=%08x want=%08x\n", h.ex_in[k], h.ex_in2[k], h.ex_got[k], h.ex_want[k]);
    (void)hipMemset(d, 0, sizeof(Res));
    return h.bad != 0;
}

int main(int argc, char** argv)
{
    const uint64_t npairs = argc > 1 ? strtoull(argv[1], nullptr, 10) : (1ull << 32);
    Res* d;
    if (hipMalloc(&d, sizeof(Res)) != hipSuccess) return 2;
    (void)hipMemset(d, 0, sizeof(Res));
    int bad = 0;
    const dim3 g(256 * 64), b(256);
    hipLaunchKernelGGL(k_rcp, g, b, 0, 0, d);
    bad |= report("rcp_rn", d);
    hipLaunchKernelGGL(k_sqrt, g, b, 0, 0, d);
    bad |= report("sqrt_rn", d);
    for (int cls = 0; cls < 3; ++cls) {
        hipLaunchKernelGGL(k_div, g, b, 0, 0, d, npairs, cls);
        char name[32];
        snprintf(name, sizeof(name), "div_rn.class%d", cls);
        bad |= report(name, d);
    }
    (void)hipFree(d);
    return bad;
}
