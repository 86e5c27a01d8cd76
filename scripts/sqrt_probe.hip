// scripts/sqrt_probe.hip -- exhaustive GPU comparison of correctly rounded f32 square-root
// sequences against the compiler's IEEE sqrtf, every f32 x in [2^-100, FLT_MAX] (dev tool).
//   A  Markstein: y = v_rsq(x); s = x y; h = y / 2; r = fma(-s, s, x); fma(r, h, s)
//   B  as A with h = 0.5 * y folded as r * y * 0.5 (two roundings)
//   C  v_sqrt alone (how far the hardware root is from RN)
#include <hip/hip_runtime.h>
#include <stdio.h>

struct Res {
    unsigned long long checked, bad[3], lo[3], hi[3];
    unsigned int ex[3][4];
};

__global__ void k(Res* r)
{
    unsigned long long n = 0, bad[3] = {0, 0, 0}, lo[3] = {0, 0, 0}, hi[3] = {0, 0, 0};
    for (uint64_t u = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; u < (1ull << 31);
         u += (uint64_t)gridDim.x * blockDim.x) {
        const float x = __builtin_bit_cast(float, (uint32_t)u);
        if (!(x >= 0x1p-100f && x <= 3.4028235e38f)) continue;
        ++n;
        const float want = __builtin_sqrtf(x);
        float got[3];
        {
            const float y = __builtin_amdgcn_rsqf(x);
            const float s = x * y, h = 0.5f * y;
            const float rr = __builtin_fmaf(-s, s, x);
            got[0] = __builtin_fmaf(rr, h, s);
        }
        {
            const float y = __builtin_amdgcn_rsqf(x);
            const float s = x * y;
            const float rr = __builtin_fmaf(-s, s, x);
            got[1] = __builtin_fmaf(rr * 0.5f, y, s);
        }
        got[2] = __builtin_amdgcn_sqrtf(x);
        for (int v = 0; v < 3; ++v) {
            const int d = (int)(__builtin_bit_cast(uint32_t, got[v]) - __builtin_bit_cast(uint32_t, want));
            if (d) {
                if (bad[v] == 0 && r->bad[v] == 0) r->ex[v][0] = (uint32_t)u;
                ++bad[v];
                if (d < 0) ++lo[v]; else ++hi[v];
            }
        }
    }
    atomicAdd(&r->checked, n);
    for (int v = 0; v < 3; ++v) {
        atomicAdd(&r->bad[v], bad[v]);
        atomicAdd(&r->lo[v], lo[v]);
        atomicAdd(&r->hi[v], hi[v]);
    }
}

int main()
{
    Res* d;
    hipMalloc(&d, sizeof(Res));
    hipMemset(d, 0, sizeof(Res));
    hipLaunchKernelGGL(k, dim3(4096), dim3(256), 0, 0, d);
    Res h;
    hipMemcpy(&h, d, sizeof(Res), hipMemcpyDeviceToHost);
    const char* nm[3] = {"A markstein", "B markstein(r/2)", "C v_sqrt"};
    for (int v = 0; v < 3; ++v)
        printf("%-18s checked=%llu mismatches=%llu (below %llu, above %llu) first=0x%08x\n", nm[v], h.checked, h.bad[v],
               h.lo[v], h.hi[v], h.ex[v][0]);
    return 0;
}
