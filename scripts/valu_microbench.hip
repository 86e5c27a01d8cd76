// scripts/valu_microbench.hip -- measures VALU throughput of the instruction kinds the path tracer
// uses on gfx950 (dev tool; informs DESIGN.md).  Each kernel runs 8 independent chains per lane,
// full occupancy, and reports wave-instructions per SIMD per cycle-equivalent as ops/s.
#include <hip/hip_runtime.h>
#include <cstdio>

#define ITERS 4096
#define CHAINS 8

template <int KIND>
__global__ __launch_bounds__(256) void kern(float* out, float a, float b)
{
    float x[CHAINS];
    double dx[CHAINS];
    float2 p[CHAINS];
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) {
        x[c] = a + threadIdx.x * 1e-7f + c;
        dx[c] = x[c];
        p[c] = make_float2(x[c], x[c] + 1.0f);
    }
    for (int i = 0; i < ITERS; ++i) {
#pragma unroll
        for (int c = 0; c < CHAINS; ++c) {
            typedef float f2 __attribute__((ext_vector_type(2)));
            if (KIND == 0) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x[c]) : "v"(a), "v"(b));
            if (KIND == 1) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(x[c]) : "v"(a));
            if (KIND == 2) {
                f2 v = {p[c].x, p[c].y}, va = {a, a}, vb = {b, b};
                asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(v) : "v"(va), "v"(vb));
                p[c] = make_float2(v.x, v.y);
            }
            if (KIND == 3) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(dx[c]) : "v"((double)a), "v"((double)b));
            if (KIND == 4) asm volatile("v_rcp_f32 %0, %0" : "+v"(x[c]));
            if (KIND == 5) x[c] = b / x[c];
            if (KIND == 6) x[c] = __builtin_sqrtf(x[c] + b);
            if (KIND == 7) {
                f2 v = {p[c].x, p[c].y}, va = {a, b};
                asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(v) : "v"(va));
                p[c] = make_float2(v.x, v.y);
            }
            if (KIND == 8) asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[c]) : "v"(a));
            if (KIND == 9) asm volatile("v_sqrt_f32 %0, %0" : "+v"(x[c]));
            if (KIND == 10) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(dx[c]) : "v"((double)a));
            if (KIND == 11) x[c] = __builtin_amdgcn_div_fixupf(__builtin_amdgcn_div_fmasf(x[c], a, b, false), a, b);
            if (KIND == 12) asm volatile("v_sub_f32 %0, %1, %0" : "+v"(x[c]) : "v"(a));
            if (KIND == 13) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x[c]) : "v"(a));
            if (KIND == 14) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x[c]) : "v"(a));
            if (KIND == 15) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x[c]) : "v"(a));
            if (KIND == 16) asm volatile("v_mov_b32 %0, %1" : "=v"(x[c]) : "v"(x[(c + 1) % CHAINS]));
            if (KIND == 17) asm volatile("v_cmp_lt_f32 vcc, %0, %1" :: "v"(x[c]), "v"(a) : "vcc");
            if (KIND == 18) {   // add/mul alternation, the path tracer's dominant mix
                if (c & 1) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(x[c]) : "v"(a));
                else asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[c]) : "v"(a));
            }
            if (KIND == 19) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(x[0]) : "v"(a));   // one dependent chain
        }
    }
    float s = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) s += x[c] + (float)dx[c] + p[c].x + p[c].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// shader clock under a sustained VALU load: d(s_memtime) / d(s_memrealtime) x 100 MHz
__global__ __launch_bounds__(256) void clk(unsigned long long* t, float a)
{
    unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    float x = a + threadIdx.x;
    for (int i = 0; i < 1 << 20; ++i) asm volatile("v_add_f32 %0, %0, %1" : "+v"(x) : "v"(a));
    unsigned long long c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        t[0] = c1 - c0;
        t[1] = r1 - r0;
    }
    if (x == 12345.0f) t[2] = 1;
}

template <int KIND>
double run(float* d, int blocks, const char* name, double ops_per_iter_chain)
{
    hipLaunchKernelGGL(kern<KIND>, dim3(blocks), dim3(256), 0, 0, d, 0.999f, 1e-3f);
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(kern<KIND>, dim3(blocks), dim3(256), 0, 0, d, 0.999f, 1e-3f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    double waves = blocks * 4.0;
    double winstr = waves * ITERS * CHAINS * ops_per_iter_chain;
    double per_simd_per_ns = winstr / 1024.0 / (ms * 1e6);
    printf("%-12s %8.3f ms  %.3e wave-instr/s  %.3f wave-instr per SIMD per ns (x2.4GHz: %.2f cyc/instr)\n", name, ms,
           winstr / (ms * 1e-3), per_simd_per_ns, 2.4 / per_simd_per_ns);
    return ms;
}

int main()
{
    float* d;
    const int blocks = 256 * 8 * 4;
    hipMalloc(&d, blocks * 256 * sizeof(float));
    {
        unsigned long long* t;
        hipMalloc(&t, 64);
        hipLaunchKernelGGL(clk, dim3(256 * 8), dim3(256), 0, 0, t, 1e-3f);
        unsigned long long h[2];
        hipMemcpy(h, t, 16, hipMemcpyDeviceToHost);
        printf("shader clock under VALU load: %.0f MHz (memtime %llu, realtime %llu)\n",
               (double)h[0] / (double)h[1] * 100.0, h[0], h[1]);
        hipFree(t);
    }
    run<0>(d, blocks, "v_fma_f32", 1);
    run<1>(d, blocks, "v_mul_f32", 1);
    run<2>(d, blocks, "v_pk_fma_f32", 1);
    run<7>(d, blocks, "v_pk_mul_f32", 1);
    run<8>(d, blocks, "v_add_f32", 1);
    run<9>(d, blocks, "v_sqrt_f32", 1);
    run<10>(d, blocks, "v_mul_f64", 1);
    run<3>(d, blocks, "v_fma_f64", 1);
    run<4>(d, blocks, "v_rcp_f32", 1);
    run<5>(d, blocks, "f32 div(seq)", 1);
    run<6>(d, blocks, "f32 sqrt(seq)", 1);
    run<12>(d, blocks, "v_sub_f32", 1);
    run<13>(d, blocks, "v_cndmask", 1);
    run<14>(d, blocks, "v_xor_b32", 1);
    run<15>(d, blocks, "v_mul_lo_u32", 1);
    run<16>(d, blocks, "v_mov_b32", 1);
    run<17>(d, blocks, "v_cmp_f32", 1);
    run<18>(d, blocks, "add/mul mix", 1);
    run<19>(d, blocks, "dep mul chain", 1);
    run<18>(d, 256 * 4, "mix 4w/SIMD", 1);
    run<18>(d, 256 * 5, "mix 5w/SIMD", 1);
    run<18>(d, 256 * 2, "mix 2w/SIMD", 1);
    run<18>(d, 256, "mix 1w/SIMD", 1);
    hipFree(d);
    return 0;
}
