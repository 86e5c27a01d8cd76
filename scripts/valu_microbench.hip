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
        }
    }
    float s = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) s += x[c] + (float)dx[c] + p[c].x + p[c].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
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
    hipFree(d);
    return 0;
}
