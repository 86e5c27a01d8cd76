// scripts/select_microbench.hip -- throughput of the select idioms on gfx950 (dev tool).
// valu_microbench.hip measured v_cndmask_b32 (VCC) at ~0.12 wave-instructions per SIMD per ns,
// 8x below v_mov; this separates the possible causes: the condition register (VCC vs another
// SGPR pair), back-to-back mask reads vs mask reads interleaved with plain VALU ops, and the
// VGPR-mask alternatives (v_bfi_b32, v_and_or).
#include <hip/hip_runtime.h>
#include <cstdio>

#define ITERS 4096
#define CHAINS 8

template <int KIND>
__global__ __launch_bounds__(256) void kern(float* out, float a, float b)
{
    float x[CHAINS];
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) x[c] = a + threadIdx.x * 1e-7f + c;
    const unsigned m = (threadIdx.x & 1) ? 0xffffffffu : 0u;   // a per-lane mask in a VGPR
    unsigned long long sm = __builtin_amdgcn_read_exec() & 0x5555555555555555ull;
    asm volatile("s_mov_b64 vcc, %0" ::"s"(sm) : "vcc");
    for (int i = 0; i < ITERS; ++i) {
#pragma unroll
        for (int c = 0; c < CHAINS; ++c) {
            if (KIND == 0) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x[c]) : "v"(a) : "vcc");
            if (KIND == 1) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(x[c]) : "v"(a), "s"(sm));
            if (KIND == 2) {
                asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x[c]) : "v"(a) : "vcc");
                asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[(c + 1) % CHAINS]) : "v"(a));
                asm volatile("v_mul_f32 %0, %0, %1" : "+v"(x[(c + 2) % CHAINS]) : "v"(a));
                asm volatile("v_sub_f32 %0, %1, %0" : "+v"(x[(c + 3) % CHAINS]) : "v"(a));
            }
            if (KIND == 3) asm volatile("v_bfi_b32 %0, %1, %0, %2" : "+v"(x[c]) : "v"(m), "v"(a));
            if (KIND == 4) asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[c]) : "v"(a));
            if (KIND == 5) {
                asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[(c + 1) % CHAINS]) : "v"(a));
                asm volatile("v_mul_f32 %0, %0, %1" : "+v"(x[(c + 2) % CHAINS]) : "v"(a));
                asm volatile("v_sub_f32 %0, %1, %0" : "+v"(x[(c + 3) % CHAINS]) : "v"(a));
            }
            if (KIND == 6) asm volatile("v_cmp_lt_f32 vcc, %0, %1" ::"v"(x[c]), "v"(a) : "vcc");
            if (KIND == 7) asm volatile("v_cmp_lt_f32_e64 %0, %1, %2" : "=s"(sm) : "v"(x[c]), "v"(a));
            if (KIND == 8) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x[c]) : "v"(a), "v"(b));
            if (KIND == 9) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x[c]) : "v"(a), "v"(x[(c + 1) % CHAINS]));
            if (KIND == 10) asm volatile("v_max_f32 %0, %0, %1" : "+v"(x[c]) : "v"(a));
            if (KIND == 11) asm volatile("v_med3_f32 %0, %0, %1, %2" : "+v"(x[c]) : "v"(a), "v"(b));
        }
    }
    float s = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s + (float)(sm & 1);
}

template <int KIND>
void run(float* d, int blocks, const char* name, double per_iter_chain)
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
    const double winstr = blocks * 4.0 * ITERS * CHAINS * per_iter_chain;
    printf("%-26s %8.3f ms  %.3f wave-instr per SIMD per ns\n", name, ms, winstr / 1024.0 / (ms * 1e6));
}

int main()
{
    float* d;
    const int blocks = 256 * 8 * 4;
    hipMalloc(&d, blocks * 256 * sizeof(float));
    run<0>(d, blocks, "cndmask vcc", 1);
    run<1>(d, blocks, "cndmask_e64 sgpr pair", 1);
    run<2>(d, blocks, "cndmask vcc 1:3 add/mul/sub", 4);
    run<3>(d, blocks, "v_bfi_b32 vgpr mask", 1);
    run<4>(d, blocks, "v_add_f32", 1);
    run<5>(d, blocks, "add/mul/sub", 3);
    run<6>(d, blocks, "v_cmp vcc", 1);
    run<7>(d, blocks, "v_cmp_e64 sgpr", 1);
    run<8>(d, blocks, "v_fma_f32 (2 const)", 1);
    run<9>(d, blocks, "v_fma_f32 (chain operands)", 1);
    run<10>(d, blocks, "v_max_f32", 1);
    run<11>(d, blocks, "v_med3_f32", 1);
    for (int w : {1, 2, 3, 4, 5}) {
        char nm[64];
        snprintf(nm, sizeof nm, "cndmask vcc %dw/SIMD", w);
        run<0>(d, 256 * w, nm, 1);
    }
    hipFree(d);
    return 0;
}
