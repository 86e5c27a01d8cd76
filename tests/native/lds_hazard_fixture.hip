// Fixture for tests/test_isa_lgkm.py (test infrastructure, never linked into the product): two
// kernels that read LDS through inline asm.  `split_wait` has the round-5 quads_exact shape -- the
// ds_read_b128 and its s_waitcnt in separate asm statements, the value consumed in between -- so
// the compiler reads the destination registers before the data returns; `fused_wait` issues the
// load and its wait in one asm statement.  The ISA checker must flag the first and pass the second.
#include <hip/hip_runtime.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(64) void split_wait(float* out)
{
    __shared__ float4 s[64];
    s[threadIdx.x] = make_float4(threadIdx.x, 1.0f, 2.0f, 3.0f);
    __syncthreads();
    const uint32_t addr = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) float4*)&s[threadIdx.x ^ 1];
    f32x4 row;
    asm volatile("ds_read_b128 %0, %1" : "=v"(row) : "v"(addr));
    const float early = row.x * 2.0f;            // consumed before the wait below
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(row));
    out[threadIdx.x] = early + row.y;
}

__global__ __launch_bounds__(64) void fused_wait(float* out)
{
    __shared__ float4 s[64];
    s[threadIdx.x] = make_float4(threadIdx.x, 1.0f, 2.0f, 3.0f);
    __syncthreads();
    const uint32_t addr = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) float4*)&s[threadIdx.x ^ 1];
    f32x4 row;
    asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(row) : "v"(addr));
    out[threadIdx.x] = row.x * 2.0f + row.y;
}
