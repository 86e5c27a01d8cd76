// scripts/anyorder_probe.hip -- does a kernel launched with hipExtAnyOrderLaunch start before the
// previous kernel on its stream has completed (gfx950)?  Dev probe, bounded waits only.
//   kernel A: one block; lane 0 polls a flag (relaxed agent loads) for at most ~50 ms of s_memrealtime
//   kernel B: one block; lane 0 stores the flag
// A sees the flag only if B ran while A was still running.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>

__global__ void kA(unsigned* flag, unsigned* out)
{
    if (threadIdx.x == 0) {
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        unsigned seen = 0;
        while (__builtin_amdgcn_s_memrealtime() - t0 < 5000000ull) {   // 100 MHz: 50 ms
            if (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) {
                seen = 1;
                break;
            }
            __builtin_amdgcn_s_sleep(10);
        }
        out[0] = seen;
        out[1] = (unsigned)((__builtin_amdgcn_s_memrealtime() - t0) / 100ull);   // us
    }
}

__global__ void kB(unsigned* flag)
{
    if (threadIdx.x == 0) __hip_atomic_store(flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

static void run(const char* name, unsigned flagsA, unsigned flagsB, bool two_streams)
{
    unsigned *flag, *out;
    hipMalloc(&flag, 4);
    hipMalloc(&out, 8);
    hipMemset(flag, 0, 4);
    hipMemset(out, 0xff, 8);
    hipStream_t s1, s2;
    hipStreamCreate(&s1);
    hipStreamCreate(&s2);
    hipDeviceSynchronize();
    void* argsA[] = {&flag, &out};
    void* argsB[] = {&flag};
    hipError_t ea = hipExtLaunchKernel((const void*)kA, dim3(1), dim3(64), argsA, 0, s1, nullptr, nullptr, flagsA);
    hipError_t eb = hipExtLaunchKernel((const void*)kB, dim3(1), dim3(64), argsB, 0, two_streams ? s2 : s1, nullptr, nullptr, flagsB);
    hipDeviceSynchronize();
    unsigned h[2];
    hipMemcpy(h, out, 8, hipMemcpyDeviceToHost);
    printf("%-34s launchA=%s launchB=%s  A saw B's flag: %u after %u us\n", name, hipGetErrorString(ea), hipGetErrorString(eb), h[0], h[1]);
    hipStreamDestroy(s1);
    hipStreamDestroy(s2);
    hipFree(flag);
    hipFree(out);
}

int main()
{
    int v = -1;
    hipDeviceGetAttribute(&v, hipDeviceAttributeCanUseStreamWaitValue, 0);
    printf("hipDeviceAttributeCanUseStreamWaitValue = %d\n", v);
    run("same stream, plain", 0, 0, false);
    run("same stream, B any-order", 0, hipExtAnyOrderLaunch, false);
    run("same stream, both any-order", hipExtAnyOrderLaunch, hipExtAnyOrderLaunch, false);
    run("two streams, plain", 0, 0, true);
    return 0;
}
