// scripts/waitvalue_probe.hip -- latency of a stream gate on a device counter (dev probe):
// stream 1 runs kernel A (64 blocks: each adds 1 to a 64-bit counter at its start, then spins
// ~200 us), stream 2 waits with hipStreamWaitValue64(counter >= 64) and then runs kernel B, which
// stamps s_memrealtime.  Reports B's start minus A's last block start, for the counter in plain
// hipMalloc memory and in hipMallocSignalMemory memory.  Bounded: A spins a fixed time.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>

__global__ void kA(unsigned long long* cnt, unsigned long long* stamp)
{
    if (threadIdx.x == 0) {
        const unsigned long long t = __builtin_amdgcn_s_memrealtime();
        __hip_atomic_fetch_add(cnt, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        atomicMax(stamp, t);
        while (__builtin_amdgcn_s_memrealtime() - t < 20000ull) __builtin_amdgcn_s_sleep(10);   // 200 us
    }
}
__global__ void kB(unsigned long long* stamp)
{
    if (threadIdx.x == 0) stamp[1] = __builtin_amdgcn_s_memrealtime();
}

static void run(const char* name, bool signal)
{
    unsigned long long *cnt, *stamp;
    hipError_t ea = signal ? hipExtMallocWithFlags((void**)&cnt, 8, hipMallocSignalMemory) : hipMalloc(&cnt, 8);
    hipMalloc(&stamp, 16);
    hipMemset(cnt, 0, 8);
    hipMemset(stamp, 0, 16);
    hipStream_t s1, s2;
    hipStreamCreateWithFlags(&s1, hipStreamNonBlocking);
    hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
    hipDeviceSynchronize();
    hipError_t ew = hipStreamWaitValue64(s2, cnt, 64, hipStreamWaitValueGte, ~0ull);
    hipLaunchKernelGGL(kB, dim3(1), dim3(64), 0, s2, stamp);
    hipLaunchKernelGGL(kA, dim3(64), dim3(64), 0, s1, cnt, stamp);
    hipError_t es = hipDeviceSynchronize();
    unsigned long long h[2], c;
    hipMemcpy(h, stamp, 16, hipMemcpyDeviceToHost);
    hipMemcpy(&c, cnt, 8, hipMemcpyDeviceToHost);
    printf("%-22s alloc=%s wait=%s sync=%s count=%llu  B start - A's last block start = %.1f us\n", name,
           hipGetErrorString(ea), hipGetErrorString(ew), hipGetErrorString(es), c, ((long long)(h[1] - h[0])) * 0.01);
    hipStreamDestroy(s1);
    hipStreamDestroy(s2);
    hipFree(cnt);
    hipFree(stamp);
}

int main()
{
    for (int i = 0; i < 2; ++i) {
        run("hipMalloc counter", false);
        run("signal-memory counter", true);
    }
    return 0;
}
