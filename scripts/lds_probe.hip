// Dev tool: how many 256-thread workgroups with S bytes of LDS are co-resident per CU on gfx950,
// against what hipOccupancyMaxActiveBlocksPerMultiprocessor reports.  Each block spins 200 us and
// records its start time; the blocks that start within the first 50 us are the resident ones.
// Build: hipcc --offload-arch=gfx950 -O2 -o /tmp/lds_probe scripts/lds_probe.hip
// Measured (ROCm 7.2, MI355X): 5 per CU up to 32000 B, 4 from 32256 B (the API says 5 up to
// 32768 B), 3 above 40960 B -> LDS is allocated in 1280-B granules of the CU's 160 KiB.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>
__global__ __launch_bounds__(256) void probe(unsigned long long* t, int spin_us)
{
    extern __shared__ float lds[];
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) t[blockIdx.x] = t0;
    lds[threadIdx.x] = (float)t0;
    while (__builtin_amdgcn_s_memrealtime() - t0 < (unsigned long long)spin_us * 100ull) __builtin_amdgcn_s_sleep(10);
    if (lds[threadIdx.x] == -1.0f) t[0] = 0;
}
int main()
{
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int nb = cus * 8;
    unsigned long long* d;
    if (hipMalloc(&d, nb * sizeof(unsigned long long)) != hipSuccess) return 1;
    std::vector<unsigned long long> h(nb);
    const int sizes[] = {16384, 26000, 29648, 30720, 31000, 31744, 32000, 32256, 32512, 32720, 32768, 33000, 40000, 40912, 40960, 41000};
    for (int s : sizes) {
        int occ = 0;
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, probe, 256, s);
        hipLaunchKernelGGL(probe, dim3(nb), dim3(256), s, 0, d, 200);
        if (hipMemcpy(h.data(), d, nb * sizeof(unsigned long long), hipMemcpyDeviceToHost) != hipSuccess) return 1;
        const unsigned long long t0 = *std::min_element(h.begin(), h.end());
        int early = 0;
        for (auto v : h) early += (v - t0) < 5000;   // started within 50 us
        printf("lds %6d B: blocks started at once %5d = %.2f per CU (occupancy API says %d)\n", s, early, (double)early / cus, occ);
    }
    return 0;
}
