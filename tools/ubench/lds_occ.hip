// Workgroups resident per CU against the dynamic LDS a 256-thread workgroup
// asks for (beside 3760 B of static LDS, as the slim greedy kernels): every
// workgroup stamps s_memrealtime at start, waits ~200 us, stamps again; the
// peak number of overlapping workgroups over the launch gives the residency.
// Usage: lds_occ  (prints one line per LDS size)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <algorithm>
#include <vector>

__device__ __forceinline__ unsigned long long rt() {
    unsigned long long t;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}

__global__ __launch_bounds__(256) void occ(unsigned long long *t, uint32_t spin) {
    extern __shared__ uint32_t dyn[];
    __shared__ uint32_t stat[940];                 // 3760 B (pf_k3_greedy, round 5)
    const unsigned long long t0 = rt();
    stat[threadIdx.x] = threadIdx.x;
    dyn[threadIdx.x] = threadIdx.x;
    __syncthreads();
    while (rt() - t0 < spin) __builtin_amdgcn_s_sleep(8);
    __syncthreads();
    if (threadIdx.x == 0) {
        t[2 * blockIdx.x] = t0;
        t[2 * blockIdx.x + 1] = rt() + stat[5] + dyn[7] - 12;
    }
}

int main() {
    const uint32_t sizes[] = {36864, 36992, 37120, 37200, 37248, 37376, 37504, 37632, 37888, 38144, 38912, 40960,
                              49152, 50688};
    int dev = 0, ncu = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    const uint32_t nwg = (uint32_t)ncu * 6;
    unsigned long long *d_t = nullptr;
    hipMalloc(&d_t, 16ull * nwg);
    std::vector<unsigned long long> h(2ull * nwg);
    hipFuncSetAttribute((const void *)occ, hipFuncAttributeMaxDynamicSharedMemorySize, 81920);
    int lds_cu = 0;
    hipDeviceGetAttribute(&lds_cu, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, dev);
    printf("CUs %d, workgroups per launch %u, LDS per CU (attribute) %d\n", ncu, nwg, lds_cu);
    for (uint32_t lds : sizes) {
        hipLaunchKernelGGL(occ, dim3(nwg), dim3(256), lds, 0, d_t, 20000u);   // 200 us at 100 MHz
        if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed at %u\n", lds); return 1; }
        hipMemcpy(h.data(), d_t, 16ull * nwg, hipMemcpyDeviceToHost);
        std::vector<std::pair<unsigned long long, int>> ev;
        for (uint32_t i = 0; i < nwg; i++) { ev.push_back({h[2 * i], 1}); ev.push_back({h[2 * i + 1], -1}); }
        std::sort(ev.begin(), ev.end(), [](auto &a, auto &b) { return a.first != b.first ? a.first < b.first : a.second < b.second; });
        int cur = 0, mx = 0;
        for (auto &e : ev) { cur += e.second; mx = std::max(mx, cur); }
        printf("dynamic LDS %6u B (+3760 static): peak resident workgroups %4d = %.2f per CU\n", lds, mx,
               (double)mx / ncu);
    }
    hipFree(d_t);
    return 0;
}
