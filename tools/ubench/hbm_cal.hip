// Calibration of rocprofv3 FETCH_SIZE / WRITE_SIZE on gfx950 for the access
// widths the pomfret_amd kernels use (developer tool; see tools/pmc_traffic.py).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void rd_u32(const uint32_t *a, size_t n, uint32_t *out) {
    uint32_t s = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) s += a[i];
    if (s == 0x12345678u) out[0] = s;
}
__global__ void rd_u8(const uint8_t *a, size_t n, uint32_t *out) {
    uint32_t s = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) s += a[i];
    if (s == 0x12345678u) out[0] = s;
}
__global__ void rd_u128(const uint4 *a, size_t n, uint32_t *out) {
    uint32_t s = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = a[i];
        s += v.x + v.y + v.z + v.w;
    }
    if (s == 0x12345678u) out[0] = s;
}
__global__ void wr_u32(uint32_t *a, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) a[i] = (uint32_t)i;
}
__global__ void wr_u8(uint8_t *a, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) a[i] = (uint8_t)i;
}

int main() {
    const size_t bytes = 1ull << 30;   // 1 GiB: past the 256 MiB Infinity Cache
    void *buf;
    uint32_t *out;
    if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, 4) != hipSuccess) return 1;
    (void)hipMemset(buf, 1, bytes);
    const dim3 g(256 * 8), b(256);
    for (int rep = 0; rep < 2; rep++) {
        hipLaunchKernelGGL(rd_u32, g, b, 0, 0, (const uint32_t *)buf, bytes / 4, out);
        hipLaunchKernelGGL(rd_u8, g, b, 0, 0, (const uint8_t *)buf, bytes, out);
        hipLaunchKernelGGL(rd_u128, g, b, 0, 0, (const uint4 *)buf, bytes / 16, out);
        hipLaunchKernelGGL(wr_u32, g, b, 0, 0, (uint32_t *)buf, bytes / 4);
        hipLaunchKernelGGL(wr_u8, g, b, 0, 0, (uint8_t *)buf, bytes);
    }
    (void)hipDeviceSynchronize();
    printf("bytes per kernel: %zu\n", bytes);
    return 0;
}
