// Micro-benchmark: LDS latencies seen by one wavefront (developer tool).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void k(unsigned long long *out, int mode, int iters) {
    __shared__ uint32_t buf[16384];
    const uint32_t lane = threadIdx.x;
    for (uint32_t i = lane; i < 16384; i += 64) buf[i] = (i * 2654435761u) & 16383u;
    __syncthreads();
    uint32_t idx = lane;
    uint32_t acc = 0;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if (mode == 0) {            // dependent chain, consecutive addresses per lane
#pragma unroll 16
        for (int i = 0; i < iters; i++) { idx = (buf[idx] & 0) + ((idx + 64) & 16383); acc += idx; }
    } else if (mode == 1) {     // dependent chain, random addresses per lane (gather)
#pragma unroll 16
        for (int i = 0; i < iters; i++) { idx = buf[idx]; acc += idx; }
    } else if (mode == 2) {     // 8 independent random gathers then use
        for (int i = 0; i < iters; i += 8) {
            uint32_t v[8];
#pragma unroll
            for (int u = 0; u < 8; u++) v[u] = buf[(idx + u * 977) & 16383];
            uint32_t s = 0;
#pragma unroll
            for (int u = 0; u < 8; u++) s += v[u];
            idx = s & 16383; acc += s;
        }
    } else if (mode == 3) {     // dependent VALU chain (v_add_f32)
        float f = (float)lane;
#pragma unroll 16
        for (int i = 0; i < iters; i++) f = f + 1.0f;
        acc = (uint32_t)f;
    } else if (mode == 4) {     // store then dependent load by another lane (wave-local handoff)
        for (int i = 0; i < iters; i++) {
            buf[lane] = idx;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            idx = buf[(lane + 1) & 63] + 1;
        }
        acc = idx;
    } else if (mode == 5) {     // ds_bpermute chain
#pragma unroll 16
        for (int i = 0; i < iters; i++) idx = (uint32_t)__shfl((int)idx, (int)((lane + 1) & 63), 64) + 1;
        acc = idx;
    } else if (mode == 7) {     // empty loop (overhead), volatile-ish counter
        for (int i = 0; i < iters; i++) { acc += lane; __builtin_amdgcn_sched_barrier(0); }
    } else if (mode == 8) {     // dependent v_pk_add_f32 chain
        float2 f = make_float2((float)lane, 1.f);
#pragma unroll 16
        for (int i = 0; i < iters; i++) { f.x = f.x + 1.0f; f.y = f.y + 2.0f; }
        acc = (uint32_t)(f.x + f.y);
    } else if (mode == 9) {     // independent VALU throughput: 8 chains
        float f[8];
        for (int u = 0; u < 8; u++) f[u] = (float)(lane + u);
#pragma unroll 2
        for (int i = 0; i < iters; i += 8) {
#pragma unroll
            for (int u = 0; u < 8; u++) f[u] = f[u] * 1.0001f + 1.0f;
        }
        acc = (uint32_t)(f[0] + f[7]);
    } else if (mode == 10) {    // dpp row_shr add chain
        for (int i = 0; i < iters; i++) idx += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)idx, 0x111, 0xF, 0xF, true);
        acc = idx;
    } else if (mode == 6) {     // readlane + SALU chain
#pragma unroll 16
        for (int i = 0; i < iters; i++) idx = (uint32_t)__builtin_amdgcn_readlane((int)idx, i & 63) + lane;
        acc = idx;
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) { out[blockIdx.x * 2] = t1 - t0; out[blockIdx.x * 2 + 1] = acc; }
}

int main() {
    unsigned long long *d, h[2 * 512];
    hipMalloc(&d, sizeof(h));
    const char *names[] = {"dep ds_read consecutive", "dep ds_read random gather", "8 indep gathers (per 8)",
                           "dep v_add_f32", "store->wave handoff->load", "ds_bpermute chain", "readlane chain", "empty loop", "dep v_pk_add (2 chains)",
                           "indep fma x8 (per op)", "dpp add chain"};
    for (int mode = 0; mode < 11; mode++) {
        for (int blocks : {1, 512}) {
            const int iters = 4096;
            hipLaunchKernelGGL(k, dim3(blocks), dim3(64), 0, 0, d, mode, iters);
            hipLaunchKernelGGL(k, dim3(blocks), dim3(64), 0, 0, d, mode, iters);
            hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
            double mx = 0;
            for (int b = 0; b < blocks; b++) mx = h[2 * b] > mx ? h[2 * b] : mx;
            printf("%-28s blocks=%3d  %.1f cycles/iter (max block)\n", names[mode], blocks, mx / iters);
        }
    }
    return 0;
}
