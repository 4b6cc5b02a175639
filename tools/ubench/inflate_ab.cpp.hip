// A/B timing of pf_inflate variants (compile-time switches of
// pomfret_amd/csrc/pf_inflate.hip, INF_AB here) on the same blocks: each
// variant's output is checked against variant 0's.  Under rocprofv3 --pmc it
// gives the per-variant SQ counters.  Usage: inflate_ab <blocks file> [copies]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>
#include "../../pomfret_amd/csrc/pf_ingest.h"

namespace v0 {                          // A: _inf_a.hip (a saved earlier version) when present
#undef INF_AB
#define INF_AB 0
#if __has_include("_inf_a.hip")
#include "_inf_a.hip"
#else
#include "../../pomfret_amd/csrc/pf_inflate.hip"
#endif
}
namespace v1 {
#undef INF_AB
#define INF_AB 1
#undef INF_SPECM
#define INF_SPECM 1
#include "../../pomfret_amd/csrc/pf_inflate.hip"
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

int main(int argc, char **argv) {
    if (argc < 2) return 2;
    const int copies = argc > 2 ? atoi(argv[2]) : 256;
    FILE *f = fopen(argv[1], "rb");
    if (!f) return 2;
    std::vector<uint8_t> one;
    uint8_t buf[1 << 16];
    size_t k;
    while ((k = fread(buf, 1, sizeof buf, f)) > 0) one.insert(one.end(), buf, buf + k);
    fclose(f);
    std::vector<pf_bgzf_blk> b1;
    for (size_t o = 0; o + 18 <= one.size();) {
        const uint32_t xlen = one[o + 10] | (one[o + 11] << 8), bsize = (one[o + 16] | (one[o + 17] << 8)) + 1;
        pf_bgzf_blk b;
        b.in_off = o + 12 + xlen;
        b.in_len = bsize - 12 - xlen - 8;
        memcpy(&b.crc, &one[o + bsize - 8], 4);
        memcpy(&b.isize, &one[o + bsize - 4], 4);
        b.run = 0;
        b1.push_back(b);
        o += bsize;
    }
    std::vector<uint8_t> comp;
    std::vector<pf_bgzf_blk> blk;
    uint64_t out = 0;
    for (int c = 0; c < copies; c++) {
        for (auto b : b1) { b.in_off += comp.size(); b.out_off = out; out += b.isize; blk.push_back(b); }
        comp.insert(comp.end(), one.begin(), one.end());
    }
    comp.resize(comp.size() + 512, 0);
    const uint32_t nb = (uint32_t)blk.size();
    uint8_t *d_in, *d_out[2];
    pf_bgzf_blk *d_blk;
    uint32_t *d_st;
    CK(hipMalloc(&d_in, comp.size()));
    CK(hipMalloc(&d_out[0], out + 512));
    CK(hipMalloc(&d_out[1], out + 512));
    CK(hipMalloc(&d_blk, sizeof(pf_bgzf_blk) * nb));
    CK(hipMalloc(&d_st, 4ull * nb));
    CK(hipMemcpy(d_in, comp.data(), comp.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(d_blk, blk.data(), sizeof(pf_bgzf_blk) * nb, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    void (*kern[2])(const uint8_t *, const pf_bgzf_blk *, uint32_t, uint8_t *, uint32_t *) = {v0::pf_inflate,
                                                                                              v1::pf_inflate};
    const char *name[2] = {"A", "B"};
    for (int rep = 0; rep < 3; rep++)
        for (int v = 0; v < 2; v++) {
            CK(hipMemset(d_st, 0, 4ull * nb));
            CK(hipEventRecord(e0, 0));
            hipLaunchKernelGGL(kern[v], dim3((nb + 3) / 4), dim3(256), 0, 0, d_in, d_blk, nb, d_out[v], d_st);
            CK(hipGetLastError());
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            std::vector<uint32_t> st(nb);
            CK(hipMemcpy(st.data(), d_st, 4ull * nb, hipMemcpyDeviceToHost));
            uint32_t bad = 0;
            for (uint32_t i = 0; i < nb; i++) bad += st[i] != 0;
            printf("%-7s blocks %u out %.0f MB: %.3f ms = %.2f GB/s  bad %u\n", name[v], nb, out / 1e6, ms,
                   out / (ms * 1e6), bad);
        }
    std::vector<uint8_t> h0(out), h1(out);
    CK(hipMemcpy(h0.data(), d_out[0], out, hipMemcpyDeviceToHost));
    CK(hipMemcpy(h1.data(), d_out[1], out, hipMemcpyDeviceToHost));
    printf("outputs %s\n", memcmp(h0.data(), h1.data(), out) ? "DIFFER" : "identical");
    return 0;
}
