// A/B timing of the BGZF inflate kernels on the same blocks (a BAM file,
// replicated): pf_inflate (one wave per block, pf_inflate.hip) against the
// two-pass decoder (inflate_simt.hip, measured slower and kept out of the product) at two table sizes; per variant the
// first pass (Huffman -> tokens) and the second (LZ77 + CRC + store) timed
// with events; outputs compared with the wave kernel's.
// Usage: inflate_si <bgzf file> [copies]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>
#include "../../pomfret_amd/csrc/pf_ingest.h"

namespace w {
#include "../../pomfret_amd/csrc/pf_inflate.hip"
// the blocks the two-pass decoder left (PF_INF_FALLBACK), one wave each
__global__ __launch_bounds__(64 * INF_WAVES) void pf_inflate_fallback(const uint8_t *in, const pf_bgzf_blk *blk,
                                                                      uint32_t nblk, uint8_t *arena, uint32_t *status) {
    inflate_blocks<true>(in, blk, nblk, arena, status);
}
}
namespace vp {
#define SI_PROF 1
#define SI_LR 8u
#define SI_DR 7u
#define SI_LCAP 96u
#define SI_DCAP 32u
#define SI_RS 8u
#define SI_RP 4u
#include "inflate_simt.hip"
#undef SI_LR
#undef SI_DR
#undef SI_LCAP
#undef SI_DCAP
#undef SI_RS
#undef SI_RP
#undef SI_PROF
#undef SI_TS
}
namespace v1 {
#define SI_LR 9u
#define SI_DR 7u
#define SI_LCAP 128u
#define SI_DCAP 32u
#define SI_RS 16u
#define SI_RP 8u
#include "inflate_simt.hip"
#undef SI_LR
#undef SI_DR
#undef SI_LCAP
#undef SI_DCAP
#undef SI_RS
#undef SI_RP
}
namespace v2 {
#define SI_LR 8u
#define SI_DR 7u
#define SI_LCAP 128u
#define SI_DCAP 32u
#define SI_RS 16u
#define SI_RP 8u
#include "inflate_simt.hip"
#undef SI_LR
#undef SI_DR
#undef SI_LCAP
#undef SI_DCAP
#undef SI_RS
#undef SI_RP
}
namespace v3 {
#define SI_LR 8u
#define SI_DR 7u
#define SI_LCAP 96u
#define SI_DCAP 32u
#define SI_RS 8u
#define SI_RP 4u
#include "inflate_simt.hip"
#undef SI_LR
#undef SI_DR
#undef SI_LCAP
#undef SI_DCAP
#undef SI_RS
#undef SI_RP
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

int main(int argc, char **argv) {
    if (argc < 2) return 2;
    const int copies = argc > 2 ? atoi(argv[2]) : 1;
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
        if (b.isize) b1.push_back(b);
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
    uint8_t *d_in, *d_out[2], *d_ws;
    pf_bgzf_blk *d_blk;
    uint32_t *d_st;
    const uint64_t tok_b = 4ull * (out + 4ull * nb + 16) + 256, meta_b = ((4ull * PF_SI_META * nb) + 255) & ~255ull;
    CK(hipMalloc(&d_in, comp.size()));
    CK(hipMalloc(&d_out[0], out + 512));
    CK(hipMalloc(&d_out[1], out + 512));
    CK(hipMalloc(&d_ws, tok_b + meta_b + (uint64_t)PF_SI_SCR * nb));
    CK(hipMalloc(&d_blk, sizeof(pf_bgzf_blk) * nb));
    CK(hipMalloc(&d_st, 4ull * nb));
    CK(hipMemcpy(d_in, comp.data(), comp.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(d_blk, blk.data(), sizeof(pf_bgzf_blk) * nb, hipMemcpyHostToDevice));
    uint32_t *tok = (uint32_t *)d_ws, *meta = (uint32_t *)(d_ws + tok_b);
    uint8_t *scr = d_ws + tok_b + meta_b;
    hipEvent_t e0, e1, e2;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventCreate(&e2));
    std::vector<uint8_t> ref(out), got(out);
    std::vector<uint32_t> st(nb);
    typedef void (*tokk)(const uint8_t *, const pf_bgzf_blk *, uint32_t, uint64_t, uint32_t *, uint32_t *, uint8_t *,
                         uint32_t *);
    typedef void (*lzk)(const pf_bgzf_blk *, uint32_t, uint64_t, const uint32_t *, const uint32_t *, uint8_t *,
                        uint32_t *);
    const int NV = 5;
    tokk tk[NV] = {nullptr, v1::pf_inflate_tok, v2::pf_inflate_tok, v3::pf_inflate_tok, vp::pf_inflate_tok};
    lzk lz[NV] = {nullptr, v1::pf_inflate_lz, v2::pf_inflate_lz, v3::pf_inflate_lz, vp::pf_inflate_lz};
    const char *name[NV] = {"wave", "9/7 c128 r16", "8/7 c128 r16", "8/7 c96 r8", "prof 8/7 c96"};
    for (int rep = 0; rep < 2; rep++)
        for (int v = 0; v < NV; v++) {
            CK(hipMemset(d_st, 0, 4ull * nb));
            uint8_t *dst = d_out[v ? 1 : 0];
            CK(hipMemset(dst, 0, out));
            CK(hipEventRecord(e0, 0));
            if (v == 0) {
                hipLaunchKernelGGL(w::pf_inflate, dim3((nb + 3) / 4), dim3(256), 0, 0, d_in, d_blk, nb, dst, d_st);
                CK(hipEventRecord(e1, 0));
            } else {
                hipLaunchKernelGGL(tk[v], dim3((nb + 63) / 64), dim3(64), 0, 0, d_in, d_blk, nb, 0ull, tok, meta, scr,
                                   d_st);
                CK(hipEventRecord(e1, 0));
                hipLaunchKernelGGL(lz[v], dim3(nb), dim3(256), 0, 0, d_blk, nb, 0ull, (const uint32_t *)tok,
                                   (const uint32_t *)meta, dst, d_st);
                hipLaunchKernelGGL(w::pf_inflate_fallback, dim3((nb + 3) / 4), dim3(256), 0, 0, d_in, d_blk, nb, dst,
                                   d_st);
            }
            CK(hipGetLastError());
            CK(hipEventRecord(e2, 0));
            CK(hipEventSynchronize(e2));
            float ms1 = 0, ms2 = 0;
            CK(hipEventElapsedTime(&ms1, e0, e1));
            CK(hipEventElapsedTime(&ms2, e1, e2));
            CK(hipMemcpy(st.data(), d_st, 4ull * nb, hipMemcpyDeviceToHost));
            uint32_t bad = 0;
            for (uint32_t i = 0; i < nb; i++) bad += st[i] != 0;
            CK(hipMemcpy(v ? got.data() : ref.data(), dst, out, hipMemcpyDeviceToHost));
            const bool same = v == 0 || memcmp(got.data(), ref.data(), out) == 0;
            printf("%-13s blocks %u out %.0f MB: pass1 %.3f ms pass2 %.3f ms total %.3f ms = %.2f GB/s  bad %u %s\n",
                   name[v], nb, out / 1e6, ms1, ms2, ms1 + ms2, out / ((ms1 + ms2) * 1e6), bad,
                   same ? "identical" : "DIFFER");
            if (v == NV - 1) {                  // s_memtime sections per wave (x16 clocks), averaged
                std::vector<uint32_t> mh((size_t)nb * PF_SI_META);
                CK(hipMemcpy(mh.data(), meta, 4ull * PF_SI_META * nb, hipMemcpyDeviceToHost));
                double sn = 0, st = 0, sr = 0, sh = 0, sd = 0;
                uint32_t nw = 0;
                for (uint32_t b = 0; b + 1 < nb; b += 64, nw++) {
                    const uint32_t *m0 = &mh[(size_t)b * PF_SI_META], *m1 = &mh[(size_t)(b + 1) * PF_SI_META];
                    sn += m0[17]; st += 16.0 * m0[18]; sr += 16.0 * m0[19]; sh += 16.0 * m1[17]; sd += 16.0 * m1[18];
                }
                printf("  pass1 per wave: iterations %.0f, clocks total %.3g = %.0f per iteration: refill %.0f, header %.0f, "
                       "decode %.0f, emit/rest %.0f\n", sn / nw, st / nw, st / sn, sr / sn, sh / sn, sd / sn,
                       (st - sr - sh - sd) / sn);
                double lt = 0, lo = 0, lv = 0, lr = 0;
                uint32_t nl = 0;
                for (uint32_t b = 0; b < nb; b++) {
                    if ((b & 63u) < 2) continue;
                    const uint32_t *m = &mh[(size_t)b * PF_SI_META];
                    lt += 16.0 * m[17]; lo += 16.0 * m[18]; lv += 16.0 * (m[19] & 0xFFFFFFu); lr += m[19] >> 24; nl++;
                }
                printf("  pass2 per block: clocks %.0f: tokens+owners %.0f, values %.0f, jumps %.0f; rounds %.1f\n",
                       lt / nl, lo / nl, lv / nl, (lt - lo - lv) / nl, lr / nl);
            }
        }
    return 0;
}
