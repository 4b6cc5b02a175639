// pf_ingest.hip -- host side of the device BAM ingest: BGZF block tables and
// the device inflate entry points (kernels in pf_inflate.hip).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <vector>
#include "pf_ingest.h"
#include "../../include/pomfret_amd.h"

struct pf_ctx;
extern "C" int pf_ctx_device(const pf_ctx *c);
extern "C" hipStream_t pf_ctx_stream(const pf_ctx *c);

#define ICHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "[E::pomfret_amd] %s failed: %s (%s:%d)\n", #x, hipGetErrorString(e_), __FILE__, __LINE__); \
    rc = PF_ERR_HIP; goto out; } } while (0)

static uint32_t rd16(const uint8_t *p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8); }
static uint32_t rd32(const uint8_t *p) { return rd16(p) | (rd16(p + 2) << 16); }

// Parse the BGZF blocks of comp[0, len) (whole blocks, as bgzf_read_block
// reads them: gzip member with FEXTRA and the BC subfield) into a block table
// whose outputs are laid out back to back from out_base.  Returns the number
// of blocks, or a negative PF_ERR.
int64_t pf_bgzf_scan(const uint8_t *comp, uint64_t len, uint64_t out_base, uint32_t run,
                     std::vector<pf_bgzf_blk> &blk) {
    uint64_t o = 0, out = out_base;
    int64_t n = 0;
    while (o < len) {
        if (len - o < 18) return PF_ERR_ARG;
        const uint8_t *h = comp + o;
        if (h[0] != 31 || h[1] != 139 || h[2] != 8 || !(h[3] & 4)) return PF_ERR_ARG;
        const uint32_t xlen = rd16(h + 10);
        if (12ull + xlen > len - o) return PF_ERR_ARG;
        uint32_t bsize = 0;
        for (uint32_t x = 0; x + 4 <= xlen;) {
            const uint8_t *sf = h + 12 + x;
            const uint32_t slen = rd16(sf + 2);
            if (sf[0] == 'B' && sf[1] == 'C' && slen == 2) bsize = rd16(sf + 4) + 1;
            x += 4 + slen;
        }
        if (bsize < 12 + xlen + 8 || bsize > 65536 || bsize > len - o) return PF_ERR_ARG;
        pf_bgzf_blk b;
        b.in_off = o + 12 + xlen;
        b.in_len = bsize - 12 - xlen - 8;
        b.crc = rd32(h + bsize - 8);
        b.isize = rd32(h + bsize - 4);
        if (b.isize > 65536) return PF_ERR_ARG;
        b.out_off = out;
        b.run = run;
        out += b.isize;
        blk.push_back(b);
        n++;
        o += bsize;
    }
    return n;
}

// Inflate blocks on the device: d_in / d_blk / d_arena / d_status resident;
// status copied back; returns PF_OK or PF_ERR_ARG naming the first bad block.
int pf_inflate_launch(hipStream_t st, const uint8_t *d_in, const pf_bgzf_blk *d_blk, uint32_t nblk, uint8_t *d_arena,
                      uint32_t *d_status, hipEvent_t e0, hipEvent_t e1) {
    if (!nblk) return PF_OK;
    if (e0 && hipEventRecord(e0, st) != hipSuccess) return PF_ERR_HIP;
    hipLaunchKernelGGL(pf_inflate, dim3((nblk + 3) / 4), dim3(256), 0, st, d_in, d_blk, nblk, d_arena, d_status);
    if (hipGetLastError() != hipSuccess) return PF_ERR_HIP;
    if (e1 && hipEventRecord(e1, st) != hipSuccess) return PF_ERR_HIP;
    hipLaunchKernelGGL(pf_bgzf_crc, dim3((nblk + 3) / 4), dim3(256), 0, st, d_arena, d_blk, nblk, d_status);
    if (hipGetLastError() != hipSuccess) return PF_ERR_HIP;
    return PF_OK;
}

extern "C" int pf_bgzf_inflate(pf_ctx_t *ctx, const uint8_t *comp, uint64_t comp_len, uint8_t *out, uint64_t out_cap,
                               uint64_t *out_len, uint32_t *block_status, uint32_t status_cap, float *kernel_ms) {
    if (!ctx || (!comp && comp_len) || !out_len) return PF_ERR_ARG;
    std::vector<pf_bgzf_blk> blk;
    const int64_t nb = pf_bgzf_scan(comp, comp_len, 0, 0, blk);
    if (nb < 0) return (int)nb;
    const uint64_t total = blk.empty() ? 0 : blk.back().out_off + blk.back().isize;
    *out_len = total;
    if (total > out_cap || (total && !out)) return PF_ERR_ARG;
    if (!nb) return PF_OK;
    int rc = PF_OK;
    uint8_t *d_in = nullptr, *d_arena = nullptr;
    pf_bgzf_blk *d_blk = nullptr;
    uint32_t *d_st = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    std::vector<uint32_t> st((size_t)nb);
    hipStream_t s = pf_ctx_stream((const pf_ctx *)ctx);
    ICHK(hipSetDevice(pf_ctx_device((const pf_ctx *)ctx)));
    ICHK(hipMalloc(&d_in, comp_len + 512));
    ICHK(hipMemsetAsync(d_in + comp_len, 0, 512, s));
    ICHK(hipMemcpyAsync(d_in, comp, comp_len, hipMemcpyHostToDevice, s));
    ICHK(hipMalloc(&d_blk, sizeof(pf_bgzf_blk) * (size_t)nb));
    ICHK(hipMemcpyAsync(d_blk, blk.data(), sizeof(pf_bgzf_blk) * (size_t)nb, hipMemcpyHostToDevice, s));
    ICHK(hipMalloc(&d_arena, total + 256));
    ICHK(hipMalloc(&d_st, 4ull * (size_t)nb));
    ICHK(hipMemsetAsync(d_st, 0, 4ull * (size_t)nb, s));
    ICHK(hipEventCreate(&e0));
    ICHK(hipEventCreate(&e1));
    rc = pf_inflate_launch(s, d_in, d_blk, (uint32_t)nb, d_arena, d_st, e0, e1);
    if (rc) goto out;
    ICHK(hipMemcpyAsync(st.data(), d_st, 4ull * (size_t)nb, hipMemcpyDeviceToHost, s));
    ICHK(hipMemcpyAsync(out, d_arena, total, hipMemcpyDeviceToHost, s));
    ICHK(hipStreamSynchronize(s));
    if (kernel_ms) ICHK(hipEventElapsedTime(kernel_ms, e0, e1));
    for (int64_t i = 0; i < nb; i++) {
        if (block_status && (uint64_t)i < status_cap) block_status[i] = st[i];
        if (st[i] && rc == PF_OK) rc = PF_ERR_ARG;
    }
out:
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    (void)hipFree(d_in);
    (void)hipFree(d_blk);
    (void)hipFree(d_arena);
    (void)hipFree(d_st);
    return rc;
}
