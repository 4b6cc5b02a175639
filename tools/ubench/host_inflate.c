/* Host BGZF block decode rate: zlib vs libdeflate (dlopen'd, as pf_bam.c
 * loads it) over N consecutive blocks of a BAM, single thread, CRC included.
 *   gcc -O2 -o /tmp/host_inflate tools/ubench/host_inflate.c -lz -ldl
 *   /tmp/host_inflate file.bam 2000
 * Result for round 5: profiles/r05/host_inflate.txt */
#include <dlfcn.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <zlib.h>

static double now(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + 1e-9 * t.tv_nsec;
}

int main(int argc, char **argv) {
    if (argc < 3) { fprintf(stderr, "usage: %s file.bam n_blocks\n", argv[0]); return 2; }
    FILE *f = fopen(argv[1], "rb");
    if (!f) return 1;
    const size_t N = (size_t)atol(argv[2]);
    uint8_t **blk = malloc(N * sizeof *blk);
    uint32_t *bs = malloc(N * 4);
    size_t nb = 0;
    uint8_t h[18];
    while (nb < N && fread(h, 1, 18, f) == 18) {           /* BGZF: BSIZE at bytes 16-17 */
        const uint32_t b = (uint32_t)(h[16] | h[17] << 8) + 1;
        blk[nb] = malloc(b);
        memcpy(blk[nb], h, 18);
        if (fread(blk[nb] + 18, 1, b - 18, f) != b - 18) break;
        bs[nb++] = b;
    }
    static uint8_t u[65536];
    size_t tz_b = 0, tl_b = 0;
    double t = now();
    for (size_t i = 0; i < nb; i++) {
        z_stream zs;
        memset(&zs, 0, sizeof zs);
        inflateInit2(&zs, -15);
        zs.next_in = blk[i] + 18;
        zs.avail_in = bs[i] - 26;
        zs.next_out = u;
        zs.avail_out = sizeof u;
        inflate(&zs, Z_FINISH);
        tz_b += zs.total_out;
        (void)crc32(0, u, (uInt)zs.total_out);
        inflateEnd(&zs);
    }
    const double tz = now() - t;
    void *L = dlopen("libdeflate.so.0", RTLD_NOW);
    if (!L) { printf("blocks %zu MB %.1f zlib %.0f MB/s (no libdeflate)\n", nb, tz_b / 1e6, tz_b / 1e6 / tz); return 0; }
    void *(*al)(void) = (void *(*)(void))dlsym(L, "libdeflate_alloc_decompressor");
    int (*de)(void *, const void *, size_t, void *, size_t, size_t *) =
        (int (*)(void *, const void *, size_t, void *, size_t, size_t *))dlsym(L, "libdeflate_deflate_decompress");
    uint32_t (*cr)(uint32_t, const void *, size_t) = (uint32_t (*)(uint32_t, const void *, size_t))dlsym(L, "libdeflate_crc32");
    void *d = al();
    t = now();
    for (size_t i = 0; i < nb; i++) {
        size_t got = 0;
        de(d, blk[i] + 18, bs[i] - 26, u, sizeof u, &got);
        tl_b += got;
        (void)cr(0, u, got);
    }
    const double tl = now() - t;
    printf("blocks %zu MB %.1f zlib %.0f MB/s libdeflate %.0f MB/s (same bytes: %s)\n", nb, tz_b / 1e6,
           tz_b / 1e6 / tz, tl_b / 1e6 / tl, tz_b == tl_b ? "yes" : "NO");
    return 0;
}
