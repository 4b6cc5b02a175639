/*
 * pf_bam.c -- BAM ingest on the host: a BGZF block reader,
 * the BAM header and record decoder, the BAI index and the region fetch that
 * load_reads_given_interval does per window (reference blockjoin.c:1053-1076,
 * with htslib's hts_open / sam_index_load / sam_itr_querys / sam_itr_next
 * semantics), producing the pf_aln_batch_t that pf_batch_upload_aln takes.
 *
 * Formats follow the SAM/BAM specification (SAMv1 sections 4.1-4.2 and 5.2):
 *   - BGZF: gzip members with a BC extra subfield (BSIZE); virtual offsets
 *     (block address << 16 | offset in the block).  As in htslib, a read
 *     that ends exactly at a block's end leaves the offset at the next
 *     block's start, so chunk ends compare the same way.
 *   - BAI: per reference the bins (with the metadata pseudo-bin 37450) and
 *     the 16 kb linear index.
 * Region fetch (htslib hts_itr_query + hts_itr_next): the region string
 * "chrom:b-E" means the 0-based [max(b-1, 0), E); the chunks of the bins
 * reg2bins gives for it, minus those ending before the linear index's
 * offset, are read in file order; a record stops the fetch when its tid
 * differs or its pos >= E and is returned when pos < E and bam_endpos > beg
 * (bam_endpos: pos + reference length, 1 for unmapped or zero length).
 * bam_read1 refuses a record whose CIGAR query length differs from l_qseq
 * (mapped, l_qseq > 0): sam_itr_next then returns < 0 and the reference's
 * loop ends, so the window's fetch stops there too (counted in
 * n_truncated).  The CG:B:I long-CIGAR tag replaces a kSmN placeholder as
 * bam_tag2cigar does.
 */
#include <dlfcn.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>

#include "../../include/pomfret_amd.h"

/* ------------------------------------------------------------------ */
/* BGZF */
struct bgzf_mt;
typedef struct {
    struct bgzf_mt *mt;      /* multi-threaded read-ahead (bgzf_mt), or NULL */
    FILE *f;
    uint8_t cbuf[65536 + 64];
    uint8_t ubuf[65536];
    int ulen, upos;
    uint64_t caddr;          /* compressed address of the block in ubuf */
    uint64_t next;           /* compressed address of the following block */
    uint64_t fpos;           /* file position after the last fread */
    int eof;
    char *iobuf;
} bgzf_t;

static uint32_t rd16(const uint8_t *p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8); }
static uint32_t rd32(const uint8_t *p) { return rd16(p) | (rd16(p + 2) << 16); }
static uint64_t rd64(const uint8_t *p) { return (uint64_t)rd32(p) | ((uint64_t)rd32(p + 4) << 32); }

/* read the block at compressed address addr into cbuf: its size, or 0 at a
 * clean EOF, <0 on error */
static int bgzf_read_raw(bgzf_t *z, uint64_t addr, uint8_t *h, uint32_t *xlen_out) {
    if (addr != z->fpos) {                    /* sequential blocks keep the stdio buffer */
        if (fseeko(z->f, (off_t)addr, SEEK_SET) != 0) return -1;
        z->fpos = addr;
    }
    size_t got = fread(h, 1, 18, z->f);
    z->fpos += got;
    if (got == 0) return 0;
    if (got < 12 || h[0] != 31 || h[1] != 139 || h[2] != 8 || !(h[3] & 4)) return -2;
    const uint32_t xlen = rd16(h + 10);
    if (xlen < 6 || 12 + xlen > 65536 + 64) return -2;
    if (got < 12 + (size_t)xlen) {
        const size_t k = fread(h + got, 1, 12 + xlen - got, z->f);
        z->fpos += k;
        if (k != 12 + xlen - got) return -2;
        got = 12 + xlen;
    }
    uint32_t bsize = 0;
    for (uint32_t x = 0; x + 4 <= xlen;) {
        const uint8_t *sf = h + 12 + x;
        const uint32_t slen = rd16(sf + 2);
        if (sf[0] == 'B' && sf[1] == 'C' && slen == 2) bsize = rd16(sf + 4) + 1;
        x += 4 + slen;
    }
    if (bsize < 12 + xlen + 8 || bsize > 65536) return -2;
    if (got < bsize) {
        const size_t k = fread(h + got, 1, bsize - got, z->f);
        z->fpos += k;
        if (k != bsize - got) return -2;
    }
    *xlen_out = xlen;
    return (int)bsize;
}

/* libdeflate, when the system has its runtime library (htslib links the same
 * library for its BGZF reads): a raw-DEFLATE decoder about twice zlib's speed
 * on BAM blocks (profiles/r05/host_inflate.txt).  Loaded once with dlopen, as
 * only libdeflate.so.0 ships (no header, no link name); without it, or with
 * PF_HOST_ZLIB set, blocks go through zlib.  Both decode the same bytes. */
typedef struct {
    void *(*alloc)(void);
    void (*free)(void *);
    int (*decompress)(void *, const void *, size_t, void *, size_t, size_t *);
    uint32_t (*crc)(uint32_t, const void *, size_t);
} ldf_t;
static ldf_t g_ldf;
static pthread_once_t g_ldf_once = PTHREAD_ONCE_INIT;
static pthread_key_t g_ldf_key;

static void ldf_init(void) {
    if (getenv("PF_HOST_ZLIB")) return;
    void *L = dlopen("libdeflate.so.0", RTLD_NOW | RTLD_LOCAL);
    if (!L) return;
    void (*fr)(void *) = (void (*)(void *))dlsym(L, "libdeflate_free_decompressor");
    ldf_t t = {(void *(*)(void))dlsym(L, "libdeflate_alloc_decompressor"), fr,
               (int (*)(void *, const void *, size_t, void *, size_t, size_t *))dlsym(L, "libdeflate_deflate_decompress"),
               (uint32_t (*)(uint32_t, const void *, size_t))dlsym(L, "libdeflate_crc32")};
    if (!fr || !t.alloc || !t.decompress || !t.crc || pthread_key_create(&g_ldf_key, fr)) return;
    g_ldf = t;
}

/* this thread's libdeflate decompressor (freed at thread exit), or NULL */
static void *ldf_dec(void) {
    pthread_once(&g_ldf_once, ldf_init);
    if (!g_ldf.alloc) return NULL;
    void *d = pthread_getspecific(g_ldf_key);
    if (!d && (d = g_ldf.alloc()) != NULL && pthread_setspecific(g_ldf_key, d)) {
        g_ldf.free(d);                        /* not registered: this thread decodes through zlib */
        return NULL;
    }
    return d;
}

int pf_host_inflater(void) {
    return ldf_dec() ? 1 : 0;
}

/* inflate + CRC check of one raw block (h, bsize): output bytes or -2 */
static int bgzf_inflate_raw(const uint8_t *h, uint32_t bsize, uint32_t xlen, uint8_t *u) {
    const uint32_t isize = rd32(h + bsize - 4), crc = rd32(h + bsize - 8);
    if (isize > 65536) return -2;
    void *ld = ldf_dec();
    if (ld) {
        size_t out = 0;
        if (g_ldf.decompress(ld, h + 12 + xlen, bsize - 12 - xlen - 8, u, 65536, &out) != 0 || out != isize) return -2;
        if (g_ldf.crc(0, u, out) != crc) return -2;
        return (int)out;
    }
    z_stream zs;
    memset(&zs, 0, sizeof zs);
    if (inflateInit2(&zs, -15) != Z_OK) return -3;
    zs.next_in = (uint8_t *)h + 12 + xlen;
    zs.avail_in = bsize - 12 - xlen - 8;
    zs.next_out = u;
    zs.avail_out = 65536;
    const int rc = inflate(&zs, Z_FINISH);
    const uint32_t out = (uint32_t)zs.total_out;
    inflateEnd(&zs);
    if (rc != Z_STREAM_END || out != isize) return -2;
    if ((uint32_t)crc32(0L, u, out) != crc) return -2;
    return (int)out;
}

/* Multi-threaded read-ahead (htslib's bgzf_mt, which the reference turns on
 * with -t N for its whole-file passes, blockjoin.c:576-578): the reading
 * thread reads the compressed blocks that follow the one it consumes into a
 * ring, and n worker threads inflate them; blocks are handed out in file
 * order.  A load at an address other than the ring's next block (a seek)
 * drains the ring and restarts the read-ahead there. */
typedef struct {
    uint64_t caddr, next;
    uint32_t bsize, xlen;
    int ulen;                 /* inflated bytes, or < 0 on error */
    int state;                /* 0 free, 1 read, 2 inflating, 3 done */
    uint8_t c[65536 + 64];
    uint8_t u[65536];
} mt_blk_t;

typedef struct bgzf_mt {
    int nth, cap;
    pthread_t *th;
    pthread_mutex_t mu;
    pthread_cond_t cv_job, cv_done;
    mt_blk_t *ring;
    uint64_t head, tail, job;     /* consume / read / next-to-inflate indices */
    uint64_t raddr;               /* next compressed address to read */
    int reof, rerr, stop;
} bgzf_mt_t;

static void *mt_worker(void *arg) {
    bgzf_mt_t *M = (bgzf_mt_t *)arg;
    pthread_mutex_lock(&M->mu);
    for (;;) {
        while (!M->stop && M->job == M->tail) pthread_cond_wait(&M->cv_job, &M->mu);
        if (M->stop) break;
        mt_blk_t *B = &M->ring[M->job % (uint64_t)M->cap];
        M->job++;
        B->state = 2;
        pthread_mutex_unlock(&M->mu);
        const int n = bgzf_inflate_raw(B->c, B->bsize, B->xlen, B->u);
        pthread_mutex_lock(&M->mu);
        B->ulen = n;
        B->state = 3;
        pthread_cond_broadcast(&M->cv_done);
    }
    pthread_mutex_unlock(&M->mu);
    return NULL;
}

/* read ahead into the free slots (the consumer's thread; the lock is not held
 * while reading) */
static void mt_fill(bgzf_t *z) {
    bgzf_mt_t *M = z->mt;
    for (;;) {
        pthread_mutex_lock(&M->mu);
        const int room = !M->reof && M->tail - M->head < (uint64_t)M->cap;
        mt_blk_t *B = room ? &M->ring[M->tail % (uint64_t)M->cap] : NULL;
        pthread_mutex_unlock(&M->mu);
        if (!B) return;
        uint32_t xlen = 0;
        const int bs = bgzf_read_raw(z, M->raddr, B->c, &xlen);
        pthread_mutex_lock(&M->mu);
        if (bs <= 0) {
            M->reof = 1;
            M->rerr = bs;                          /* 0: clean EOF */
        } else {
            B->caddr = M->raddr;
            B->next = M->raddr + (uint64_t)bs;
            B->bsize = (uint32_t)bs;
            B->xlen = xlen;
            B->state = 1;
            M->raddr = B->next;
            M->tail++;
            pthread_cond_signal(&M->cv_job);
        }
        pthread_mutex_unlock(&M->mu);
        if (bs <= 0) return;
    }
}

/* wait for every inflate in flight, then empty the ring (lock held) */
static void mt_drain(bgzf_mt_t *M) {
    while (M->job != M->tail) pthread_cond_wait(&M->cv_done, &M->mu);
    for (uint64_t i = M->head; i < M->tail; i++)
        while (M->ring[i % (uint64_t)M->cap].state == 2) pthread_cond_wait(&M->cv_done, &M->mu);
    for (int i = 0; i < M->cap; i++) M->ring[i].state = 0;
    M->head = M->tail = M->job = 0;
}

static int bgzf_load_mt(bgzf_t *z, uint64_t addr) {
    bgzf_mt_t *M = z->mt;
    pthread_mutex_lock(&M->mu);
    const int hit = M->tail > M->head && M->ring[M->head % (uint64_t)M->cap].caddr == addr;
    const int at_end = M->tail == M->head && M->reof && M->raddr == addr;
    if (!hit && !at_end) {
        mt_drain(M);
        M->raddr = addr;
        M->reof = 0;
        M->rerr = 0;
    }
    pthread_mutex_unlock(&M->mu);
    mt_fill(z);
    pthread_mutex_lock(&M->mu);
    if (M->tail == M->head) {
        const int err = M->rerr;
        pthread_mutex_unlock(&M->mu);
        if (err < 0) return err;
        z->caddr = addr; z->next = addr; z->ulen = z->upos = 0; z->eof = 1;
        return 1;
    }
    mt_blk_t *B = &M->ring[M->head % (uint64_t)M->cap];
    while (B->state != 3) pthread_cond_wait(&M->cv_done, &M->mu);
    pthread_mutex_unlock(&M->mu);
    if (B->ulen < 0) return B->ulen;
    memcpy(z->ubuf, B->u, (size_t)B->ulen);
    z->caddr = B->caddr;
    z->next = B->next;
    z->ulen = B->ulen;
    z->upos = 0;
    z->eof = 0;
    pthread_mutex_lock(&M->mu);
    B->state = 0;
    M->head++;
    pthread_mutex_unlock(&M->mu);
    mt_fill(z);
    return 0;
}

/* n inflate threads for this reader (n <= 1: single-threaded) */
static int bgzf_mt(bgzf_t *z, int n) {
    if (n <= 1 || z->mt) return 0;
    bgzf_mt_t *M = (bgzf_mt_t *)calloc(1, sizeof *M);
    if (!M) return PF_ERR_NOMEM;
    M->nth = n;
    M->cap = 4 * n;
    M->ring = (mt_blk_t *)calloc((size_t)M->cap, sizeof(mt_blk_t));
    M->th = (pthread_t *)calloc((size_t)n, sizeof(pthread_t));
    if (!M->ring || !M->th) { free(M->ring); free(M->th); free(M); return PF_ERR_NOMEM; }
    pthread_mutex_init(&M->mu, NULL);
    pthread_cond_init(&M->cv_job, NULL);
    pthread_cond_init(&M->cv_done, NULL);
    /* the ring starts where the single-threaded reader stands */
    M->raddr = z->ulen > 0 && z->upos < z->ulen ? z->next : z->caddr;
    int made = 0;
    for (int i = 0; i < n; i++) made += pthread_create(&M->th[i], NULL, mt_worker, M) == 0;
    if (made < n) {
        pthread_mutex_lock(&M->mu);
        M->stop = 1;
        pthread_cond_broadcast(&M->cv_job);
        pthread_mutex_unlock(&M->mu);
        for (int i = 0; i < made; i++) pthread_join(M->th[i], NULL);
        free(M->ring); free(M->th); free(M);
        return PF_ERR_INTERNAL;
    }
    z->mt = M;
    return 0;
}

static void bgzf_mt_free(bgzf_t *z) {
    bgzf_mt_t *M = z->mt;
    if (!M) return;
    pthread_mutex_lock(&M->mu);
    mt_drain(M);
    M->stop = 1;
    pthread_cond_broadcast(&M->cv_job);
    pthread_mutex_unlock(&M->mu);
    for (int i = 0; i < M->nth; i++) pthread_join(M->th[i], NULL);
    pthread_mutex_destroy(&M->mu);
    pthread_cond_destroy(&M->cv_job);
    pthread_cond_destroy(&M->cv_done);
    free(M->ring);
    free(M->th);
    free(M);
    z->mt = NULL;
}

/* load the block at compressed address addr; 0 ok, 1 clean EOF, <0 error */
static int bgzf_load(bgzf_t *z, uint64_t addr) {
    if (z->mt) return bgzf_load_mt(z, addr);
    uint32_t xlen = 0;
    const int bsize = bgzf_read_raw(z, addr, z->cbuf, &xlen);
    if (bsize == 0) { z->caddr = addr; z->next = addr; z->ulen = z->upos = 0; z->eof = 1; return 1; }
    if (bsize < 0) return bsize;
    const int out = bgzf_inflate_raw(z->cbuf, (uint32_t)bsize, xlen, z->ubuf);
    if (out < 0) return out;
    z->caddr = addr;
    z->next = addr + (uint64_t)bsize;
    z->ulen = out;
    z->upos = 0;
    z->eof = 0;
    return 0;
}

static int bgzf_seek(bgzf_t *z, uint64_t voff) {
    const uint64_t addr = voff >> 16;
    const int off = (int)(voff & 0xFFFF);
    if (!(z->ulen > 0 && z->caddr == addr)) {
        const int rc = bgzf_load(z, addr);
        if (rc < 0) return rc;
    }
    if (off > z->ulen) return -2;
    z->upos = off;
    return 0;
}

static uint64_t bgzf_tell(const bgzf_t *z) { return (z->caddr << 16) | (uint64_t)z->upos; }

/* n bytes; returns n, 0 at a clean EOF before any byte, <0 otherwise */
static int64_t bgzf_read(bgzf_t *z, void *dst, size_t n) {
    uint8_t *d = (uint8_t *)dst;
    size_t done = 0;
    while (done < n) {
        if (z->upos >= z->ulen) {
            int rc;
            do { rc = bgzf_load(z, z->next); } while (rc == 0 && z->ulen == 0);   /* skip empty blocks */
            if (rc == 1) return done == 0 ? 0 : -2;
            if (rc < 0) return rc;
        }
        size_t k = (size_t)(z->ulen - z->upos);
        if (k > n - done) k = n - done;
        memcpy(d + done, z->ubuf + z->upos, k);
        z->upos += (int)k;
        done += k;
    }
    if (z->upos == z->ulen) {        /* htslib: the offset moves to the next block */
        z->caddr = z->next;
        z->ulen = z->upos = 0;
    }
    return (int64_t)n;
}

static void bgzf_close(bgzf_t *z) {
    bgzf_mt_free(z);
    if (z->f) fclose(z->f);
    z->f = NULL;
    free(z->iobuf);
    z->iobuf = NULL;
}

static int bgzf_open(bgzf_t *z, const char *path) {
    memset(z, 0, sizeof *z);
    z->f = fopen(path, "rb");
    if (!z->f) return -1;
    z->iobuf = (char *)malloc(1 << 20);
    if (z->iobuf) setvbuf(z->f, z->iobuf, _IOFBF, 1 << 20);
    const int rc = bgzf_load(z, 0);
    if (rc != 0) {
        fclose(z->f);
        z->f = NULL;
        free(z->iobuf);
        z->iobuf = NULL;
        return rc == 1 ? PF_ERR_ARG : rc == -1 ? -1 : PF_ERR_ARG;
    }
    return 0;
}

/* ------------------------------------------------------------------ */
/* index */
typedef struct { uint64_t u, v; } chunk_t;
typedef struct {
    uint32_t bin;
    uint32_t n;
    chunk_t *c;
} bin_t;
typedef struct {
    uint32_t n_bin, n_intv;
    bin_t *bins;                 /* sorted by bin number */
    uint64_t *intv;
    int has_meta;
    uint64_t mapped, unmapped;
} ref_idx_t;

struct pf_bam {
    char *path;
    int32_t n_ref;
    char **names;
    uint32_t *lens;
    uint64_t data_off;           /* virtual offset of the first record */
    int32_t n_ref_idx;
    ref_idx_t *idx;
    int64_t n_no_coor;           /* the index's count of unplaced records; -1 when it has none */
    int n_threads;               /* inflate threads of the whole-file / whole-contig passes */
};

static int cmp_bin(const void *a, const void *b) {
    const uint32_t x = ((const bin_t *)a)->bin, y = ((const bin_t *)b)->bin;
    return x < y ? -1 : x > y;
}

static uint8_t *slurp(const char *path, size_t *n) {
    FILE *f = fopen(path, "rb");
    if (!f) return NULL;
    size_t cap = 1 << 16, len = 0;
    uint8_t *buf = (uint8_t *)malloc(cap);
    for (;;) {
        if (!buf) { fclose(f); return NULL; }
        const size_t k = fread(buf + len, 1, cap - len, f);
        len += k;
        if (len < cap) break;
        cap *= 2;
        uint8_t *nb = (uint8_t *)realloc(buf, cap);
        if (!nb) { free(buf); fclose(f); return NULL; }
        buf = nb;
    }
    fclose(f);
    *n = len;
    return buf;
}

static int load_bai(pf_bam_t *b, const char *path) {
    size_t n = 0;
    uint8_t *d = slurp(path, &n);
    if (!d) return -1;
    int rc = PF_ERR_ARG;
    size_t o = 8;
    if (n < 8 || memcmp(d, "BAI\1", 4) != 0) goto out;
    const int32_t nr = (int32_t)rd32(d + 4);
    if (nr < 0) goto out;
    b->n_ref_idx = nr;
    b->idx = (ref_idx_t *)calloc(nr ? (size_t)nr : 1, sizeof(ref_idx_t));
    if (!b->idx) { rc = PF_ERR_NOMEM; goto out; }
    for (int32_t r = 0; r < nr; r++) {
        ref_idx_t *ri = &b->idx[r];
        if (o + 4 > n) goto out;
        const uint32_t nb = rd32(d + o);
        o += 4;
        ri->bins = (bin_t *)calloc(nb ? nb : 1, sizeof(bin_t));
        if (!ri->bins) { rc = PF_ERR_NOMEM; goto out; }
        uint32_t k = 0;
        for (uint32_t i = 0; i < nb; i++) {
            if (o + 8 > n) goto out;
            const uint32_t bin = rd32(d + o), nc = rd32(d + o + 4);
            o += 8;
            if (nc > (n - o) / 16) goto out;
            if (bin == 37450) {                       /* metadata pseudo-bin */
                if (nc >= 2) {
                    ri->has_meta = 1;
                    ri->mapped = rd64(d + o + 16);
                    ri->unmapped = rd64(d + o + 24);
                }
                o += 16ull * nc;
                continue;
            }
            bin_t *bb = &ri->bins[k++];
            bb->bin = bin;
            bb->n = nc;
            bb->c = (chunk_t *)malloc((nc ? nc : 1) * sizeof(chunk_t));
            if (!bb->c) { rc = PF_ERR_NOMEM; goto out; }
            for (uint32_t c = 0; c < nc; c++) {
                bb->c[c].u = rd64(d + o);
                bb->c[c].v = rd64(d + o + 8);
                o += 16;
            }
        }
        ri->n_bin = k;
        qsort(ri->bins, k, sizeof(bin_t), cmp_bin);
        if (o + 4 > n) goto out;
        const uint32_t ni = rd32(d + o);
        o += 4;
        if (ni > (n - o) / 8) goto out;
        ri->n_intv = ni;
        ri->intv = (uint64_t *)malloc((ni ? ni : 1) * sizeof(uint64_t));
        if (!ri->intv) { rc = PF_ERR_NOMEM; goto out; }
        for (uint32_t i = 0; i < ni; i++) ri->intv[i] = rd64(d + o + 8ull * i);
        o += 8ull * ni;
    }
    b->n_no_coor = o + 8 <= n ? (int64_t)(rd64(d + o) & 0x7FFFFFFFFFFFFFFFull) : -1;
    rc = PF_OK;
out:
    free(d);
    return rc;
}

static int load_header(pf_bam_t *b) {
    bgzf_t *z = (bgzf_t *)malloc(sizeof(bgzf_t));
    if (!z) return PF_ERR_NOMEM;
    int rc = bgzf_open(z, b->path);
    if (rc) { free(z); return rc; }
    uint8_t h[8];
    rc = PF_ERR_ARG;
    if (bgzf_read(z, h, 8) != 8 || memcmp(h, "BAM\1", 4) != 0) goto out;
    {
        const uint32_t lt = rd32(h + 4);
        char *text = (char *)malloc(lt ? lt : 1);
        if (!text) { rc = PF_ERR_NOMEM; goto out; }
        const int64_t g = bgzf_read(z, text, lt);
        free(text);
        if (g != (int64_t)lt) goto out;
    }
    uint8_t w[4];
    if (bgzf_read(z, w, 4) != 4) goto out;
    b->n_ref = (int32_t)rd32(w);
    if (b->n_ref < 0) goto out;
    b->names = (char **)calloc(b->n_ref ? (size_t)b->n_ref : 1, sizeof(char *));
    b->lens = (uint32_t *)calloc(b->n_ref ? (size_t)b->n_ref : 1, sizeof(uint32_t));
    if (!b->names || !b->lens) { rc = PF_ERR_NOMEM; goto out; }
    for (int32_t r = 0; r < b->n_ref; r++) {
        if (bgzf_read(z, w, 4) != 4) goto out;
        const uint32_t ln = rd32(w);
        if (ln == 0 || ln > (1u << 20)) goto out;
        b->names[r] = (char *)malloc(ln);
        if (!b->names[r]) { rc = PF_ERR_NOMEM; goto out; }
        if (bgzf_read(z, b->names[r], ln) != (int64_t)ln) goto out;
        b->names[r][ln - 1] = 0;
        if (bgzf_read(z, w, 4) != 4) goto out;
        b->lens[r] = rd32(w);
    }
    b->data_off = bgzf_tell(z);
    rc = PF_OK;
out:
    bgzf_close(z);
    free(z);
    return rc;
}

int pf_bam_open(const char *bam_path, const char *bai_path, pf_bam_t **out) {
    if (!out || (!bam_path && !bai_path)) return PF_ERR_ARG;
    *out = NULL;
    pf_bam_t *b = (pf_bam_t *)calloc(1, sizeof(pf_bam_t));
    if (!b) return PF_ERR_NOMEM;
    int rc = PF_OK;
    if (bam_path) {
        b->path = strdup(bam_path);
        if (!b->path) { pf_bam_close(b); return PF_ERR_NOMEM; }
        rc = load_header(b);
        if (rc) { pf_bam_close(b); return rc; }
    }
    if (bai_path) rc = load_bai(b, bai_path);
    else {
        const size_t L = strlen(bam_path);
        char *p = (char *)malloc(L + 5);
        if (!p) { pf_bam_close(b); return PF_ERR_NOMEM; }
        memcpy(p, bam_path, L);
        memcpy(p + L, ".bai", 5);
        rc = load_bai(b, p);
        if (rc == -1 && L > 4 && strcmp(bam_path + L - 4, ".bam") == 0) {
            memcpy(p + L - 4, ".bai", 5);
            rc = load_bai(b, p);
        }
        free(p);
    }
    if (rc) { pf_bam_close(b); return rc; }
    if (bam_path && b->n_ref_idx != b->n_ref) { pf_bam_close(b); return PF_ERR_ARG; }
    *out = b;
    return PF_OK;
}

void pf_bam_close(pf_bam_t *b) {
    if (!b) return;
    for (int32_t r = 0; r < b->n_ref; r++) free(b->names ? b->names[r] : NULL);
    free(b->names);
    free(b->lens);
    for (int32_t r = 0; b->idx && r < b->n_ref_idx; r++) {
        for (uint32_t i = 0; i < b->idx[r].n_bin; i++) free(b->idx[r].bins[i].c);
        free(b->idx[r].bins);
        free(b->idx[r].intv);
    }
    free(b->idx);
    free(b->path);
    free(b);
}

const char *pf_bam_path(const pf_bam_t *b) { return b ? b->path : NULL; }
void pf_bam_set_threads(pf_bam_t *b, int n) { if (b) b->n_threads = n; }
int64_t pf_bam_n_no_coor(const pf_bam_t *b) { return b ? b->n_no_coor : -1; }

int32_t pf_bam_n_targets(const pf_bam_t *b) { return b ? (b->path ? b->n_ref : b->n_ref_idx) : 0; }
const char *pf_bam_target_name(const pf_bam_t *b, int32_t tid) {
    return b && b->names && tid >= 0 && tid < b->n_ref ? b->names[tid] : NULL;
}
uint32_t pf_bam_target_len(const pf_bam_t *b, int32_t tid) {
    return b && b->lens && tid >= 0 && tid < b->n_ref ? b->lens[tid] : 0;
}
int32_t pf_bam_tid(const pf_bam_t *b, const char *name) {
    if (!b || !name || !b->names) return -1;
    for (int32_t r = 0; r < b->n_ref; r++)
        if (strcmp(b->names[r], name) == 0) return r;
    return -1;
}
int pf_bam_index_stats(const pf_bam_t *b, int32_t tid, uint64_t *mapped, uint64_t *unmapped) {
    if (!b || tid < 0 || tid >= b->n_ref_idx || !b->idx[tid].has_meta) return PF_ERR_ARG;
    if (mapped) *mapped = b->idx[tid].mapped;
    if (unmapped) *unmapped = b->idx[tid].unmapped;
    return PF_OK;
}

/* ------------------------------------------------------------------ */
/* growable arrays of one fetch */
typedef struct {
    uint8_t *p;
    size_t n, cap;
} vbuf_t;

static int vb_put(vbuf_t *v, const void *src, size_t n) {
    if (v->n + n > v->cap) {
        size_t c = v->cap ? v->cap : 256;
        while (c < v->n + n) c *= 2;
        uint8_t *np = (uint8_t *)realloc(v->p, c);
        if (!np) return PF_ERR_NOMEM;
        v->p = np;
        v->cap = c;
    }
    if (n) memcpy(v->p + v->n, src, n);
    v->n += n;
    return 0;
}

enum { F_FLAG, F_MAPQ, F_POS, F_LQ, F_DE, F_HP, F_HPTAG, F_END, F_CIG, F_SEQ, F_MM, F_ML, F_QN,
       F_CIGOFF, F_SEQOFF, F_MMOFF, F_MLOFF, F_QNOFF, NF };
/* reads mode (-u pre-pass): F_POS start, F_END bam_endpos, F_LQ l_qseq, F_MM the MD text */

typedef struct {
    vbuf_t f[NF];
    uint64_t n_recs;
    uint64_t truncated;
} recbuf_t;

static void rb_free(recbuf_t *r) {
    for (int i = 0; i < NF; i++) free(r->f[i].p);
    memset(r, 0, sizeof *r);
}

/* aux field size past its 3-byte tag+type header; 0 for an unknown type */
static size_t aux_size(const uint8_t *p, const uint8_t *end) {
    const uint8_t t = p[2];
    const uint8_t *v = p + 3;
    switch (t) {
    case 'A': case 'c': case 'C': return 1;
    case 's': case 'S': return 2;
    case 'i': case 'I': case 'f': return 4;
    case 'd': return 8;
    case 'Z': case 'H': {
        const uint8_t *q = v;
        while (q < end && *q) q++;
        return q < end ? (size_t)(q - v) + 1 : 0;
    }
    case 'B': {
        if (v + 5 > end) return 0;
        const uint32_t cnt = rd32(v + 1);
        size_t es;
        switch (v[0]) {
        case 'c': case 'C': es = 1; break;
        case 's': case 'S': es = 2; break;
        case 'i': case 'I': case 'f': es = 4; break;
        default: return 0;
        }
        return 5 + (size_t)cnt * es;
    }
    default: return 0;
    }
}

static const uint8_t *aux_find(const uint8_t *aux, const uint8_t *end, const char tag[2]) {
    const uint8_t *p = aux;
    while (p + 3 <= end) {
        const size_t s = aux_size(p, end);
        if (s == 0 || p + 3 + s > end) return NULL;
        if (p[0] == (uint8_t)tag[0] && p[1] == (uint8_t)tag[1]) return p;
        p += 3 + s;
    }
    return NULL;
}

static int aux_int(const uint8_t *p, int64_t *out) {     /* bam_aux2i for integer types */
    const uint8_t *v = p + 3;
    switch (p[2]) {
    case 'c': *out = (int8_t)v[0]; return 1;
    case 'C': *out = v[0]; return 1;
    case 's': *out = (int16_t)rd16(v); return 1;
    case 'S': *out = rd16(v); return 1;
    case 'i': *out = (int32_t)rd32(v); return 1;
    case 'I': *out = rd32(v); return 1;
    default: return 0;
    }
}

static double aux_f(const uint8_t *p) {                  /* bam_aux2f */
    const uint8_t *v = p + 3;
    int64_t x;
    if (p[2] == 'd') { double d; memcpy(&d, v, 8); return d; }
    if (p[2] == 'f') { float f; memcpy(&f, v, 4); return f; }
    if (aux_int(p, &x)) return (double)x;
    return 0.0;
}

/* one decoded record, pointing into the caller's buffer */
typedef struct {
    int32_t tid, pos;
    uint32_t l_qseq, n_cigar;
    uint16_t flag;
    uint8_t mapq;
    const char *qname;
    uint32_t l_qname;
    const uint8_t *cigar;     /* n_cigar little-endian u32 */
    const uint8_t *seq;
    const uint8_t *aux, *aux_end;
} rec_t;

/* decode; 0 ok, <0 corrupt */
static int rec_decode(const uint8_t *d, uint32_t bs, rec_t *r) {
    if (bs < 32) return -1;
    r->tid = (int32_t)rd32(d);
    r->pos = (int32_t)rd32(d + 4);
    const uint32_t lrn = d[8];
    r->mapq = d[9];
    r->n_cigar = rd16(d + 12);
    r->flag = (uint16_t)rd16(d + 14);
    const int32_t lseq = (int32_t)rd32(d + 16);
    if (lseq < 0 || lrn == 0) return -1;
    r->l_qseq = (uint32_t)lseq;
    uint64_t o = 32;
    r->qname = (const char *)(d + o);
    r->l_qname = lrn;
    o += lrn;
    r->cigar = d + o;
    o += 4ull * r->n_cigar;
    r->seq = d + o;
    o += (r->l_qseq + 1ull) / 2;
    o += r->l_qseq;                                     /* qual */
    if (o > bs) return -1;
    r->aux = d + o;
    r->aux_end = d + bs;
    return 0;
}

static uint64_t cigar_rlen(const uint8_t *cg, uint32_t n, uint64_t *qlen) {
    uint64_t rl = 0, ql = 0;
    for (uint32_t i = 0; i < n; i++) {
        const uint32_t c = rd32(cg + 4ull * i), op = c & 15u, ln = c >> 4;
        if (op == 0 || op == 2 || op == 3 || op == 7 || op == 8) rl += ln;
        if (op == 0 || op == 1 || op == 4 || op == 7 || op == 8) ql += ln;
    }
    if (qlen) *qlen = ql;
    return rl;
}

/* the records of one region [beg, end) of tid into rb */
typedef struct {
    const pf_bam_t *b;
    int32_t tid;
    bgzf_t z;
    uint8_t *rec;
    size_t rec_cap;
    chunk_t *chunks;
    size_t chunk_cap;
    int reads_mode;           /* 1: pre_haplotagging_read_in_one_ref's records (1869-1871);
                                 2: every record (the rescue pass, 2510-2545) */
} fetcher_t;

static int push_record(recbuf_t *rb, const rec_t *r, const uint8_t *cg, uint32_t ncg) {
    int rc = 0;
    const uint32_t pos = (uint32_t)r->pos, lq = r->l_qseq;
    float de = -1.f;
    const uint8_t *t = aux_find(r->aux, r->aux_end, "de");
    if (t) de = (float)aux_f(t);
    int32_t hp_tag = INT32_MIN;
    uint8_t hp = 254;
    t = aux_find(r->aux, r->aux_end, "HP");
    if (t) {
        int64_t v = 0;
        if (!aux_int(t, &v)) v = 0;                     /* bam_aux2i of a non-integer: 0 */
        hp_tag = v < INT32_MIN ? INT32_MIN + 1 : v > INT32_MAX ? INT32_MAX : (int32_t)v;
        /* get_hp_from_aln: 0 -> unphased, else HP-1 (an int); values outside
         * 1..255 are kept as unphased (the batch holds u8 tags) */
        hp = (v >= 1 && v <= 255) ? (uint8_t)(v - 1) : 254;
    }
    const uint8_t *mm = aux_find(r->aux, r->aux_end, "MM");
    if (!mm) mm = aux_find(r->aux, r->aux_end, "Mm");
    const uint8_t *ml = aux_find(r->aux, r->aux_end, "ML");
    if (!ml) ml = aux_find(r->aux, r->aux_end, "Ml");
    const char *mmz = NULL;
    size_t mml = 0;
    const uint8_t *mlv = NULL;
    uint32_t mln = 0;
    int mods_ok = 1;
    if (mm && mm[2] != 'Z') mods_ok = 0;
    if (ml && (ml[2] != 'B' || ml[3] != 'C')) mods_ok = 0;
    if (mods_ok && mm) {
        mmz = (const char *)(mm + 3);
        mml = strlen(mmz);
        if (ml) { mln = rd32(ml + 4); mlv = ml + 8; }
    }
    uint64_t off;
#define PUTV(fi, ptr, nb) do { if ((rc = vb_put(&rb->f[fi], (ptr), (nb)))) return rc; } while (0)
    PUTV(F_FLAG, &r->flag, 2);
    PUTV(F_MAPQ, &r->mapq, 1);
    PUTV(F_POS, &pos, 4);
    PUTV(F_LQ, &lq, 4);
    PUTV(F_DE, &de, 4);
    PUTV(F_HP, &hp, 1);
    PUTV(F_HPTAG, &hp_tag, 4);
    off = rb->f[F_CIG].n / 4; PUTV(F_CIGOFF, &off, 8);
    PUTV(F_CIG, cg, 4ull * ncg);
    off = rb->f[F_SEQ].n; PUTV(F_SEQOFF, &off, 8);
    PUTV(F_SEQ, r->seq, (lq + 1ull) / 2);
    off = rb->f[F_MM].n; PUTV(F_MMOFF, &off, 8);
    if (mml) PUTV(F_MM, mmz, mml);
    off = rb->f[F_ML].n; PUTV(F_MLOFF, &off, 8);
    if (mln) PUTV(F_ML, mlv, mln);
    off = rb->f[F_QN].n; PUTV(F_QNOFF, &off, 8);
    PUTV(F_QN, r->qname, strnlen(r->qname, r->l_qname));
#undef PUTV
    rb->n_recs++;
    return 0;
}

/* -u pre-pass record: primary mapped only, MD:Z required (the reference
 * asserts on it, 1594-1595) */
static int push_read(recbuf_t *rb, const rec_t *r, const uint8_t *cg, uint32_t ncg, uint32_t end) {
    int rc = 0;
    const uint8_t *md = aux_find(r->aux, r->aux_end, "MD");
    if (!md || md[2] != 'Z') return PF_ERR_ARG;
    const char *mdz = (const char *)(md + 3);
    const size_t mdl = strlen(mdz);
    const uint32_t pos = (uint32_t)r->pos, lq = r->l_qseq;
    uint64_t off;
#define PUTV(fi, ptr, nb) do { if ((rc = vb_put(&rb->f[fi], (ptr), (nb)))) return rc; } while (0)
    PUTV(F_POS, &pos, 4);
    PUTV(F_END, &end, 4);
    PUTV(F_LQ, &lq, 4);
    off = rb->f[F_CIG].n / 4; PUTV(F_CIGOFF, &off, 8);
    PUTV(F_CIG, cg, 4ull * ncg);
    off = rb->f[F_SEQ].n; PUTV(F_SEQOFF, &off, 8);
    PUTV(F_SEQ, r->seq, (lq + 1ull) / 2);
    off = rb->f[F_MM].n; PUTV(F_MMOFF, &off, 8);
    if (mdl) PUTV(F_MM, mdz, mdl);
    off = rb->f[F_QN].n; PUTV(F_QNOFF, &off, 8);
    PUTV(F_QN, r->qname, strnlen(r->qname, r->l_qname));
#undef PUTV
    rb->n_recs++;
    return 0;
}

/* rescue pass record: pos, get_hp_from_aln, CIGAR, MD (F_FLAG = 1 when present), qname */
static int push_any(recbuf_t *rb, const rec_t *r, const uint8_t *cg, uint32_t ncg) {
    int rc = 0;
    const uint8_t *md = aux_find(r->aux, r->aux_end, "MD");
    const uint16_t has_md = (md && md[2] == 'Z') ? 1 : 0;
    const char *mdz = has_md ? (const char *)(md + 3) : "";
    const size_t mdl = strlen(mdz);
    uint8_t hp = 254;
    const uint8_t *t = aux_find(r->aux, r->aux_end, "HP");
    if (t) {
        int64_t v = 0;
        if (!aux_int(t, &v)) v = 0;
        hp = (v >= 1 && v <= 255) ? (uint8_t)(v - 1) : 254;
    }
    const uint32_t pos = (uint32_t)r->pos;
    uint64_t off;
#define PUTV(fi, ptr, nb) do { if ((rc = vb_put(&rb->f[fi], (ptr), (nb)))) return rc; } while (0)
    PUTV(F_POS, &pos, 4);
    PUTV(F_FLAG, &has_md, 2);
    PUTV(F_HP, &hp, 1);
    off = rb->f[F_CIG].n / 4; PUTV(F_CIGOFF, &off, 8);
    PUTV(F_CIG, cg, 4ull * ncg);
    off = rb->f[F_MM].n; PUTV(F_MMOFF, &off, 8);
    if (mdl) PUTV(F_MM, mdz, mdl);
    off = rb->f[F_QN].n; PUTV(F_QNOFF, &off, 8);
    PUTV(F_QN, r->qname, strnlen(r->qname, r->l_qname));
#undef PUTV
    rb->n_recs++;
    return 0;
}

static int cmp_chunk(const void *a, const void *b) {
    const uint64_t x = ((const chunk_t *)a)->u, y = ((const chunk_t *)b)->u;
    return x < y ? -1 : x > y;
}

/* the index chunks of region [beg, end) of tid, sorted by start offset
 * (hts_itr_query's chunk list before it walks them) */
static int64_t region_chunks(const pf_bam_t *b, int32_t tid, int64_t beg, int64_t end, chunk_t **buf, size_t *cap) {
    const ref_idx_t *ri = &b->idx[tid];
    if (end <= beg) return 0;
    /* the bins reg2bins(beg, end) lists are exactly the index bins whose
     * interval overlaps [beg, end): level l bin k covers
     * [(k - first_l) << shift_l, (k - first_l + 1) << shift_l) */
    uint64_t min_off = 0;
    if (ri->n_intv) {
        const int64_t li = beg >> 14;
        min_off = li >= (int64_t)ri->n_intv ? ri->intv[ri->n_intv - 1] : ri->intv[li];
    }
    size_t nc = 0;
    static const uint32_t first[6] = {0, 1, 9, 73, 585, 4681};
    static const int shift[6] = {29, 26, 23, 20, 17, 14};
    for (uint32_t i = 0; i < ri->n_bin; i++) {
        const bin_t *bb = &ri->bins[i];
        if (bb->bin > 37449) continue;
        int l = 5;
        while (l > 0 && bb->bin < first[l]) l--;
        const int64_t lo = (int64_t)(bb->bin - first[l]) << shift[l], hi = lo + ((int64_t)1 << shift[l]);
        if (!(lo < end && hi > beg)) continue;
        for (uint32_t c = 0; c < bb->n; c++) {
            if (bb->c[c].v <= min_off) continue;
            if (nc == *cap) {
                const size_t ncap = *cap ? 2 * *cap : 64;
                chunk_t *np = (chunk_t *)realloc(*buf, ncap * sizeof(chunk_t));
                if (!np) return PF_ERR_NOMEM;
                *buf = np;
                *cap = ncap;
            }
            (*buf)[nc++] = bb->c[c];
        }
    }
    if (nc) qsort(*buf, nc, sizeof(chunk_t), cmp_chunk);
    return (int64_t)nc;
}

int64_t pf_bam_query_chunks(const pf_bam_t *b, int32_t tid, int64_t beg, int64_t end, uint64_t *uv, uint64_t cap) {
    if (!b || tid < 0 || tid >= b->n_ref_idx || (cap && !uv)) return PF_ERR_ARG;
    chunk_t *buf = NULL;
    size_t bcap = 0;
    const int64_t n = region_chunks(b, tid, beg, end, &buf, &bcap);
    for (int64_t i = 0; i < n && (uint64_t)i < cap; i++) { uv[2 * i] = buf[i].u; uv[2 * i + 1] = buf[i].v; }
    free(buf);
    return n;
}

static int fetch_region(fetcher_t *F, int64_t beg, int64_t end, recbuf_t *rb) {
    const int64_t nci = region_chunks(F->b, F->tid, beg, end, &F->chunks, &F->chunk_cap);
    if (nci <= 0) return (int)nci;
    const size_t nc = (size_t)nci;
    uint64_t done = 0;                          /* records before this offset were read */
    for (size_t c = 0; c < nc; c++) {
        uint64_t at = F->chunks[c].u > done ? F->chunks[c].u : done;
        if (at >= F->chunks[c].v) continue;
        int rc = bgzf_seek(&F->z, at);
        if (rc) return PF_ERR_ARG;
        while (bgzf_tell(&F->z) < F->chunks[c].v) {
            uint8_t w[4];
            const int64_t g = bgzf_read(&F->z, w, 4);
            if (g == 0) return 0;
            if (g != 4) return PF_ERR_ARG;
            const uint32_t bs = rd32(w);
            if (bs < 32 || bs > (1u << 30)) return PF_ERR_ARG;
            if (bs > F->rec_cap) {
                uint8_t *np = (uint8_t *)realloc(F->rec, bs);
                if (!np) return PF_ERR_NOMEM;
                F->rec = np;
                F->rec_cap = bs;
            }
            if (bgzf_read(&F->z, F->rec, bs) != (int64_t)bs) return PF_ERR_ARG;
            done = bgzf_tell(&F->z);
            rec_t r;
            if (rec_decode(F->rec, bs, &r)) return PF_ERR_ARG;
            /* bam_tag2cigar: a kSmN placeholder with a CG:B:I / B:i tag */
            const uint8_t *cg = r.cigar;
            uint32_t ncg = r.n_cigar;
            if (ncg > 0 && r.tid >= 0 && r.pos >= 0 && (rd32(cg) & 15u) == 4u && (rd32(cg) >> 4) == r.l_qseq) {
                const uint8_t *t = aux_find(r.aux, r.aux_end, "CG");
                if (t && t[2] == 'B' && (t[3] == 'I' || t[3] == 'i')) {
                    const uint32_t n = rd32(t + 4);
                    if (n >= r.n_cigar && n < (1u << 29)) { cg = t + 8; ncg = n; }
                }
            }
            uint64_t qlen = 0;
            uint64_t rlen = cigar_rlen(cg, ncg, &qlen);
            if (ncg > 0 && r.l_qseq > 0 && !(r.flag & 4) && qlen != r.l_qseq) {
                rb->truncated++;                        /* bam_read1 -> -4: the fetch ends */
                return 0;
            }
            if ((r.flag & 4) || ncg == 0) rlen = 0;
            if (rlen == 0) rlen = 1;
            if (r.tid != F->tid || (int64_t)r.pos >= end) return 0;
            if ((int64_t)r.pos + (int64_t)rlen > beg) {
                if (!F->reads_mode) rc = push_record(rb, &r, cg, ncg);
                else if (F->reads_mode == 2) rc = push_any(rb, &r, cg, ncg);
                else if (!(r.flag & (4 | 256 | 2048))) rc = push_read(rb, &r, cg, ncg, (uint32_t)(r.pos + rlen));
                if (rc) return rc;
            }
        }
    }
    return 0;
}

typedef struct {
    const pf_bam_t *b;
    int32_t tid;
    const uint32_t *ws, *we;
    uint32_t w0, w1, readback;
    recbuf_t *out;            /* one per window */
    uint64_t *win_n;
    int rc;
} job_t;

static void *fetch_job(void *arg) {
    job_t *j = (job_t *)arg;
    fetcher_t F;
    memset(&F, 0, sizeof F);
    F.b = j->b;
    F.tid = j->tid;
    int rc = bgzf_open(&F.z, j->b->path);
    for (uint32_t w = j->w0; !rc && w < j->w1; w++) {
        /* "%s:%d-%d" with (s-readback)>0 ? s-readback : 0 and e+readback (int
         * arithmetic, 1053-1054); htslib reads b-E as the 0-based [b-1, E) */
        const int64_t s = (int32_t)j->ws[w], e = (int32_t)j->we[w], rb = (int32_t)j->readback;
        const int64_t b1 = s - rb > 0 ? s - rb : 0;
        const int64_t beg = b1 > 0 ? b1 - 1 : 0, end = e + rb;
        const uint64_t n0 = j->out->n_recs;
        rc = fetch_region(&F, beg, end, j->out);
        j->win_n[w] = j->out->n_recs - n0;
    }
    bgzf_close(&F.z);
    free(F.rec);
    free(F.chunks);
    j->rc = rc;
    return NULL;
}

struct pf_bam_records_own {
    pf_bam_records_t pub;
    recbuf_t rb;
    uint32_t *ws, *we, *wro;
};

void pf_bam_records_free(pf_bam_records_t *r) {
    if (!r) return;
    struct pf_bam_records_own *o = (struct pf_bam_records_own *)r;
    rb_free(&o->rb);
    free(o->ws);
    free(o->we);
    free(o->wro);
    free(o);
}

int pf_bam_fetch_windows(pf_bam_t *b, const char *chrom, uint32_t W, const uint32_t *ws, const uint32_t *we,
                         uint32_t readback, int n_threads, pf_bam_records_t **out) {
    if (!b || !chrom || !out || (W && (!ws || !we)) || !b->path) return PF_ERR_ARG;
    *out = NULL;
    const int32_t tid = pf_bam_tid(b, chrom);
    if (tid < 0 || tid >= b->n_ref_idx) return PF_ERR_ARG;
    if (n_threads < 1) n_threads = 1;
    if ((uint32_t)n_threads > W) n_threads = W ? (int)W : 1;
    struct pf_bam_records_own *o = (struct pf_bam_records_own *)calloc(1, sizeof *o);
    if (!o) return PF_ERR_NOMEM;
    o->ws = (uint32_t *)malloc((W ? W : 1) * 4ull);
    o->we = (uint32_t *)malloc((W ? W : 1) * 4ull);
    o->wro = (uint32_t *)malloc((W + 1ull) * 4);
    uint64_t *win_n = (uint64_t *)calloc(W ? W : 1, 8);
    recbuf_t *parts = (recbuf_t *)calloc((size_t)n_threads, sizeof(recbuf_t));
    job_t *jobs = (job_t *)calloc((size_t)n_threads, sizeof(job_t));
    pthread_t *th = (pthread_t *)calloc((size_t)n_threads, sizeof(pthread_t));
    int rc = PF_OK;
    if (!o->ws || !o->we || !o->wro || !win_n || !parts || !jobs || !th) rc = PF_ERR_NOMEM;
    if (!rc) {
        if (W) { memcpy(o->ws, ws, 4ull * W); memcpy(o->we, we, 4ull * W); }
        /* contiguous window ranges per thread, so the parts concatenate in window order */
        for (int t = 0; t < n_threads; t++) {
            jobs[t].b = b; jobs[t].tid = tid; jobs[t].ws = ws; jobs[t].we = we; jobs[t].readback = readback;
            jobs[t].w0 = (uint32_t)((uint64_t)W * t / n_threads);
            jobs[t].w1 = (uint32_t)((uint64_t)W * (t + 1) / n_threads);
            jobs[t].out = &parts[t];
            jobs[t].win_n = win_n;
        }
        char *made = (char *)calloc((size_t)n_threads, 1);
        for (int t = 1; t < n_threads; t++)
            if (made) made[t] = pthread_create(&th[t], NULL, fetch_job, &jobs[t]) == 0;
        fetch_job(&jobs[0]);
        for (int t = 1; t < n_threads; t++) {
            if (made && made[t]) pthread_join(th[t], NULL);
            else fetch_job(&jobs[t]);              /* no thread: run it here */
        }
        free(made);
        for (int t = 0; t < n_threads && !rc; t++) rc = jobs[t].rc;
    }
    if (!rc) {
        /* concatenate the parts, rebasing the offsets */
        recbuf_t *R = &o->rb;
        uint64_t base[NF] = {0};
        for (int t = 0; t < n_threads && !rc; t++) {
            recbuf_t *P = &parts[t];
            for (int f = 0; f < F_CIGOFF && !rc; f++) {
                base[f] = R->f[f].n;
                rc = vb_put(&R->f[f], P->f[f].p, P->f[f].n);
            }
            static const int offs[5][2] = {{F_CIGOFF, F_CIG}, {F_SEQOFF, F_SEQ}, {F_MMOFF, F_MM},
                                           {F_MLOFF, F_ML}, {F_QNOFF, F_QN}};
            for (int k = 0; k < 5 && !rc; k++) {
                const uint64_t add = offs[k][1] == F_CIG ? base[F_CIG] / 4 : base[offs[k][1]];
                const uint64_t *src = (const uint64_t *)P->f[offs[k][0]].p;
                for (uint64_t i = 0; i < P->n_recs && !rc; i++) {
                    const uint64_t v = src[i] + add;
                    rc = vb_put(&R->f[offs[k][0]], &v, 8);
                }
            }
            R->n_recs += P->n_recs;
            R->truncated += P->truncated;
        }
        /* closing offsets */
        static const int offs2[5][2] = {{F_CIGOFF, F_CIG}, {F_SEQOFF, F_SEQ}, {F_MMOFF, F_MM}, {F_MLOFF, F_ML},
                                        {F_QNOFF, F_QN}};
        for (int k = 0; k < 5 && !rc; k++) {
            const uint64_t v = offs2[k][1] == F_CIG ? R->f[F_CIG].n / 4 : R->f[offs2[k][1]].n;
            rc = vb_put(&R->f[offs2[k][0]], &v, 8);
        }
        if (!rc && R->n_recs > 0xFFFFFFFFull) rc = PF_ERR_LIMIT;
    }
    if (!rc) {
        uint64_t acc = 0;
        for (uint32_t w = 0; w < W; w++) { o->wro[w] = (uint32_t)acc; acc += win_n[w]; }
        o->wro[W] = (uint32_t)acc;
        recbuf_t *R = &o->rb;
        pf_aln_batch_t *a = &o->pub.aln;
        memset(a, 0, sizeof *a);
        a->n_windows = W;
        a->n_recs = (uint32_t)R->n_recs;
        a->win_start = o->ws;
        a->win_end = o->we;
        a->win_rec_off = o->wro;
        a->flag = (const uint16_t *)R->f[F_FLAG].p;
        a->mapq = R->f[F_MAPQ].p;
        a->pos = (const uint32_t *)R->f[F_POS].p;
        a->l_qseq = (const uint32_t *)R->f[F_LQ].p;
        a->de = (const float *)R->f[F_DE].p;
        a->hp = R->f[F_HP].p;
        a->cigar_off = (const uint64_t *)R->f[F_CIGOFF].p;
        a->cigar = (const uint32_t *)R->f[F_CIG].p;
        a->seq_off = (const uint64_t *)R->f[F_SEQOFF].p;
        a->seq = R->f[F_SEQ].p;
        a->mm_off = (const uint64_t *)R->f[F_MMOFF].p;
        a->mm = (const char *)R->f[F_MM].p;
        a->ml_off = (const uint64_t *)R->f[F_MLOFF].p;
        a->ml = R->f[F_ML].p;
        o->pub.qname_off = (const uint64_t *)R->f[F_QNOFF].p;
        o->pub.qname = (const char *)R->f[F_QN].p;
        o->pub.hp_tag = (const int32_t *)R->f[F_HPTAG].p;
        o->pub.n_truncated = R->truncated;
        /* empty arrays still get a valid pointer */
        static const uint8_t dummy[8] = {0};
        if (!a->flag) a->flag = (const uint16_t *)dummy;
        if (!a->mapq) a->mapq = dummy;
        if (!a->pos) a->pos = (const uint32_t *)dummy;
        if (!a->l_qseq) a->l_qseq = (const uint32_t *)dummy;
        if (!a->de) a->de = (const float *)dummy;
        if (!a->hp) a->hp = dummy;
        if (!a->cigar) a->cigar = (const uint32_t *)dummy;
        if (!a->seq) a->seq = dummy;
        if (!a->mm) a->mm = (const char *)dummy;
        if (!a->ml) a->ml = dummy;
        if (!o->pub.qname) o->pub.qname = (const char *)dummy;
        if (!o->pub.hp_tag) o->pub.hp_tag = (const int32_t *)dummy;
    }
    for (int t = 0; parts && t < n_threads; t++) rb_free(&parts[t]);
    free(parts);
    free(jobs);
    free(th);
    free(win_n);
    if (rc) { pf_bam_records_free(&o->pub); return rc; }
    *out = &o->pub;
    return PF_OK;
}

/* ------------------------------------------------------------------ */
/* -u pre-pass reads of one contig */
struct pf_bam_reads_own {
    pf_bam_reads_t pub;
    recbuf_t rb;
};

void pf_bam_reads_free(pf_bam_reads_t *r) {
    if (!r) return;
    struct pf_bam_reads_own *o = (struct pf_bam_reads_own *)r;
    rb_free(&o->rb);
    free(o);
}

int pf_bam_fetch_contig_reads(pf_bam_t *b, const char *chrom, pf_bam_reads_t **out) {
    if (!b || !chrom || !out || !b->path) return PF_ERR_ARG;
    *out = NULL;
    const int32_t tid = pf_bam_tid(b, chrom);
    if (tid < 0 || tid >= b->n_ref_idx) return PF_ERR_ARG;
    struct pf_bam_reads_own *o = (struct pf_bam_reads_own *)calloc(1, sizeof *o);
    if (!o) return PF_ERR_NOMEM;
    fetcher_t F;
    memset(&F, 0, sizeof F);
    F.b = b;
    F.tid = tid;
    F.reads_mode = 1;
    int rc = bgzf_open(&F.z, b->path);
    if (!rc) rc = bgzf_mt(&F.z, b->n_threads);
    /* sam_itr_querys(idx, hdr, chrom): the whole reference, [0, HTS_POS_MAX) */
    if (!rc) rc = fetch_region(&F, 0, INT64_MAX, &o->rb);
    bgzf_close(&F.z);
    free(F.rec);
    free(F.chunks);
    recbuf_t *R = &o->rb;
    static const int offs[4][2] = {{F_CIGOFF, F_CIG}, {F_SEQOFF, F_SEQ}, {F_MMOFF, F_MM}, {F_QNOFF, F_QN}};
    for (int k = 0; k < 4 && !rc; k++) {
        const uint64_t v = offs[k][1] == F_CIG ? R->f[F_CIG].n / 4 : R->f[offs[k][1]].n;
        rc = vb_put(&R->f[offs[k][0]], &v, 8);
    }
    if (!rc && R->n_recs > 0xFFFFFFFFull) rc = PF_ERR_LIMIT;
    if (rc) { pf_bam_reads_free(&o->pub); return rc; }
    static const uint8_t dummy[8] = {0};
    pf_read_aln_batch_t *a = &o->pub.reads;
    a->n_reads = (uint32_t)R->n_recs;
    a->start = R->f[F_POS].p ? (const uint32_t *)R->f[F_POS].p : (const uint32_t *)dummy;
    a->end = R->f[F_END].p ? (const uint32_t *)R->f[F_END].p : (const uint32_t *)dummy;
    a->seq_len = R->f[F_LQ].p ? (const uint32_t *)R->f[F_LQ].p : (const uint32_t *)dummy;
    a->cigar_off = (const uint64_t *)R->f[F_CIGOFF].p;
    a->cigar = R->f[F_CIG].p ? (const uint32_t *)R->f[F_CIG].p : (const uint32_t *)dummy;
    a->seq_off = (const uint64_t *)R->f[F_SEQOFF].p;
    a->seq = R->f[F_SEQ].p ? R->f[F_SEQ].p : dummy;
    a->md_off = (const uint64_t *)R->f[F_MMOFF].p;
    a->md = R->f[F_MM].p ? (const char *)R->f[F_MM].p : (const char *)dummy;
    o->pub.qname_off = (const uint64_t *)R->f[F_QNOFF].p;
    o->pub.qname = R->f[F_QN].p ? (const char *)R->f[F_QN].p : (const char *)dummy;
    o->pub.n_truncated = R->truncated;
    *out = &o->pub;
    return PF_OK;
}

/* ------------------------------------------------------------------ */
/* recover_variant_phase_in_dropped_intervals (2618-2694) and
 * recover_variant_phase_in_one_interval (2475-2616) for one contig */

typedef struct {                      /* open-addressing qname -> hp table */
    uint64_t *key_off;                /* index into the caller's arrays, or ~0 */
    uint32_t mask;
    const pf_qname_tags_t *t;
} qtab_t;

static uint64_t fnv(const char *s, size_t n) {
    uint64_t h = 1469598103934665603ull;
    for (size_t i = 0; i < n; i++) { h ^= (uint8_t)s[i]; h *= 1099511628211ull; }
    return h;
}

static int qtab_build(qtab_t *q, const pf_qname_tags_t *t) {
    q->t = t;
    uint32_t cap = 16;
    while (cap < 2ull * t->n + 16) cap <<= 1;
    q->mask = cap - 1;
    q->key_off = (uint64_t *)malloc(cap * sizeof(uint64_t));
    if (!q->key_off) return PF_ERR_NOMEM;
    for (uint32_t i = 0; i < cap; i++) q->key_off[i] = ~0ull;
    for (uint32_t i = 0; i < t->n; i++) {       /* first wins */
        const char *nm = t->names + t->off[i];
        const size_t l = t->off[i + 1] - t->off[i];
        uint32_t h = (uint32_t)fnv(nm, l) & q->mask;
        for (;;) {
            const uint64_t k = q->key_off[h];
            if (k == ~0ull) { q->key_off[h] = i; break; }
            if (t->off[k + 1] - t->off[k] == l && memcmp(t->names + t->off[k], nm, l) == 0) break;
            h = (h + 1) & q->mask;
        }
    }
    return 0;
}

static int qtab_get(const qtab_t *q, const char *nm, size_t l) {   /* hp or -1 */
    const pf_qname_tags_t *t = q->t;
    uint32_t h = (uint32_t)fnv(nm, l) & q->mask;
    for (;;) {
        const uint64_t k = q->key_off[h];
        if (k == ~0ull) return -1;
        if (t->off[k + 1] - t->off[k] == l && memcmp(t->names + t->off[k], nm, l) == 0) return t->hp[k];
        h = (h + 1) & q->mask;
    }
}

static int md_type(uint8_t c) {       /* md_op_table (blockjoin.c:94-): digit 0, '^' 1, bases 2, else 4 */
    if (c >= '0' && c <= '9') return 0;
    if (c == '^') return 1;
    switch (c) {
    case 'A': case 'T': case 'C': case 'G': case 'a': case 't': case 'c': case 'g':
    case 'U': case 'u': case 'N': case 'n': return 2;
    default: return 4;
    }
}

typedef struct { uint64_t *a; size_t n, m; } u64v_t;
static int u64_push(u64v_t *v, uint64_t x) {
    if (v->n == v->m) {
        const size_t nm = v->m ? 2 * v->m : 256;
        uint64_t *p = (uint64_t *)realloc(v->a, nm * 8);
        if (!p) return PF_ERR_NOMEM;
        v->a = p;
        v->m = nm;
    }
    v->a[v->n++] = x;
    return 0;
}
static int cmp_u64(const void *a, const void *b) {
    const uint64_t x = *(const uint64_t *)a, y = *(const uint64_t *)b;
    return x < y ? -1 : x > y;
}

/* the positions parse_variants_for_one_read (1545-1691) gives a record's
 * variants: CIGAR I at the current reference position, MD mismatches and
 * ^-deletion runs closed by a number; each pushed as pos<<33 | 1<<32 | hap
 * (the vote needs only the methphased tag).  Returns PF_ERR_ARG for an MD
 * character outside md_op_table (the reference exits, 1621-1624, or asserts
 * on the first character, 1616). */
static int read_var_positions(uint32_t pos0, const uint32_t *cig, uint32_t ncig, const char *md, size_t mdl,
                              uint32_t hap, u64v_t *out) {
    uint32_t ref = pos0;
    int rc;
    for (uint32_t i = 0; i < ncig; i++) {
        const uint32_t op = cig[i] & 15u, l = cig[i] >> 4;
        if (op == 3 || op == 0 || op == 7 || op == 8 || op == 2) ref += l;
        else if (op == 1) { if ((rc = u64_push(out, ((uint64_t)ref << 33) | (1ull << 32) | hap))) return rc; }
    }
    /* md_s[0] is asserted < 4 (1616): an empty MD or a bad first character aborts */
    if (mdl == 0 || md_type((uint8_t)md[0]) == 4) return PF_ERR_ARG;
    ref = pos0;
    int prev = md_type((uint8_t)md[0]);
    size_t prev_i = 0;
    if (prev == 2) {
        if ((rc = u64_push(out, ((uint64_t)ref << 33) | (1ull << 32) | hap))) return rc;
        ref++;
        prev = -1;
    }
    for (size_t i = 1; i < mdl; i++) {
        const int t = md_type((uint8_t)md[i]);
        if (t == 4) return PF_ERR_ARG;
        if (t == prev) continue;
        if (prev == 0) {
            uint32_t l = 0;                  /* natoi of the digit run */
            for (size_t k = prev_i; k < i; k++) l = l * 10u + (uint32_t)(md[k] - '0');
            ref += l;
        } else if (prev == 1) {
            if (t == 0) {
                if ((rc = u64_push(out, ((uint64_t)ref << 33) | (1ull << 32) | hap))) return rc;
                ref += (uint32_t)(i - prev_i - 1);
                prev = t;
                prev_i = i;
            }
            continue;
        }
        if (t == 2) {
            if ((rc = u64_push(out, ((uint64_t)ref << 33) | (1ull << 32) | hap))) return rc;
            ref++;
            prev = -1;
            prev_i = i;
        } else {
            prev = t;
            prev_i = i;
        }
    }
    return 0;
}

struct pf_rescue_own {
    pf_rescue_map_t pub;
    uint32_t *pos;
    uint8_t *hap;
};

void pf_rescue_map_free(pf_rescue_map_t *m) {
    if (!m) return;
    struct pf_rescue_own *o = (struct pf_rescue_own *)m;
    free(o->pos);
    free(o->hap);
    free(o);
}

/* the rescue's dropped intervals of one contig: its known positions per
 * interval (pushed before the reads' variants, 2653-2663) and, per interval,
 * (rp << 8 | hap) in vote order */
typedef struct {
    int32_t tid;
    uint32_t n_drop;
    const uint32_t *drop_start, *drop_end;
    uint64_t *kpos_off;               /* [n_drop + 1] into kpos */
    u64v_t kpos;                      /* known positions as pos << 33 */
    u64v_t *per;                      /* [n_drop] */
} rescue_ctg_t;

typedef struct {
    const pf_bam_t *b;
    const qtab_t *qm, *qr;
    rescue_ctg_t *ctg;
    const uint64_t *item_off;         /* [n_ctg + 1]: intervals of the contigs before */
    uint32_t n_ctg;
    uint64_t n_items;
    atomic_uint_fast64_t *next;
    int rc;
} rescue_job_t;

static int rescue_one(rescue_job_t *J, fetcher_t *F, const rescue_ctg_t *R, uint32_t k, u64v_t *pb) {
    const uint32_t start = R->drop_start[k] - 1u, end = R->drop_end[k] + 1u;
    pb->n = 0;
    int rc = 0;
    for (uint64_t i = R->kpos_off[k]; i < R->kpos_off[k + 1] && !rc; i++) rc = u64_push(pb, R->kpos.a[i]);
    if (rc) return rc;
    /* "%s:%d-%d" of (start, end): htslib's 0-based [start-1, end) */
    const int64_t b1 = (int32_t)start, e1 = (int32_t)end;
    const int64_t beg = b1 > 0 ? b1 - 1 : 0;
    recbuf_t rb;
    memset(&rb, 0, sizeof rb);
    if (R->tid >= 0 && R->tid < J->b->n_ref_idx) {
        F->tid = R->tid;
        rc = fetch_region(F, beg, e1, &rb);
    }
    {                                                              /* closing offsets */
        const uint64_t vq = rb.f[F_QN].n, vc = rb.f[F_CIG].n / 4, vm = rb.f[F_MM].n;
        if (!rc) rc = vb_put(&rb.f[F_QNOFF], &vq, 8);
        if (!rc) rc = vb_put(&rb.f[F_CIGOFF], &vc, 8);
        if (!rc) rc = vb_put(&rb.f[F_MMOFF], &vm, 8);
    }
    const size_t nk = pb->n;
    for (uint64_t r = 0; r < rb.n_recs && !rc; r++) {
        const uint64_t *qo = (const uint64_t *)rb.f[F_QNOFF].p;
        const char *qn = (const char *)rb.f[F_QN].p + qo[r];
        const size_t ql = (size_t)(qo[r + 1] - qo[r]);
        const int hm = qtab_get(J->qm, qn, ql);
        if (hm < 0) continue;
        int hr;
        if (J->qr) { hr = qtab_get(J->qr, qn, ql); if (hr < 0) continue; }
        else hr = ((const uint8_t *)rb.f[F_HP].p)[r];
        if (hr == 254) continue;
        if (!((const uint16_t *)rb.f[F_FLAG].p)[r]) { rc = PF_ERR_ARG; break; }   /* assert(tagd), 1596 */
        const uint64_t *co = (const uint64_t *)rb.f[F_CIGOFF].p, *mo = (const uint64_t *)rb.f[F_MMOFF].p;
        rc = read_var_positions(((const uint32_t *)rb.f[F_POS].p)[r],
                                (const uint32_t *)rb.f[F_CIG].p + co[r], (uint32_t)(co[r + 1] - co[r]),
                                (const char *)rb.f[F_MM].p + mo[r], (size_t)(mo[r + 1] - mo[r]),
                                (uint32_t)hm & 0xFFu, pb);
    }
    rb_free(&rb);
    if (rc || nk == 0) return rc;                                  /* pb.n == 0: goto done */
    qsort(pb->a, pb->n, 8, cmp_u64);
    /* for (i = 0; i < pb.n-1;): a known position sorted last is never visited */
    u64v_t *o = &R->per[k];
    for (size_t i = 0; i + 1 < pb->n && !rc;) {
        if (pb->a[i] & (1ull << 32)) { i++; continue; }
        const uint32_t rp = (uint32_t)(pb->a[i] >> 33);
        uint32_t c[2] = {0, 0};
        size_t j;
        for (j = i + 1; j < pb->n; j++) {
            if (!(pb->a[j] & (1ull << 32))) break;
            if ((uint32_t)(pb->a[j] >> 33) != rp) break;
            const uint32_t h = (uint32_t)pb->a[j] & 0xFFu;
            if (h < 2) c[h]++;
        }
        const uint32_t hap = c[0] > c[1] ? 1u : c[1] > c[0] ? 0u : 254u;
        rc = u64_push(o, ((uint64_t)rp << 8) | hap);
        i = j;
    }
    return rc;
}

static void *rescue_main(void *arg) {
    rescue_job_t *J = (rescue_job_t *)arg;
    fetcher_t F;
    memset(&F, 0, sizeof F);
    F.b = J->b;
    F.reads_mode = 2;
    u64v_t pb = {0};
    int rc = 0, open = 0;
    for (;;) {
        const uint64_t it = atomic_fetch_add(J->next, 1);
        if (it >= J->n_items || rc) break;
        uint32_t c = 0;
        while (J->item_off[c + 1] <= it) c++;
        const rescue_ctg_t *R = &J->ctg[c];
        if (!open && R->tid >= 0 && R->tid < J->b->n_ref_idx) {
            if ((rc = bgzf_open(&F.z, J->b->path))) break;
            open = 1;
        }
        rc = rescue_one(J, &F, R, (uint32_t)(it - J->item_off[c]), &pb);
    }
    if (open) bgzf_close(&F.z);
    free(F.rec);
    free(F.chunks);
    free(pb.a);
    J->rc = rc;
    return NULL;
}

/* recover_variant_phase_in_dropped_intervals (2475-2694) for several contigs
 * at once: the qname tables are built once, every (contig, interval) is a
 * work item taken by `threads` host threads (each with its own file handle),
 * and each contig's results are then taken in interval order, so the last
 * write per position is the serial pass's */
int pf_rescue_dropped_multi(pf_bam_t *b, uint32_t n_ctg, const char *const *chroms, const uint32_t *n_drop,
                            const uint32_t *const *drop_start, const uint32_t *const *drop_end,
                            const pf_known_vars_t *const *known, const pf_qname_tags_t *methphased,
                            const pf_qname_tags_t *raw, int threads, pf_rescue_map_t **out) {
    if (!b || !b->path || !methphased || !out || (n_ctg && (!chroms || !n_drop || !drop_start || !drop_end || !known)))
        return PF_ERR_ARG;
    for (uint32_t c = 0; c < n_ctg; c++) {
        out[c] = NULL;
        if (!chroms[c] || !known[c] || (n_drop[c] && (!drop_start[c] || !drop_end[c]))) return PF_ERR_ARG;
    }
    qtab_t qm = {0}, qr = {0};
    rescue_ctg_t *R = (rescue_ctg_t *)calloc(n_ctg ? n_ctg : 1, sizeof(rescue_ctg_t));
    uint64_t *item_off = (uint64_t *)calloc((size_t)n_ctg + 1, sizeof(uint64_t));
    int rc = (!R || !item_off) ? PF_ERR_NOMEM : 0;
    if (!rc) rc = qtab_build(&qm, methphased);
    if (!rc && raw) rc = qtab_build(&qr, raw);
    for (uint32_t c = 0; c < n_ctg && !rc; c++) {
        rescue_ctg_t *r = &R[c];
        r->tid = pf_bam_tid(b, chroms[c]);
        r->n_drop = n_drop[c];
        r->drop_start = drop_start[c];
        r->drop_end = drop_end[c];
        r->kpos_off = (uint64_t *)calloc((size_t)r->n_drop + 1, sizeof(uint64_t));
        r->per = (u64v_t *)calloc(r->n_drop ? r->n_drop : 1, sizeof(u64v_t));
        if (!r->kpos_off || !r->per) { rc = PF_ERR_NOMEM; break; }
        /* the known-position cursor runs across a contig's intervals in order (2653-2663) */
        const pf_known_vars_t *kv = known[c];
        uint32_t prev_i = 0;
        for (uint32_t k = 0; k < r->n_drop && !rc; k++) {
            const uint32_t start = r->drop_start[k] - 1u, end = r->drop_end[k] + 1u;
            for (uint32_t i = prev_i; i < kv->n; i++) {
                const uint32_t p = kv->pos[i];
                if (p >= start && p < end && (rc = u64_push(&r->kpos, (uint64_t)p << 33))) break;
                if (p >= end) { prev_i = i; break; }
            }
            r->kpos_off[k + 1] = r->kpos.n;
        }
        item_off[c + 1] = item_off[c] + r->n_drop;
    }
    const uint64_t n_items = n_ctg ? item_off[n_ctg] : 0;
    if (!rc && n_items) {
        int nt = threads > 0 ? threads : 1;
        if ((uint64_t)nt > n_items) nt = (int)n_items;
        atomic_uint_fast64_t next;
        atomic_init(&next, 0);
        rescue_job_t *J = (rescue_job_t *)calloc((size_t)nt, sizeof(rescue_job_t));
        pthread_t *th = (pthread_t *)calloc((size_t)nt, sizeof(pthread_t));
        char *made = (char *)calloc((size_t)nt, 1);
        if (!J || !th || !made) rc = PF_ERR_NOMEM;
        for (int t = 0; t < nt && !rc; t++)
            J[t] = (rescue_job_t){b, &qm, raw ? &qr : NULL, R, item_off, n_ctg, n_items, &next, 0};
        if (!rc) {
            for (int t = 1; t < nt; t++) made[t] = pthread_create(&th[t], NULL, rescue_main, &J[t]) == 0;
            rescue_main(&J[0]);
            for (int t = 1; t < nt; t++) {
                if (made[t]) pthread_join(th[t], NULL);
                else rescue_main(&J[t]);
            }
            for (int t = 0; t < nt && !rc; t++) rc = J[t].rc;
        }
        free(J); free(th); free(made);
    }
    for (uint32_t c = 0; c < n_ctg && !rc; c++) {
        /* in interval order: pos << 40 | sequence << 8 | hap; the sort keeps
         * the last write per position (the hash's) */
        const rescue_ctg_t *r = &R[c];
        u64v_t res = {0};
        uint64_t seq = 0;
        for (uint32_t k = 0; k < r->n_drop && !rc; k++)
            for (size_t i = 0; i < r->per[k].n && !rc; i++)
                rc = u64_push(&res, ((r->per[k].a[i] >> 8) << 40) | (seq++ << 8) | (r->per[k].a[i] & 0xFFu));
        struct pf_rescue_own *o = NULL;
        if (!rc) {
            qsort(res.a, res.n, 8, cmp_u64);
            o = (struct pf_rescue_own *)calloc(1, sizeof *o);
            if (o) { o->pos = (uint32_t *)malloc((res.n ? res.n : 1) * 4); o->hap = (uint8_t *)malloc(res.n ? res.n : 1); }
            if (!o || !o->pos || !o->hap) rc = PF_ERR_NOMEM;
            else {
                uint32_t n = 0;
                for (size_t i = 0; i < res.n; i++) {
                    const uint32_t p = (uint32_t)(res.a[i] >> 40);
                    if (i + 1 < res.n && (uint32_t)(res.a[i + 1] >> 40) == p) continue;
                    o->pos[n] = p;
                    o->hap[n] = (uint8_t)(res.a[i] & 0xFFu);
                    n++;
                }
                o->pub.n = n;
                o->pub.pos = o->pos;
                o->pub.hap_of_ref = o->hap;
                out[c] = &o->pub;
            }
        }
        if (rc && o) pf_rescue_map_free(&o->pub);
        free(res.a);
    }
    for (uint32_t c = 0; R && c < n_ctg; c++) {
        for (uint32_t k = 0; R[c].per && k < R[c].n_drop; k++) free(R[c].per[k].a);
        free(R[c].per);
        free(R[c].kpos_off);
        free(R[c].kpos.a);
    }
    free(R);
    free(item_off);
    free(qm.key_off);
    free(qr.key_off);
    if (rc)
        for (uint32_t c = 0; c < n_ctg; c++) { pf_rescue_map_free(out[c]); out[c] = NULL; }
    return rc;
}

int pf_rescue_dropped_mt(pf_bam_t *b, const char *chrom, uint32_t n_drop, const uint32_t *drop_start,
                         const uint32_t *drop_end, const pf_known_vars_t *known, const pf_qname_tags_t *methphased,
                         const pf_qname_tags_t *raw, int threads, pf_rescue_map_t **out) {
    if (!b || !chrom || !known || !methphased || !out || (n_drop && (!drop_start || !drop_end)) || !b->path)
        return PF_ERR_ARG;
    return pf_rescue_dropped_multi(b, 1, &chrom, &n_drop, &drop_start, &drop_end, &known, methphased, raw, threads,
                                   out);
}

int pf_rescue_dropped(pf_bam_t *b, const char *chrom, uint32_t n_drop, const uint32_t *drop_start,
                      const uint32_t *drop_end, const pf_known_vars_t *known, const pf_qname_tags_t *methphased,
                      const pf_qname_tags_t *raw, pf_rescue_map_t **out) {
    return pf_rescue_dropped_mt(b, chrom, n_drop, drop_start, drop_end, known, methphased, raw, 1, out);
}

/* ------------------------------------------------------------------ */
/* estimate_read_coverage_dirtyfast (951-1040): every record from the first
 * one (region "."), per contig bins of 5000 bp (target_len / 5000 of them):
 * a record passing flag 4/256/2048, mapq >= 5, l_qseq >= 15000 and
 * de <= 0.1 adds 1 to the bins of start, start + 5000, ... < bam_endpos;
 * a contig's estimate is the integer mean over its bins, taken when the next
 * contig starts and, for the last one, only when the last record read has a
 * tid >= 0 (refID is reassigned by unplaced reads).  Counts that fall past
 * the last whole bin are dropped (the reference writes past buf.n: they are
 * never summed).  Contigs without reads stay 0. */
int pf_bam_estimate_coverage(pf_bam_t *b, int32_t *covs, int32_t n) {
    if (!b || !b->path || !covs || n < b->n_ref) return PF_ERR_ARG;
    for (int32_t i = 0; i < n; i++) covs[i] = 0;
    bgzf_t *z = (bgzf_t *)malloc(sizeof(bgzf_t));
    if (!z) return PF_ERR_NOMEM;
    int rc = bgzf_open(z, b->path);
    if (rc) { free(z); return rc; }
    rc = bgzf_mt(z, b->n_threads);
    if (!rc) rc = bgzf_seek(z, b->data_off) ? PF_ERR_ARG : 0;
    uint8_t *rec = NULL;
    size_t cap = 0;
    uint64_t *bins = NULL;
    size_t nb = 0, mb = 0;
    int32_t prev = -1, refid = -1;
    const int mod = 5000;
    while (!rc) {
        uint8_t w[4];
        const int64_t g = bgzf_read(z, w, 4);
        if (g == 0) break;
        if (g != 4) { rc = PF_ERR_ARG; break; }
        const uint32_t bs = rd32(w);
        if (bs < 32 || bs > (1u << 30)) { rc = PF_ERR_ARG; break; }
        if (bs > cap) {
            uint8_t *np = (uint8_t *)realloc(rec, bs);
            if (!np) { rc = PF_ERR_NOMEM; break; }
            rec = np;
            cap = bs;
        }
        if (bgzf_read(z, rec, bs) != (int64_t)bs) { rc = PF_ERR_ARG; break; }
        rec_t r;
        if (rec_decode(rec, bs, &r)) { rc = PF_ERR_ARG; break; }
        const uint8_t *cg = r.cigar;
        uint32_t ncg = r.n_cigar;
        if (ncg > 0 && r.tid >= 0 && r.pos >= 0 && (rd32(cg) & 15u) == 4u && (rd32(cg) >> 4) == r.l_qseq) {
            const uint8_t *t = aux_find(r.aux, r.aux_end, "CG");
            if (t && t[2] == 'B' && (t[3] == 'I' || t[3] == 'i')) {
                const uint32_t nn = rd32(t + 4);
                if (nn >= r.n_cigar && nn < (1u << 29)) { cg = t + 8; ncg = nn; }
            }
        }
        uint64_t qlen = 0;
        uint64_t rlen = cigar_rlen(cg, ncg, &qlen);
        if (ncg > 0 && r.l_qseq > 0 && !(r.flag & 4) && qlen != r.l_qseq) break;   /* sam_itr_next < 0 */
        refid = r.tid;
        if (refid < 0) continue;
        if (refid > b->n_ref) continue;                 /* the reference's check is '>' */
        if (refid == b->n_ref) continue;                /* (target_len[n_targets] is out of range) */
        if (refid != prev) {
            if (prev >= 0) {
                uint64_t tot = 0;
                for (size_t i = 0; i < nb; i++) tot += bins[i];
                covs[prev] = nb ? (int32_t)(tot / nb) : 0;
            }
            nb = b->lens[refid] / (uint32_t)mod;
            if (nb > mb) {
                uint64_t *np = (uint64_t *)realloc(bins, nb * 8);
                if (!np) { rc = PF_ERR_NOMEM; break; }
                bins = np;
                mb = nb;
            }
            for (size_t i = 0; i < nb; i++) bins[i] = 0;
            prev = refid;
        }
        if ((r.flag & 4) || (r.flag & 256) || (r.flag & 2048)) continue;
        if (r.mapq < 5) continue;
        float de = -1.f;
        const uint8_t *t = aux_find(r.aux, r.aux_end, "de");
        if (t) de = (float)aux_f(t);
        if (r.l_qseq < 15000) continue;
        if ((double)de > 0.1) continue;
        if ((r.flag & 4) || ncg == 0) rlen = 0;
        if (rlen == 0) rlen = 1;
        const uint32_t st = (uint32_t)r.pos, en = (uint32_t)(r.pos + rlen);
        for (int64_t i = (int32_t)st; i < (int64_t)en; i += mod) {
            const uint64_t k = (uint64_t)i / (uint64_t)mod;
            if (i >= 0 && k < nb) bins[k]++;
        }
    }
    if (!rc && refid >= 0 && refid < b->n_ref && prev >= 0) {
        uint64_t tot = 0;
        for (size_t i = 0; i < nb; i++) tot += bins[i];
        covs[refid] = nb ? (int32_t)(tot / nb) : 0;
    }
    free(bins);
    free(rec);
    bgzf_close(z);
    free(z);
    return rc;
}

/* ------------------------------------------------------------------ */
/* BAM writer: --write-bam (output_modify_bam, blockjoin.c:3022-3103, and
 * the sam_index_build3 call at 4723) and varhaptag (main_varhaptag,
 * 4737-4836).
 *
 * BGZF as htslib's bgzf_write writes it: 0xff00-byte blocks, raw deflate
 * (zlib, window 15, memLevel 8, default strategy) at the given level (htslib's
 * "w" mode: Z_DEFAULT_COMPRESSION), the header flushed into its own block(s)
 * by bam_hdr_write, and bam_write1's bgzf_flush_try: a record that does not
 * fit the current block starts a new one (only records larger than a block
 * straddle blocks).  The index is built as hts_idx_push / hts_idx_finish
 * build it while the file is written (chunks per bin, the 16 kb linear index
 * with leading holes set to the first record's offset and later holes to the
 * previous window's, the metadata pseudo-bin, the unplaced-read count); bins
 * are written in ascending order and htslib's compress_binning (merging bins
 * whose chunks span < 64 KiB of compressed file into their parent, in khash
 * order) is not applied, so the index answers every query alike but is not
 * byte-identical to htslib's -- parity unpinned (htslib is absent here).  The
 * records themselves are copied byte for byte except the HP tag and the bin
 * field, which bam_read1 recomputes from the CIGAR; a CG:B:I
 * long-CIGAR record keeps its placeholder layout (htslib's bam_write1 would
 * re-append the CG tag at the end of the aux data). */

#define BGZF_BLK 0xff00
static const uint8_t BGZF_EOF[28] = {31, 139, 8, 4, 0, 0, 0, 0, 0, 255, 6, 0, 66, 67, 2, 0, 27, 0, 3, 0,
                                     0, 0, 0, 0, 0, 0, 0, 0};

/* one BGZF block: n bytes of ubuf deflated into cbuf; its size, or 0 on error */
static uint32_t bgzf_block(const uint8_t *ubuf, int n, int level, uint8_t *cbuf) {
    z_stream zs;
    memset(&zs, 0, sizeof zs);
    if (deflateInit2(&zs, level, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY) != Z_OK) return 0;
    zs.next_in = (Bytef *)ubuf;
    zs.avail_in = (uInt)n;
    zs.next_out = cbuf + 18;
    zs.avail_out = (uInt)(65536 - 18 - 8);
    const int rc = deflate(&zs, Z_FINISH);
    const uint32_t clen = (uint32_t)zs.total_out;
    deflateEnd(&zs);
    if (rc != Z_STREAM_END) return 0;
    const uint32_t bsize = 18 + clen + 8;
    const uint8_t hdr[16] = {31, 139, 8, 4, 0, 0, 0, 0, 0, 255, 6, 0, 66, 67, 2, 0};
    memcpy(cbuf, hdr, 16);
    cbuf[16] = (uint8_t)((bsize - 1) & 0xff);
    cbuf[17] = (uint8_t)((bsize - 1) >> 8);
    const uint32_t crc = (uint32_t)crc32(crc32(0L, Z_NULL, 0), ubuf, (uInt)n);
    uint8_t *t = cbuf + 18 + clen;
    for (int i = 0; i < 4; i++) { t[i] = (uint8_t)(crc >> (8 * i)); t[4 + i] = (uint8_t)((uint32_t)n >> (8 * i)); }
    return bsize;
}

/* -T / --bam-threads (htslib's bgzf_mt for the output, cli.c:261-264): blocks
 * are queued, deflated by a pool of threads in batches and written in order.
 * Each block is deflated alone with the same parameters, so the file is the
 * same bytes at any thread count.  The index's virtual offsets are taken in
 * block-number space while writing (bgzfw_tell) and moved to file addresses
 * when the last block is written (bgzfw_vmap). */
#define BGZFW_BATCH 16                /* queued blocks per thread */
typedef struct {
    int nt, nq, cap;                  /* threads, queued blocks, queue capacity */
    uint8_t *u, *c;                   /* cap x BGZF_BLK input, cap x 65536 output */
    int *un;
    uint32_t *cs;
    pthread_t *th;
    int made;
    pthread_mutex_t mu;
    pthread_cond_t go, done;
    uint64_t gen;                     /* batch generation */
    int next, left, quit, level;
} bgzfw_pool_t;

typedef struct {
    FILE *f;
    uint8_t ubuf[BGZF_BLK];
    uint8_t cbuf[65536];
    int n;
    uint64_t caddr;              /* compressed address of the block being filled (threaded: its number) */
    int level;
    int err;
    bgzfw_pool_t *pool;          /* NULL: deflated in this thread as it fills */
    uint64_t *baddr;             /* threaded: file address of block i (i <= the blocks written) */
    uint64_t nb, mb;
} bgzfw_t;

static void *bgzfw_worker(void *arg) {
    bgzfw_pool_t *P = (bgzfw_pool_t *)arg;
    uint64_t seen = 0;
    pthread_mutex_lock(&P->mu);
    for (;;) {
        while (!P->quit && P->gen == seen) pthread_cond_wait(&P->go, &P->mu);
        if (P->quit) break;
        seen = P->gen;
        while (P->next < P->nq) {
            const int i = P->next++;
            pthread_mutex_unlock(&P->mu);
            P->cs[i] = bgzf_block(P->u + (size_t)i * BGZF_BLK, P->un[i], P->level, P->c + (size_t)i * 65536);
            pthread_mutex_lock(&P->mu);
            if (--P->left == 0) pthread_cond_signal(&P->done);
        }
    }
    pthread_mutex_unlock(&P->mu);
    return NULL;
}

/* deflate the queued blocks (the pool and this thread), write them in order */
static int bgzfw_drain(bgzfw_t *w) {
    bgzfw_pool_t *P = w->pool;
    if (!P->nq) return 0;
    pthread_mutex_lock(&P->mu);
    P->next = 0;
    P->left = P->nq;
    P->gen++;
    pthread_cond_broadcast(&P->go);
    while (P->next < P->nq) {                         /* this thread takes blocks too */
        const int i = P->next++;
        pthread_mutex_unlock(&P->mu);
        P->cs[i] = bgzf_block(P->u + (size_t)i * BGZF_BLK, P->un[i], P->level, P->c + (size_t)i * 65536);
        pthread_mutex_lock(&P->mu);
        P->left--;
    }
    while (P->left > 0) pthread_cond_wait(&P->done, &P->mu);
    pthread_mutex_unlock(&P->mu);
    for (int i = 0; i < P->nq && !w->err; i++) {
        if (!P->cs[i]) { w->err = PF_ERR_INTERNAL; break; }
        if (fwrite(P->c + (size_t)i * 65536, 1, P->cs[i], w->f) != P->cs[i]) { w->err = -1; break; }
        if (w->nb + 1 >= w->mb) {
            const uint64_t m = w->mb ? 2 * w->mb : 1024;
            uint64_t *a = (uint64_t *)realloc(w->baddr, m * sizeof(uint64_t));
            if (!a) { w->err = PF_ERR_NOMEM; break; }
            w->baddr = a;
            w->mb = m;
        }
        w->baddr[w->nb + 1] = w->baddr[w->nb] + P->cs[i];
        w->nb++;
    }
    P->nq = 0;
    return w->err;
}

static int bgzfw_flush(bgzfw_t *w) {
    if (w->err) return w->err;
    if (w->n == 0) return 0;
    if (w->pool) {
        bgzfw_pool_t *P = w->pool;
        memcpy(P->u + (size_t)P->nq * BGZF_BLK, w->ubuf, (size_t)w->n);
        P->un[P->nq++] = w->n;
        w->caddr++;
        w->n = 0;
        return P->nq == P->cap ? bgzfw_drain(w) : 0;
    }
    const uint32_t bsize = bgzf_block(w->ubuf, w->n, w->level, w->cbuf);
    if (!bsize) return w->err = PF_ERR_INTERNAL;
    if (fwrite(w->cbuf, 1, bsize, w->f) != bsize) return w->err = -1;
    w->caddr += bsize;
    w->n = 0;
    return 0;
}

/* threads > 1: start the pool (on failure the writer stays single-threaded) */
static void bgzfw_start_pool(bgzfw_t *w, int threads) {
    if (threads <= 1) return;
    bgzfw_pool_t *P = (bgzfw_pool_t *)calloc(1, sizeof(bgzfw_pool_t));
    if (!P) return;
    P->nt = threads;
    P->cap = BGZFW_BATCH * threads;
    P->level = w->level;
    P->u = (uint8_t *)malloc((size_t)P->cap * BGZF_BLK);
    P->c = (uint8_t *)malloc((size_t)P->cap * 65536);
    P->un = (int *)malloc((size_t)P->cap * sizeof(int));
    P->cs = (uint32_t *)malloc((size_t)P->cap * sizeof(uint32_t));
    P->th = (pthread_t *)calloc((size_t)threads, sizeof(pthread_t));
    w->baddr = (uint64_t *)calloc(1024, sizeof(uint64_t));
    w->mb = 1024;
    if (!P->u || !P->c || !P->un || !P->cs || !P->th || !w->baddr || pthread_mutex_init(&P->mu, NULL)) goto fail;
    pthread_cond_init(&P->go, NULL);
    pthread_cond_init(&P->done, NULL);
    for (int i = 0; i < threads - 1; i++) P->made += pthread_create(&P->th[i], NULL, bgzfw_worker, P) == 0;
    w->pool = P;
    w->baddr[0] = w->caddr;                           /* the first queued block's file address */
    w->caddr = 0;                                     /* block numbers from here */
    return;
fail:
    free(P->u); free(P->c); free(P->un); free(P->cs); free(P->th); free(P);
    free(w->baddr); w->baddr = NULL; w->mb = 0;
}

static void bgzfw_stop_pool(bgzfw_t *w) {
    bgzfw_pool_t *P = w->pool;
    if (!P) return;
    pthread_mutex_lock(&P->mu);
    P->quit = 1;
    pthread_cond_broadcast(&P->go);
    pthread_mutex_unlock(&P->mu);
    for (int i = 0; i < P->made; i++) pthread_join(P->th[i], NULL);
    pthread_mutex_destroy(&P->mu);
    pthread_cond_destroy(&P->go);
    pthread_cond_destroy(&P->done);
    free(P->u); free(P->c); free(P->un); free(P->cs); free(P->th); free(P);
    w->pool = NULL;
}

/* a virtual offset of the threaded writer (block number << 16 | offset) as a
 * file one (after the last drain); the single-threaded writer's as is */
static uint64_t bgzfw_vmap(const bgzfw_t *w, uint64_t v) {
    if (!w->baddr || v == ~0ull) return v;
    const uint64_t b = v >> 16;
    return b <= w->nb ? (w->baddr[b] << 16) | (v & 0xffffu) : v;
}

static int bgzfw_write(bgzfw_t *w, const void *src, size_t n) {
    const uint8_t *s = (const uint8_t *)src;
    while (n && !w->err) {
        size_t k = (size_t)(BGZF_BLK - w->n);
        if (k > n) k = n;
        memcpy(w->ubuf + w->n, s, k);
        w->n += (int)k;
        s += k;
        n -= k;
        if (w->n == BGZF_BLK) bgzfw_flush(w);
    }
    return w->err;
}

static uint64_t bgzfw_tell(const bgzfw_t *w) { return (w->caddr << 16) | (uint64_t)w->n; }

/* hts_idx_push / hts_idx_finish for a BAI (min_shift 14, 5 levels) */
typedef struct { uint32_t bin; uint64_t u, v; } ichunk_t;
typedef struct {
    ichunk_t *c; size_t n, m;
    uint64_t *lin; size_t nl, ml;
    int has_meta;
    uint64_t off_beg, off_end, n_mapped, n_unmapped;
} iref_t;
typedef struct {
    int32_t n_ref;
    iref_t *r;
    uint64_t n_no_coor;
    int32_t last_tid, save_tid;
    uint32_t last_bin, save_bin;
    uint64_t save_off, last_off, off_beg;
    uint64_t n_mapped, n_unmapped;
    int finished;
    int err;
} bai_t;

static uint32_t reg2bin14(int64_t beg, int64_t end) {
    end--;
    if (beg >> 14 == end >> 14) return (uint32_t)(((1 << 15) - 1) / 7 + (beg >> 14));
    if (beg >> 17 == end >> 17) return (uint32_t)(((1 << 12) - 1) / 7 + (beg >> 17));
    if (beg >> 20 == end >> 20) return (uint32_t)(((1 << 9) - 1) / 7 + (beg >> 20));
    if (beg >> 23 == end >> 23) return (uint32_t)(((1 << 6) - 1) / 7 + (beg >> 23));
    if (beg >> 26 == end >> 26) return (uint32_t)(((1 << 3) - 1) / 7 + (beg >> 26));
    return 0;
}

static void bai_chunk(bai_t *x, int32_t tid, uint32_t bin, uint64_t u, uint64_t v) {
    if (x->err || tid < 0 || tid >= x->n_ref) return;
    iref_t *r = &x->r[tid];
    if (r->n == r->m) {
        const size_t m = r->m ? 2 * r->m : 64;
        ichunk_t *c = (ichunk_t *)realloc(r->c, m * sizeof(ichunk_t));
        if (!c) { x->err = PF_ERR_NOMEM; return; }
        r->c = c;
        r->m = m;
    }
    r->c[r->n].bin = bin; r->c[r->n].u = u; r->c[r->n].v = v;
    r->n++;
}

static void bai_meta(bai_t *x, int32_t tid, uint64_t beg, uint64_t end) {
    if (tid < 0 || tid >= x->n_ref) return;
    iref_t *r = &x->r[tid];
    r->has_meta = 1;
    r->off_beg = beg; r->off_end = end;
    r->n_mapped = x->n_mapped; r->n_unmapped = x->n_unmapped;
}

static void bai_finish(bai_t *x, uint64_t final_off) {
    if (x->finished) return;
    if (x->save_tid >= 0) {
        bai_chunk(x, x->save_tid, x->save_bin, x->save_off, final_off);
        bai_meta(x, x->save_tid, x->off_beg, final_off);
    }
    x->finished = 1;
}

static void bai_push(bai_t *x, int32_t tid, int64_t beg, int64_t end, uint64_t offset, int mapped) {
    if (tid < 0) x->n_no_coor++;
    if (x->finished || x->err) return;
    if (x->last_tid != tid || (x->last_tid >= 0 && tid < 0)) {
        x->last_tid = tid;
        x->last_bin = 0xffffffffu;
    }
    if (tid >= 0 && tid < x->n_ref && mapped) {          /* insert_to_l */
        if (beg < 0) beg = 0;
        if (end <= 0) end = 1;
        iref_t *r = &x->r[tid];
        const int64_t b = beg >> 14, e = (end - 1) >> 14;
        if ((size_t)e + 1 > r->ml) {
            size_t m = r->ml ? r->ml : 64;
            while (m < (size_t)e + 1) m *= 2;
            uint64_t *l = (uint64_t *)realloc(r->lin, m * sizeof(uint64_t));
            if (!l) { x->err = PF_ERR_NOMEM; return; }
            for (size_t i = r->ml; i < m; i++) l[i] = ~0ull;
            r->lin = l;
            r->ml = m;
        }
        for (int64_t i = b; i <= e; i++) if (r->lin[i] == ~0ull) r->lin[i] = x->last_off;
        if (r->nl < (size_t)e + 1) r->nl = (size_t)e + 1;
    }
    const uint32_t bin = reg2bin14(beg, end);
    if (x->last_bin != bin) {
        if (x->save_bin != 0xffffffffu) bai_chunk(x, x->save_tid, x->save_bin, x->save_off, x->last_off);
        if (x->last_bin == 0xffffffffu && x->save_bin != 0xffffffffu) {   /* change of contig */
            bai_meta(x, x->save_tid, x->off_beg, x->last_off);
            x->n_mapped = x->n_unmapped = 0;
            x->off_beg = x->last_off;
        }
        x->save_off = x->last_off;
        x->save_bin = x->last_bin = bin;
        x->save_tid = tid;
        if (tid < 0) { bai_finish(x, offset); return; }
    }
    if (mapped) x->n_mapped++;
    else x->n_unmapped++;
    x->last_off = offset;
}

static int cmp_ichunk(const void *a, const void *b) {
    const ichunk_t *x = (const ichunk_t *)a, *y = (const ichunk_t *)b;
    if (x->bin != y->bin) return x->bin < y->bin ? -1 : 1;
    return x->u < y->u ? -1 : x->u > y->u;
}

static int bai_write(bai_t *x, const char *path) {
    FILE *f = fopen(path, "wb");
    if (!f) return -1;
    int rc = 0;
#define W(p, n) do { if (!rc && fwrite((p), 1, (n), f) != (size_t)(n)) rc = -1; } while (0)
    W("BAI\1", 4);
    int32_t nr = x->n_ref;
    W(&nr, 4);
    for (int32_t t = 0; t < x->n_ref; t++) {
        iref_t *r = &x->r[t];
        qsort(r->c, r->n, sizeof(ichunk_t), cmp_ichunk);
        int32_t nb = 0;
        for (size_t i = 0; i < r->n; i++) if (i == 0 || r->c[i].bin != r->c[i - 1].bin) nb++;
        const int32_t nbt = nb + (r->has_meta ? 1 : 0);
        W(&nbt, 4);
        for (size_t i = 0; i < r->n;) {
            size_t j = i;
            while (j < r->n && r->c[j].bin == r->c[i].bin) j++;
            const uint32_t bin = r->c[i].bin;
            const int32_t nc = (int32_t)(j - i);
            W(&bin, 4);
            W(&nc, 4);
            for (size_t k = i; k < j; k++) { W(&r->c[k].u, 8); W(&r->c[k].v, 8); }
            i = j;
        }
        if (r->has_meta) {
            const uint32_t mb = 37450;
            const int32_t two = 2;
            W(&mb, 4); W(&two, 4);
            W(&r->off_beg, 8); W(&r->off_end, 8); W(&r->n_mapped, 8); W(&r->n_unmapped, 8);
        }
        /* update_loff: leading holes -> the contig's first record offset, others -> previous */
        size_t l = 0;
        const uint64_t offset0 = r->has_meta ? r->off_beg : 0;
        for (; l < r->nl && r->lin[l] == ~0ull; l++) r->lin[l] = offset0;
        for (; l < r->nl; l++) if (r->lin[l] == ~0ull) r->lin[l] = r->lin[l - 1];
        const int32_t ni = (int32_t)r->nl;
        W(&ni, 4);
        for (size_t i = 0; i < r->nl; i++) W(&r->lin[i], 8);
    }
    W(&x->n_no_coor, 8);
#undef W
    if (fclose(f) && !rc) rc = -1;
    return rc;
}

/* bam_aux_update_int(b, "HP", val) on a record's bytes: rewrite into out */
static int hp_update(const uint8_t *d, uint32_t bs, const rec_t *r, int64_t val, vbuf_t *out) {
    out->n = 0;
    uint8_t type;
    uint32_t sz;
    if (val < INT16_MIN || val > UINT16_MAX) { type = val < 0 ? 'i' : 'I'; sz = 4; }
    else if (val < INT8_MIN || val > UINT8_MAX) { type = val < 0 ? 's' : 'S'; sz = 2; }
    else { type = val < 0 ? 'c' : 'C'; sz = 1; }
    /* bam_aux_get: the first HP, or ENOENT at the end, or EINVAL on corrupt aux */
    const uint8_t *p = r->aux, *hp = NULL;
    int corrupt = 0;
    while (p + 3 <= r->aux_end) {
        const size_t s = aux_size(p, r->aux_end);
        if (s == 0 || p + 3 + s > r->aux_end) { corrupt = 1; break; }
        if (p[0] == 'H' && p[1] == 'P') { hp = p; break; }
        p += 3 + s;
    }
    if (!hp && (corrupt || p != r->aux_end)) return vb_put(out, d, bs);      /* invalid aux: unchanged */
    uint8_t v8[8];
    for (int i = 0; i < 8; i++) v8[i] = (uint8_t)((uint64_t)val >> (8 * i));
    if (!hp) {                                                   /* new tag at the end */
        const uint8_t t3[3] = {'H', 'P', type};
        int rc = vb_put(out, d, bs);
        if (!rc) rc = vb_put(out, t3, 3);
        if (!rc) rc = vb_put(out, v8, sz);
        return rc;
    }
    uint32_t old_sz;
    switch (hp[2]) {
    case 'c': case 'C': old_sz = 1; break;
    case 's': case 'S': old_sz = 2; break;
    case 'i': case 'I': old_sz = 4; break;
    default: return vb_put(out, d, bs);                          /* not an integer: unchanged */
    }
    if (old_sz >= sz) {                                          /* reuse the old space */
        sz = old_sz;
        type = (uint8_t)(val < 0 ? "\0cs\0i"[old_sz] : "\0CS\0I"[old_sz]);
    }
    const size_t at = (size_t)(hp - d);
    int rc = vb_put(out, d, at + 2);
    if (!rc) rc = vb_put(out, &type, 1);
    if (!rc) rc = vb_put(out, v8, sz);
    if (!rc) rc = vb_put(out, hp + 3 + old_sz, bs - (at + 3 + old_sz));
    return rc;
}

int pf_retag_bam(const char *bam_in, const char *bam_out, const char *bai_out, const char *tsv_out, int mode,
                 const pf_gaps_t *g, const pf_blocks_t *blk, const pf_tags_t *methphased, const pf_tags_t *raw,
                 int level, uint64_t *n_records) {
    return pf_retag_bam_threads(bam_in, bam_out, bai_out, tsv_out, mode, g, blk, methphased, raw, level, 1, n_records);
}

int pf_retag_bam_threads(const char *bam_in, const char *bam_out, const char *bai_out, const char *tsv_out, int mode,
                         const pf_gaps_t *g, const pf_blocks_t *blk, const pf_tags_t *methphased, const pf_tags_t *raw,
                         int level, int threads, uint64_t *n_records) {
    if (!bam_in || (!bam_out && !tsv_out) ||
        (mode != PF_RETAG_METHPHASE && mode != PF_RETAG_VARHAPTAG && mode != PF_RETAG_INPUT_HAPTAG))
        return PF_ERR_ARG;
    if (mode == PF_RETAG_METHPHASE && (!g || !blk || !methphased)) return PF_ERR_ARG;
    if (mode != PF_RETAG_METHPHASE && !raw) return PF_ERR_ARG;
    if (mode == PF_RETAG_INPUT_HAPTAG && (bam_out || !tsv_out)) return PF_ERR_ARG;
    if (n_records) *n_records = 0;
    bgzf_t *z = (bgzf_t *)malloc(sizeof(bgzf_t));
    bgzfw_t *w = bam_out ? (bgzfw_t *)calloc(1, sizeof(bgzfw_t)) : NULL;
    FILE *tsv = NULL;
    bai_t X;
    memset(&X, 0, sizeof X);
    uint8_t *rec = NULL, *hdr = NULL;
    size_t cap = 0;
    vbuf_t ob = {0};
    char **names = NULL;
    int32_t *vcf_of_tid = NULL;
    int32_t n_ref = 0;
    int rc = (!z || (bam_out && !w)) ? PF_ERR_NOMEM : 0;
    if (!rc) { rc = bgzf_open(z, bam_in); if (rc) { free(z); z = NULL; } }
    if (!rc && w) {
        w->f = fopen(bam_out, "wb");
        w->level = level;
        if (!w->f) rc = -1;
    }
    if (!rc && tsv_out) {
        tsv = fopen(tsv_out, "w");
        if (!tsv) rc = -1;
        else if (mode == PF_RETAG_INPUT_HAPTAG) fprintf(tsv, "#qname\treal_hp\ttagged_hp\n");   /* 4498 */
        else fprintf(tsv, "#qname\thaptag_input\thaptag_new\n");
    }
    /* header: copied as read, then flushed into its own block (bam_hdr_write) */
    if (!rc) {
        uint8_t h8[8], w4[4];
        if (bgzf_read(z, h8, 8) != 8 || memcmp(h8, "BAM\1", 4) != 0) rc = PF_ERR_ARG;
        const uint32_t lt = rc ? 0 : rd32(h8 + 4);
        if (!rc) { hdr = (uint8_t *)malloc(lt ? lt : 1); if (!hdr) rc = PF_ERR_NOMEM; }
        if (!rc && bgzf_read(z, hdr, lt) != (int64_t)lt) rc = PF_ERR_ARG;
        if (!rc && w) { bgzfw_write(w, h8, 8); bgzfw_write(w, hdr, lt); }
        if (!rc && bgzf_read(z, w4, 4) != 4) rc = PF_ERR_ARG;
        if (!rc) {
            n_ref = (int32_t)rd32(w4);
            if (n_ref < 0) rc = PF_ERR_ARG;
            if (w) bgzfw_write(w, w4, 4);
        }
        if (!rc) {
            names = (char **)calloc(n_ref ? (size_t)n_ref : 1, sizeof(char *));
            vcf_of_tid = (int32_t *)malloc((n_ref ? (size_t)n_ref : 1) * sizeof(int32_t));
            if (!names || !vcf_of_tid) rc = PF_ERR_NOMEM;
        }
        for (int32_t t = 0; t < n_ref && !rc; t++) {
            if (bgzf_read(z, w4, 4) != 4) { rc = PF_ERR_ARG; break; }
            const uint32_t ln = rd32(w4);
            if (ln == 0 || ln > (1u << 20)) { rc = PF_ERR_ARG; break; }
            names[t] = (char *)malloc(ln);
            uint8_t l4[4];
            if (!names[t]) { rc = PF_ERR_NOMEM; break; }
            if (bgzf_read(z, names[t], ln) != (int64_t)ln || bgzf_read(z, l4, 4) != 4) { rc = PF_ERR_ARG; break; }
            names[t][ln - 1] = 0;
            if (w) { bgzfw_write(w, w4, 4); bgzfw_write(w, names[t], ln); bgzfw_write(w, l4, 4); }
            vcf_of_tid[t] = -1;                          /* the contig's VCF index, by name */
            if (g) for (uint32_t c = 0; c < g->n_contigs; c++) if (!strcmp(g->names[c], names[t])) { vcf_of_tid[t] = (int32_t)c; break; }
        }
        if (!rc && w) rc = bgzfw_flush(w);
    }
    if (!rc && w) bgzfw_start_pool(w, threads);       /* the header's block is written: numbers start at 0 */
    if (!rc && w) {
        X.n_ref = n_ref;
        X.r = (iref_t *)calloc(n_ref ? (size_t)n_ref : 1, sizeof(iref_t));
        if (!X.r) rc = PF_ERR_NOMEM;
        X.last_tid = -1; X.save_tid = -1;
        X.last_bin = X.save_bin = 0xffffffffu;
        X.last_off = X.off_beg = bgzfw_tell(w);
    }
    /* output_modify_bam's cursor state (3038-3040, 3059-3064) */
    int prev_unphased_idx = 1, need_flip = 0;
    int32_t prev_tid = 0;
    uint64_t nrec = 0;
    while (!rc) {
        uint8_t w4[4];
        const int64_t gr = bgzf_read(z, w4, 4);
        if (gr == 0) break;
        if (gr != 4) { rc = PF_ERR_ARG; break; }
        const uint32_t bs = rd32(w4);
        if (bs < 32 || bs > (1u << 30)) { rc = PF_ERR_ARG; break; }
        if (bs > cap) {
            uint8_t *np = (uint8_t *)realloc(rec, bs);
            if (!np) { rc = PF_ERR_NOMEM; break; }
            rec = np;
            cap = bs;
        }
        if (bgzf_read(z, rec, bs) != (int64_t)bs) { rc = PF_ERR_ARG; break; }
        rec_t r;
        if (rec_decode(rec, bs, &r)) { rc = PF_ERR_ARG; break; }
        const uint8_t *cg = r.cigar;
        uint32_t ncg = r.n_cigar;
        if (ncg > 0 && r.tid >= 0 && r.pos >= 0 && (rd32(cg) & 15u) == 4u && (rd32(cg) >> 4) == r.l_qseq) {
            const uint8_t *t = aux_find(r.aux, r.aux_end, "CG");
            if (t && t[2] == 'B' && (t[3] == 'I' || t[3] == 'i')) {
                const uint32_t nn = rd32(t + 4);
                if (nn >= r.n_cigar && nn < (1u << 29)) { cg = t + 8; ncg = nn; }
            }
        }
        uint64_t qlen = 0;
        const uint64_t rlen = cigar_rlen(cg, ncg, &qlen);
        if (ncg > 0 && r.l_qseq > 0 && !(r.flag & 4) && qlen != r.l_qseq) break;   /* sam_itr_next < 0 */
        const size_t lq = r.l_qname > 0 ? r.l_qname - 1 : 0;
        uint64_t qoff[2] = {0, (uint64_t)lq};
        /* the raw tag: the -u table (absent -> unphased) or get_hp_from_aln (910-923) */
        int hp_tag;
        {
            int64_t v = 0;
            const uint8_t *t = aux_find(r.aux, r.aux_end, "HP");
            hp_tag = (t && aux_int(t, &v) && v != 0) ? (int)(v - 1) : 254;
            if (t && !aux_int(t, &v)) hp_tag = 254;      /* bam_aux2i of a non-integer: 0 */
        }
        int hp_raw = hp_tag;
        if (raw) {
            uint8_t h;
            pf_tags_get(raw, 1, qoff, r.qname, 254, &h);
            hp_raw = h;
        }
        int hp;
        if (mode != PF_RETAG_METHPHASE) {
            hp = hp_raw;                                 /* st->qname2haptag_raw, 4787-4795 / 4504-4512 */
        } else {
            if (r.tid != prev_tid) { prev_unphased_idx = 1; prev_tid = r.tid; }
            /* check_if_in_phased_intervals (2406-2426) on the contig's merged gaps */
            const int32_t c = (r.tid >= 0 && r.tid < n_ref) ? vcf_of_tid[r.tid] : -1;
            int updated = 0;
            if (c >= 0) {
                const uint64_t go = g->gap_off[c], gn = g->gap_off[c + 1] - go;
                for (uint64_t j = (uint64_t)prev_unphased_idx; j < gn; j++) {
                    if ((int)r.pos >= (int)g->gap_end[go + j - 1] && (int)r.pos <= (int)g->gap_start[go + j]) {
                        if ((int)j != prev_unphased_idx) { updated = 1; prev_unphased_idx = (int)j; }
                        break;
                    }
                }
            }
            if (updated) {       /* get_flip_status_by_idx: flips_onraw indexed by the merged index - 1 */
                const uint64_t fo = blk->dec_off[c], fn = blk->dec_off[c + 1] - fo;
                const uint64_t k = (uint64_t)(prev_unphased_idx - 1);
                need_flip = k < fn ? blk->flip[fo + k] : 0;
            }
            /* get_read_new_haplotag (2990-3020) */
            uint8_t hm;
            if (pf_tags_get(methphased, 1, qoff, r.qname, 0, &hm) > 0) {
                hp = hm;
                if (need_flip) hp ^= 1;
            } else {
                hp = hp_raw;
                if ((hp == 0 || hp == 1) && need_flip) hp ^= 1;
            }
        }
        if (tsv) fprintf(tsv, "%s\t%d\t%d\n", r.qname, hp_tag + 1, hp + 1);
        if (w) {
            rc = hp_update(rec, bs, &r, (int64_t)hp + 1, &ob);
            if (rc) break;
            if (ncg > 0) {       /* bam_read1 recomputes bin from the CIGAR (hts_reg2bin(pos, pos + rlen, 14, 5)) */
                const int64_t rl = ((r.flag & 4) || rlen == 0) ? 1 : (int64_t)rlen;
                const uint32_t bin = reg2bin14(r.pos, r.pos + rl);
                ob.p[10] = (uint8_t)bin;
                ob.p[11] = (uint8_t)(bin >> 8);
            }
            uint8_t o4[4];
            const uint32_t nb = (uint32_t)ob.n;
            for (int i = 0; i < 4; i++) o4[i] = (uint8_t)(nb >> (8 * i));
            if (w->n + 4 + nb > BGZF_BLK) bgzfw_flush(w);          /* bgzf_flush_try */
            bgzfw_write(w, o4, 4);
            bgzfw_write(w, ob.p, nb);
            if (w->err) { rc = w->err; break; }
            const int mapped = !(r.flag & 4);
            const int64_t end = r.pos + ((mapped && rlen) ? (int64_t)rlen : 1);      /* bam_endpos */
            bai_push(&X, r.tid, r.pos, end, bgzfw_tell(w), mapped);
            if (X.err) { rc = X.err; break; }
        }
        nrec++;
    }
    if (!rc && w) {
        rc = bgzfw_flush(w);
        if (!rc) bai_finish(&X, bgzfw_tell(w));
        if (!rc && w->pool) rc = bgzfw_drain(w);
        if (!rc && w->baddr) {                        /* block numbers -> file addresses */
            for (int32_t t = 0; t < X.n_ref; t++) {
                iref_t *r = &X.r[t];
                for (size_t i = 0; i < r->n; i++) { r->c[i].u = bgzfw_vmap(w, r->c[i].u); r->c[i].v = bgzfw_vmap(w, r->c[i].v); }
                for (size_t i = 0; i < r->nl; i++) r->lin[i] = bgzfw_vmap(w, r->lin[i]);
                r->off_beg = bgzfw_vmap(w, r->off_beg);
                r->off_end = bgzfw_vmap(w, r->off_end);
            }
        }
        if (!rc && fwrite(BGZF_EOF, 1, sizeof BGZF_EOF, w->f) != sizeof BGZF_EOF) rc = -1;
    }
    if (w) {
        bgzfw_stop_pool(w);
        if (w->f && fclose(w->f) && !rc) rc = -1;
        free(w->baddr);
        free(w);
    }
    if (!rc && bam_out && bai_out) rc = bai_write(&X, bai_out);
    if (tsv && fclose(tsv) && !rc) rc = -1;
    for (int32_t t = 0; t < X.n_ref; t++) { free(X.r[t].c); free(X.r[t].lin); }
    free(X.r);
    if (names) for (int32_t t = 0; t < n_ref; t++) free(names[t]);
    free(names); free(vcf_of_tid); free(rec); free(hdr); free(ob.p);
    if (z) { bgzf_close(z); free(z); }
    if (n_records) *n_records = nrec;
    return rc;
}
