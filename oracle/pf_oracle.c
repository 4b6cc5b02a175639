/*
 * pf_oracle.c -- CPU oracle: plain-C restatement of the reference hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see pf_oracle.h).  Used by tests/ as the checker
 * of the HIP path and by bench.py as the CPU baseline ("port").  Never linked
 * into libpomfret_amd.so.
 *
 * Parity: methylation core UNPINNED (the reference cannot be built here:
 * blockjoin.c needs htslib, which this image lacks, and the reference holds
 * no test vectors for this path because example/phased.bam is missing).  Each
 * function restates the reference lines it cites, keeping the reference's
 * data structures (per-site methmer key lists with linear search, stable
 * merge sort of candidates, u64 piggy-back radix sorts) so that its cost
 * profile is that of the reference, too.
 *
 * Line numbers: /root/reference/blockjoin.c unless noted.
 */
#define _GNU_SOURCE
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>
#include <pthread.h>
#include <zlib.h>
#include "pf_oracle.h"

#define HAPTAG_UNPHASED 254           /* :26 */
#define HARD_COV_THRESHOLD 15         /* :20 */
#define HARD_CONTAMINATE_THRESHOLD 5  /* :21 */
#define EVAL_P_THRE 0.001             /* :24 */
#define VAR_DIFF_OVERRIDE_RATIO 5     /* :32 */
#define MAXV(a,b) ((a)>(b)?(a):(b))
#define MINV(a,b) ((a)<=(b)?(a):(b))

/* ---------------------------------------------------------------- */
/* growable vectors (kvec.h analogue)                                */
typedef struct { uint32_t *a; size_t n, m; } vu32;
typedef struct { uint64_t *a; size_t n, m; } vu64;
typedef struct { uint16_t *a; size_t n, m; } vu16;
typedef struct { float *a; size_t n, m; } vf32;
#define VPUSH(v, x) do { if ((v).n == (v).m) { (v).m = (v).m ? (v).m * 2 : 16; \
    (v).a = realloc((v).a, sizeof(*(v).a) * (v).m); } (v).a[(v).n++] = (x); } while (0)
#define VFREE(v) do { free((v).a); (v).a = 0; (v).n = (v).m = 0; } while (0)

/* LSD radix sort, ascending (same order as klib radix_sort_ksu64, ksort.h). */
static void radix_u64(uint64_t *a, size_t n, uint64_t *tmp) {
    if (n < 2) return;
    uint64_t *src = a, *dst = tmp;
    uint64_t x_or = 0, first = a[0];
    for (size_t i = 0; i < n; i++) x_or |= a[i] ^ first;
    for (int shift = 0; shift < 64; shift += 8) {
        if (((x_or >> shift) & 0xff) == 0) continue;
        size_t cnt[257] = {0};
        for (size_t i = 0; i < n; i++) cnt[((src[i] >> shift) & 0xff) + 1]++;
        for (int b = 0; b < 256; b++) cnt[b + 1] += cnt[b];
        for (size_t i = 0; i < n; i++) dst[cnt[(src[i] >> shift) & 0xff]++] = src[i];
        uint64_t *t = src; src = dst; dst = t;
    }
    if (src != a) memcpy(a, src, n * sizeof(uint64_t));
}
static void radix_u64_alloc(uint64_t *a, size_t n) {
    if (n < 2) return;
    uint64_t *tmp = malloc(n * sizeof(uint64_t));
    radix_u64(a, n, tmp);
    free(tmp);
}

/* ---------------------------------------------------------------- */
/* search_arr1 / search_arr  (:339-421), restated literally           */
static int search_arr1(const uint32_t *a, uint32_t l, uint32_t v, uint32_t *idx) {
    if (l == 0) return -3;
    if (v < a[0]) { *idx = UINT32_MAX; return -1; }
    if (v > a[l - 1]) { *idx = UINT32_MAX; return -2; }
    if (l < 16) {
        for (uint32_t i = 0; i < l; i++) {
            if (a[i] == v) { *idx = i; return 1; }
            if (a[i] > v) { *idx = i; return 0; }
        }
        fprintf(stderr, "[E::%s] impossible 1\n", __func__); abort();
    } else {
        uint32_t low = 0, mid, high = l - 1;
        while (low < high) {
            mid = low + (high - low) / 2;
            if (v <= a[mid]) high = mid; else low = mid + 1;
        }
        if (a[high] == v) { *idx = high; return 1; }
        else if (a[high] > v) { *idx = high; return 0; }
        fprintf(stderr, "[E::%s] impossible 2\n", __func__); abort();
    }
    return -4;
}
int orc_search_arr(const uint32_t *a, uint32_t l, uint32_t v, uint32_t *idx, int which_end) {
    uint32_t i = 0;
    int stat = search_arr1(a, l, v, &i);
    if (which_end < 0) { *idx = i; return stat; }
    if (stat <= 0) { *idx = i; return stat; }
    if (which_end == 0) {
        for (int j = (int)i - 1; j >= 0; j--) { if (a[j] == v) i = j; else break; }
    } else {
        for (int j = (int)i + 1; j < (int)l; j++) { if (a[j] == v) i = j; else break; }
    }
    *idx = i;
    return stat;
}

/* ---------------------------------------------------------------- */
/* read set: rs_t (:442-464) restricted to what the hot path reads     */
typedef struct {
    int hp;                 /* read_t.hp */
    uint32_t calls_n;
    const uint32_t *calls;  /* meth.calls */
    const uint8_t *quals;   /* meth.quals (categories) */
    uint32_t *mmr;          /* read_t.mmr */
    int mmr_n;
    uint32_t mmr_start_i;
} o_read_t;

typedef struct {
    o_read_t *a;
    uint32_t n;                 /* rs->n (0 after the left-coverage check fails) */
    uint32_t n_loaded;          /* reads in the window before the check          */
    uint32_t ref_start, ref_end;
    vu32 left, left_strict, right, right_strict;  /* refreads_t (:212-219)     */
    uint64_t *revbuf;           /* end<<32|id, sorted (:1126, :1140)             */
} o_rs_t;

/* one site's methmer table: mmr_t (:3106-3110) */
typedef struct { vu32 keys; vu16 cnt[2]; uint16_t sum[2]; } o_mmr_t;
typedef struct {
    int n;
    uint32_t *sites_real_poss, *sites_starts;
    uint8_t *mmr_lens;
    o_mmr_t *mmr_a;
    uint32_t mmr_min_i, mmr_max_i;
} o_ms_t;

typedef struct {
    int k, k_span, cov_sel, cov_rt, n_cand, hard_cov;
} o_par_t;

static void ms_free(o_ms_t *ms) {
    if (!ms) return;
    free(ms->sites_real_poss); free(ms->sites_starts); free(ms->mmr_lens);
    if (ms->mmr_a) {
        for (int i = 0; i < ms->n; i++) {
            VFREE(ms->mmr_a[i].keys); VFREE(ms->mmr_a[i].cnt[0]); VFREE(ms->mmr_a[i].cnt[1]);
        }
        free(ms->mmr_a);
    }
    free(ms);
}

/* get_methmer_sites_and_ranges (:3202-3354).  Counting is restated with a
 * sort instead of the khashl table; the per-category counter semantics are
 * kept: cnt[call] is a uint16 holding count<<4 (plus strand bits), so the
 * count wraps at 4096 (:3210-3253).  masked_positions is always NULL on the
 * hot path (:4250-4251). */
static o_ms_t *get_methmer_sites_and_ranges(const o_rs_t *rs, const o_par_t *par, int direction) {
    size_t tot = 0;
    for (uint32_t i = 0; i < rs->n; i++) tot += rs->a[i].calls_n;
    uint64_t *keys = malloc(sizeof(uint64_t) * (tot ? tot : 1));
    size_t t = 0;
    for (uint32_t i = 0; i < rs->n; i++)
        for (uint32_t j = 0; j < rs->a[i].calls_n; j++)
            keys[t++] = ((uint64_t)rs->a[i].calls[j] << 2) | (rs->a[i].quals[j] & 3);
    radix_u64_alloc(keys, tot);
    vu32 ok; memset(&ok, 0, sizeof(ok));
    for (size_t i = 0; i < tot;) {
        uint32_t pos = (uint32_t)(keys[i] >> 2);
        uint16_t cnt[3] = {0, 0, 0};
        size_t j = i;
        for (; j < tot && (uint32_t)(keys[j] >> 2) == pos; j++) {
            int call = keys[j] & 3;
            if (call > 2) continue;        /* categories are 0..2 */
            cnt[call] = (uint16_t)(cnt[call] + 16);  /* += incre on uint16 (:3232, :3237) */
        }
        if ((cnt[0] >> 4) >= par->cov_sel && (cnt[1] >> 4) >= par->cov_sel) VPUSH(ok, pos);
        i = j;
    }
    free(keys);

    o_ms_t *ret = calloc(1, sizeof(o_ms_t));
    int n = (int)ok.n;
    ret->n = n;
    ret->sites_real_poss = calloc(n ? n : 1, sizeof(uint32_t));
    ret->sites_starts = calloc(n ? n : 1, sizeof(uint32_t));
    ret->mmr_lens = calloc(n ? n : 1, 1);
    ret->mmr_a = calloc(n ? n : 1, sizeof(o_mmr_t));
    if (n) memcpy(ret->sites_real_poss, ok.a, n * sizeof(uint32_t));  /* already ascending */
    VFREE(ok);
    uint32_t *sites = ret->sites_real_poss;
    if (direction == 1) {  /* reverse_arr (:3299) */
        for (int i = 0; i < n / 2; i++) { uint32_t x = sites[i]; sites[i] = sites[n - 1 - i]; sites[n - 1 - i] = x; }
    }
    for (int i = 0; i < n; i++) {           /* :3310-3322 */
        int j = i + par->k;
        j = j > n - 1 ? n - 1 : j;
        while (1) {
            if ((direction == 0 && (uint32_t)(sites[j] - sites[i]) <= (uint32_t)par->k_span) ||
                (direction == 1 && (uint32_t)(sites[i] - sites[j]) <= (uint32_t)par->k_span)) break;
            j--;
        }
        ret->mmr_lens[i] = j - i == 0 ? 1 : j - i;
        ret->sites_starts[i] = direction == 0 ? sites[i] : sites[j];
    }
    if (direction == 1) {                   /* :3325-3329 */
        for (int i = 0; i < n / 2; i++) {
            uint32_t x = sites[i]; sites[i] = sites[n - 1 - i]; sites[n - 1 - i] = x;
            x = ret->sites_starts[i]; ret->sites_starts[i] = ret->sites_starts[n - 1 - i]; ret->sites_starts[n - 1 - i] = x;
            uint8_t y = ret->mmr_lens[i]; ret->mmr_lens[i] = ret->mmr_lens[n - 1 - i]; ret->mmr_lens[n - 1 - i] = y;
        }
    }
    return ret;
}

/* methmer_to_uint32 (:3186-3194) with chars already coded m=0,u=1,-=2 */
static uint32_t mmr_code(const uint8_t *c, int l) {
    uint32_t r = 0;
    for (int i = 0; i < l; i++) r = r << 2 | (c[i] == 0 ? 0u : c[i] == 1 ? 1u : 2u);
    return r;
}

/* get_mmr_of_read (:3357-3451), restated literally. */
static int get_mmr_of_read(const o_read_t *read, const o_ms_t *ms, vu32 *buf_mmr, uint32_t *start_i) {
    buf_mmr->n = 0;
    const uint32_t *sites = ms->sites_starts;
    uint32_t sites_n = (uint32_t)ms->n;
    const uint32_t *calls = read->calls;
    const uint8_t *quals = read->quals;
    uint32_t calls_n = read->calls_n;
    *start_i = UINT32_MAX;
    if (calls_n == 0) return 0;
    uint32_t x_i_left = 0, x_i_right = 0;
    int stat = orc_search_arr(sites, sites_n, calls[0], &x_i_left, 0);
    if (stat == -2 || stat == -3) return 0;
    if (stat == 0) x_i_left = x_i_left == 0 ? 0 : x_i_left - 1;
    stat = orc_search_arr(sites, sites_n, calls[calls_n - 1], &x_i_right, 0);
    if (stat == -1 || stat == -3) return 0;
    if (x_i_left == UINT32_MAX) x_i_left = 0;
    if (x_i_right == UINT32_MAX) x_i_right = sites_n;

    size_t cap = (x_i_right > x_i_left ? x_i_right - x_i_left : 0) + calls_n + 1;
    uint64_t *buf = malloc(sizeof(uint64_t) * cap * 2);
    uint64_t *tmp = buf + cap;
    size_t bn = 0;
    for (uint32_t i = x_i_left; i < x_i_right; i++) {
        if (i > 1 && sites[i] == sites[i - 1]) continue;           /* :3391 */
        buf[bn++] = ((uint64_t)sites[i]) << 35 | i;
    }
    for (uint32_t i = 0; i < calls_n; i++)
        buf[bn++] = ((uint64_t)((uint32_t)(calls[i] << 3 | 4 | quals[i]))) << 32;  /* :3398 */
    radix_u64(buf, bn, tmp);

    uint8_t mmr[16];
    uint32_t start_pos_i = UINT32_MAX;
    const uint64_t maskbit = ((uint64_t)4) << 32;
    for (size_t i = 0; i < bn; i++) {
        if ((buf[i] & maskbit) != 0) continue;
        uint32_t pos_i = (uint32_t)buf[i];
        for (int j = (int)pos_i; j < ms->n; j++) {                  /* :3410 */
            if (sites[j] != sites[pos_i]) break;
            int mmr_len = ms->mmr_lens[j];
            int n = 0;
            for (size_t jj = i; bn > 0 && jj < bn - 1;) {           /* :3420 */
                if ((buf[jj] & maskbit) != 0) { jj++; continue; }
                if ((buf[jj] >> 35) == (buf[jj + 1] >> 35) && (buf[jj + 1] & maskbit) != 0) {
                    mmr[n] = (uint8_t)((buf[jj + 1] >> 32) & 3);   /* "mu-"[...] */
                    n++; jj += 2;
                } else {
                    mmr[n] = 2; n++; jj++;
                }
                if (n >= mmr_len) break;
            }
            if (n != mmr_len) continue;                              /* :3438 */
            if (start_pos_i == UINT32_MAX) start_pos_i = (uint32_t)j;
            VPUSH(*buf_mmr, mmr_code(mmr, n));
        }
    }
    free(buf);
    *start_i = buf_mmr->n ? start_pos_i : UINT32_MAX;
    return (int)buf_mmr->n;
}

/* store_mmr_of_reads / store_mmr_of_one_read (:3518-3550) */
static void store_mmr_of_reads(o_rs_t *rs, const o_ms_t *ms) {
    vu32 b; memset(&b, 0, sizeof(b));
    for (uint32_t i = 0; i < rs->n; i++) {
        uint32_t st = 0;
        int n = get_mmr_of_read(&rs->a[i], ms, &b, &st);
        o_read_t *r = &rs->a[i];
        if (n == 0 || st == UINT32_MAX) { r->mmr_n = 0; r->mmr = 0; r->mmr_start_i = 0; }
        else {
            r->mmr_n = n; r->mmr_start_i = st;
            r->mmr = malloc(sizeof(uint32_t) * n);
            memcpy(r->mmr, b.a, sizeof(uint32_t) * n);
        }
    }
    VFREE(b);
}
static void wipe_mmr_of_reads(o_rs_t *rs) {
    for (uint32_t i = 0; i < rs->n; i++) {
        free(rs->a[i].mmr); rs->a[i].mmr = 0; rs->a[i].mmr_n = 0; rs->a[i].mmr_start_i = 0;
    }
}

/* insert_mmrs_to_counts (:3453-3486).  A methmer whose assigned site index
 * falls outside [0, n) is skipped: the reference indexes mmr_a out of bounds
 * there (undefined behaviour); see DESIGN.md "reference UB". */
static void insert_mmrs_to_counts(o_ms_t *ms, const uint32_t *m, int n_mmr, int start, int hap) {
    for (int i0 = 0, j; i0 < n_mmr; i0++) {
        int i = i0 + start;
        if (i < 0 || i >= ms->n) continue;
        uint32_t q = m[i0];
        o_mmr_t *t = &ms->mmr_a[i];
        int found = 0;
        for (j = 0; j < (int)t->keys.n; j++) {
            if (q == t->keys.a[j]) { t->cnt[hap].a[j]++; t->sum[hap]++; found = 1; break; }
        }
        if (!found) {
            VPUSH(t->keys, q); VPUSH(t->cnt[0], 0); VPUSH(t->cnt[1], 0);
            t->cnt[hap].a[j]++; t->sum[hap]++;
        }
    }
}

/* query_counts_of_mmrs (:3487-3515) */
static void query_counts_of_mmrs(const o_ms_t *ms, const uint32_t *m, int n_mmr, uint32_t start,
                                 int hap, vf32 *buf) {
    buf->n = 0;
    for (int i0 = 0; i0 < n_mmr; i0++) {
        int i = (int)start + i0;
        if ((uint32_t)i < ms->mmr_min_i || (uint32_t)i >= ms->mmr_max_i) continue;  /* int vs u32 */
        uint32_t q = m[i0];
        const o_mmr_t *t = &ms->mmr_a[i];
        for (size_t j = 0; j < t->keys.n; j++) {
            if (t->keys.a[j] == q) {
                uint32_t cnt = t->cnt[hap].a[j];
                uint32_t sum = t->sum[hap];
                if (sum != 0) VPUSH(*buf, (float)cnt / sum);
                break;
            }
        }
    }
}

/* use_mmr_count_predict_tag_for_one_read (:3594-3656) */
static int predict_one(const o_read_t *r, const o_ms_t *ms, float *best, float diff_min, int l_min, vf32 *buf) {
    float score0 = 0, score1 = 0;
    int l0, l1;
    query_counts_of_mmrs(ms, r->mmr, r->mmr_n, r->mmr_start_i, 0, buf);
    l0 = (int)buf->n;
    for (size_t i = 0; i < buf->n; i++) if (buf->a[i] > 0) { score0 += buf->a[i]; l0++; }  /* double count (:3619-3624) */
    query_counts_of_mmrs(ms, r->mmr, r->mmr_n, r->mmr_start_i, 1, buf);
    l1 = (int)buf->n;
    for (size_t i = 0; i < buf->n; i++) if (buf->a[i] > 0) { score1 += buf->a[i]; l1++; }
    float diff = score0 > score1 ? score0 - score1 : score1 - score0;
    if (diff < diff_min && (l0 < l_min || l1 < l_min)) { *best = 0; return -1; }
    *best = diff;
    return score0 > score1 ? 0 : 1;
}

/* update_available_methmer_range (:3669-3691) */
static int update_range(o_ms_t *ms, int cov) {
    int updated = 0;
    for (int i = (int)ms->mmr_min_i; i >= 0; i--) {
        int sum = ms->mmr_a[i].sum[0] + ms->mmr_a[i].sum[1];
        if (sum >= cov) { ms->mmr_min_i = (uint32_t)i; updated++; } else break;
    }
    for (int i = (int)ms->mmr_max_i; i < ms->n; i++) {
        if (ms->mmr_a[i].sum[0] + ms->mmr_a[i].sum[1] >= cov) { ms->mmr_max_i = (uint32_t)i; updated++; }
        else break;
    }
    return updated;
}

typedef struct { float score; int tag; uint32_t readID; uint32_t idx; } forpred_t;

/* stable merge sort ascending by score (ks_mergesort, ksort.h:77-125) */
static void mergesort_forpred(forpred_t *a, size_t n, forpred_t *tmp) {
    if (n < 2) return;
    size_t h = n / 2;
    mergesort_forpred(a, h, tmp);
    mergesort_forpred(a + h, n - h, tmp);
    size_t i = 0, j = h, k = 0;
    while (i < h && j < n) { if (a[j].score < a[i].score) tmp[k++] = a[j++]; else tmp[k++] = a[i++]; }
    while (i < h) tmp[k++] = a[i++];
    while (j < n) tmp[k++] = a[j++];
    memcpy(a, tmp, n * sizeof(forpred_t));
}

typedef struct {
    uint32_t cap, cnt;
    uint32_t *ids; uint8_t *tags; float *scores;
} o_trace_t;

/* predict_tags_of_reads (:3693-3774) with insert_best_n = 1 */
static int predict_tags_of_reads(o_rs_t *rs, o_ms_t *ms, const uint32_t *ids, int nids, int cov_rt,
                                 forpred_t *fp, forpred_t *fptmp, vf32 *buf, o_trace_t *tr) {
    for (int i = 0; i < nids; i++) {
        float s;
        int tag = predict_one(&rs->a[ids[i]], ms, &s, 3, 3, buf);
        fp[i].score = s; fp[i].tag = tag; fp[i].readID = ids[i]; fp[i].idx = (uint32_t)i;
    }
    mergesort_forpred(fp, (size_t)nids, fptmp);
    int n = 0;
    for (int i = nids - 1; i >= 0; i--) {
        uint32_t id = fp[i].readID;
        int hap = fp[i].tag;
        if ((hap == 0 || hap == 1) && rs->a[id].mmr_start_i != UINT32_MAX) {
            rs->a[id].hp = hap;
            insert_mmrs_to_counts(ms, rs->a[id].mmr, rs->a[id].mmr_n, (int)rs->a[id].mmr_start_i, hap);
            if (tr) {
                if (tr->cnt < tr->cap) { tr->ids[tr->cnt] = id; tr->tags[tr->cnt] = (uint8_t)hap; tr->scores[tr->cnt] = fp[i].score; }
                tr->cnt++;
            }
            n++;
            break;
        }
    }
    if (n > 0) update_range(ms, cov_rt);
    return n;
}

/* insert_ref_reads_methmer_counts (:3776-3810) */
static void insert_ref_reads(o_rs_t *rs, o_ms_t *ms, const uint32_t *ids, int n, int cov_rt) {
    for (int i = 0; i < ms->n; i++) {
        ms->mmr_a[i].keys.n = 0; ms->mmr_a[i].cnt[0].n = 0; ms->mmr_a[i].cnt[1].n = 0;
        ms->mmr_a[i].sum[0] = ms->mmr_a[i].sum[1] = 0;
    }
    for (int i = 0; i < n; i++) {
        uint32_t id = ids[i];
        int hap = rs->a[id].hp;
        if ((hap == 0 || hap == 1) && rs->a[id].mmr_start_i != UINT32_MAX)
            insert_mmrs_to_counts(ms, rs->a[id].mmr, rs->a[id].mmr_n, (int)rs->a[id].mmr_start_i, hap);
    }
    update_range(ms, cov_rt);
}

/* haplotag_region1 (:3958-4080) */
static void haplotag_region1(o_rs_t *rs, o_ms_t *ms, int n_cand, int cov_rt, int direction, o_trace_t *tr) {
    const uint32_t *ref_ids; int ref_n;
    int nreads = (int)rs->n;
    if (direction == 0) {
        ms->mmr_min_i = 0; ms->mmr_max_i = 0;
        ref_ids = rs->left.a; ref_n = (int)rs->left.n;
    } else {
        ms->mmr_min_i = (uint32_t)(ms->n - 1); ms->mmr_max_i = (uint32_t)(ms->n - 1);
        ref_ids = rs->right.a; ref_n = (int)rs->right.n;
    }
    if (direction == 0) {
        for (int i = (int)ms->mmr_max_i; i < ms->n; i++) {
            if (ms->sites_real_poss[i] <= rs->ref_start) ms->mmr_max_i++; else break;
        }
    } else {
        for (int i = (int)ms->mmr_min_i; i >= 0; i--) {
            if (ms->sites_real_poss[i] > rs->ref_end) ms->mmr_min_i--; else break;
        }
    }
    insert_ref_reads(rs, ms, ref_ids, ref_n, cov_rt);

    /* step1.5 (:4010-4025): (readID<<2)|hp round trip, set all unphased, restore */
    uint32_t *tmp = malloc(sizeof(uint32_t) * (size_t)(ref_n > 0 ? ref_n : 1));
    for (int i = 0; i < ref_n; i++) tmp[i] = (ref_ids[i] << 2) | (uint32_t)rs->a[ref_ids[i]].hp;
    for (uint32_t i = 0; i < rs->n; i++) rs->a[i].hp = 2;
    for (int i = 0; i < ref_n; i++) {
        uint32_t id = tmp[i] >> 2;
        int hp = (int)(tmp[i] & 3);
        if (id < rs->n) rs->a[id].hp = hp;   /* id>=n writes a spare slot in the reference */
    }
    free(tmp);

    int i_last = direction == 0 ? 0 : nreads - 1;
    int inc = direction == 0 ? 1 : -1;
    int failed = 0;
    uint32_t *cand = malloc(sizeof(uint32_t) * (n_cand > 0 ? n_cand : 1));
    forpred_t *fp = malloc(sizeof(forpred_t) * (n_cand > 0 ? n_cand : 1) * 2);
    vf32 buf; memset(&buf, 0, sizeof(buf));
    while (1) {
        int nc = 0;
        if ((direction == 0 && i_last >= nreads) || (direction != 0 && i_last <= 0)) break;
        for (int i0 = i_last; direction == 0 ? i0 < nreads : i0 >= 0; i0 += inc) {
            int i = direction == 0 ? i0 : (int)(uint32_t)rs->revbuf[i0];
            if (rs->a[i].hp != 0 && rs->a[i].hp != 1) {
                cand[nc++] = (uint32_t)i;
                if (nc >= n_cand) break;
            }
        }
        if (nc == 0) {
            failed++;
            if (failed > 10) break;
            i_last += n_cand * inc;
            continue;
        }
        int ins = predict_tags_of_reads(rs, ms, cand, nc, cov_rt, fp, fp + n_cand, &buf, tr);
        if (ins == 0) {
            failed++;
            if (failed > 10) break;
            i_last += n_cand * inc;
            continue;
        }
        failed = 0;
    }
    VFREE(buf);
    free(cand); free(fp);
}

/* ---------------------------------------------------------------- */
/* htslib kfunc.c kt_fisher_exact, restated (third-party, unpinned)   */
static double lbinom(int n, int k) {
    if (k == 0 || n == k) return 0;
    return lgamma(n + 1) - lgamma(k + 1) - lgamma(n - k + 1);
}
static double hypergeo(int n11, int n1_, int n_1, int n) {
    return exp(lbinom(n1_, n11) + lbinom(n - n1_, n_1 - n11) - lbinom(n, n_1));
}
typedef struct { int n11, n1_, n_1, n; double p; } hgacc_t;
static double hypergeo_acc(int n11, int n1_, int n_1, int n, hgacc_t *aux) {
    if (n1_ || n_1 || n) {
        aux->n11 = n11; aux->n1_ = n1_; aux->n_1 = n_1; aux->n = n;
    } else {
        if (n11 % 11 && n11 + aux->n - aux->n1_ - aux->n_1) {
            if (n11 == aux->n11 + 1) {
                aux->p *= (double)(aux->n1_ - aux->n11) / n11
                        * (aux->n_1 - aux->n11) / (n11 + aux->n - aux->n1_ - aux->n_1);
                aux->n11 = n11;
                return aux->p;
            }
            if (n11 == aux->n11 - 1) {
                aux->p *= (double)aux->n11 / (aux->n1_ - n11)
                        * (aux->n11 + aux->n - aux->n1_ - aux->n_1) / (aux->n_1 - n11);
                aux->n11 = n11;
                return aux->p;
            }
        }
        aux->n11 = n11;
    }
    aux->p = hypergeo(aux->n11, aux->n1_, aux->n_1, aux->n);
    return aux->p;
}
double orc_fisher_exact(int n11, int n12, int n21, int n22, double *_left, double *_right, double *two) {
    int i, j, max, min;
    double p, q, left, right;
    hgacc_t aux;
    int n1_ = n11 + n12, n_1 = n11 + n21, n = n11 + n12 + n21 + n22;
    max = (n_1 < n1_) ? n_1 : n1_;
    min = n1_ + n_1 - n;
    if (min < 0) min = 0;
    *two = *_left = *_right = 1.;
    if (min == max) return 1.;
    q = hypergeo_acc(n11, n1_, n_1, n, &aux);
    if (q == 0.0) {
        if ((double)n11 * (n + 2) < (double)(n_1 + 1) * (n1_ + 1)) { *_left = 0.0; *_right = 1.0; }
        else { *_left = 1.0; *_right = 0.0; }
        *two = 0.0;
        return 0.0;
    }
    p = hypergeo_acc(min, 0, 0, 0, &aux);
    for (left = 0., i = min + 1; p < 0.99999999 * q && i <= max; ++i)
        left += p, p = hypergeo_acc(i, 0, 0, 0, &aux);
    --i;
    if (p < 1.00000001 * q) left += p; else --i;
    p = hypergeo_acc(max, 0, 0, 0, &aux);
    for (right = 0., j = max - 1; p < 0.99999999 * q && j >= 0; --j)
        right += p, p = hypergeo_acc(j, 0, 0, 0, &aux);
    ++j;
    if (p < 1.00000001 * q) right += p; else ++j;
    *two = left + right;
    if (*two > 1.) *two = 1.;
    if (abs(i - n11) < abs(j - n11)) right = 1. - left + q;
    else left = 1.0 - right + q;
    *_left = left; *_right = right;
    return q;
}

/* evaluate_separation1 (:3881-3939) */
static float evaluate_separation1(const int buf[2][2], int *join_dir, double *p_out) {
    int hard_coverage_fail = (MINV(buf[0][0], buf[0][1]) > HARD_COV_THRESHOLD ||
                              MINV(buf[1][0], buf[1][1]) > HARD_COV_THRESHOLD);
    float min, max, scores[2];
    int which_way = 0;
    *p_out = 1.0;
    for (int i = 0; i < 2; i++) {
        if (buf[i][0] > buf[i][1]) { min = buf[i][1]; max = buf[i][0]; which_way = i == 0 ? which_way + 1 : which_way - 1; }
        else { min = buf[i][0]; max = buf[i][1]; which_way = i == 0 ? which_way - 1 : which_way + 1; }
        if (MINV(buf[0][0], buf[0][1]) > HARD_CONTAMINATE_THRESHOLD ||
            MINV(buf[1][0], buf[1][1]) > HARD_CONTAMINATE_THRESHOLD) { *join_dir = -9; return 1.0f; }
        if (max == 0) { *join_dir = -9; return 1.0f; }
        min = min == 0 ? 1 : min;
        if (max / min < 3) { *join_dir = -9; return 1.0f; }
        scores[i] = max / min;
    }
    double l, r, two;
    orc_fisher_exact(buf[0][0], buf[0][1], buf[1][0], buf[1][1], &l, &r, &two);
    *p_out = two;
    if (two < EVAL_P_THRE && !hard_coverage_fail) { *join_dir = which_way; return MINV(scores[0], scores[1]); }
    *join_dir = -9;
    return 1.0f;
}

/* haplotag_region2 (:4088-4214) at n_permutations = 1 (the only value the
 * hot path passes: :4675, :5063).  Returns join; tags left as the reference
 * leaves them (do_reset restores the entry state). */
static int haplotag_region2(o_rs_t *rs, o_ms_t *ms, const o_par_t *par, int dir, int do_reset,
                            int table[4], int *which_way_out, double *p_out, float *score_out,
                            o_trace_t *tr) {
    uint8_t *initial = malloc(rs->n ? rs->n : 1);
    for (uint32_t i = 0; i < rs->n; i++) initial[i] = (uint8_t)rs->a[i].hp;   /* store_haplotags */
    haplotag_region1(rs, ms, par->n_cand, par->cov_rt, dir, tr);
    uint8_t *after = malloc(rs->n ? rs->n : 1);
    for (uint32_t i = 0; i < rs->n; i++) after[i] = (uint8_t)rs->a[i].hp;
    /* evaluate_separation (:3940-3956) on the opposite side's strict reads */
    const vu32 *rf = dir == 0 ? &rs->right_strict : &rs->left_strict;
    int buf[2][2] = {{0, 0}, {0, 0}};
    for (size_t i = 0; i < rf->n; i++) {
        uint8_t ref = initial[rf->a[i]], q = (uint8_t)rs->a[rf->a[i]].hp;
        if (ref != 0 && ref != 1) continue;
        if (q != 0 && q != 1) continue;
        buf[ref][q]++;
    }
    table[0] = buf[0][0]; table[1] = buf[0][1]; table[2] = buf[1][0]; table[3] = buf[1][1];
    int which_way;
    float score = evaluate_separation1((const int (*)[2])buf, &which_way, p_out);
    *which_way_out = which_way;
    *score_out = score;
    int ret = -1;
    float best_score[2] = {1, 1};
    int best_i[2] = {-1, -1};
    if (score >= 2 && which_way != 0) {
        int w = which_way > 0 ? 0 : 1;
        if (score > best_score[w]) { best_score[w] = score; best_i[w] = 0; }
    }
    for (uint32_t i = 0; i < rs->n; i++) rs->a[i].hp = initial[i];     /* restore_haplotags */
    if (best_i[0] >= 0) { ret = 0; for (uint32_t i = 0; i < rs->n; i++) rs->a[i].hp = after[i]; }
    else if (best_i[1] >= 0) { ret = 1; for (uint32_t i = 0; i < rs->n; i++) rs->a[i].hp = after[i]; }
    else { ret = -1; for (uint32_t i = 0; i < rs->n; i++) rs->a[i].hp = 2; }
    if (do_reset) for (uint32_t i = 0; i < rs->n; i++) rs->a[i].hp = initial[i];
    free(initial); free(after);
    return ret;
}

/* ---------------------------------------------------------------- */
/* window driver: load_reads_given_interval bookkeeping (:1111-1163) + */
/* haplotag_region_given_bam (:4217-4335)                              */
static o_par_t window_par(const pf_cfg_t *cfg, const pf_window_batch_t *b, uint32_t w) {
    o_par_t p;
    p.k = cfg->k; p.k_span = cfg->k_span;
    p.cov_sel = b->win_cov_sel ? b->win_cov_sel[w] : cfg->cov_for_selection;
    p.cov_rt = b->win_cov_rt ? b->win_cov_rt[w] : cfg->cov_for_runtime;
    p.n_cand = b->win_n_cand ? b->win_n_cand[w] : cfg->n_cand;
    p.hard_cov = cfg->hard_cov > 0 ? cfg->hard_cov : HARD_COV_THRESHOLD;
    return p;
}

static void rs_build(o_rs_t *rs, const pf_window_batch_t *b, uint32_t w, const o_par_t *par) {
    memset(rs, 0, sizeof(*rs));
    uint32_t r0 = b->win_read_off[w], r1 = b->win_read_off[w + 1];
    uint32_t n = r1 - r0;
    int s = (int)b->win_start[w], e = (int)b->win_end[w];
    rs->a = calloc(n ? n : 1, sizeof(o_read_t));
    rs->revbuf = malloc(sizeof(uint64_t) * (n ? n : 1));
    rs->n = n; rs->n_loaded = n;
    rs->ref_start = s >= 0 ? (uint32_t)s : 0;
    rs->ref_end = (uint32_t)e;
    int left_cov[2] = {0, 0};
    for (uint32_t i = 0; i < n; i++) {
        uint32_t r = r0 + i;
        o_read_t *rd = &rs->a[i];
        rd->hp = b->read_hp[r];
        uint64_t c0 = b->read_call_off[r], c1 = b->read_call_off[r + 1];
        rd->calls_n = (uint32_t)(c1 - c0);
        rd->calls = b->call_pos + c0;
        rd->quals = b->call_cat + c0;
        uint32_t start_pos = b->read_start[r];
        uint64_t end_pos = b->read_end[r];
        rs->revbuf[i] = (end_pos << 32) | i;
        if (start_pos <= (uint32_t)s) {
            VPUSH(rs->left, i);
            if (end_pos > (uint64_t)(int64_t)s) VPUSH(rs->left_strict, i);
            if (rd->hp == 0 || rd->hp == 1) left_cov[rd->hp]++;
        } else if (end_pos >= (uint64_t)(int64_t)e) {
            VPUSH(rs->right, i);
            if (start_pos < (uint32_t)e) VPUSH(rs->right_strict, i);
        }
    }
    radix_u64_alloc(rs->revbuf, n);
    if (left_cov[0] < par->hard_cov || left_cov[1] < par->hard_cov) rs->n = 0;
}
static void rs_free(o_rs_t *rs) {
    for (uint32_t i = 0; i < rs->n_loaded; i++) free(rs->a[i].mmr);
    free(rs->a); free(rs->revbuf);
    VFREE(rs->left); VFREE(rs->left_strict); VFREE(rs->right); VFREE(rs->right_strict);
}

typedef struct {
    int table[2][4], join[2], which_way[2];
    double p[2]; float score[2];
    uint32_t n_sites, n_reads;
    int decision;
} o_winres_t;

static void run_window(const pf_cfg_t *cfg, const pf_window_batch_t *b, uint32_t w,
                       o_winres_t *res, uint8_t *hp_out, o_trace_t tr[2]) {
    o_par_t par = window_par(cfg, b, w);
    if (par.cov_sel <= 0) par.cov_sel = 1;         /* clamp (:4381-4385) */
    if (par.n_cand <= 1) par.n_cand = 2;           /* clamp (:4386-4390) */
    o_rs_t rs;
    rs_build(&rs, b, w, &par);
    memset(res, 0, sizeof(*res));
    for (int d = 0; d < 2; d++) { res->join[d] = -1; res->which_way[d] = -9; res->p[d] = 1.0; res->score[d] = 1.0f; }
    res->decision = -1;
    res->n_reads = rs.n;
    o_ms_t *ms = get_methmer_sites_and_ranges(&rs, &par, 0);
    o_ms_t *ms_bwd = get_methmer_sites_and_ranges(&rs, &par, 1);
    res->n_sites = (uint32_t)ms->n;
    if (ms->n == 0 || ms_bwd->n == 0) goto cleanup;            /* :4266-4270 */
    store_mmr_of_reads(&rs, ms_bwd);
    res->join[1] = haplotag_region2(&rs, ms_bwd, &par, 1, 1, res->table[1], &res->which_way[1],
                                    &res->p[1], &res->score[1], tr ? &tr[1] : NULL);
    wipe_mmr_of_reads(&rs);
    store_mmr_of_reads(&rs, ms);
    res->join[0] = haplotag_region2(&rs, ms, &par, 0, 0, res->table[0], &res->which_way[0],
                                    &res->p[0], &res->score[0], tr ? &tr[0] : NULL);
    if (res->join[0] != res->join[1] || (res->join[0] == -1 && res->join[1] == -1)) {
        for (uint32_t i = 0; i < rs.n; i++) rs.a[i].hp = 2;
        res->decision = -1;
    } else res->decision = res->join[0];
cleanup:
    if (hp_out) {
        uint32_t r0 = b->win_read_off[w];
        for (uint32_t i = 0; i < rs.n_loaded; i++) hp_out[r0 + i] = (uint8_t)rs.a[i].hp;
    }
    ms_free(ms); ms_free(ms_bwd);
    rs_free(&rs);
}

typedef struct {
    const pf_cfg_t *cfg; const pf_window_batch_t *b; pf_window_out_t *out;
    uint32_t next; pthread_mutex_t mu;
} o_job_t;

static void store_res(pf_window_out_t *out, uint32_t w, const o_winres_t *r) {
    if (out->decision) out->decision[w] = (int8_t)r->decision;
    for (int d = 0; d < 2; d++) {
        if (out->dir_table) for (int t = 0; t < 4; t++) out->dir_table[(w * 2 + d) * 4 + t] = r->table[d][t];
        if (out->dir_join) out->dir_join[w * 2 + d] = r->join[d];
        if (out->dir_which_way) out->dir_which_way[w * 2 + d] = r->which_way[d];
        if (out->dir_fisher_p) out->dir_fisher_p[w * 2 + d] = r->p[d];
        if (out->dir_score) out->dir_score[w * 2 + d] = r->score[d];
    }
    if (out->win_n_sites) out->win_n_sites[w] = r->n_sites;
    if (out->win_n_reads) out->win_n_reads[w] = r->n_reads;
}

static void *worker(void *arg) {
    o_job_t *j = (o_job_t *)arg;
    for (;;) {
        pthread_mutex_lock(&j->mu);
        uint32_t w = j->next++;
        pthread_mutex_unlock(&j->mu);
        if (w >= j->b->n_windows) break;
        o_winres_t r;
        run_window(j->cfg, j->b, w, &r, j->out->read_hp, NULL);
        store_res(j->out, w, &r);
    }
    return NULL;
}

int orc_methphase_windows(const pf_cfg_t *cfg, const pf_window_batch_t *b, pf_window_out_t *out, int n_threads) {
    if (!cfg || !b || !out) return PF_ERR_ARG;
    if (cfg->k < 1 || cfg->k > 15) return PF_ERR_ARG;
    o_job_t job = {cfg, b, out, 0, PTHREAD_MUTEX_INITIALIZER};
    if (n_threads <= 1) { worker(&job); return 0; }
    pthread_t *tid = malloc(sizeof(pthread_t) * n_threads);
    for (int i = 0; i < n_threads; i++) pthread_create(&tid[i], NULL, worker, &job);
    for (int i = 0; i < n_threads; i++) pthread_join(tid[i], NULL);
    free(tid);
    return 0;
}

typedef struct {
    const pf_cfg_t *cfg; const pf_load_cfg_t *lc; const pf_aln_batch_t *A; pf_window_out_t *out;
    uint32_t next; int fatal; pthread_mutex_t mu;
} o_ajob_t;

static void *aln_worker(void *arg) {
    o_ajob_t *j = (o_ajob_t *)arg;
    for (;;) {
        pthread_mutex_lock(&j->mu);
        uint32_t w = j->next++;
        pthread_mutex_unlock(&j->mu);
        if (w >= j->A->n_windows) break;
        orc_window_t lw;
        if (orc_load_window(j->lc, j->A, w, &lw) < 0) {
            pthread_mutex_lock(&j->mu); j->fatal = 1; pthread_mutex_unlock(&j->mu);
        }
        o_winres_t r;
        run_window(j->cfg, &lw.b, 0, &r, NULL, NULL);
        store_res(j->out, w, &r);
        orc_window_free(&lw);
    }
    return NULL;
}

int orc_methphase_aln(const pf_cfg_t *cfg, const pf_load_cfg_t *lc, const pf_aln_batch_t *A,
                      pf_window_out_t *out, int n_threads) {
    if (!cfg || !lc || !A || !out) return PF_ERR_ARG;
    o_ajob_t job = {cfg, lc, A, out, 0, 0, PTHREAD_MUTEX_INITIALIZER};
    if (n_threads <= 1) aln_worker(&job);
    else {
        pthread_t *tid = malloc(sizeof(pthread_t) * n_threads);
        for (int i = 0; i < n_threads; i++) pthread_create(&tid[i], NULL, aln_worker, &job);
        for (int i = 0; i < n_threads; i++) pthread_join(tid[i], NULL);
        free(tid);
    }
    return job.fatal ? -1 : 0;
}

int orc_methphase_trace(const pf_cfg_t *cfg, const pf_window_batch_t *b, uint32_t cap,
                        uint32_t *read_ids, uint8_t *tags, float *scores, uint32_t *counts) {
    for (uint32_t w = 0; w < b->n_windows; w++) {
        o_trace_t tr[2];
        for (int d = 0; d < 2; d++) {
            size_t o = ((size_t)w * 2 + d) * cap;
            tr[d].cap = cap; tr[d].cnt = 0;
            tr[d].ids = read_ids + o; tr[d].tags = tags + o; tr[d].scores = scores + o;
        }
        o_winres_t r;
        run_window(cfg, b, w, &r, NULL, tr);
        counts[w * 2] = tr[0].cnt; counts[w * 2 + 1] = tr[1].cnt;
    }
    return 0;
}

int orc_window_sites(const pf_cfg_t *cfg, const pf_window_batch_t *b, uint32_t w, int dir,
                     uint32_t *sites_real, uint32_t *sites_starts, uint8_t *lens) {
    o_par_t par = window_par(cfg, b, w);
    if (par.cov_sel <= 0) par.cov_sel = 1;
    o_rs_t rs;
    rs_build(&rs, b, w, &par);
    o_ms_t *ms = get_methmer_sites_and_ranges(&rs, &par, dir);
    int n = ms->n;
    memcpy(sites_real, ms->sites_real_poss, n * sizeof(uint32_t));
    memcpy(sites_starts, ms->sites_starts, n * sizeof(uint32_t));
    memcpy(lens, ms->mmr_lens, n);
    ms_free(ms);
    rs_free(&rs);
    return n;
}

long orc_window_methmers(const pf_cfg_t *cfg, const pf_window_batch_t *b, uint32_t w, int dir,
                         uint32_t *mmr_n, uint32_t *start_i, uint32_t *keys, long cap) {
    o_par_t par = window_par(cfg, b, w);
    if (par.cov_sel <= 0) par.cov_sel = 1;
    o_rs_t rs;
    rs_build(&rs, b, w, &par);
    o_ms_t *ms = get_methmer_sites_and_ranges(&rs, &par, dir);
    long tot = 0;
    for (uint32_t i = 0; i < rs.n_loaded; i++) { mmr_n[i] = 0; start_i[i] = 0; }
    if (ms->n > 0) {
        store_mmr_of_reads(&rs, ms);
        for (uint32_t i = 0; i < rs.n; i++) {
            mmr_n[i] = (uint32_t)rs.a[i].mmr_n;
            start_i[i] = rs.a[i].mmr_start_i;
            if (tot + rs.a[i].mmr_n > cap) { tot = -1; break; }
            memcpy(keys + tot, rs.a[i].mmr, sizeof(uint32_t) * rs.a[i].mmr_n);
            tot += rs.a[i].mmr_n;
        }
    }
    ms_free(ms);
    rs_free(&rs);
    return tot;
}

/* ---------------------------------------------------------------- */
/* -u pre-pass: parse_variants_for_one_read (:1545-1691),              */
/* haptag_one_read_with_variants (:1693-1840)                          */
static const char seq_nt16_str[] = "=ACMGRSVTWYHKDBN";   /* htslib */
static uint8_t nt4(char c) {                            /* seq_nt4_table (:74-92) */
    switch (c) { case 'A': case 'a': return 0; case 'C': case 'c': return 1;
                 case 'G': case 'g': return 2; case 'T': case 't': case 'U': case 'u': return 3;
                 default: return 4; }
}
static int md_op(char c) {                              /* md_op_table (:94-115) */
    if (c >= '0' && c <= '9') return 0;
    if (c == '^') return 1;
    switch (c) { case 'A': case 'C': case 'G': case 'T': case 'U': case 'N':
                 case 'a': case 'c': case 'g': case 't': case 'u': case 'n': return 2; }
    return 4;
}
static int natoi(const char *s, int l) {                /* :117-130 */
    if (l <= 0) return -1;
    int ret = 0;
    for (int i = 0; i < l; i++) { int e = 1; for (int j = 0; j < l - 1 - i; j++) e *= 10; ret += ((int)s[i] - 48) * e; }
    return ret;
}
typedef struct { uint32_t pos, len; uint8_t op; uint8_t ch[64]; uint8_t *chx; } o_var_t;
typedef struct { o_var_t *a; size_t n, m; } o_vvar_t;
static void vvar_push(o_vvar_t *v, uint32_t pos, int op, uint32_t len, const uint8_t *codes) {
    if (v->n == v->m) { v->m = v->m ? v->m * 2 : 32; v->a = realloc(v->a, sizeof(o_var_t) * v->m); }
    o_var_t *x = &v->a[v->n++];
    x->pos = pos; x->op = (uint8_t)op; x->len = len; x->chx = NULL;
    uint8_t *dst = x->ch;
    if (len > sizeof(x->ch)) { x->chx = malloc(len); dst = x->chx; }
    memcpy(dst, codes, len);
}
static const uint8_t *var_chars(const o_var_t *x) { return x->chx ? x->chx : x->ch; }
static void vvar_clear(o_vvar_t *v) { for (size_t i = 0; i < v->n; i++) free(v->a[i].chx); v->n = 0; }

static uint8_t seq_base_code(const uint8_t *seq, uint32_t l_qseq, uint32_t i) {
    if (i >= l_qseq) return 4;      /* past the end: reference reads past SEQ (UB); coded N */
    int nib = (seq[i >> 1] >> ((~i & 1) << 2)) & 0xf;
    return nt4(seq_nt16_str[nib]);
}

static int parse_variants_for_one_read(const pf_read_aln_batch_t *R, uint32_t r, o_vvar_t *buf) {
    uint32_t self_start = 0, ref_start = R->start[r];
    const uint32_t *cigar = R->cigar + R->cigar_off[r];
    uint32_t n_cigar = (uint32_t)(R->cigar_off[r + 1] - R->cigar_off[r]);
    const uint8_t *seq = R->seq + R->seq_off[r];
    uint32_t lq = R->seq_len[r];
    uint32_t ref_pos = ref_start, self_pos = 0;
    vu64 ins; memset(&ins, 0, sizeof(ins));
    uint8_t *tmpc = malloc(16); size_t tmpm = 16;
    for (uint32_t i = 0; i < n_cigar; i++) {
        uint32_t op = cigar[i] & 0xf, l = cigar[i] >> 4;
        if (op == 3) ref_pos += l;                               /* N */
        else if (op == 4) { if (i == 0) self_start = l; self_pos += l; }   /* S */
        else if (op == 0 || op == 7 || op == 8) { ref_pos += l; self_pos += l; }
        else if (op == 1) {                                      /* I */
            if (l > tmpm) { tmpm = l; tmpc = realloc(tmpc, tmpm); }
            for (uint32_t j = 0; j < l; j++) tmpc[j] = seq_base_code(seq, lq, self_pos + j);
            vvar_push(buf, ref_pos, PF_VAR_I, l, tmpc);
            VPUSH(ins, ((uint64_t)l) << 32 | self_pos);
            self_pos += l;
        } else if (op == 2) ref_pos += l;                        /* D */
    }
    const char *md = R->md + R->md_off[r];
    int md_l = (int)(R->md_off[r + 1] - R->md_off[r]);
    size_t prev_ins_idx = 0;
    int prev_md_i = 0, prev_md_type, md_type;
    int ret = 0;
    self_pos = self_start;
    ref_pos = ref_start;
    if (md_l <= 0) { ret = -1; goto done; }                      /* assert(tagd) (:1596) */
    prev_md_type = md_op(md[0]);
    if (prev_md_type == 2) {
        uint8_t c = seq_base_code(seq, lq, self_pos);
        vvar_push(buf, ref_pos, PF_VAR_X, 1, &c);
        ref_pos++; self_pos++;
        prev_md_type = -1;
    }
    if (prev_md_type >= 4) { ret = -1; goto done; }
    for (int i = 1; i < md_l; i++) {
        md_type = md_op(md[i]);
        if (md_type == 4) { ret = -1; goto done; }               /* fatal in reference (:1621-1624) */
        if (md_type != prev_md_type) {
            if (prev_md_type == 0) {
                int l = natoi(md + prev_md_i, i - prev_md_i);
                ref_pos += l; self_pos += l;
                while (prev_ins_idx < ins.n && self_pos > (uint32_t)ins.a[prev_ins_idx]) {
                    self_pos += (uint32_t)(ins.a[prev_ins_idx] >> 32);
                    prev_ins_idx++;
                }
            } else if (prev_md_type == 1) {
                if (md_type == 0) {
                    int l = i - prev_md_i - 1;
                    if ((size_t)l > tmpm) { tmpm = l; tmpc = realloc(tmpc, tmpm); }
                    for (int j = 0; j < l; j++) tmpc[j] = nt4(md[prev_md_i + 1 + j]);
                    vvar_push(buf, ref_pos, PF_VAR_D, (uint32_t)l, tmpc);
                    ref_pos += l;
                    prev_md_type = md_type;
                    prev_md_i = i;
                }
                continue;
            }
            if (md_type == 2) {
                uint8_t c = seq_base_code(seq, lq, self_pos);
                vvar_push(buf, ref_pos, PF_VAR_X, 1, &c);
                ref_pos++; self_pos++;
                prev_md_type = -1;
                prev_md_i = i;
            } else {
                prev_md_type = md_type;
                prev_md_i = i;
            }
        }
    }
done:
    VFREE(ins); free(tmpc);
    return ret;
}

static int haptag_one_read(const pf_known_vars_t *K, const o_vvar_t *rv, uint32_t start_pos, uint32_t end_pos,
                           int *prev_i_left, vu64 *pb) {
    if (K->n == 0) return HAPTAG_UNPHASED;
    int i_left = *prev_i_left;
    while (i_left < (int)K->n && K->pos[i_left] < start_pos) i_left++;
    *prev_i_left = i_left == 0 ? 0 : i_left - 1;
    pb->n = 0;
    const uint64_t typebit = 1ULL << 32;
    for (uint32_t i = (uint32_t)i_left; i < K->n; i++) {
        if (K->pos[i] >= end_pos) break;
        VPUSH(*pb, ((uint64_t)K->pos[i]) << 33 | i);
    }
    for (uint32_t i = 0; i < rv->n; i++) VPUSH(*pb, ((uint64_t)rv->a[i].pos) << 33 | typebit | i);
    radix_u64_alloc(pb->a, pb->n);
    int hp_cnt[2] = {0, 0}, hp;
    for (size_t i = 0; i < pb->n;) {
        if (pb->a[i] & typebit) { i++; continue; }
        uint32_t ref_pos = (uint32_t)(pb->a[i] >> 33);
        uint32_t ref_i = (uint32_t)pb->a[i];
        if (i + 1 == pb->n) { hp = K->haptag[ref_i]; hp_cnt[hp & 1]++; break; }
        uint32_t self_pos = (uint32_t)(pb->a[i + 1] >> 33);
        uint32_t self_i = (uint32_t)pb->a[i + 1];
        if (ref_pos != self_pos) {
            int skip_due_del = 0;
            if (i > 0 && (pb->a[i - 1] & typebit)) {
                uint32_t last_self_pos = (uint32_t)(pb->a[i - 1] >> 33);
                uint32_t last_self_i = (uint32_t)pb->a[i - 1];
                if (rv->a[last_self_i].op == PF_VAR_D && last_self_pos + rv->a[last_self_i].len >= ref_pos)
                    skip_due_del = 1;
            }
            if (!skip_due_del) { hp = K->haptag[ref_i]; hp_cnt[hp & 1]++; }
            i++;
        } else {
            if (!(pb->a[i + 1] & typebit)) { i += 2; }
            else {
                int ok = 1;
                const o_var_t *s = &rv->a[self_i];
                if (K->len[ref_i] == s->len) {
                    const uint8_t *kc = K->chars + K->char_off[ref_i];
                    const uint8_t *sc = var_chars(s);
                    for (uint32_t j = 0; j < s->len; j++) if (kc[j] != sc[j]) { ok = 0; break; }
                } else ok = 0;
                if (ok) { hp = K->haptag[ref_i] ^ 1; hp_cnt[hp & 1]++; }
                i += 2;
            }
        }
    }
    float mx = MAXV(hp_cnt[0], hp_cnt[1]);
    int mn = MINV(hp_cnt[0], hp_cnt[1]);
    float ratio = mn == 0 ? 0 : mx / (float)mn;
    if ((hp_cnt[0] > 3 && hp_cnt[1] > 3 && ratio < VAR_DIFF_OVERRIDE_RATIO) || hp_cnt[0] == hp_cnt[1])
        return HAPTAG_UNPHASED;
    return hp_cnt[0] > hp_cnt[1] ? 0 : 1;
}

int orc_haptag_reads(const pf_known_vars_t *known, const pf_read_aln_batch_t *reads, uint8_t *hp_out) {
    o_vvar_t rv; memset(&rv, 0, sizeof(rv));
    vu64 pb; memset(&pb, 0, sizeof(pb));
    int prev_i_left = 0;
    int rc = 0;
    for (uint32_t r = 0; r < reads->n_reads; r++) {
        vvar_clear(&rv);
        if (parse_variants_for_one_read(reads, r, &rv) < 0) { rc = PF_ERR_ARG; hp_out[r] = HAPTAG_UNPHASED; continue; }
        hp_out[r] = (uint8_t)haptag_one_read(known, &rv, reads->start[r], reads->end[r], &prev_i_left, &pb);
    }
    vvar_clear(&rv); free(rv.a); VFREE(pb);
    return rc;
}

/* ---------------------------------------------------------------- */
/* VCF -> gaps: load_intervals_from_file (:1977-2176, VCF branch),     */
/* insert_vcf_line (:1348-1430), merge_close_intervals (:2190-2218)    */
static int search_substr_idx(const char *s, const char *q, char delim) {  /* :283-314 (get_idx=1) */
    int i = 0, start = 0, col = 0, lr = (int)strlen(s), lq = (int)strlen(q);
    while (i <= lr) {
        if (s[i] == delim || i == lr) {
            if ((i - start) == lq && strncmp(q, s + start, lq) == 0) return col;
            if (i == lr) break;
            start = i + 1; col++;
        }
        i++;
    }
    return -1;
}
static int get_substr_by_idx(const char *s, int idx, char delim, int *st, int *len) {  /* :315-337 */
    int i = 0, col = 0, start = 0, lr = (int)strlen(s);
    while (i <= lr) {
        if (s[i] == delim || i == lr) {
            if (col == idx) { *st = start; *len = i - start; return 0; }
            if (i == lr) break;
            start = i + 1; col++;
        }
        i++;
    }
    return -1;
}
typedef struct {
    char name[256];
    uint32_t abs_start, abs_end;
    vu32 starts, ends;
    vu32 dropped_s, dropped_e;
    vu32 raw_s, raw_e;
} o_ref_t;

static void insert_vcf_line(char *s, const char *chrom, o_ref_t *iv, uint32_t *prev_pos, uint32_t *prev_group) {
    char *save = NULL;
    char *tok = strtok_r(s, "\t", &save);
    int i = 0, i_ps = -1, use = 0;
    uint32_t pos = 0;
    while (tok) {
        if (i == 0) { i_ps = -1; use = strcmp(tok, chrom) == 0; }
        else if (i == 1 && use) {
            pos = (uint32_t)strtoul(tok, NULL, 10);
            if (*prev_pos != UINT32_MAX && pos < *prev_pos) { fprintf(stderr, "[E::orc] vcf not sorted\n"); }
        } else if (i == 8 && use) i_ps = search_substr_idx(tok, "PS", ':');
        else if (i == 9 && use) {
            if (i_ps >= 0) {
                int ps_start = 0, ps_l = 0;
                if (get_substr_by_idx(tok, i_ps, ':', &ps_start, &ps_l) == 0 &&
                    !(ps_l == 1 && tok[ps_start] == '.')) {
                    char gid[32];
                    snprintf(gid, sizeof(gid), "%.*s", ps_l < 31 ? ps_l : 31, tok + ps_start);
                    uint32_t g = (uint32_t)strtoul(gid, NULL, 10);
                    if (*prev_group == UINT32_MAX) { *prev_group = g; *prev_pos = pos; iv->abs_start = pos; }
                    if (g == *prev_group) *prev_pos = pos;
                    else {
                        if (*prev_pos != UINT32_MAX) { VPUSH(iv->starts, *prev_pos); VPUSH(iv->ends, g); }
                        *prev_group = g; *prev_pos = pos;
                    }
                }
            }
        }
        tok = strtok_r(NULL, "\t", &save);
        i++;
    }
}

/* insert_gtf_line (:1305-1345): GTF columns 3/4 or TSV columns 1/2 (strtok
 * tokens); a block's start closes the gap [prev_end, start] when a block was
 * seen before on this contig, else it is the contig's abs_start; a block's end
 * becomes prev_end */
static void insert_gtf_line(char *s, const char *chrom, o_ref_t *iv, uint32_t *prev_end, int is_tsv) {
    char *save = NULL;
    char *tok = strtok_r(s, "\t", &save);
    const int col_s = is_tsv ? 1 : 3, col_e = is_tsv ? 2 : 4;
    int i = 0, use = 0;
    while (tok) {
        if (i == 0) use = strcmp(chrom, tok) == 0;
        else if (i == col_s && use) {
            if (*prev_end != UINT32_MAX) { VPUSH(iv->starts, *prev_end); VPUSH(iv->ends, (uint32_t)strtoul(tok, NULL, 10)); }
            else iv->abs_start = (uint32_t)strtoul(tok, NULL, 10);
        } else if (i == col_e && use) *prev_end = (uint32_t)strtoul(tok, NULL, 10);
        tok = strtok_r(NULL, "\t", &save);
        i++;
    }
}

int orc_vcf_gaps(const char *vcf_path, int readback, const char *out_path) {
    return orc_interval_gaps(vcf_path, 0, readback, out_path);
}

/* load_intervals_from_file (:1977-2176) for fmt 0 VCF, 1 GTF, 2 TSV */
int orc_interval_gaps(const char *vcf_path, int fmt, int readback, const char *out_path) {
    gzFile fp = gzopen(vcf_path, "rb");
    if (!fp) return -1;
    size_t m = 1 << 16, n = 0;
    char *all = malloc(m);
    int nr;
    char tmp[1 << 16];
    while ((nr = gzread(fp, tmp, sizeof(tmp))) > 0) {
        if (n + nr + 1 > m) { while (n + nr + 1 > m) m *= 2; all = realloc(all, m); }
        memcpy(all + n, tmp, nr); n += nr;
    }
    gzclose(fp);
    o_ref_t *refs = NULL; int ref_n = 0, ref_m = 0;
    int rp = -1;
    uint32_t prev_end = UINT32_MAX, prev_group = UINT32_MAX;
    size_t start = 0;
    for (size_t i = 0; i < n; i++) {
        if (all[i] != '\n') continue;     /* a trailing line without '\n' is never read (:2019-2020) */
        all[i] = 0;
        char *line = all + start;
        start = i + 1;
        if (line[0] == '#') continue;
        char name[256];
        size_t tl = strcspn(line, "\t");
        if (tl == 0 || tl >= sizeof(name)) continue;
        memcpy(name, line, tl); name[tl] = 0;
        int found = -1;
        for (int k = ref_n - 1; k >= 0; k--) if (strcmp(refs[k].name, name) == 0) { found = k; break; }
        if (found >= 0) rp = found;
        else {
            if (ref_n > 0 && prev_end != UINT32_MAX) refs[ref_n - 1].abs_end = prev_end;
            if (ref_n == ref_m) { ref_m = ref_m ? ref_m * 2 : 8; refs = realloc(refs, sizeof(o_ref_t) * ref_m); }
            memset(&refs[ref_n], 0, sizeof(o_ref_t));
            snprintf(refs[ref_n].name, sizeof(refs[ref_n].name), "%s", name);
            rp = ref_n++;
            prev_end = UINT32_MAX;     /* prev_group is NOT reset (:2098) */
        }
        if (fmt == 0) insert_vcf_line(line, refs[rp].name, &refs[rp], &prev_end, &prev_group);
        else insert_gtf_line(line, refs[rp].name, &refs[rp], &prev_end, fmt == 2);
    }
    if (prev_end != UINT32_MAX && rp >= 0) refs[rp].abs_end = prev_end;
    free(all);
    FILE *fo = fopen(out_path, "w");
    if (!fo) return -2;
    for (int k = 0; k < ref_n; k++) {
        o_ref_t *r = &refs[k];
        fprintf(fo, "contig\t%s\t%u\t%u\n", r->name, r->abs_start, r->abs_end);
        for (size_t i = 0; i < r->starts.n; i++) fprintf(fo, "raw\t%u\t%u\n", r->starts.a[i], r->ends.a[i]);
        if (r->starts.n > 1) {                  /* merge_close_intervals */
            size_t j = 0;
            for (size_t i = 1; i < r->starts.n; i++) {
                if ((uint32_t)(r->starts.a[i] - r->ends.a[j]) < (uint32_t)readback) {
                    VPUSH(r->dropped_s, r->ends.a[j]); VPUSH(r->dropped_e, r->starts.a[i]);
                    r->ends.a[j] = r->ends.a[i];
                } else { j++; r->starts.a[j] = r->starts.a[i]; r->ends.a[j] = r->ends.a[i]; }
            }
            r->starts.n = r->ends.n = j + 1;
        }
        for (size_t i = 0; i < r->starts.n; i++) fprintf(fo, "gap\t%u\t%u\n", r->starts.a[i], r->ends.a[i]);
        for (size_t i = 0; i < r->dropped_s.n; i++) fprintf(fo, "dropped\t%u\t%u\n", r->dropped_s.a[i], r->dropped_e.a[i]);
        VFREE(r->starts); VFREE(r->ends); VFREE(r->dropped_s); VFREE(r->dropped_e);
    }
    fclose(fo);
    free(refs);
    return ref_n;
}
