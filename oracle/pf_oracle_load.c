/*
 * pf_oracle_load.c -- CPU oracle of the window loader: read filters and 5mC
 * call extraction (reference a3/a4).
 *
 * TEST INFRASTRUCTURE ONLY (see pf_oracle.h): the checker of kernel K0.
 *
 * Restates, line by line of /root/reference/blockjoin.c:
 *   load_reads_given_interval            1043-1173 (filters, keep rule, hp)
 *   fill_read_meth_record_from_bam_line   794-908  (5mC at CpG, has_implicit)
 *   get_mod_poss_on_ref                   605-792  (CIGAR walk, implicit calls)
 *
 * The MM/ML decoding itself is htslib's (bam_parse_basemod /
 * bam_mods_at_next_pos, htslib >= 1.13, not vendored in the reference, version
 * unpinned by its Makefile:7).  It is restated here from the SAM optional-tag
 * specification that htslib implements -- PARITY UNPINNED for this part: no
 * reference test or fixture covers it.  Definitions where htslib's behaviour
 * on malformed input is not observable from the reference:
 *   - every MM entry with canonical base C and the single-letter code 'm'
 *     among its codes gives 5mC calls, whatever its strand: htslib matches an
 *     entry's canonical base against the read's base (complemented for a
 *     reverse read) and reports the strand only as a field, so a `C-m` entry
 *     counts the same C's as `C+m` (round 5; rounds 1-4 read the first C+
 *     entry alone).  At one read position the calls come in MM order
 *     (bam_mods_at_next_pos walks the entries in parse order) and the
 *     reference pushes each (blockjoin.c:846-880); get_mod_poss_on_ref then
 *     keeps the last one's quality (704-706).  Other entries (G-m, C+h, ...)
 *     only advance the ML cursor.  A position with more than N_MODS = 10
 *     modification codes (skipped whole at 840-844) is not restated: no
 *     basecaller writes that many;
 *   - an entry whose deltas run past the last C of the read (G, counted from
 *     the end, for a reverse-strand read), or an ML array shorter than the MM
 *     tag needs, yields no calls (htslib reports a parse error; the reference
 *     ignores the return code);
 *   - an absent ML tag gives every call quality 255 (HTS_MOD_UNKNOWN cast to
 *     uint8_t by blockjoin.c:869).
 */
#define _GNU_SOURCE
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "pf_oracle.h"

typedef struct { uint32_t *a; size_t n, m; } lv32;
typedef struct { uint8_t *a; size_t n, m; } lv8;
#define LPUSH(v, x) do { if ((v).n == (v).m) { (v).m = (v).m ? (v).m * 2 : 64; \
    (v).a = realloc((v).a, sizeof(*(v).a) * (v).m); } (v).a[(v).n++] = (x); } while (0)

static inline uint8_t nib(const uint8_t *s, uint32_t i) { return (s[i >> 1] >> ((~i & 1) << 2)) & 0xf; }
#define NT_C 2   /* seq_nt16 codes: "=ACMGRSVTWYHKDBN" */
#define NT_G 4

/* 5mC triggers (read position in stored orientation, ML value) in ascending
 * position order, as the reference's mod_pos loop sees them (832-882).
 * Returns the number of triggers, 0 when there are none or on a parse error. */
static int cmp_u64k(const void *a, const void *b) {
    const uint64_t x = *(const uint64_t *)a, y = *(const uint64_t *)b;
    return x < y ? -1 : x > y;
}

static size_t mm_triggers(const char *mm, size_t mm_n, const uint8_t *ml, size_t ml_n, const uint8_t *seq,
                          uint32_t len, int rev, lv32 *tpos, lv8 *tq) {
    tpos->n = tq->n = 0;
    size_t ml_cur = 0, i = 0;
    uint32_t n_ent = 0;                                 /* target entries so far (MM order) */
    lv32 ent = {0};                                     /* each trigger's entry */
    while (i < mm_n) {
        size_t e = i;
        while (e < mm_n && mm[e] != ';') e++;
        /* header: base, strand, codes, optional '.'/'?' */
        if (e - i < 3) goto fail;
        const char base = mm[i], strand = mm[i + 1];
        if (strand != '+' && strand != '-') goto fail;
        size_t h = i + 2;
        int ncodes = 0, m_idx = -1;
        if (mm[h] >= '0' && mm[h] <= '9') {            /* ChEBI code */
            while (h < e && mm[h] >= '0' && mm[h] <= '9') h++;
            ncodes = 1;
        } else {
            while (h < e && ((mm[h] >= 'a' && mm[h] <= 'z') || (mm[h] >= 'A' && mm[h] <= 'Z'))) {
                if (mm[h] == 'm' && m_idx < 0) m_idx = ncodes;
                ncodes++;
                h++;
            }
        }
        if (ncodes == 0) goto fail;
        if (h < e && (mm[h] == '.' || mm[h] == '?')) h++;
        size_t nd = 0;
        for (size_t k = h; k < e; k++) nd += mm[k] == ',';
        const int target = base == 'C' && m_idx >= 0 && nd > 0 && n_ent < 255;
        if (target) {
            if (ml_n && ml_cur + nd * (size_t)ncodes > ml_n) goto fail;
            /* ranks of the called C's among the read's C's (original orientation) */
            uint64_t rank = 0;
            lv32 ranks = {0};
            size_t k = h;
            for (size_t d = 0; d < nd; d++) {
                if (k >= e || mm[k] != ',') { free(ranks.a); goto fail; }
                k++;
                uint64_t v = 0;
                size_t k0 = k;
                while (k < e && mm[k] >= '0' && mm[k] <= '9') v = v * 10 + (uint64_t)(mm[k++] - '0');
                if (k == k0 || v > 0xFFFFFFFFull) { free(ranks.a); goto fail; }
                rank += v + (d ? 1 : 0);
                if (rank > 0xFFFFFFFFull) { free(ranks.a); goto fail; }
                LPUSH(ranks, (uint32_t)rank);
            }
            /* count the target bases: C forward, G (= complement of C) reverse */
            const uint8_t tb = rev ? NT_G : NT_C;
            uint64_t n_t = 0;
            for (uint32_t p = 0; p < len; p++) n_t += nib(seq, p) == tb;
            if (nd && ranks.a[nd - 1] >= n_t) { free(ranks.a); goto fail; }
            /* walk positions in stored order; a reverse read's C ranks count from the end */
            size_t d = rev ? nd : 0;
            uint64_t seen = 0;
            for (uint32_t p = 0; p < len; p++) {
                if (nib(seq, p) != tb) continue;
                const uint64_t r = rev ? n_t - 1 - seen : seen;
                seen++;
                if (rev) {
                    if (d > 0 && ranks.a[d - 1] == r) {
                        d--;
                        LPUSH(*tpos, p);
                        LPUSH(*tq, ml_n ? ml[ml_cur + d * ncodes + m_idx] : 255);
                        LPUSH(ent, n_ent);
                    }
                } else if (d < nd && ranks.a[d] == r) {
                    LPUSH(*tpos, p);
                    LPUSH(*tq, ml_n ? ml[ml_cur + d * ncodes + m_idx] : 255);
                    LPUSH(ent, n_ent);
                    d++;
                }
            }
            free(ranks.a);
            n_ent++;
        }
        ml_cur += nd * (size_t)ncodes;
        i = e + 1;
    }
    if (ml_n && ml_cur > ml_n) { tpos->n = tq->n = 0; }
    if (n_ent > 1 && tpos->n) {                        /* several entries: position order, ties in MM order */
        uint64_t *k = (uint64_t *)malloc(tpos->n * sizeof(uint64_t));
        for (size_t j = 0; j < tpos->n; j++)
            k[j] = ((uint64_t)tpos->a[j] << 40) | ((uint64_t)ent.a[j] << 32) | ((uint64_t)tq->a[j] << 24) | j;
        qsort(k, tpos->n, sizeof(uint64_t), cmp_u64k);
        for (size_t j = 0; j < tpos->n; j++) { tpos->a[j] = (uint32_t)(k[j] >> 40); tq->a[j] = (uint8_t)(k[j] >> 24); }
        free(k);
    }
    free(ent.a);
    return tpos->n;
fail:
    free(ent.a);
    tpos->n = tq->n = 0;
    return 0;
}

/* get_mod_poss_on_ref (605-792).  calls/quals are appended to out_pos/out_q.
 * Returns 0 when the read has no CIGAR or no 5mC call, -1 on a CIGAR
 * operation the reference treats as fatal (776-779), 1 otherwise. */
static int mod_poss_on_ref(lv32 *cp, lv8 *cq, const uint32_t *cigar, uint32_t cigar_l, uint32_t qs,
                           int strand, const uint32_t *mod_poss, const uint8_t *mod_q, uint32_t mod_l,
                           const uint8_t *seqi, uint32_t aln_len) {
    if (cigar_l == 0 || mod_l == 0) return 0;
    const uint32_t cgoffset = strand ? (uint32_t)-1 : 0;
    uint32_t i_read = 0, i_ref = qs, i_trigger = 0;
    uint32_t next_trigger = mod_poss[0];
    uint8_t next_qual = mod_q[0];
    uint32_t i_cigar = 0;
#define PUSH(v, q) do { LPUSH(*cp, (v)); LPUSH(*cq, (q)); } while (0)
    if ((cigar[0] & 15) == 4) {                          /* leading soft clip (629-652) */
        i_read = cigar[0] >> 4;
        while (next_trigger < i_read) {
            i_trigger++;
            if (i_trigger < mod_l) { next_trigger = mod_poss[i_trigger]; next_qual = mod_q[i_trigger]; }
            else break;
        }
        if (next_trigger == i_read) {
            PUSH(i_ref + cgoffset, next_qual);
            i_trigger++;
            if (i_trigger < mod_l) { next_trigger = mod_poss[i_trigger]; next_qual = mod_q[i_trigger]; }
        }
        i_ref -= cigar[0] >> 4;
        i_cigar = 1;
    }
    uint32_t offset = 0;                                 /* int in the reference; same bits */
    for (; i_cigar < cigar_l; i_cigar++) {
        const uint32_t op = cigar[i_cigar] & 15, length = cigar[i_cigar] >> 4;
        if (op <= 1) {                                   /* M, I (660-769) */
            uint32_t pos_canonical = i_read;
            while (i_read + length >= next_trigger) {
                if (op == 0 && next_trigger != UINT32_MAX) {
                    if (seqi) {                          /* implicit canonicals before the call (666-700) */
                        const uint32_t a = next_trigger - 1, b = i_read + length;
                        const uint32_t until = a < b ? a : b;
                        for (uint32_t t = pos_canonical; t < until; t++) {
                            if (t < aln_len - 1 && nib(seqi, t) == NT_C && nib(seqi, t + 1) == NT_G) {
                                const uint32_t pc = i_ref + t + offset;
                                if (!(cp->n > 0 && cp->a[cp->n - 1] == pc)) PUSH(pc, 1);
                                t++;
                            }
                        }
                    }
                    const uint32_t pt = i_ref + next_trigger + cgoffset + offset;   /* (703-710) */
                    if (cp->n > 0 && cp->a[cp->n - 1] == pt) cq->a[cq->n - 1] = next_qual;
                    else PUSH(pt, next_qual);
                    pos_canonical = cgoffset == 0 ? next_trigger + 1 : next_trigger + 2;
                }
                i_trigger++;
                if (i_trigger >= mod_l) { next_trigger = UINT32_MAX; break; }
                next_trigger = mod_poss[i_trigger];
                next_qual = mod_q[i_trigger];
            }
            if (op == 0) {
                if (seqi) {                              /* implicit canonicals to the op's end (727-761) */
                    const uint32_t until = i_read + length;
                    for (uint32_t t = pos_canonical; t < until; t++) {
                        if (t < aln_len - 1 && nib(seqi, t) == NT_C && nib(seqi, t + 1) == NT_G) {
                            const uint32_t pc = i_ref + t + offset;
                            if (!(cp->n > 0 && cp->a[cp->n - 1] == pc)) PUSH(pc, 1);
                            t++;
                        }
                    }
                }
                i_read += length;
            } else {
                i_read += length;
                offset -= length;
            }
        } else if (op == 2) {                            /* D */
            offset += length;
        } else if (op == 3 || op == 4) {                 /* N, S: stop (771-775) */
            break;
        } else {
            return -1;                                   /* fatal in the reference (776-779) */
        }
    }
#undef PUSH
    return 1;
}

/* fill_read_meth_record_from_bam_line (794-908) for record r. */
static int fill_read(const pf_aln_batch_t *A, uint32_t r, uint8_t lo, uint8_t hi, lv32 *tp, lv8 *tq, lv32 *mp,
                     lv8 *mq, lv32 *cp, lv8 *cq) {
    const uint32_t len = A->l_qseq[r];
    const int strand = !!(A->flag[r] & 16);
    const uint8_t *seq = A->seq + A->seq_off[r];
    const size_t nt = mm_triggers(A->mm + A->mm_off[r], A->mm_off[r + 1] - A->mm_off[r], A->ml + A->ml_off[r],
                                  A->ml_off[r + 1] - A->ml_off[r], seq, len, strand, tp, tq);
    int has_implicit = 0;
    mp->n = mq->n = 0;
    for (size_t i = 0; i < nt; i++) {                   /* 845-880 */
        const uint32_t p = tp->a[i];
        if (!(p < len - 1 && p > 0)) continue;
        const int ok = nib(seq, p) == NT_C ? nib(seq, p + 1) == NT_G : nib(seq, p - 1) == NT_C;
        if (!ok) { has_implicit = 1; continue; }
        LPUSH(*mp, p);
        const uint8_t q = tq->a[i];
        LPUSH(*mq, q < lo ? 1 : q >= hi ? 0 : 2);
    }
    return mod_poss_on_ref(cp, cq, A->cigar + A->cigar_off[r], (uint32_t)(A->cigar_off[r + 1] - A->cigar_off[r]),
                           A->pos[r], strand, mp->a, mq->a, (uint32_t)mp->n, has_implicit ? seq : NULL, len);
}

static uint32_t bam_endpos_(const pf_aln_batch_t *A, uint32_t r) {
    const uint64_t c0 = A->cigar_off[r], c1 = A->cigar_off[r + 1];
    if ((A->flag[r] & 4) || c1 == c0) return A->pos[r] + 1;
    uint32_t rl = 0;
    for (uint64_t c = c0; c < c1; c++) {
        const uint32_t op = A->cigar[c] & 15;
        if (op == 0 || op == 2 || op == 3 || op == 7 || op == 8) rl += A->cigar[c] >> 4;
    }
    return A->pos[r] + rl;
}

int orc_load_reads(const pf_load_cfg_t *lc, const pf_aln_batch_t *A, uint32_t *rec_read, uint32_t *win_read_off,
                   uint32_t *read_start, uint32_t *read_end, uint8_t *read_hp, uint64_t *call_off,
                   uint32_t *call_pos, uint8_t *call_cat, uint64_t call_cap, uint64_t *n_calls_out) {
    lv32 tp = {0}, mp = {0}, cp = {0};
    lv8 tq = {0}, mq = {0}, cq = {0};
    const uint8_t lo = (uint8_t)lc->qual_lo, hi = (uint8_t)lc->qual_hi;
    uint32_t R = 0;
    uint64_t N = 0;
    int rc = 0;
    if (win_read_off) win_read_off[0] = 0;
    for (uint32_t w = 0; w < A->n_windows; w++) {
        for (uint32_t r = A->win_rec_off[w]; r < A->win_rec_off[w + 1]; r++) {
            rec_read[r] = UINT32_MAX;
            const uint32_t flag = A->flag[r], mapq = A->mapq[r], len = A->l_qseq[r];
            const float de = A->de[r];
            if ((flag & 4) || (flag & 256) || (flag & 2048)) continue;      /* 1081 */
            if (mapq < (uint32_t)lc->min_mapq) continue;                   /* 1082 */
            if (len < 2 || len < (uint32_t)lc->min_len) continue;          /* 1083 */
            if ((double)de > 0.1) continue;                                /* 1084, MIN_ALN_DE */
            cp.n = cq.n = 0;
            const int st = fill_read(&A[0], r, lo, hi, &tp, &tq, &mp, &mq, &cp, &cq);
            if (st < 0) { rc = -1; goto done; }
            if (st == 0) continue;                                         /* 933-936 */
            rec_read[r] = R;
            if (read_start) read_start[R] = A->pos[r];
            if (read_end) read_end[R] = bam_endpos_(A, r);
            if (read_hp) read_hp[R] = A->hp[r];
            if (call_off) call_off[R] = N;
            if (N + cp.n <= call_cap) {
                memcpy(call_pos + N, cp.a, cp.n * 4);
                memcpy(call_cat + N, cq.a, cq.n);
            }
            N += cp.n;
            R++;
        }
        if (win_read_off) win_read_off[w + 1] = R;
    }
    if (call_off) call_off[R] = N;
    rc = (int)R;
    if (N > call_cap) rc = -2;
done:
    if (n_calls_out) *n_calls_out = N;
    free(tp.a); free(tq.a); free(mp.a); free(mq.a); free(cp.a); free(cq.a);
    return rc;
}

/* One window loaded into a self-owned single-window batch (the per-window
 * load_reads_given_interval call of haplotag_region_given_bam, 4217-4240):
 * used by orc_methphase_aln, the record-level CPU path. */
int orc_load_window(const pf_load_cfg_t *lc, const pf_aln_batch_t *A, uint32_t w, orc_window_t *o) {
    lv32 tp = {0}, mp = {0}, cp = {0}, rs = {0}, re = {0}, pos = {0};
    lv8 tq = {0}, mq = {0}, cq = {0}, hp = {0}, cat = {0};
    typedef struct { uint64_t *a; size_t n, m; } lv64;
    lv64 off = {0};
    const uint8_t lo = (uint8_t)lc->qual_lo, hi = (uint8_t)lc->qual_hi;
    int rc = 0;
    LPUSH(off, 0);
    for (uint32_t r = A->win_rec_off[w]; r < A->win_rec_off[w + 1]; r++) {
        const uint32_t flag = A->flag[r], mapq = A->mapq[r], len = A->l_qseq[r];
        if ((flag & 4) || (flag & 256) || (flag & 2048)) continue;
        if (mapq < (uint32_t)lc->min_mapq) continue;
        if (len < 2 || len < (uint32_t)lc->min_len) continue;
        if ((double)A->de[r] > 0.1) continue;
        cp.n = cq.n = 0;
        const int st = fill_read(A, r, lo, hi, &tp, &tq, &mp, &mq, &cp, &cq);
        if (st < 0) { rc = -1; break; }
        if (st == 0) continue;
        LPUSH(rs, A->pos[r]);
        LPUSH(re, bam_endpos_(A, r));
        LPUSH(hp, A->hp[r]);
        for (size_t i = 0; i < cp.n; i++) { LPUSH(pos, cp.a[i]); LPUSH(cat, cq.a[i]); }
        LPUSH(off, (uint64_t)pos.n);
    }
    free(tp.a); free(tq.a); free(mp.a); free(mq.a); free(cp.a); free(cq.a);
    memset(o, 0, sizeof(*o));
    o->win_start = A->win_start[w];
    o->win_end = A->win_end[w];
    o->win_read_off[0] = 0;
    o->win_read_off[1] = (uint32_t)rs.n;
    o->read_start = rs.a; o->read_end = re.a; o->read_hp = hp.a;
    o->read_call_off = off.a; o->call_pos = pos.a; o->call_cat = cat.a;
    memset(&o->b, 0, sizeof(o->b));
    o->b.n_windows = 1;
    o->b.n_reads = (uint32_t)rs.n;
    o->b.n_calls = pos.n;
    o->b.win_start = &o->win_start;
    o->b.win_end = &o->win_end;
    o->b.win_read_off = o->win_read_off;
    o->b.win_cov_sel = A->win_cov_sel ? A->win_cov_sel + w : NULL;
    o->b.win_cov_rt = A->win_cov_rt ? A->win_cov_rt + w : NULL;
    o->b.win_n_cand = A->win_n_cand ? A->win_n_cand + w : NULL;
    o->b.read_start = rs.a; o->b.read_end = re.a; o->b.read_hp = hp.a;
    o->b.read_call_off = off.a; o->b.call_pos = pos.a; o->b.call_cat = cat.a;
    return rc;
}

void orc_window_free(orc_window_t *o) {
    free(o->read_start); free(o->read_end); free(o->read_hp);
    free((void *)o->read_call_off); free(o->call_pos); free(o->call_cat);
    memset(o, 0, sizeof(*o));
}
