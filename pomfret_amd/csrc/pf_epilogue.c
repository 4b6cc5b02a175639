/*
 * pf_epilogue.c -- the methphase output epilogue on the host.
 *
 * From the per-window join decisions of pf_methphase_* and the gaps of
 * pf_vcf_gaps, in the order main_blockjoin runs them (reference
 * blockjoin.c:4685-4712):
 *   pf_phase_blocks: lift_decisions (:2250-2310) -> make_decisions_flippings_
 *                    onraw (:2312-2324) -> generate_new_phase_blocks(use_raw=1)
 *                    (:2326-2362);
 *   pf_write_gtf / pf_write_tsv: output_gtf (:2721-2756) / output_tsv (:2696-2719);
 *   pf_write_vcf:    output_modify_vcf (:2918-2988) over alter_vcf_line
 *                    (:2758-2916), with get_new_phaseblock_ID (:2366-2395),
 *                    tmp_check_if_in_dropped_intervals (:2397-2409) and
 *                    get_flip_status (:2444-2481).
 *
 * Behaviour kept from the reference:
 *   - merge_close_intervals leaves decisions.n at the raw gap count
 *     (:2219), so lift_decisions also visits indices past the merged gaps,
 *     with decision -1 and the stale raw end there;
 *   - the last phase block starts at the last unjoined gap's START
 *     (:2355-2360), a contig without gaps gets no block at all, GTF skips
 *     blocks starting or ending at 0 (:2743);
 *   - the flip cursor of get_flip_status only resets when POS decreases
 *     (:2811-2815) and moves down by one per call when it is past the end;
 *   - the GT edits index the rewritten line with the ORIGINAL column offsets
 *     (:2898-2912), so a FORMAT with PS before GT gets its bytes shifted, and
 *     a flip writes GT[2] from the already flipped GT[0] (0|0 -> 1|0);
 *   - a phased line inside a dropped interval is left untouched unless the
 *     rescue map (recover_variant_phase_in_dropped_intervals, :2618-2694,
 *     supplied by the caller) has its 0-based position with hap 0 or 1: then
 *     PS becomes "." and GT's separator '/' (:2875-2889);
 *   - a final line without '\n' is never processed nor written.
 * Reference undefined behaviour, defined here: a FORMAT PS/GT index without a
 * matching sample field leaves the line as is (the reference reads
 * uninitialised offsets); flips_onraw reads out of range (a contig with
 * phased lines but no gaps: NULL dereference in the reference) give 0; a GT
 * edit past the end of the rewritten line is skipped; a missing raw gap in
 * lift_decisions (assert) is PF_ERR_ARG.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>

#include "../../include/pomfret_amd.h"

void pf_blocks_free(pf_blocks_t *b) {
    if (!b) return;
    free(b->raw_off); free(b->raw_start); free(b->raw_end);
    free(b->dec_off); free(b->dec_onraw); free(b->flip);
    free(b->blk_off); free(b->blk_start); free(b->blk_end);
    free(b);
}

int pf_phase_blocks(const pf_gaps_t *g, const int8_t *decision, pf_blocks_t **out) {
    if (!g || !out || (g->gap_off[g->n_contigs] && !decision)) return PF_ERR_ARG;
    *out = NULL;
    const uint32_t C = g->n_contigs;
    const uint64_t NR = g->raw_off[C];
    pf_blocks_t *b = (pf_blocks_t *)calloc(1, sizeof(pf_blocks_t));
    if (!b) return PF_ERR_NOMEM;
    b->n_contigs = C;
    b->raw_off = (uint64_t *)calloc(C + 1, 8);
    b->dec_off = (uint64_t *)calloc(C + 1, 8);
    b->blk_off = (uint64_t *)calloc(C + 1, 8);
    /* every count is bounded by the raw gap count (+1 block per contig) */
    b->raw_start = (uint32_t *)malloc((NR + 1) * 4);
    b->raw_end = (uint32_t *)malloc((NR + 1) * 4);
    b->dec_onraw = (int32_t *)malloc((NR + 1) * 4);
    b->flip = (int32_t *)malloc((NR + 1) * 4);
    b->blk_start = (uint32_t *)malloc((NR + C + 1) * 4);
    b->blk_end = (uint32_t *)malloc((NR + C + 1) * 4);
    if (!b->raw_off || !b->dec_off || !b->blk_off || !b->raw_start || !b->raw_end || !b->dec_onraw ||
        !b->flip || !b->blk_start || !b->blk_end) {
        pf_blocks_free(b);
        return PF_ERR_NOMEM;
    }
    uint64_t kr = 0, kd = 0, kb = 0;
    for (uint32_t c = 0; c < C; c++) {
        const uint64_t r0 = g->raw_off[c], nr = g->raw_off[c + 1] - r0;
        const uint64_t g0 = g->gap_off[c], ng = g->gap_off[c + 1] - g0;
        /* rawunphasedblocks (store_raw_intervals, :2178-2188), edited in place */
        uint32_t *rs = b->raw_start + kr, *re = b->raw_end + kr;
        memcpy(rs, g->raw_start + r0, nr * 4);
        memcpy(re, g->raw_end + r0, nr * 4);
        uint64_t n = nr;
        int32_t *don = b->dec_onraw + kd;
        uint64_t nd = 0;
        /* lift_decisions (:2250-2310) over decisions.n = the raw gap count */
        uint64_t j = 0;
        for (uint64_t i = 0; i < nr; i++) {
            const int32_t d = i < ng ? (int32_t)decision[g0 + i] : -1;
            const uint32_t endi = i < ng ? g->gap_end[g0 + i] : g->raw_end[r0 + i];
            if (d < 0) {
                while (j < n && re[j] <= endi) { don[nd++] = d; j++; }
            } else {
                if (j >= n) { pf_blocks_free(b); return PF_ERR_ARG; }
                if (re[j] < endi) {
                    uint64_t j2 = j;
                    while (j2 < n && re[j2] != endi) j2++;
                    if (j2 == n) { pf_blocks_free(b); return PF_ERR_ARG; }  /* assert(found) */
                    re[j] = endi;
                    for (uint64_t l = j + 1, r = j2 + 1; r < n; l++, r++) { rs[l] = rs[r]; re[l] = re[r]; }
                    n -= j2 - j;
                }
                don[nd++] = d;
                j++;
            }
        }
        /* make_decisions_flippings_onraw (:2312-2324) */
        int32_t flip = 0;
        for (uint64_t i = 0; i < nd; i++) {
            flip = don[i] < 0 ? 0 : flip ^ don[i];
            b->flip[kd + i] = flip;
        }
        /* generate_new_phase_blocks, use_raw = 1 (:2326-2362) */
        uint32_t start = g->abs_start[c], end = UINT32_MAX;
        for (uint64_t i = 0; i < nd; i++) {
            if (don[i] >= 0) continue;
            end = rs[i];
            b->blk_start[kb] = start;
            b->blk_end[kb] = end;
            kb++;
            start = re[i];
        }
        if (nd > 0 && end != g->abs_end[c]) {
            end = end == UINT32_MAX ? g->abs_start[c] : end;
            b->blk_start[kb] = end;
            b->blk_end[kb] = g->abs_end[c];
            kb++;
        }
        kr += n;
        kd += nd;
        b->raw_off[c + 1] = kr;
        b->dec_off[c + 1] = kd;
        b->blk_off[c + 1] = kb;
    }
    *out = b;
    return PF_OK;
}

int pf_write_gtf(const pf_gaps_t *g, const pf_blocks_t *b, const char *path) {
    if (!g || !b || !path || b->n_contigs != g->n_contigs) return PF_ERR_ARG;
    FILE *fp = fopen(path, "w");
    if (!fp) return -1;
    for (uint32_t c = 0; c < g->n_contigs; c++)
        for (uint64_t i = b->blk_off[c]; i < b->blk_off[c + 1]; i++) {
            const int s = (int)b->blk_start[i], e = (int)b->blk_end[i];
            if (s == 0 || e == 0) continue;                  /* placeholders (:2743) */
            fprintf(fp, "%s\tPhasing\texon\t%d\t%d\t.\t+\t.\tgene_id \"%d\"; transcript_id \"%d.1\"\n",
                    g->names[c], s, e, s, s);
        }
    return fclose(fp) == 0 ? PF_OK : -1;
}

int pf_write_tsv(const pf_gaps_t *g, const pf_blocks_t *b, const char *path) {
    if (!g || !b || !path || b->n_contigs != g->n_contigs) return PF_ERR_ARG;
    FILE *fp = fopen(path, "w");
    if (!fp) return -1;
    for (uint32_t c = 0; c < g->n_contigs; c++)
        for (uint64_t i = b->blk_off[c]; i < b->blk_off[c + 1]; i++)
            fprintf(fp, "%s\t%d\t%d\n", g->names[c], (int)b->blk_start[i], (int)b->blk_end[i]);
    return fclose(fp) == 0 ? PF_OK : -1;
}

/* ---------------------------------------------------------------- VCF */

typedef struct {
    const pf_gaps_t *g;
    const pf_blocks_t *b;
    const pf_rescue_t *rescue;
    int prev_group_idx, prev_block_idx, last_pos;
    char *nl;               /* rewritten line */
    size_t nl_cap;
    int64_t n_mod, n_drop, n_tot;
} vcf_state_t;

/* search_substr_idx(s, q, ':', 1, s_l, 0) (:283-313) for a 2-letter tag */
static int tag_index(const char *s, size_t l, const char *q) {
    size_t start = 0;
    int col = 0;
    for (size_t i = 0; i <= l; i++) {
        if (i == l || s[i] == ':') {
            if (i - start == 2 && s[start] == q[0] && s[start + 1] == q[1]) return col;
            if (i == l) break;
            start = i + 1;
            col++;
        }
    }
    return -1;
}

/* get_substr_by_idx (:315-337) */
static int sub_by_idx(const char *s, size_t l, int idx, size_t *fs, size_t *fl) {
    size_t start = 0;
    int col = 0;
    for (size_t i = 0; i <= l; i++) {
        if (i == l || s[i] == ':') {
            if (col == idx) { *fs = start; *fl = i - start; return 0; }
            if (i == l) break;
            start = i + 1;
            col++;
        }
    }
    return -1;
}

static int32_t flip_at(const pf_blocks_t *b, uint32_t c, int64_t k) {
    const uint64_t d0 = b->dec_off[c], nd = b->dec_off[c + 1] - d0;
    return k >= 0 && (uint64_t)k < nd ? b->flip[d0 + k] : 0;
}

/* get_flip_status (:2444-2481) */
static int32_t flip_status(vcf_state_t *v, uint32_t c, int pos) {
    const pf_blocks_t *b = v->b;
    const uint64_t r0 = b->raw_off[c];
    const int64_t n = (int64_t)(b->raw_off[c + 1] - r0);
    int64_t j = v->prev_block_idx;
    /* (int j < size_t n: a negative cursor skips the loop) */
    for (; j >= 0 && j < n; j++) {
        const int start = (int)b->raw_start[r0 + j];
        if (start >= pos) {
            v->prev_block_idx = j == 0 ? 0 : (int)(j - 1);
            int32_t stat = flip_at(b, c, v->prev_block_idx);
            if (n > 0 && (uint32_t)pos <= b->raw_start[r0]) stat = 0;   /* before the first gap */
            return stat;
        }
    }
    v->prev_block_idx = (int)(j - 1);
    return flip_at(b, c, n == 0 ? 0 : n - 1);
}

/* hap of the REF allele at 0-based pos in the caller's rescue map, or -1 */
static int rescue_hap(const pf_rescue_t *r, uint32_t c, uint32_t pos0) {
    if (!r) return -1;
    uint64_t lo = r->off[c], hi = r->off[c + 1];
    while (lo < hi) {
        const uint64_t mid = (lo + hi) / 2;
        if (r->pos[mid] < pos0) lo = mid + 1;
        else hi = mid;
    }
    return lo < r->off[c + 1] && r->pos[lo] == pos0 ? r->hap_of_ref[lo] : -1;
}

static int grow_nl(vcf_state_t *v, size_t need) {
    if (need <= v->nl_cap) return 0;
    char *p = (char *)realloc(v->nl, need);
    if (!p) return -1;
    v->nl = p;
    v->nl_cap = need;
    return 0;
}

/* alter_vcf_line (:2758-2916): 0 unchanged, 1 rewritten, 2 rescued to
 * unphased (v->nl holds the new line), PF_ERR_ARG on a bad #CHROM header */
static int alter_line(vcf_state_t *v, const char *s, size_t l, size_t *nl_len) {
    if (l > 0 && s[0] == '#') {
        if (l > 1 && s[1] == '#') return 0;
        int n = 1;
        for (size_t i = 0; i < l; i++) n += s[i] == '\t';
        return n == 10 ? 0 : PF_ERR_ARG;
    }
    const pf_gaps_t *g = v->g;
    int col = 0;
    size_t start = 0;
    int pos = 0, i_ps = -1, i_gt = -1;
    uint32_t c = 0;
    for (size_t i = 0; i < l; i++) {
        if (s[i] != '\t') continue;
        if (col == 0) {
            const size_t nl = i - start;
            for (c = 0; c < g->n_contigs; c++)
                if (strlen(g->names[c]) == nl && memcmp(g->names[c], s + start, nl) == 0) break;
            pos = 0;
            i_ps = -1;
            i_gt = -1;
            if (c == g->n_contigs) break;
        } else if (col == 1) {
            char tmp[21];
            const size_t tl = i - start < 20 ? i - start : 20;
            memcpy(tmp, s + start, tl);
            tmp[tl] = 0;
            pos = atoi(tmp);
            if (pos < v->last_pos) {                       /* a new chromosome (:2811-2815) */
                v->prev_group_idx = 0;
                v->prev_block_idx = 0;
            }
            v->last_pos = pos;
        } else if (col == 8) {
            /* search_substr_idx with s_l = 0 scans to the end of the line */
            const size_t fl = i - start ? i - start : l - start;
            i_ps = tag_index(s + start, fl, "PS");
            i_gt = tag_index(s + start, fl, "GT");
        }
        col++;
        start = i + 1;
    }
    if (pos == 0 || i_ps < 0) return 0;
    const char *smp = s + start;
    const size_t sl = l - start;
    size_t ps_s, ps_l, gt_s, gt_l;
    if (sub_by_idx(smp, sl, i_ps, &ps_s, &ps_l) || sub_by_idx(smp, sl, i_gt, &gt_s, &gt_l)) return 0;
    if (ps_l == 1 && smp[ps_s] == '.') return 0;
    char GT[10] = {0};
    memcpy(GT, smp + gt_s, gt_l < 9 ? gt_l : 9);
    if (GT[1] != '|') return 0;
    if (GT[0] != '0' && GT[0] != '1') return 0;
    if (GT[2] != '0' && GT[2] != '1') return 0;

    /* get_new_phaseblock_ID1 (:2366-2383) */
    int group = -1;
    {
        const pf_blocks_t *b = v->b;
        for (uint64_t i = b->blk_off[c]; i < b->blk_off[c + 1]; i++) {
            const uint32_t bs = b->blk_start[i], be = b->blk_end[i];
            if (bs == UINT32_MAX || be == 0 || be == UINT32_MAX) continue;
            if ((uint32_t)pos >= bs && (uint32_t)pos < be) {
                v->prev_group_idx = (int)(i - b->blk_off[c]);
                group = (int)bs;
                break;
            }
        }
    }
    /* tmp_check_if_in_dropped_intervals (:2397-2409), inclusive ends */
    int dropped = 0;
    for (uint64_t i = g->drop_off[c]; i < g->drop_off[c + 1]; i++)
        if ((uint32_t)pos >= g->drop_start[i] && (uint32_t)pos <= g->drop_end[i]) { dropped = 1; break; }
    const int32_t need_flip = flip_status(v, c, pos);
    int middle = 0;
    if (group >= 0 && dropped) {
        const int h = rescue_hap(v->rescue, c, (uint32_t)pos - 1u);
        middle = h == 0 || h == 1;
    }
    const size_t off = start + ps_s;
    if (group < 0 || dropped) {
        if (!middle) return 0;
        const size_t len = off + 1 + (l - off - ps_l);
        if (grow_nl(v, len + 1)) return PF_ERR_NOMEM;
        memcpy(v->nl, s, off);
        v->nl[off] = '.';
        memcpy(v->nl + off + 1, s + off + ps_l, l - off - ps_l);
        v->nl[len] = 0;
        if (start + gt_s + 1 < len) v->nl[start + gt_s + 1] = '/';
        *nl_len = len;
        return 2;
    }
    char num[16];
    const int nd = snprintf(num, sizeof num, "%d", group);
    const size_t len = off + (size_t)nd + (l - off - ps_l);
    if (grow_nl(v, len + 1)) return PF_ERR_NOMEM;
    memcpy(v->nl, s, off);
    memcpy(v->nl + off, num, (size_t)nd);
    memcpy(v->nl + off + nd, s + off + ps_l, l - off - ps_l);
    v->nl[len] = 0;
    if (need_flip) {
        const size_t a = start + gt_s;
        if (a < len) v->nl[a] = v->nl[a] == '0' ? '1' : '0';
        if (a + 2 < len) v->nl[a + 2] = v->nl[a] == '0' ? '1' : '0';
    }
    *nl_len = len;
    return 1;
}

int pf_write_vcf(const char *vcf_in, const pf_gaps_t *g, const pf_blocks_t *b, const pf_rescue_t *rescue,
                 const char *vcf_out, int64_t *counts) {
    if (!vcf_in || !g || !b || !vcf_out || b->n_contigs != g->n_contigs) return PF_ERR_ARG;
    gzFile in = gzopen(vcf_in, "rb");
    if (!in) return -1;
    FILE *out = fopen(vcf_out, "w");
    if (!out) { gzclose(in); return -1; }
    vcf_state_t v;
    memset(&v, 0, sizeof v);
    v.g = g;
    v.b = b;
    v.rescue = rescue;
    v.last_pos = -1;
    size_t cap = 1 << 16, len = 0;
    char *buf = (char *)malloc(cap);
    int rc = buf ? 0 : PF_ERR_NOMEM;
    while (!rc) {
        if (len == cap) {
            char *p = (char *)realloc(buf, cap * 2);
            if (!p) { rc = PF_ERR_NOMEM; break; }
            buf = p;
            cap *= 2;
        }
        const int nr = gzread(in, buf + len, (unsigned)(cap - len));
        if (nr < 0) { rc = -1; break; }
        if (nr == 0) break;                                 /* a trailing partial line is dropped */
        len += (size_t)nr;
        size_t start = 0;
        for (size_t i = 0; i < len && !rc; i++) {
            if (buf[i] != '\n') continue;
            size_t nl_len = 0;
            const int a = alter_line(&v, buf + start, i - start, &nl_len);
            if (a < 0) { rc = a; break; }
            v.n_tot++;
            if (a == 0) {
                fwrite(buf + start, 1, i - start + 1, out);
            } else {
                if (a == 2) v.n_drop++;
                else v.n_mod++;
                fwrite(v.nl, 1, nl_len, out);
                fputc('\n', out);
            }
            start = i + 1;
        }
        memmove(buf, buf + start, len - start);
        len -= start;
    }
    free(buf);
    free(v.nl);
    gzclose(in);
    if (fclose(out) != 0 && !rc) rc = -1;
    if (counts) { counts[0] = v.n_mod; counts[1] = v.n_drop; counts[2] = v.n_tot; }
    return rc;
}
