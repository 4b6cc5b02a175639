/*
 * pf_windows.c -- window definition on the host.
 *
 * pf_vcf_gaps: the phase-block gaps a phased VCF defines for
 * `pomfret methphase`: load_intervals_from_file (reference blockjoin.c:
 * 1977-2170) driving insert_vcf_line (:1348-1430) over every complete line,
 * then store_raw_intervals + merge_close_intervals(READBACK) per contig
 * (:2178-2220, called at :4520-4521).  Behaviour kept from the reference:
 *   - a gap is [last POS of a phase block, PS value of the next block];
 *   - only lines with a PS in the sample column count (the SNP test is
 *     commented out in the reference, :1389-1393); PS "." is skipped;
 *   - abs_start is set by the first phased variant of the FIRST contig only:
 *     prev_group_ID is never reset, so later contigs keep abs_start = 0;
 *   - abs_end of a contig is the last phased POS seen before the next new
 *     contig name (or EOF); a contig name seen again only switches back;
 *   - a final line without '\n' is never parsed (the reference's buffered
 *     reader only handles complete lines);
 *   - merging compares (start_i - end_j) as uint32 against the threshold, so
 *     an out-of-order start never merges.
 * Every line starting with '#' is skipped before insert_vcf_line sees it
 * (:2023-2026), so the #CHROM column check of insert_vcf_line (:1355-1371) is
 * never reached on this path (the VCF writer keeps it, alter_vcf_line).
 * Fatal exits of the reference become error codes: PF_ERR_ARG for an
 * unsorted POS within a contig (:1383-1387), PF_ERR_NOMEM, -1 for an
 * unreadable file.  Differences (reference UB): a PS value longer than 10
 * characters is cut at 10 (the reference overflows char[11]); a sample
 * column with fewer fields than FORMAT's PS index counts as PS "." (the
 * reference reads uninitialised values); empty (or all-tab) lines are skipped
 * (the reference calls strlen(NULL)).
 *
 * pf_interval_gaps: the same loader on a GTF (`--gtf`, e.g. whatshap stats
 * --block-list output) or a 3-column TSV (`--tsv`): insert_gtf_line
 * (:1305-1345) on columns 3/4 (GTF) or 1/2 (TSV) of the strtok tokens.  A
 * block's start closes the gap [end of the previous block, this start] when
 * the contig has seen a block, else it sets the contig's abs_start; its end
 * becomes the previous end.  The previous end is reset at every new contig
 * name (:2098), so unlike the VCF path every contig gets its own abs_start; a
 * contig name seen again only switches back (its gaps continue from the
 * other contig's last end, as the reference's shared prev_end does).
 *
 * pf_report_windows: the chunk windows of `pomfret report` (main_methreport,
 * :4963-4991): per contig, for each raw gap [start, end] in order with prev
 * starting at abs_start, when start - prev > chunk (uint32) emit
 * [i, i + chunk) for i = prev; i + stride < start; i += stride (uint32);
 * then prev = end.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>

#include "../../include/pomfret_amd.h"

typedef struct {
    uint32_t *a;
    size_t n, m;
} u32v;

static int u32v_push(u32v *v, uint32_t x) {
    if (v->n == v->m) {
        size_t nm = v->m ? v->m * 2 : 64;
        uint32_t *p = (uint32_t *)realloc(v->a, nm * sizeof(uint32_t));
        if (!p) return -1;
        v->a = p;
        v->m = nm;
    }
    v->a[v->n++] = x;
    return 0;
}

typedef struct {
    char *name;
    uint32_t abs_start, abs_end;
    u32v s, e;          /* raw gaps, in VCF order */
} contig_t;

typedef struct {
    contig_t *c;
    size_t n, m;
    int cur;            /* index of the contig lines are attributed to */
    uint32_t prev_pos, prev_group;   /* prev_pos is the GTF/TSV path's prev_end */
    int fmt;            /* PF_INTERVALS_* */
} gap_state_t;

/* the idx-th ':'-separated field of [s, s+l) */
static int field_of(const char *s, size_t l, int idx, size_t *fs, size_t *fl) {
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

static int index_of_ps(const char *s, size_t l) {
    size_t start = 0;
    int col = 0;
    for (size_t i = 0; i <= l; i++) {
        if (i == l || s[i] == ':') {
            if (i - start == 2 && s[start] == 'P' && s[start + 1] == 'S') return col;
            if (i == l) break;
            start = i + 1;
            col++;
        }
    }
    return -1;
}

static uint32_t parse_u32(const char *s, size_t l) {
    /* (uint32_t)strtoul(token, NULL, 10): leading white space, an optional
     * sign (a '-' negates in unsigned arithmetic), the leading digits;
     * ULONG_MAX on overflow */
    unsigned long v = 0;
    int neg = 0, over = 0;
    size_t i = 0;
    while (i < l && (s[i] == ' ' || (s[i] >= '\t' && s[i] <= '\r'))) i++;
    if (i < l && (s[i] == '+' || s[i] == '-')) neg = s[i++] == '-';
    for (; i < l && s[i] >= '0' && s[i] <= '9'; i++) {
        const unsigned long d = (unsigned long)(s[i] - '0');
        if (v > (~0ul - d) / 10) over = 1;
        v = v * 10 + d;
    }
    if (over) return (uint32_t)~0ul;
    return (uint32_t)(neg ? 0ul - v : v);
}

static int new_contig(gap_state_t *g, const char *name, size_t l) {
    if (g->n == g->m) {
        size_t nm = g->m ? g->m * 2 : 8;
        contig_t *p = (contig_t *)realloc(g->c, nm * sizeof(contig_t));
        if (!p) return -1;
        g->c = p;
        g->m = nm;
    }
    contig_t *c = &g->c[g->n];
    memset(c, 0, sizeof(*c));
    c->name = (char *)malloc(l + 1);
    if (!c->name) return -1;
    memcpy(c->name, name, l);
    c->name[l] = 0;
    g->cur = (int)g->n;
    g->n++;
    return 0;
}

/* one complete data line (no '\n'); returns 0, PF_ERR_ARG or PF_ERR_NOMEM */
static int gap_line(gap_state_t *g, const char *s, size_t l) {
    if (l == 0 || s[0] == '#') return 0;                 /* :2023-2026 */
    /* split on tabs (empty tokens are skipped, as strtok does) */
    const char *tok[10];
    size_t tl[10];
    int nt = 0;
    size_t i = 0;
    while (i < l && nt < 10) {
        while (i < l && s[i] == '\t') i++;
        if (i >= l) break;
        size_t j = i;
        while (j < l && s[j] != '\t') j++;
        tok[nt] = s + i;
        tl[nt] = j - i;
        nt++;
        i = j;
    }
    if (nt == 0) return 0;
    /* contig bookkeeping of load_intervals_from_file (:2027-2104) */
    int found = -1;
    for (int c = (int)g->n - 1; c >= 0; c--)
        if (strlen(g->c[c].name) == tl[0] && memcmp(g->c[c].name, tok[0], tl[0]) == 0) { found = c; break; }
    if (g->n == 0) {
        if (new_contig(g, tok[0], tl[0])) return PF_ERR_NOMEM;
    } else if (found >= 0) {
        g->cur = found;
    } else {
        if (g->prev_pos != UINT32_MAX) g->c[g->n - 1].abs_end = g->prev_pos;
        if (new_contig(g, tok[0], tl[0])) return PF_ERR_NOMEM;
        g->prev_pos = UINT32_MAX;
    }
    contig_t *c = &g->c[g->cur];
    if (g->fmt != PF_INTERVALS_VCF) {                    /* insert_gtf_line (:1305-1345) */
        const int cs = g->fmt == PF_INTERVALS_TSV ? 1 : 3, ce = cs + 1;
        if (nt > cs) {
            const uint32_t v = parse_u32(tok[cs], tl[cs]);
            if (g->prev_pos != UINT32_MAX) {
                if (u32v_push(&c->s, g->prev_pos) || u32v_push(&c->e, v)) return PF_ERR_NOMEM;
            } else {
                c->abs_start = v;
            }
        }
        if (nt > ce) g->prev_pos = parse_u32(tok[ce], tl[ce]);
        return 0;
    }
    /* insert_vcf_line (:1348-1430) */
    uint32_t pos = 0;
    if (nt > 1) {
        pos = parse_u32(tok[1], tl[1]);
        if (g->prev_pos != UINT32_MAX && pos < g->prev_pos) return PF_ERR_ARG;
    }
    if (nt < 10) return 0;
    const int ips = index_of_ps(tok[8], tl[8]);
    if (ips < 0) return 0;
    size_t fs, fl;
    if (field_of(tok[9], tl[9], ips, &fs, &fl) != 0) return 0;
    if (fl == 1 && tok[9][fs] == '.') return 0;
    const uint32_t group = parse_u32(tok[9] + fs, fl > 10 ? 10 : fl);
    if (g->prev_group == UINT32_MAX) {
        g->prev_group = group;
        g->prev_pos = pos;
        c->abs_start = pos;
    }
    if (group == g->prev_group) {
        g->prev_pos = pos;
    } else {
        if (g->prev_pos != UINT32_MAX) {
            if (u32v_push(&c->s, g->prev_pos) || u32v_push(&c->e, group)) return PF_ERR_NOMEM;
        }
        g->prev_group = group;
        g->prev_pos = pos;
    }
    return 0;
}

static void free_state(gap_state_t *g) {
    for (size_t i = 0; i < g->n; i++) {
        free(g->c[i].name);
        free(g->c[i].s.a);
        free(g->c[i].e.a);
    }
    free(g->c);
}

int pf_vcf_gaps(const char *vcf_path, int32_t readback, pf_gaps_t **out) {
    return pf_interval_gaps(vcf_path, PF_INTERVALS_VCF, readback, out);
}

int pf_interval_gaps(const char *path, int32_t format, int32_t readback, pf_gaps_t **out) {
    if (!path || !out || format < PF_INTERVALS_VCF || format > PF_INTERVALS_TSV) return PF_ERR_ARG;
    *out = NULL;
    gzFile fp = gzopen(path, "rb");
    if (!fp) return -1;
    gap_state_t g;
    memset(&g, 0, sizeof(g));
    g.fmt = format;
    g.cur = -1;
    g.prev_pos = UINT32_MAX;
    g.prev_group = UINT32_MAX;
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
        const int nr = gzread(fp, buf + len, (unsigned)(cap - len));
        if (nr < 0) { rc = -1; break; }
        if (nr == 0) break;                                /* a trailing partial line is dropped */
        len += (size_t)nr;
        size_t start = 0;
        for (size_t i = 0; i < len && !rc; i++) {
            if (buf[i] == '\n') {
                rc = gap_line(&g, buf + start, i - start);
                start = i + 1;
            }
        }
        memmove(buf, buf + start, len - start);
        len -= start;
    }
    gzclose(fp);
    free(buf);
    if (!rc && g.prev_pos != UINT32_MAX && g.cur >= 0) g.c[g.cur].abs_end = g.prev_pos;
    if (rc) { free_state(&g); return rc; }

    /* flatten; merge_close_intervals (:2190-2220) per contig */
    size_t nraw = 0;
    for (size_t i = 0; i < g.n; i++) nraw += g.c[i].s.n;
    pf_gaps_t *r = (pf_gaps_t *)calloc(1, sizeof(pf_gaps_t));
    const size_t nc = g.n;
    if (r) {
        r->n_contigs = (uint32_t)nc;
        r->names = (char **)calloc(nc ? nc : 1, sizeof(char *));
        r->abs_start = (uint32_t *)calloc(nc ? nc : 1, 4);
        r->abs_end = (uint32_t *)calloc(nc ? nc : 1, 4);
        r->raw_off = (uint64_t *)calloc(nc + 1, 8);
        r->gap_off = (uint64_t *)calloc(nc + 1, 8);
        r->drop_off = (uint64_t *)calloc(nc + 1, 8);
        r->raw_start = (uint32_t *)malloc((nraw ? nraw : 1) * 4);
        r->raw_end = (uint32_t *)malloc((nraw ? nraw : 1) * 4);
        r->gap_start = (uint32_t *)malloc((nraw ? nraw : 1) * 4);
        r->gap_end = (uint32_t *)malloc((nraw ? nraw : 1) * 4);
        r->drop_start = (uint32_t *)malloc((nraw ? nraw : 1) * 4);
        r->drop_end = (uint32_t *)malloc((nraw ? nraw : 1) * 4);
    }
    if (!r || !r->names || !r->abs_start || !r->abs_end || !r->raw_off || !r->gap_off || !r->drop_off ||
        !r->raw_start || !r->raw_end || !r->gap_start || !r->gap_end || !r->drop_start || !r->drop_end) {
        pf_gaps_free(r);
        free_state(&g);
        return PF_ERR_NOMEM;
    }
    size_t kr = 0, kg = 0, kd = 0;
    for (size_t i = 0; i < nc; i++) {
        contig_t *c = &g.c[i];
        r->names[i] = c->name;
        c->name = NULL;
        r->abs_start[i] = c->abs_start;
        r->abs_end[i] = c->abs_end;
        const size_t n = c->s.n;
        for (size_t j = 0; j < n; j++) { r->raw_start[kr + j] = c->s.a[j]; r->raw_end[kr + j] = c->e.a[j]; }
        kr += n;
        if (n > 0) {
            uint32_t js = c->s.a[0], je = c->e.a[0];
            for (size_t j = 1; j < n; j++) {
                if (c->s.a[j] - je < (uint32_t)readback) {       /* uint32 compare (:2198) */
                    r->drop_start[kd] = je;
                    r->drop_end[kd] = c->s.a[j];
                    kd++;
                    je = c->e.a[j];
                } else {
                    r->gap_start[kg] = js;
                    r->gap_end[kg] = je;
                    kg++;
                    js = c->s.a[j];
                    je = c->e.a[j];
                }
            }
            r->gap_start[kg] = js;
            r->gap_end[kg] = je;
            kg++;
        }
        r->raw_off[i + 1] = kr;
        r->gap_off[i + 1] = kg;
        r->drop_off[i + 1] = kd;
    }
    free_state(&g);
    *out = r;
    return PF_OK;
}

void pf_gaps_free(pf_gaps_t *g) {
    if (!g) return;
    if (g->names)
        for (uint32_t i = 0; i < g->n_contigs; i++) free(g->names[i]);
    free(g->names);
    free(g->abs_start);
    free(g->abs_end);
    free(g->raw_off);
    free(g->gap_off);
    free(g->drop_off);
    free(g->raw_start);
    free(g->raw_end);
    free(g->gap_start);
    free(g->gap_end);
    free(g->drop_start);
    free(g->drop_end);
    free(g);
}

int64_t pf_report_windows(uint32_t abs_start, const uint32_t *gap_start, const uint32_t *gap_end, uint64_t n_gaps,
                          uint32_t chunk_size, uint32_t chunk_stride, uint32_t *win_start, uint32_t *win_end,
                          uint64_t cap) {
    if ((n_gaps && (!gap_start || !gap_end)) || chunk_stride == 0) return PF_ERR_ARG;
    uint64_t n = 0;
    uint32_t prev = abs_start;
    for (uint64_t k = 0; k < n_gaps; k++) {
        const uint32_t start = gap_start[k], end = gap_end[k];
        if (start - prev > chunk_size) {
            for (uint32_t i = prev; i + chunk_stride < start; i += chunk_stride) {
                if (win_start && n < cap) { win_start[n] = i; win_end[n] = i + chunk_size; }
                n++;
            }
        }
        prev = end;
    }
    return (int64_t)n;
}

/* ------------------------------------------------------------------ */
/* pf_vcf_known_vars: the -u known-variant table of one contig
 * (insert_variant_from_vcf_line, :1432-1543).  Quirks kept: tokens are
 * strtok_r's (runs of tabs collapse); POS is strtoul(POS) - 1 in uint32
 * arithmetic; GT is the FORMAT-indexed sample field and must be exactly
 * "a|b" with a, b in {0,1}; a deletion moves POS one base right and takes
 * its chars from REF+1, an insertion its chars from ALT+1 (a multi-allelic
 * ALT is one string here too, commas included); chars are seq_nt4 codes
 * (A0 C1 G2 T3, else 4).  A sample column with fewer fields than FORMAT's
 * GT index is skipped (the reference reads uninitialised values).  Lines
 * starting with '#' never reach insert_variant_from_vcf_line on the paths
 * that collect variants (load_intervals_from_file, :2023-2026), so its
 * #CHROM column check (:1441-1455) is not applied. */
typedef struct {
    u32v pos, len, hp;
    uint8_t *op;
    size_t n_op, m_op;
    uint8_t *ch;
    size_t n_ch, m_ch;
    uint64_t *off;
    size_t n_off, m_off;
} known_acc_t;

static int grow(void **p, size_t *m, size_t need, size_t es) {
    if (need <= *m) return 0;
    size_t nm = *m ? *m : 64;
    while (nm < need) nm *= 2;
    void *q = realloc(*p, nm * es);
    if (!q) return -1;
    *p = q;
    *m = nm;
    return 0;
}

static uint8_t nt4(char c) {
    switch (c) {
    case 'A': case 'a': return 0;
    case 'C': case 'c': return 1;
    case 'G': case 'g': return 2;
    case 'T': case 't': return 3;
    default: return 4;
    }
}

static int known_line(known_acc_t *K, const char *contig, const char *s, size_t l) {
    if (l > 0 && s[0] == '#') return 0;              /* skipped by the caller (:2023-2026) */
    const char *tok[10];
    size_t tl[10];
    int nt = 0;
    for (size_t i = 0; i < l && nt < 10;) {
        while (i < l && s[i] == '\t') i++;
        if (i >= l) break;
        tok[nt] = s + i;
        const size_t st = i;
        while (i < l && s[i] != '\t') i++;
        tl[nt] = i - st;
        nt++;
    }
    if (nt < 1 || tl[0] != strlen(contig) || memcmp(tok[0], contig, tl[0]) != 0) return 0;
    if (nt < 10) return 0;
    uint32_t pos = parse_u32(tok[1], tl[1]) - 1u;
    const size_t ref_l = tl[3], alt_l = tl[4];
    /* GT index in FORMAT, then that field of the sample */
    int i_gt = -1;
    {
        size_t start = 0;
        int col = 0;
        for (size_t i = 0; i <= tl[8]; i++) {
            if (i == tl[8] || tok[8][i] == ':') {
                if (i - start == 2 && tok[8][start] == 'G' && tok[8][start + 1] == 'T') { i_gt = col; break; }
                if (i == tl[8]) break;
                start = i + 1;
                col++;
            }
        }
    }
    if (i_gt < 0) return 0;
    size_t fs, fl;
    if (field_of(tok[9], tl[9], i_gt, &fs, &fl)) return 0;
    if (fl != 3) return 0;
    const char *gt = tok[9] + fs;
    if (gt[1] != '|' || (gt[0] != '0' && gt[0] != '1') || (gt[2] != '0' && gt[2] != '1')) return 0;
    uint8_t op;
    uint32_t op_l;
    const char *vs;
    if (ref_l == 1 && alt_l == 1) { op = PF_VAR_X; op_l = 1; vs = tok[4]; }
    else if (ref_l == alt_l) return 0;                    /* unhandled variant case (:1528-1532) */
    else if (ref_l > alt_l) { op = PF_VAR_D; op_l = (uint32_t)(ref_l - alt_l); pos += 1; vs = tok[3] + 1; }
    else { op = PF_VAR_I; op_l = (uint32_t)(alt_l - ref_l); vs = tok[4] + 1; }
    if (u32v_push(&K->pos, pos) || u32v_push(&K->len, op_l) || u32v_push(&K->hp, (uint32_t)(gt[0] - '0')))
        return PF_ERR_NOMEM;
    if (grow((void **)&K->op, &K->m_op, K->n_op + 1, 1)) return PF_ERR_NOMEM;
    K->op[K->n_op++] = op;
    if (grow((void **)&K->ch, &K->m_ch, K->n_ch + op_l, 1)) return PF_ERR_NOMEM;
    for (uint32_t i = 0; i < op_l; i++) K->ch[K->n_ch++] = nt4(vs[i]);
    if (grow((void **)&K->off, &K->m_off, K->n_off + 1, 8)) return PF_ERR_NOMEM;
    K->off[K->n_off++] = K->n_ch;
    return 0;
}

struct pf_known_own {
    pf_known_table_t pub;
    known_acc_t k;
    uint8_t *hp8;
    uint64_t *off;
};

void pf_known_table_free(pf_known_table_t *t) {
    if (!t) return;
    struct pf_known_own *o = (struct pf_known_own *)t;
    free(o->k.pos.a);
    free(o->k.len.a);
    free(o->k.hp.a);
    free(o->k.op);
    free(o->k.ch);
    free(o->k.off);
    free(o->hp8);
    free(o->off);
    free(o);
}

/* the public view of an accumulated table */
static int known_finish(struct pf_known_own *o) {
    const size_t n = o->k.pos.n;
    o->hp8 = (uint8_t *)malloc(n ? n : 1);
    o->off = (uint64_t *)malloc((n + 1) * 8);
    if (!o->hp8 || !o->off) return PF_ERR_NOMEM;
    o->off[0] = 0;
    for (size_t i = 0; i < n; i++) { o->hp8[i] = (uint8_t)o->k.hp.a[i]; o->off[i + 1] = o->k.off[i]; }
    static const uint8_t dummy[8] = {0};
    pf_known_vars_t *v = &o->pub.vars;
    v->n = (uint32_t)n;
    v->pos = n ? o->k.pos.a : (const uint32_t *)dummy;
    v->len = n ? o->k.len.a : (const uint32_t *)dummy;
    v->op = n ? o->k.op : dummy;
    v->haptag = o->hp8;
    v->char_off = o->off;
    v->chars = o->k.n_ch ? o->k.ch : dummy;
    return PF_OK;
}

/* every complete line of a (gzipped) text file through fn(arg, line, len) */
static int each_line(const char *path, int (*fn)(void *, const char *, size_t), void *arg) {
    gzFile fp = gzopen(path, "rb");
    if (!fp) return -1;
    size_t cap = 1 << 16, len = 0;
    char *buf = (char *)malloc(cap);
    int rc = buf ? 0 : PF_ERR_NOMEM;
    while (!rc) {
        if (len == cap) {
            char *q = (char *)realloc(buf, cap * 2);
            if (!q) { rc = PF_ERR_NOMEM; break; }
            buf = q;
            cap *= 2;
        }
        const int nr = gzread(fp, buf + len, (unsigned)(cap - len));
        if (nr < 0) { rc = -1; break; }
        if (nr == 0) break;                                /* a trailing partial line is dropped */
        len += (size_t)nr;
        size_t start = 0;
        for (size_t i = 0; i < len && !rc; i++) {
            if (buf[i] == '\n') {
                rc = fn(arg, buf + start, i - start);
                start = i + 1;
            }
        }
        memmove(buf, buf + start, len - start);
        len -= start;
    }
    gzclose(fp);
    free(buf);
    return rc;
}

/* one pass for several contigs: a line goes to the table of the contig its
 * CHROM names, or -- when that name is not in `names` -- to the table the
 * previous line went to (none before the first match).  This is the
 * var_storage branch of load_intervals_from_file (2150-2163) that
 * recover_variant_phase_in_dropped_intervals drives (2639): i_ref_cache is
 * only updated by a name it finds.  With every VCF contig in `names` each
 * table is that contig's pf_vcf_known_vars. */
typedef struct {
    uint32_t n;
    const char *const *names;
    struct pf_known_own **o;
    int32_t cache;
    int sticky;         /* 0: a name not in `names` is skipped (one contig's table) */
} known_multi_t;

static int known_multi_line(void *arg, const char *s, size_t l) {
    known_multi_t *M = (known_multi_t *)arg;
    if (l == 0 || s[0] == '#') return 0;
    size_t i = 0;
    while (i < l && s[i] == '\t') i++;
    if (i >= l) return 0;
    size_t j = i;
    while (j < l && s[j] != '\t') j++;
    char nm[1024];
    const size_t nl = j - i < sizeof nm - 1 ? j - i : sizeof nm - 1;
    memcpy(nm, s + i, nl);
    nm[nl] = 0;
    int32_t hit = -1;
    for (uint32_t c = 0; c < M->n && hit < 0; c++)
        if (!strcmp(M->names[c], nm)) hit = (int32_t)c;
    if (hit >= 0 || !M->sticky) M->cache = hit;
    if (M->cache < 0) return 0;
    return known_line(&M->o[M->cache]->k, nm, s, l);
}

int pf_vcf_known_vars_multi(const char *vcf_path, uint32_t n, const char *const *names, pf_known_table_t **out) {
    if (!vcf_path || !out || (n && !names)) return PF_ERR_ARG;
    struct pf_known_own **o = (struct pf_known_own **)calloc(n ? n : 1, sizeof *o);
    int rc = o ? 0 : PF_ERR_NOMEM;
    for (uint32_t c = 0; c < n && !rc; c++) {
        out[c] = NULL;
        if (!names[c]) rc = PF_ERR_ARG;
        else if (!(o[c] = (struct pf_known_own *)calloc(1, sizeof **o))) rc = PF_ERR_NOMEM;
    }
    known_multi_t M = {n, names, o, -1, 1};
    if (!rc) rc = each_line(vcf_path, known_multi_line, &M);
    for (uint32_t c = 0; c < n && !rc; c++) rc = known_finish(o[c]);
    for (uint32_t c = 0; c < n && o; c++) {
        if (rc) pf_known_table_free(o[c] ? &o[c]->pub : NULL);
        else out[c] = &o[c]->pub;
    }
    free(o);
    return rc;
}

int pf_vcf_known_vars(const char *vcf_path, const char *contig, pf_known_table_t **out) {
    if (!vcf_path || !contig || !out) return PF_ERR_ARG;
    *out = NULL;
    struct pf_known_own *o = (struct pf_known_own *)calloc(1, sizeof *o);
    if (!o) return PF_ERR_NOMEM;
    known_multi_t M = {1, &contig, &o, -1, 0};
    int rc = each_line(vcf_path, known_multi_line, &M);
    if (!rc) rc = known_finish(o);
    if (rc) { pf_known_table_free(&o->pub); return rc; }
    *out = &o->pub;
    return PF_OK;
}
