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
 * Fatal exits of the reference become error codes: PF_ERR_ARG for an
 * unsorted POS within a contig (:1383-1387) or a #CHROM header without
 * exactly 10 columns (:1361-1368), PF_ERR_NOMEM, -1 for an unreadable file.
 * Differences (reference UB): a PS value longer than 10 characters is cut at
 * 10 (the reference overflows char[11]); a sample column with fewer fields
 * than FORMAT's PS index counts as PS "." (the reference reads
 * uninitialised values); empty lines are skipped (the reference calls
 * strlen(NULL)).
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
    uint32_t prev_pos, prev_group;
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
    /* strtoul semantics on a token: leading digits, truncated to 32 bits */
    unsigned long v = 0;
    size_t i = 0;
    while (i < l && (s[i] == ' ' || s[i] == '\t')) i++;
    if (i < l && s[i] == '+') i++;
    for (; i < l && s[i] >= '0' && s[i] <= '9'; i++) v = v * 10 + (unsigned long)(s[i] - '0');
    return (uint32_t)v;
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
    if (l == 0) return 0;
    if (s[0] == '#') {
        if (l > 1 && s[1] == '#') return 0;
        int n = 1;                                       /* #CHROM header: column count */
        for (size_t i = 0; i < l; i++) n += s[i] == '\t';
        return n == 10 ? 0 : PF_ERR_ARG;
    }
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
    /* insert_vcf_line (:1348-1430) */
    contig_t *c = &g->c[g->cur];
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
    if (!vcf_path || !out) return PF_ERR_ARG;
    *out = NULL;
    gzFile fp = gzopen(vcf_path, "rb");
    if (!fp) return -1;
    gap_state_t g;
    memset(&g, 0, sizeof(g));
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
 * GT index is skipped (the reference reads uninitialised values). */
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
    if (l > 0 && s[0] == '#') {
        if (l > 1 && s[1] == '#') return 0;
        int n = 0;                                   /* strtok token count */
        for (size_t i = 0; i < l;) {
            while (i < l && s[i] == '\t') i++;
            if (i >= l) break;
            n++;
            while (i < l && s[i] != '\t') i++;
        }
        return n == 10 ? 0 : PF_ERR_ARG;
    }
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

int pf_vcf_known_vars(const char *vcf_path, const char *contig, pf_known_table_t **out) {
    if (!vcf_path || !contig || !out) return PF_ERR_ARG;
    *out = NULL;
    gzFile fp = gzopen(vcf_path, "rb");
    if (!fp) return -1;
    struct pf_known_own *o = (struct pf_known_own *)calloc(1, sizeof *o);
    size_t cap = 1 << 16, len = 0;
    char *buf = (char *)malloc(cap);
    int rc = (buf && o) ? 0 : PF_ERR_NOMEM;
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
                rc = known_line(&o->k, contig, buf + start, i - start);
                start = i + 1;
            }
        }
        memmove(buf, buf + start, len - start);
        len -= start;
    }
    gzclose(fp);
    free(buf);
    if (!rc) {
        const size_t n = o->k.pos.n;
        o->hp8 = (uint8_t *)malloc(n ? n : 1);
        o->off = (uint64_t *)malloc((n + 1) * 8);
        if (!o->hp8 || !o->off) rc = PF_ERR_NOMEM;
        else {
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
        }
    }
    if (rc) { pf_known_table_free(o ? &o->pub : NULL); return rc; }
    *out = &o->pub;
    return PF_OK;
}
