/*
 * pf_pipeline.c -- `pomfret methphase` / `pomfret report` end to end in host C
 * around the device hot path (f1-f3 glue).
 *
 * Reference structure (line numbers: /root/reference/blockjoin.c):
 *   main_blockjoin (4643-4736) -> blockjoin_parallel (4427-4641):
 *     load_intervals_from_file + merge_close_intervals      -> pf_interval_gaps
 *       (--tsv, then --gtf, then --vcf, 4661-4666; with -u the VCF names
 *        the pre-pass contigs and a GTF/TSV then overrides the intervals,
 *        4445-4465)
 *     (-u) pre_haplotagging_read_in_one_ref per contig (1841-1898),
 *          qname first-wins per contig, merged in contig order     -> K4 jobs
 *     estimate_read_coverage_dirtyfast when -c is absent (4547)     -> pf_bam_estimate_coverage_dev
 *                                                   (pf_bam_estimate_coverage with --host-fetch / no device)
 *     kt_for(blockjoin_one_chrom_callback) over contigs (4560):
 *       per-contig parameters and clamps (4357-4390), one
 *       haplotag_region_given_bam per merged gap, and for a joined gap
 *       every read's tag into the contig's qname table, first wins
 *       (4396-4423)                                                  -> window jobs on the devices
 *     per-contig tables merged into st->qname2haptag in contig order,
 *     first wins (4571-4595)                                         -> pf_mp_finish
 *   lift_decisions .. output_modify_vcf (4685-4717)                  -> pf_phase_blocks, pf_write_*,
 *                                                                       pf_rescue_dropped
 *   main_methreport (4901-5089): chunk windows of the raw gaps, one
 *     haplotag_region_given_bam each, report.tsv rows and the running
 *     correct/switch/fail totals                                      -> mode PF_MODE_REPORT
 *
 * MI355X-first shape.  The reference fans contigs out to CPU threads and
 * re-opens the BAM per gap.  Here the windows of all contigs are cut into
 * jobs (runs of consecutive windows of one contig), ordered by
 * longest-processing-time first on their fetch span, and consumed by one
 * host thread per GPU: the thread fetches a job's records on the host
 * (pf_bam_fetch_windows, threaded) while its device runs the previous job
 * (K0..K3, pf_methphase_run), so host ingest and device compute overlap.
 * Within one process the device threads share a work queue; across
 * processes (one per GPU, torch.distributed) `rank/world` picks a static
 * LPT shard and the job results -- per-window decisions plus the joined
 * windows' (qname, tag) lists -- are exported, gathered and imported on the
 * writer rank, whose merge in (contig, window) order reproduces the
 * reference's first-wins tables exactly.
 *
 * Windows whose record count exceeds the device limit (65,535 reads per
 * window) are left undecided (-1) with a warning instead of failing the run.
 */
#include <errno.h>
#include <math.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../../include/pomfret_amd.h"

#define PF_JOB_WINDOWS_DEFAULT 1024u
#define PF_MAX_WIN_RECS 65535u

/* ------------------------------------------------------------------ */
/* qname -> hp, first wins (htstri_t of the reference)                  */

struct pf_tags {
    uint64_t *slot;        /* entry index + 1, 0 = empty */
    uint64_t mask;
    uint64_t n, cap;       /* entries */
    uint64_t *off;         /* [cap+1] name offsets */
    char *names;
    uint64_t names_n, names_cap;
    uint8_t *hp;
};

static uint64_t fnv1a(const char *s, size_t n) {
    uint64_t h = 1469598103934665603ull;
    for (size_t i = 0; i < n; i++) { h ^= (uint8_t)s[i]; h *= 1099511628211ull; }
    return h ^ (h >> 29);
}

pf_tags_t *pf_tags_new(void) {
    pf_tags_t *t = (pf_tags_t *)calloc(1, sizeof *t);
    if (!t) return NULL;
    t->mask = 1023;
    t->slot = (uint64_t *)calloc(t->mask + 1, sizeof(uint64_t));
    t->cap = 256;
    t->off = (uint64_t *)calloc(t->cap + 1, sizeof(uint64_t));
    t->hp = (uint8_t *)malloc(t->cap);
    t->names_cap = 4096;
    t->names = (char *)malloc(t->names_cap);
    if (!t->slot || !t->off || !t->hp || !t->names) { pf_tags_free(t); return NULL; }
    return t;
}

void pf_tags_free(pf_tags_t *t) {
    if (!t) return;
    free(t->slot); free(t->off); free(t->hp); free(t->names);
    free(t);
}

uint64_t pf_tags_size(const pf_tags_t *t) { return t ? t->n : 0; }

static int64_t tags_find(const pf_tags_t *t, const char *nm, size_t l, uint64_t *slot_out) {
    uint64_t h = fnv1a(nm, l) & t->mask;
    for (;;) {
        const uint64_t s = t->slot[h];
        if (!s) { if (slot_out) *slot_out = h; return -1; }
        const uint64_t k = s - 1;
        if (t->off[k + 1] - t->off[k] == l && memcmp(t->names + t->off[k], nm, l) == 0) return (int64_t)k;
        h = (h + 1) & t->mask;
    }
}

static int tags_rehash(pf_tags_t *t) {
    const uint64_t nm = (t->mask + 1) * 2 - 1;
    uint64_t *ns = (uint64_t *)calloc(nm + 1, sizeof(uint64_t));
    if (!ns) return PF_ERR_NOMEM;
    for (uint64_t k = 0; k < t->n; k++) {
        uint64_t h = fnv1a(t->names + t->off[k], t->off[k + 1] - t->off[k]) & nm;
        while (ns[h]) h = (h + 1) & nm;
        ns[h] = k + 1;
    }
    free(t->slot);
    t->slot = ns;
    t->mask = nm;
    return PF_OK;
}

/* insert (nm, hp) unless present; 1 inserted, 0 present, < 0 error */
static int tags_put(pf_tags_t *t, const char *nm, size_t l, uint8_t hp) {
    uint64_t slot;
    if (tags_find(t, nm, l, &slot) >= 0) return 0;
    if (2 * (t->n + 1) > t->mask + 1) {
        int rc = tags_rehash(t);
        if (rc) return rc;
        (void)tags_find(t, nm, l, &slot);
    }
    if (t->n + 1 > t->cap) {
        const uint64_t nc = t->cap * 2;
        uint64_t *no = (uint64_t *)realloc(t->off, (nc + 1) * sizeof(uint64_t));
        if (!no) return PF_ERR_NOMEM;
        t->off = no;
        uint8_t *nh = (uint8_t *)realloc(t->hp, nc);
        if (!nh) return PF_ERR_NOMEM;
        t->hp = nh;
        t->cap = nc;
    }
    if (t->names_n + l > t->names_cap) {
        uint64_t nc = t->names_cap * 2;
        while (nc < t->names_n + l) nc *= 2;
        char *nn = (char *)realloc(t->names, nc);
        if (!nn) return PF_ERR_NOMEM;
        t->names = nn;
        t->names_cap = nc;
    }
    memcpy(t->names + t->names_n, nm, l);
    t->names_n += l;
    t->hp[t->n] = hp;
    t->n++;
    t->off[t->n] = t->names_n;
    t->slot[slot] = t->n;
    return 1;
}

int64_t pf_tags_put_first(pf_tags_t *t, uint32_t n, const uint64_t *off, const char *names, const uint8_t *hp) {
    if (!t || (n && (!off || !names || !hp))) return PF_ERR_ARG;
    int64_t ins = 0;
    for (uint32_t i = 0; i < n; i++) {
        if (off[i + 1] < off[i]) return PF_ERR_ARG;
        const int rc = tags_put(t, names + off[i], (size_t)(off[i + 1] - off[i]), hp[i]);
        if (rc < 0) return rc;
        ins += rc;
    }
    return ins;
}

int64_t pf_tags_get(const pf_tags_t *t, uint32_t n, const uint64_t *off, const char *names, uint8_t dflt,
                    uint8_t *hp_out) {
    if (!t || (n && (!off || !names || !hp_out))) return PF_ERR_ARG;
    int64_t found = 0;
    for (uint32_t i = 0; i < n; i++) {
        const int64_t k = tags_find(t, names + off[i], (size_t)(off[i + 1] - off[i]), NULL);
        hp_out[i] = k >= 0 ? t->hp[k] : dflt;
        found += k >= 0;
    }
    return found;
}

int pf_tags_view(const pf_tags_t *t, pf_qname_tags_t *out) {
    if (!t || !out) return PF_ERR_ARG;
    if (t->n > UINT32_MAX) return PF_ERR_LIMIT;
    out->n = (uint32_t)t->n;
    out->off = t->off;
    out->names = t->names;
    out->hp = t->hp;
    return PF_OK;
}

/* ------------------------------------------------------------------ */
/* plan                                                                 */

typedef struct {
    uint32_t contig, w0, w1;   /* windows [w0, w1) of the plan's global window list */
    int64_t lo, hi;            /* window jobs: the union of the windows' fetch regions */
    int32_t bc;                /* -u jobs: the window contig whose piece bounds the fetch uses (-1: none) */
    double cost;
    int32_t rank;
    int done;
    /* result */
    int8_t *dec;               /* [w1-w0] */
    uint64_t *tag_off;         /* [w1-w0+1] entry ranges per window */
    uint64_t n_ent;
    uint64_t *name_off;        /* [n_ent+1] */
    char *names;
    uint8_t *hp;
    uint32_t n_limit;          /* windows left undecided for a device limit */
} job_t;

/* pf_ingest.hip / pf_api.hip */
int pf_fetch_cache_scope_ctx(void);
int pf_fetch_cache_home(pf_ctx_t *const *ctxs, int n, const char *path, int32_t tid);
int pf_fetch_cache_home_range(pf_ctx_t *const *ctxs, int n, const char *path, int32_t tid, int64_t lo, int64_t hi);
int pf_ctx_device(const pf_ctx_t *ctx);

struct pf_mp_plan {
    pf_methphase_opts_t o;
    char *bam_path, *vcf_path, *out_prefix;
    pf_gaps_t *gaps;           /* the windows' phase blocks: --tsv / --gtf / --vcf */
    uint32_t n_contigs;
    pf_gaps_t *ugaps_own;      /* -u with --gtf / --tsv: the VCF's own gaps */
    const pf_gaps_t *ug;       /* contigs of the -u pre-pass (the VCF's): ugaps_own or gaps */
    int32_t *utid;             /* [ug->n_contigs] their BAM tids or -1 */
    /* -u pre-pass pieces of a chromosome-scale contig (window contig c's
     * bounds bnd[bnd_off[c], bnd_off[c+1])): placed between the contig's
     * windows' fetch regions, so every window job -- cut at the bounds --
     * is served by one kept piece arena */
    uint64_t *bnd_off;
    int64_t *bnd, *bext;       /* bound k and how far piece k's fetch reaches past it */
    char *interval_path;
    int32_t *tid;              /* [n_contigs] BAM tid or -1 */
    pf_cfg_t *cfg;             /* [n_contigs] */
    uint32_t n_windows;
    uint64_t *win_off;         /* [n_contigs+1] */
    uint32_t *win_start, *win_end;
    uint32_t n_jobs, n_ujobs;
    job_t *jobs, *ujobs;       /* window jobs; -u pre-pass jobs (one per contig, w0=w1=0) */
    uint32_t *order, *uorder;  /* LPT order */
    pf_tags_t *raw;            /* merged -u table */
    int raw_merged;
    int8_t *decision;          /* [n_windows] after finish */
    pf_tags_t *qname_hp;
    pf_blocks_t *blocks;
    int finished;
    uint32_t n_limit;
    double report_counts[3];   /* correct, switch, fail */
    pf_mp_stats_t st;          /* measurement hook (pf_mp_stats) */
    int keeps_arenas;          /* the -u pre-pass's arenas stay on the devices for the window jobs */
    pthread_mutex_t st_mu;
    /* -u without -c, one process: the coverage estimate comes from the -u
     * pre-pass's whole-contig fetches (pf_haptag_bam_cov), per VCF contig */
    int est_deferred;
    int32_t *ucov, *utrunc;
    uint8_t *uhave;
};

static double now_s(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

/* add a device fetch's timings to the run's stats (kind 0 windows, 1 -u) */
static void st_fetch(pf_mp_plan_t *p, int kind, const pf_bam_dev_fetch_t *F, double run_ms) {
    pthread_mutex_lock(&p->st_mu);
    pf_mp_stats_t *s = &p->st;
    if (F) {
        const double m[7] = {F->ms_read, F->ms_inflate, F->ms_chain, F->ms_decode, F->ms_select, F->ms_build,
                             F->ms_total};
        for (int i = 0; i < 7; i++) s->fetch_ms[kind][i] += m[i];
        s->comp_bytes[kind] += F->comp_bytes;
        s->inflated_bytes[kind] += F->inflated_bytes;
        s->n_fetch[kind]++;
        if (kind == 0 && p->keeps_arenas) {
            if (F->from_arena) s->arena_hits++;
            else { s->arena_misses++; s->reread_bytes += F->comp_bytes; }
        }
    }
    s->run_ms[kind] += run_ms;
    pthread_mutex_unlock(&p->st_mu);
}

int pf_mp_stats(const pf_mp_plan_t *p, pf_mp_stats_t *s) {
    if (!p || !s) return PF_ERR_ARG;
    pthread_mutex_lock((pthread_mutex_t *)&p->st_mu);
    *s = p->st;
    pthread_mutex_unlock((pthread_mutex_t *)&p->st_mu);
    return PF_OK;
}

static char *dupstr(const char *s) {
    if (!s) return NULL;
    const size_t l = strlen(s);
    char *d = (char *)malloc(l + 1);
    if (d) memcpy(d, s, l + 1);
    return d;
}

static void job_clear(job_t *j) {
    free(j->dec); free(j->tag_off); free(j->name_off); free(j->names); free(j->hp);
    j->dec = NULL; j->tag_off = NULL; j->name_off = NULL; j->names = NULL; j->hp = NULL;
    j->n_ent = 0;
    j->done = 0;
}

void pf_mp_free(pf_mp_plan_t *p) {
    if (!p) return;
    for (uint32_t j = 0; j < p->n_jobs; j++) job_clear(&p->jobs[j]);
    for (uint32_t j = 0; j < p->n_ujobs; j++) job_clear(&p->ujobs[j]);
    free(p->jobs); free(p->ujobs); free(p->order); free(p->uorder);
    free(p->tid); free(p->cfg); free(p->win_off); free(p->win_start); free(p->win_end);
    free(p->decision);
    pf_tags_free(p->raw);
    pf_tags_free(p->qname_hp);
    if (p->blocks) pf_blocks_free(p->blocks);
    if (p->gaps) pf_gaps_free(p->gaps);
    if (p->ugaps_own) pf_gaps_free(p->ugaps_own);
    free(p->utid); free(p->bnd_off); free(p->bnd); free(p->bext);
    free(p->bam_path); free(p->vcf_path); free(p->out_prefix); free(p->interval_path);
    free(p->ucov); free(p->utrunc); free(p->uhave);
    pthread_mutex_destroy(&p->st_mu);
    free(p);
}

static int cmp_cost_desc(const void *a, const void *b, void *ctx) {
    const job_t *J = (const job_t *)ctx;
    const uint32_t x = *(const uint32_t *)a, y = *(const uint32_t *)b;
    const double cx = J[x].cost, cy = J[y].cost;
    if (cx != cy) return cx > cy ? -1 : 1;
    return x < y ? -1 : x > y;
}

/* LPT order and static rank assignment */
static int lpt(job_t *J, uint32_t n, int32_t world, uint32_t **order_out) {
    uint32_t *ord = (uint32_t *)malloc((n ? n : 1) * sizeof(uint32_t));
    double *load = (double *)calloc(world > 0 ? world : 1, sizeof(double));
    if (!ord || !load) { free(ord); free(load); return PF_ERR_NOMEM; }
    for (uint32_t i = 0; i < n; i++) ord[i] = i;
    qsort_r(ord, n, sizeof(uint32_t), cmp_cost_desc, J);
    const int32_t W = world > 0 ? world : 1;
    for (uint32_t i = 0; i < n; i++) {
        int32_t best = 0;
        for (int32_t r = 1; r < W; r++) if (load[r] < load[best]) best = r;
        J[ord[i]].rank = best;
        load[best] += J[ord[i]].cost;
    }
    free(load);
    *order_out = ord;
    return PF_OK;
}

static void mp_log(const pf_mp_plan_t *p, const char *fmt, const char *a, long x, long y) {
    if (p->o.verbose) { fprintf(stderr, fmt, a, x, y); fputc('\n', stderr); }
}

/* the methphase parameters of contig c from its coverage estimate (or -c) */
static void methphase_cfg(pf_cfg_t *cf, const pf_methphase_opts_t *o, int cov_est) {
    int sel = o->cov_for_selection, nc = o->n_cand, rt = o->cov_for_runtime;
    if (sel <= 0) {                                   /* 4357-4374 */
        sel = cov_est / 10 + 1;
        rt = 2 * sel;
        nc = cov_est / 4 + 1;
    } else if (rt <= 0) {
        rt = 2 * sel;                                  /* config.cov_for_runtime, 4655 */
    }
    if (sel <= 0) sel = 1;                             /* clamps, 4381-4390 */
    if (nc <= 1) nc = 2;
    cf->cov_for_selection = sel; cf->cov_for_runtime = rt; cf->n_cand = nc;
}

static int mp_plan(const pf_methphase_opts_t *o, pf_mp_plan_t **out, int defer_est);

int pf_mp_plan(const pf_methphase_opts_t *o, pf_mp_plan_t **out) { return mp_plan(o, out, 0); }

/* the phase-block file the windows come from (main_blockjoin 4661-4666) */
static int interval_file(const pf_methphase_opts_t *o, const char **path) {
    if (o->interval_path && o->interval_format != PF_INTERVALS_VCF) { *path = o->interval_path; return o->interval_format; }
    *path = o->vcf_path;
    return PF_INTERVALS_VCF;
}

static int mp_plan(const pf_methphase_opts_t *o, pf_mp_plan_t **out, int defer_est) {
    if (!o || !out || !o->bam_path) return PF_ERR_ARG;
    if (o->mode != PF_MODE_METHPHASE && o->mode != PF_MODE_REPORT) return PF_ERR_ARG;
    const char *ipath = NULL;
    const int ifmt = interval_file(o, &ipath);
    if (!ipath || ifmt < PF_INTERVALS_VCF || ifmt > PF_INTERVALS_TSV) return PF_ERR_ARG;
    /* -u needs the VCF's variants; report reads only the VCF (main_methreport 4916-4919) */
    if ((o->untagged || o->mode == PF_MODE_REPORT) && !o->vcf_path) return PF_ERR_ARG;
    if (o->mode == PF_MODE_REPORT && ifmt != PF_INTERVALS_VCF) return PF_ERR_ARG;
    if (o->mode == PF_MODE_REPORT && (o->chunk_size <= 0 || o->chunk_stride <= 0)) return PF_ERR_ARG;
    *out = NULL;
    const double t_plan0 = now_s();
    pf_mp_plan_t *p = (pf_mp_plan_t *)calloc(1, sizeof *p);
    if (!p) return PF_ERR_NOMEM;
    pthread_mutex_init(&p->st_mu, NULL);
    p->o = *o;
    p->bam_path = dupstr(o->bam_path);
    p->vcf_path = dupstr(o->vcf_path);
    p->out_prefix = dupstr(o->out_prefix);
    p->interval_path = dupstr(o->interval_path);
    p->o.bam_path = p->bam_path;
    p->o.vcf_path = p->vcf_path;
    p->o.out_prefix = p->out_prefix;
    p->o.interval_path = p->interval_path;
    p->o.ctxs = NULL;
    p->o.n_ctxs = 0;
    /* -u: the VCF's contigs are pre-haplotagged (load_intervals_from_file with
     * load_vcf_variants_too, 4446); a GTF / TSV then replaces the intervals
     * (wipe_intervals_of_storage_t + reload, 4460-4465) */
    int rc = PF_OK;
    if (o->untagged && ifmt != PF_INTERVALS_VCF) rc = pf_vcf_gaps(o->vcf_path, PF_READBACK, &p->ugaps_own);
    if (!rc) rc = pf_interval_gaps(ipath, ifmt, PF_READBACK, &p->gaps);
    if (rc) { pf_mp_free(p); return rc; }
    p->ug = p->ugaps_own ? p->ugaps_own : p->gaps;
    const pf_gaps_t *g = p->gaps;
    const uint32_t C = g->n_contigs;
    p->n_contigs = C;
    p->tid = (int32_t *)calloc(C ? C : 1, sizeof(int32_t));
    p->cfg = (pf_cfg_t *)calloc(C ? C : 1, sizeof(pf_cfg_t));
    p->win_off = (uint64_t *)calloc(C + 1, sizeof(uint64_t));
    p->ucov = (int32_t *)calloc(C ? C : 1, sizeof(int32_t));
    p->utrunc = (int32_t *)calloc(C ? C : 1, sizeof(int32_t));
    p->uhave = (uint8_t *)calloc(C ? C : 1, 1);
    p->utid = (int32_t *)calloc(p->ug->n_contigs ? p->ug->n_contigs : 1, sizeof(int32_t));
    if (!p->tid || !p->cfg || !p->win_off || !p->ucov || !p->utrunc || !p->uhave || !p->utid) {
        pf_mp_free(p);
        return PF_ERR_NOMEM;
    }

    pf_bam_t *bam = NULL;
    rc = pf_bam_open(o->bam_path, NULL, &bam);
    if (!rc) pf_bam_set_threads(bam, o->threads);
    if (rc) { pf_mp_free(p); return rc; }
    const int32_t nt = pf_bam_n_targets(bam);
    int32_t *covs = NULL;
    const int need_est = o->mode == PF_MODE_METHPHASE ? o->cov_for_selection <= 0 : o->cov <= 0;
    const double t_est0 = now_s();
    p->est_deferred = need_est && defer_est && o->mode == PF_MODE_METHPHASE && o->untagged && !o->host_fetch &&
                      o->n_ctxs > 0 && p->ug == p->gaps;
    if (need_est) {
        covs = (int32_t *)calloc(nt > 0 ? nt : 1, sizeof(int32_t));
        if (!covs) rc = PF_ERR_NOMEM;
        if (!rc && p->est_deferred) {
            /* estimated from the -u pre-pass's fetches (finish_deferred_estimate) */
        } else if (!rc && !o->host_fetch && (o->n_ctxs > 0 || pf_device_count() > 0)) {
            /* the pass over the whole BAM on the device (the first context or
             * device of the run); runs without a device scan on the host */
            pf_ctx_t *ec = o->n_ctxs > 0 ? o->ctxs[0] : NULL;
            int own = 0;
            if (!ec) { rc = pf_ctx_create(o->devices ? o->devices[0] : 0, &ec); own = !rc; }
            if (!rc) rc = pf_bam_estimate_coverage_dev(ec, bam, covs, nt > 0 ? nt : 1, 0);
            if (own) pf_ctx_destroy(ec);
        } else if (!rc) {
            rc = pf_bam_estimate_coverage(bam, covs, nt > 0 ? nt : 1);
        }
    }
    p->st.s_estimate = now_s() - t_est0;
    /* windows: merged gaps (methphase) or report chunks of the raw gaps */
    uint64_t nw = 0, cap = 0;
    for (uint32_t c = 0; c < p->ug->n_contigs; c++) p->utid[c] = pf_bam_tid(bam, p->ug->names[c]);
    for (uint32_t c = 0; c < C && !rc; c++) {
        p->tid[c] = pf_bam_tid(bam, g->names[c]);
        pf_cfg_t *cf = &p->cfg[c];
        cf->k = o->k > 0 ? o->k : 3;
        cf->k_span = o->k_span > 0 ? o->k_span : 5000;
        cf->hard_cov = 15;
        if (o->mode == PF_MODE_METHPHASE) {
            methphase_cfg(cf, o, need_est && (p->tid[c] >= 0 && p->tid[c] < nt) ? covs[p->tid[c]] : 0);
        } else {                                               /* 5045-5051: no clamps */
            /* covs is indexed by the VCF contig index here, as the reference
             * does (covs[i_ref], 5046); out of range reads as 0 */
            const int cov = o->cov > 0 ? o->cov : ((int32_t)c < nt ? covs[c] : 0);
            cf->cov_for_selection = cov / 10 + 1;
            cf->cov_for_runtime = 2 * cf->cov_for_selection;
            cf->n_cand = cov / 4 + 1;
        }
        uint64_t n_c;
        if (o->mode == PF_MODE_METHPHASE) {
            n_c = g->gap_off[c + 1] - g->gap_off[c];
        } else {
            const int64_t r = pf_report_windows(g->abs_start[c], g->raw_start + g->raw_off[c], g->raw_end + g->raw_off[c],
                                                g->raw_off[c + 1] - g->raw_off[c], (uint32_t)o->chunk_size,
                                                (uint32_t)o->chunk_stride, NULL, NULL, 0);
            if (r < 0) { rc = (int)r; break; }
            n_c = (uint64_t)r;
        }
        if (nw + n_c > cap) {
            uint64_t nc2 = cap ? cap : 1024;
            while (nc2 < nw + n_c) nc2 *= 2;
            uint32_t *a = (uint32_t *)realloc(p->win_start, nc2 * sizeof(uint32_t));
            if (!a) { rc = PF_ERR_NOMEM; break; }
            p->win_start = a;
            a = (uint32_t *)realloc(p->win_end, nc2 * sizeof(uint32_t));
            if (!a) { rc = PF_ERR_NOMEM; break; }
            p->win_end = a;
            cap = nc2;
        }
        if (o->mode == PF_MODE_METHPHASE) {
            memcpy(p->win_start + nw, g->gap_start + g->gap_off[c], n_c * sizeof(uint32_t));
            memcpy(p->win_end + nw, g->gap_end + g->gap_off[c], n_c * sizeof(uint32_t));
        } else if (n_c) {
            const int64_t r = pf_report_windows(g->abs_start[c], g->raw_start + g->raw_off[c], g->raw_end + g->raw_off[c],
                                                g->raw_off[c + 1] - g->raw_off[c], (uint32_t)o->chunk_size,
                                                (uint32_t)o->chunk_stride, p->win_start + nw, p->win_end + nw, n_c);
            if (r != (int64_t)n_c) { rc = PF_ERR_INTERNAL; break; }
        }
        nw += n_c;
        p->win_off[c + 1] = nw;
        if (o->mode == PF_MODE_REPORT && o->verbose >= 0)
            fprintf(stderr, "[M::%s] %s has %d intervals\n", "main_methreport", g->names[c], (int)n_c);
    }
    free(covs);
    pf_bam_close(bam);
    if (rc) { pf_mp_free(p); return rc; }
    if (nw > UINT32_MAX) { pf_mp_free(p); return PF_ERR_LIMIT; }
    p->n_windows = (uint32_t)nw;

    /* -u pre-pass pieces (device fetch): a contig past the piece size is
     * fetched in position pieces whose arenas are kept one by one; each bound
     * moves from k * step to the nearest position outside every window's
     * fetch region (within half a step), so no window straddles two pieces */
    p->bnd_off = (uint64_t *)calloc(C + 1, sizeof(uint64_t));
    if (!p->bnd_off) { pf_mp_free(p); return PF_ERR_NOMEM; }
    if (o->untagged && !o->host_fetch && o->mode == PF_MODE_METHPHASE) {
        pf_bam_t *bb = NULL;
        rc = pf_bam_open(o->bam_path, NULL, &bb);
        uint64_t nb = 0, bcap = 0;
        for (uint32_t c = 0; c < C && !rc; c++) {
            p->bnd_off[c] = nb;
            if (p->tid[c] < 0) continue;
            int64_t step = 0;
            const uint64_t K = pf_bam_contig_pieces(bb, p->tid[c], 0, &step);
            if (K <= 1 || step <= 0) continue;
            /* the windows' fetch regions, merged into clusters */
            const uint64_t w0 = p->win_off[c], w1 = p->win_off[c + 1];
            int64_t *ca = (int64_t *)malloc(2 * (w1 - w0 + 1) * sizeof(int64_t));
            if (!ca) { rc = PF_ERR_NOMEM; break; }
            uint64_t ncl = 0;
            for (uint64_t w = w0; w < w1; w++) {          /* windows are in file order: starts ascending */
                const int64_t a = p->win_start[w] > PF_READBACK ? (int64_t)p->win_start[w] - PF_READBACK : 0;
                const int64_t b = (int64_t)p->win_end[w] + PF_READBACK;
                if (ncl && a < ca[2 * ncl - 1]) { if (b > ca[2 * ncl - 1]) ca[2 * ncl - 1] = b; }
                else { ca[2 * ncl] = a; ca[2 * ncl + 1] = b; ncl++; }
            }
            int64_t prev = 0;
            for (uint64_t k = 1; k < K; k++) {
                const int64_t t = (int64_t)k * step;
                int64_t x = t;
                for (uint64_t q = 0; q < ncl; q++) {
                    if (ca[2 * q] < t && t < ca[2 * q + 1]) {
                        const int64_t A = ca[2 * q], B = ca[2 * q + 1];
                        x = (t - A <= B - t && A > prev) ? A : B;
                        if (x - t > step / 2 || t - x > step / 2) x = t;
                        break;
                    }
                }
                if (x <= prev) continue;
                if (nb == bcap) {
                    bcap = bcap ? 2 * bcap : 64;
                    int64_t *nbp = (int64_t *)realloc(p->bnd, bcap * sizeof(int64_t));
                    if (nbp) p->bnd = nbp;
                    int64_t *nbe = nbp ? (int64_t *)realloc(p->bext, bcap * sizeof(int64_t)) : NULL;
                    if (!nbp || !nbe) { rc = PF_ERR_NOMEM; break; }
                    p->bext = nbe;
                }
                /* piece k-1 serves the windows whose fetch region starts
                 * before x (the job cut below): its fetch reaches the
                 * furthest of their ends, not the end of their cluster --
                 * dense windows merge into one cluster per contig */
                int64_t ext = x;
                for (uint64_t w = w0; w < w1; w++) {
                    const int64_t a = p->win_start[w] > PF_READBACK ? (int64_t)p->win_start[w] - PF_READBACK : 0;
                    if (a >= x) break;
                    const int64_t b = (int64_t)p->win_end[w] + PF_READBACK;
                    if (b > ext) ext = b;
                }
                p->bnd[nb] = x;
                p->bext[nb] = ext;
                nb++;
                prev = x;
            }
            free(ca);
        }
        p->bnd_off[C] = nb;
        if (bb) pf_bam_close(bb);
        if (rc) { pf_mp_free(p); return rc; }
    }

    /* window jobs: runs of consecutive windows of one contig, at most
     * job_windows windows and, with several devices or ranks, small enough
     * that every one gets several jobs; never across a -u piece bound */
    const uint32_t jw = o->job_windows ? o->job_windows : PF_JOB_WINDOWS_DEFAULT;
    double tot_span = 0;
    for (uint64_t w = 0; w < nw; w++) tot_span += (double)(p->win_end[w] - p->win_start[w]) + 2.0 * PF_READBACK;
    const int32_t par = (o->world > 1 ? o->world : 1) * (o->n_devices > 1 ? o->n_devices : 1);
    const double span_cap = par > 1 ? tot_span / (4.0 * par) : 1e300;
    uint32_t nj = 0, jcap = 64;
    p->jobs = (job_t *)calloc(jcap, sizeof(job_t));
    if (!p->jobs) { pf_mp_free(p); return PF_ERR_NOMEM; }
    for (uint32_t c = 0; c < C; c++) {
        uint64_t w = p->win_off[c];
        const int64_t *bd = p->bnd + p->bnd_off[c];
        const uint64_t nbd = p->bnd_off[c + 1] - p->bnd_off[c];
        /* the piece a window's fetch region starts in */
        #define WIN_LO(w_) ((int64_t)(p->win_start[w_] > PF_READBACK ? p->win_start[w_] - PF_READBACK : 0))
        #define WIN_HI(w_) ((int64_t)p->win_end[w_] + PF_READBACK)
        while (w < p->win_off[c + 1]) {
            const uint64_t w0 = w;
            double span = 0;
            uint64_t pc = 0;
            while (pc < nbd && bd[pc] <= WIN_LO(w0)) pc++;
            int64_t lo = WIN_LO(w0), hi = WIN_HI(w0);
            while (w < p->win_off[c + 1] && w - w0 < jw && (w == w0 || span < span_cap) &&
                   (w == w0 || pc >= nbd || WIN_LO(w) < bd[pc])) {
                span += (double)(p->win_end[w] - p->win_start[w]) + 2.0 * PF_READBACK;
                if (WIN_LO(w) < lo) lo = WIN_LO(w);
                if (WIN_HI(w) > hi) hi = WIN_HI(w);
                w++;
            }
            if (nj == jcap) {
                job_t *nj2 = (job_t *)realloc(p->jobs, 2 * jcap * sizeof(job_t));
                if (!nj2) { pf_mp_free(p); return PF_ERR_NOMEM; }
                memset(nj2 + jcap, 0, jcap * sizeof(job_t));
                p->jobs = nj2;
                jcap *= 2;
            }
            job_t *J = &p->jobs[nj++];
            J->contig = c; J->w0 = (uint32_t)w0; J->w1 = (uint32_t)w; J->cost = span;
            J->lo = lo; J->hi = hi; J->bc = -1;
        }
    }
    p->n_jobs = nj;
    rc = lpt(p->jobs, nj, o->world, &p->order);
    /* -u pre-pass jobs: one per VCF contig present in the BAM (cost: contig length) */
    if (!rc && o->untagged) {
        const uint32_t UC = p->ug->n_contigs;
        p->ujobs = (job_t *)calloc(UC ? UC : 1, sizeof(job_t));
        if (!p->ujobs) rc = PF_ERR_NOMEM;
        uint32_t nu = 0;
        pf_bam_t *b2 = NULL;
        if (!rc) rc = pf_bam_open(o->bam_path, NULL, &b2);
        for (uint32_t c = 0; c < UC && !rc; c++) {
            if (p->utid[c] < 0) continue;
            job_t *J = &p->ujobs[nu++];
            J->contig = c;
            J->cost = (double)pf_bam_target_len(b2, p->utid[c]);
            J->bc = -1;                                          /* the window contig of the same name */
            for (uint32_t wc = 0; wc < C; wc++)
                if (!strcmp(g->names[wc], p->ug->names[c])) { J->bc = (int32_t)wc; break; }
        }
        if (b2) pf_bam_close(b2);
        p->n_ujobs = nu;
        if (!rc) rc = lpt(p->ujobs, nu, o->world, &p->uorder);
    }
    p->raw = pf_tags_new();
    p->qname_hp = pf_tags_new();
    if (!rc && (!p->raw || !p->qname_hp)) rc = PF_ERR_NOMEM;
    if (rc) { pf_mp_free(p); return rc; }
    mp_log(p, "[M::pf_mp_plan] %s: %ld windows in %ld jobs", o->mode == PF_MODE_REPORT ? "report" : "methphase",
           (long)p->n_windows, (long)p->n_jobs);
    p->st.s_plan = now_s() - t_plan0;
    *out = p;
    return PF_OK;
}

uint32_t pf_mp_n_jobs(const pf_mp_plan_t *p, int kind) {
    if (!p) return 0;
    return kind == PF_JOB_HAPTAG ? p->n_ujobs : p->n_jobs;
}

static job_t *job_of(const pf_mp_plan_t *p, int kind, uint32_t j) {
    if (!p) return NULL;
    if (kind == PF_JOB_HAPTAG) return j < p->n_ujobs ? &p->ujobs[j] : NULL;
    return j < p->n_jobs ? &p->jobs[j] : NULL;
}

int pf_mp_job_info(const pf_mp_plan_t *p, int kind, uint32_t j, pf_mp_job_info_t *info) {
    const job_t *J = job_of(p, kind, j);
    if (!J || !info) return PF_ERR_ARG;
    const uint32_t *ord = kind == PF_JOB_HAPTAG ? p->uorder : p->order;
    const uint32_t n = kind == PF_JOB_HAPTAG ? p->n_ujobs : p->n_jobs;
    uint32_t pos = 0;
    for (uint32_t i = 0; i < n; i++) if (ord[i] == j) { pos = i; break; }
    info->contig = J->contig;
    info->contig_name = (kind == PF_JOB_HAPTAG ? p->ug : p->gaps)->names[J->contig];
    info->w0 = J->w0;
    info->w1 = J->w1;
    info->rank = J->rank;
    info->lpt_pos = pos;
    info->cost = J->cost;
    info->done = J->done;
    if (kind == PF_JOB_HAPTAG && p->ug != p->gaps) memset(&info->cfg, 0, sizeof info->cfg);
    else info->cfg = p->cfg[J->contig];
    return PF_OK;
}

int pf_mp_windows(const pf_mp_plan_t *p, const uint32_t **win_start, const uint32_t **win_end,
                  const uint64_t **contig_win_off, uint32_t *n_windows) {
    if (!p) return PF_ERR_ARG;
    if (win_start) *win_start = p->win_start;
    if (win_end) *win_end = p->win_end;
    if (contig_win_off) *contig_win_off = p->win_off;
    if (n_windows) *n_windows = p->n_windows;
    return PF_OK;
}

const pf_gaps_t *pf_mp_gaps(const pf_mp_plan_t *p) { return p ? p->gaps : NULL; }
const pf_blocks_t *pf_mp_blocks(const pf_mp_plan_t *p) { return p ? p->blocks : NULL; }
const pf_tags_t *pf_mp_qname_hp(const pf_mp_plan_t *p) { return p ? p->qname_hp : NULL; }
const pf_tags_t *pf_mp_raw_hp(const pf_mp_plan_t *p) { return p && p->o.untagged ? p->raw : NULL; }

int pf_mp_decisions(const pf_mp_plan_t *p, const int8_t **dec, uint32_t *n, uint32_t *n_limit) {
    if (!p) return PF_ERR_ARG;
    if (!p->finished) {                         /* varhaptag: no windows were run */
        if (dec) *dec = NULL;
        if (n) *n = 0;
        if (n_limit) *n_limit = 0;
        return PF_OK;
    }
    if (dec) *dec = p->decision;
    if (n) *n = p->n_windows;
    if (n_limit) *n_limit = p->n_limit;
    return PF_OK;
}

/* ------------------------------------------------------------------ */
/* job results                                                          */

int pf_mp_get_job_result(const pf_mp_plan_t *p, int kind, uint32_t j, pf_mp_job_result_t *r) {
    const job_t *J = job_of(p, kind, j);
    if (!J || !r) return PF_ERR_ARG;
    if (!J->done) return PF_ERR_ARG;
    if (J->n_ent > UINT32_MAX) return PF_ERR_LIMIT;
    r->n_windows = J->w1 - J->w0;
    r->decision = J->dec;
    r->tag_off = J->tag_off;
    r->tags.n = (uint32_t)J->n_ent;
    r->tags.off = J->name_off;
    r->tags.names = J->names;
    r->tags.hp = J->hp;
    r->n_limit = J->n_limit;
    return PF_OK;
}

static int job_store(job_t *J, uint32_t n_win, const int8_t *dec, const uint64_t *tag_off, uint64_t n_ent,
                     const uint64_t *name_off, const char *names, const uint8_t *hp, uint32_t n_limit) {
    job_clear(J);
    J->dec = (int8_t *)malloc(n_win ? n_win : 1);
    J->tag_off = (uint64_t *)malloc((n_win + 1) * sizeof(uint64_t));
    J->name_off = (uint64_t *)malloc((n_ent + 1) * sizeof(uint64_t));
    const uint64_t nb = n_ent ? name_off[n_ent] - name_off[0] : 0;
    J->names = (char *)malloc(nb ? nb : 1);
    J->hp = (uint8_t *)malloc(n_ent ? n_ent : 1);
    if (!J->dec || !J->tag_off || !J->name_off || !J->names || !J->hp) { job_clear(J); return PF_ERR_NOMEM; }
    if (n_win) memcpy(J->dec, dec, n_win);
    if (tag_off) for (uint32_t w = 0; w <= n_win; w++) J->tag_off[w] = tag_off[w] - tag_off[0];
    else for (uint32_t w = 0; w <= n_win; w++) J->tag_off[w] = 0;
    for (uint64_t i = 0; i <= n_ent; i++) J->name_off[i] = n_ent ? name_off[i] - name_off[0] : 0;
    if (nb) memcpy(J->names, names + name_off[0], nb);
    if (n_ent) memcpy(J->hp, hp, n_ent);
    J->n_ent = n_ent;
    J->n_limit = n_limit;
    J->done = 1;
    return PF_OK;
}

int pf_mp_set_job_result(pf_mp_plan_t *p, int kind, uint32_t j, const pf_mp_job_result_t *r) {
    job_t *J = job_of(p, kind, j);
    if (!J || !r) return PF_ERR_ARG;
    if (r->n_windows != J->w1 - J->w0) return PF_ERR_ARG;
    if (r->n_windows && !r->decision) return PF_ERR_ARG;
    if (r->tags.n && (!r->tags.off || !r->tags.names || !r->tags.hp)) return PF_ERR_ARG;
    if (kind != PF_JOB_HAPTAG && r->tag_off && r->tag_off[r->n_windows] - r->tag_off[0] != r->tags.n)
        return PF_ERR_ARG;
    if (kind != PF_JOB_HAPTAG && r->tags.n && !r->tag_off) return PF_ERR_ARG;
    static const uint64_t zero = 0;
    return job_store(J, r->n_windows, r->decision, kind == PF_JOB_HAPTAG ? NULL : r->tag_off, r->tags.n,
                     r->tags.n ? r->tags.off : &zero, r->tags.names, r->tags.hp, r->n_limit);
}

/* ------------------------------------------------------------------ */
/* running jobs on a device                                             */

typedef struct {                /* a growable (qname, hp) list */
    uint64_t n, cap;
    uint64_t *off;
    char *names;
    uint64_t nb, nbcap;
    uint8_t *hp;
} entlist_t;

static void ent_free(entlist_t *e) { free(e->off); free(e->names); free(e->hp); memset(e, 0, sizeof *e); }

static int ent_push(entlist_t *e, const char *nm, size_t l, uint8_t hp) {
    if (!e->off) {
        e->cap = 1024;
        e->off = (uint64_t *)malloc((e->cap + 1) * sizeof(uint64_t));
        e->hp = (uint8_t *)malloc(e->cap);
        e->nbcap = 16384;
        e->names = (char *)malloc(e->nbcap);
        if (!e->off || !e->hp || !e->names) return PF_ERR_NOMEM;
        e->off[0] = 0;
    }
    if (e->n + 1 > e->cap) {
        e->cap *= 2;
        uint64_t *o = (uint64_t *)realloc(e->off, (e->cap + 1) * sizeof(uint64_t));
        uint8_t *h = o ? (uint8_t *)realloc(e->hp, e->cap) : NULL;
        if (o) e->off = o;
        if (!o || !h) return PF_ERR_NOMEM;
        e->hp = h;
    }
    if (e->nb + l > e->nbcap) {
        while (e->nb + l > e->nbcap) e->nbcap *= 2;
        char *s = (char *)realloc(e->names, e->nbcap);
        if (!s) return PF_ERR_NOMEM;
        e->names = s;
    }
    memcpy(e->names + e->nb, nm, l);
    e->nb += l;
    e->hp[e->n++] = hp;
    e->off[e->n] = e->nb;
    return PF_OK;
}

int pf_mp_run_haptag_job(pf_mp_plan_t *p, pf_ctx_t *ctx, uint32_t j) {
    job_t *J = job_of(p, PF_JOB_HAPTAG, j);
    if (!J || !ctx) return PF_ERR_ARG;
    const char *contig = p->ug->names[J->contig];
    pf_known_table_t *kt = NULL;
    pf_bam_t *bam = NULL;
    pf_bam_reads_t *rd = NULL;
    uint8_t *hp = NULL;
    entlist_t e = {0};
    pf_tags_t *seen = NULL;
    int rc = pf_vcf_known_vars(p->vcf_path, contig, &kt);
    if (!rc && kt->vars.n) rc = pf_bam_open(p->bam_path, NULL, &bam);
    if (!rc && bam) pf_bam_set_threads(bam, p->o.threads);
    if (!rc && kt->vars.n && !p->o.host_fetch) {
        /* device fetch + K4 on the device (pf_haptag_bam) */
        pf_bam_dev_fetch_t *F = NULL;
        const double t0 = now_s();
        /* the contig's pieces: the plan's bounds (between its windows), or
         * the default equal-length pieces when it has none */
        const uint64_t b0 = J->bc >= 0 ? p->bnd_off[J->bc] : 0, b1 = J->bc >= 0 ? p->bnd_off[J->bc + 1] : 0;
        if (p->est_deferred) {                  /* the contig's coverage estimate from the same fetch */
            rc = pf_haptag_bam_pieces(ctx, &kt->vars, bam, contig, (uint32_t)(b1 - b0), b1 > b0 ? p->bnd + b0 : NULL,
                                      b1 > b0 ? p->bext + b0 : NULL, &F, &p->ucov[J->contig], &p->utrunc[J->contig]);
            if (!rc) p->uhave[J->contig] = 1;
        } else {
            rc = pf_haptag_bam_pieces(ctx, &kt->vars, bam, contig, (uint32_t)(b1 - b0), b1 > b0 ? p->bnd + b0 : NULL,
                                      b1 > b0 ? p->bext + b0 : NULL, &F, NULL, NULL);
        }
        if (!rc) st_fetch(p, 1, F, (now_s() - t0) * 1e3 - F->ms_total);
        if (!rc && F->n_recs) {
            seen = pf_tags_new();
            if (!seen) rc = PF_ERR_NOMEM;
            for (uint64_t r = 0; r < F->n_recs && !rc; r++) {
                const char *nm = F->qname + F->qname_off[r];
                const size_t l = (size_t)(F->qname_off[r + 1] - F->qname_off[r]);
                const int ins = tags_put(seen, nm, l, F->read_hp[r]);
                if (ins < 0) rc = ins;
                else if (ins) rc = ent_push(&e, nm, l, F->read_hp[r]);
            }
        }
        pf_bam_dev_fetch_free(F);
    } else if (!rc && kt->vars.n) rc = pf_bam_fetch_contig_reads(bam, contig, &rd);
    if (!rc && rd && rd->reads.n_reads) {
        hp = (uint8_t *)malloc(rd->reads.n_reads);
        seen = pf_tags_new();
        if (!hp || !seen) rc = PF_ERR_NOMEM;
        if (!rc) rc = pf_haptag_reads(ctx, &kt->vars, &rd->reads, hp);
        /* the contig's table, first wins (1880-1889), kept in BAM order */
        for (uint32_t r = 0; r < rd->reads.n_reads && !rc; r++) {
            const char *nm = rd->qname + rd->qname_off[r];
            const size_t l = (size_t)(rd->qname_off[r + 1] - rd->qname_off[r]);
            const int ins = tags_put(seen, nm, l, hp[r]);
            if (ins < 0) rc = ins;
            else if (ins) rc = ent_push(&e, nm, l, hp[r]);
        }
    }
    if (!rc) {
        static const uint64_t zero = 0;
        rc = job_store(J, 0, NULL, NULL, e.n, e.off ? e.off : &zero, e.names, e.hp, 0);
    }
    ent_free(&e);
    pf_tags_free(seen);
    free(hp);
    if (rd) pf_bam_reads_free(rd);
    if (bam) pf_bam_close(bam);
    if (kt) pf_known_table_free(kt);
    return rc;
}

int pf_mp_merge_raw(pf_mp_plan_t *p) {
    if (!p) return PF_ERR_ARG;
    if (!p->o.untagged) { p->raw_merged = 1; return PF_OK; }
    const double t0 = now_s();
    /* contig order, first wins across contigs (the -u table is one hash
     * filled contig by contig, 2069-2080) */
    const uint32_t UC = p->ug->n_contigs;
    uint32_t *by_contig = (uint32_t *)malloc((UC ? UC : 1) * sizeof(uint32_t));
    if (!by_contig) return PF_ERR_NOMEM;
    for (uint32_t c = 0; c < UC; c++) by_contig[c] = UINT32_MAX;
    for (uint32_t j = 0; j < p->n_ujobs; j++) {
        if (!p->ujobs[j].done) { free(by_contig); return PF_ERR_ARG; }
        by_contig[p->ujobs[j].contig] = j;
    }
    int rc = PF_OK;
    for (uint32_t c = 0; c < UC && !rc; c++) {
        if (by_contig[c] == UINT32_MAX) continue;
        const job_t *J = &p->ujobs[by_contig[c]];
        if (J->n_ent > UINT32_MAX) { rc = PF_ERR_LIMIT; break; }
        const int64_t r = pf_tags_put_first(p->raw, (uint32_t)J->n_ent, J->name_off, J->names, J->hp);
        if (r < 0) rc = (int)r;
    }
    free(by_contig);
    if (!rc) p->raw_merged = 1;
    p->st.s_haptag += now_s() - t0;
    return rc;
}

/* fetch of one job (host), separate from the device part so that the next
 * job's fetch overlaps this job's kernels */
typedef struct {
    pf_bam_records_t *recs;
    int rc;
} fetch_t;

static int job_fetch(const pf_mp_plan_t *p, pf_bam_t *bam, const job_t *J, fetch_t *f) {
    f->recs = NULL;
    f->rc = PF_OK;
    if (p->tid[J->contig] < 0) return PF_OK;
    f->rc = pf_bam_fetch_windows(bam, p->gaps->names[J->contig], J->w1 - J->w0, p->win_start + J->w0,
                                 p->win_end + J->w0, PF_READBACK, p->o.threads > 0 ? p->o.threads : 1, &f->recs);
    if (!f->rc && p->o.untagged) {              /* the -u table replaces HP (1114-1122) */
        pf_aln_batch_t *a = &f->recs->aln;
        f->rc = (int)pf_tags_get(p->raw, a->n_recs, f->recs->qname_off, f->recs->qname, 254, (uint8_t *)a->hp);
        if (f->rc > 0) f->rc = 0;
    }
    return f->rc;
}

/* upload + run a sub-batch of windows [a, b) of the fetched records */
static int run_windows(const pf_mp_plan_t *p, pf_ctx_t *ctx, const job_t *J, const pf_bam_records_t *R,
                       const uint32_t *sel, uint32_t n_sel, int8_t *dec, entlist_t *ent, uint64_t *win_ent) {
    const pf_aln_batch_t *A = &R->aln;
    const pf_cfg_t *cf = &p->cfg[J->contig];
    pf_load_cfg_t lc = p->o.load;
    /* gather the selected windows (usually all of them, in order) */
    pf_aln_batch_t a = *A;
    uint32_t *wro = NULL;
    int all = n_sel == A->n_windows;
    for (uint32_t i = 0; all && i < n_sel; i++) all = sel[i] == i;
    if (!all) {
        /* a single window: slice the arrays (offsets stay absolute) */
        if (n_sel != 1) return PF_ERR_INTERNAL;
        const uint32_t w = sel[0];
        const uint32_t r0 = A->win_rec_off[w], r1 = A->win_rec_off[w + 1];
        wro = (uint32_t *)malloc(2 * sizeof(uint32_t));
        if (!wro) return PF_ERR_NOMEM;
        wro[0] = 0; wro[1] = r1 - r0;
        a.n_windows = 1; a.n_recs = r1 - r0;
        a.win_start = A->win_start + w; a.win_end = A->win_end + w; a.win_rec_off = wro;
        a.flag = A->flag + r0; a.mapq = A->mapq + r0; a.pos = A->pos + r0; a.l_qseq = A->l_qseq + r0;
        a.de = A->de + r0; a.hp = A->hp + r0;
        a.cigar_off = A->cigar_off + r0; a.seq_off = A->seq_off + r0; a.mm_off = A->mm_off + r0;
        a.ml_off = A->ml_off + r0;
    }
    pf_dbatch_t *db = NULL;
    int rc = pf_batch_upload_aln(ctx, cf, &lc, &a, &db);
    /* the kept reads are known after a run (K0 sizes the batch on the
     * device); the records bound them */
    const uint32_t W = a.n_windows, cap = a.n_recs ? a.n_recs : 1;
    uint32_t R_ = 0;
    uint32_t *rec_of = NULL;
    uint8_t *rhp = NULL;
    int8_t *d = NULL;
    if (!rc) {
        rec_of = (uint32_t *)malloc(cap * sizeof(uint32_t));
        rhp = (uint8_t *)malloc(cap);
        d = (int8_t *)malloc(W ? W : 1);
        if (!rec_of || !rhp || !d) rc = PF_ERR_NOMEM;
    }
    if (!rc) {
        pf_window_out_t o;
        memset(&o, 0, sizeof o);
        o.decision = d;
        o.read_hp = rhp;
        rc = pf_methphase_run(ctx, db, &o);
    }
    if (!rc) {
        R_ = pf_batch_n_reads(db);
        if (R_ > cap) rc = PF_ERR_INTERNAL;
    }
    if (!rc) rc = pf_batch_read_recs(db, rec_of, cap);
    if (!rc) {
        /* reads are the kept records in record order; window w's reads are
         * those whose record lies in [win_rec_off[w], win_rec_off[w+1]) */
        const uint64_t rbase = a.win_rec_off == wro ? A->win_rec_off[sel[0]] : 0;
        uint32_t i = 0;
        for (uint32_t w = 0; w < W && !rc; w++) {
            const uint32_t gw = all ? w : sel[0];
            dec[gw] = d[w];
            const uint32_t rend = a.win_rec_off[w + 1];
            const uint64_t e0 = ent->n;
            for (; i < R_ && rec_of[i] < rend; i++) {
                if (d[w] < 0 || p->o.mode == PF_MODE_REPORT) continue;
                const uint64_t rec = rbase + rec_of[i];
                rc = ent_push(ent, R->qname + R->qname_off[rec], (size_t)(R->qname_off[rec + 1] - R->qname_off[rec]),
                              rhp[i]);
                if (rc) break;
            }
            win_ent[gw] = ent->n - e0;
        }
    }
    if (db) pf_batch_free(db);
    free(rec_of); free(rhp); free(d); free(wro);
    return rc;
}

static int job_device(pf_mp_plan_t *p, pf_ctx_t *ctx, job_t *J, fetch_t *f) {
    if (f->rc) return f->rc;
    const uint32_t n = J->w1 - J->w0;
    int8_t *dec = (int8_t *)malloc(n ? n : 1);
    uint64_t *cnt = (uint64_t *)calloc(n + 1, sizeof(uint64_t));
    uint64_t *toff = (uint64_t *)calloc(n + 1, sizeof(uint64_t));
    uint32_t *sel = (uint32_t *)malloc((n ? n : 1) * sizeof(uint32_t));
    entlist_t ent = {0};
    uint32_t n_limit = 0;
    int rc = (!dec || !cnt || !toff || !sel) ? PF_ERR_NOMEM : PF_OK;
    for (uint32_t w = 0; w < n && !rc; w++) dec[w] = -1;
    if (!rc && f->recs && n) {
        const pf_aln_batch_t *A = &f->recs->aln;
        /* windows over the device's per-window read limit stay undecided */
        uint32_t ns = 0, big = 0;
        for (uint32_t w = 0; w < n; w++) {
            if (A->win_rec_off[w + 1] - A->win_rec_off[w] > PF_MAX_WIN_RECS) { big++; continue; }
            sel[ns++] = w;
        }
        if (big == 0) {
            rc = run_windows(p, ctx, J, f->recs, sel, ns, dec, &ent, cnt);
        }
        if (big || rc == PF_ERR_LIMIT) {
            /* window by window; a window the device refuses stays -1 */
            ent.n = 0; ent.nb = 0;
            if (ent.off) ent.off[0] = 0;
            memset(cnt, 0, (n + 1) * sizeof(uint64_t));
            for (uint32_t w = 0; w < n; w++) dec[w] = -1;
            rc = PF_OK;
            for (uint32_t w = 0; w < n && !rc; w++) {
                if (A->win_rec_off[w + 1] - A->win_rec_off[w] > PF_MAX_WIN_RECS) {
                    fprintf(stderr, "[W::pomfret_amd] %s:%u-%u: %u records exceed the device limit of %u reads "
                            "per window; left undecided\n", p->gaps->names[J->contig], A->win_start[w],
                            A->win_end[w], A->win_rec_off[w + 1] - A->win_rec_off[w], PF_MAX_WIN_RECS);
                    n_limit++;
                    continue;
                }
                const uint32_t one = w;
                rc = run_windows(p, ctx, J, f->recs, &one, 1, dec, &ent, cnt);
                if (rc == PF_ERR_LIMIT) {
                    fprintf(stderr, "[W::pomfret_amd] %s:%u-%u exceeds a device limit; left undecided\n",
                            p->gaps->names[J->contig], A->win_start[w], A->win_end[w]);
                    dec[w] = -1;
                    cnt[w] = 0;
                    n_limit++;
                    rc = PF_OK;
                }
            }
        }
    }
    if (!rc) {
        toff[0] = 0;
        for (uint32_t w = 0; w < n; w++) toff[w + 1] = toff[w] + cnt[w];
        static const uint64_t zero = 0;
        rc = job_store(J, n, dec, toff, ent.n, ent.off ? ent.off : &zero, ent.names, ent.hp, n_limit);
    }
    ent_free(&ent);
    free(dec); free(cnt); free(toff); free(sel);
    return rc;
}

/* one job through the device fetch (pf_batch_upload_bam): the host plans the
 * fetch from the BAI and reads compressed blocks, the device inflates,
 * selects and gathers the windows' records; a window over the record limit
 * stays undecided (as job_device), a batch the device refuses for another
 * limit goes through the host path window by window */
static int job_device_fetch(pf_mp_plan_t *p, pf_ctx_t *ctx, pf_bam_t *bam, job_t *J) {
    const uint32_t n = J->w1 - J->w0;
    if (p->tid[J->contig] < 0 || !n) {
        fetch_t f = {NULL, PF_OK};
        return job_device(p, ctx, J, &f);
    }
    const pf_cfg_t *cf = &p->cfg[J->contig];
    pf_load_cfg_t lc = p->o.load;
    pf_dbatch_t *db = NULL;
    pf_bam_dev_fetch_t *F = NULL;
    int rc = pf_batch_upload_bam(ctx, cf, &lc, bam, p->gaps->names[J->contig], n, p->win_start + J->w0,
                                 p->win_end + J->w0, PF_READBACK, PF_MAX_WIN_RECS, &db, &F);
    if (!rc) st_fetch(p, 0, F, 0.0);
    if (rc == PF_ERR_LIMIT) {                   /* per window on the host path */
        fetch_t f;
        rc = job_fetch(p, bam, J, &f);
        if (!rc) rc = job_device(p, ctx, J, &f);
        if (f.recs) pf_bam_records_free(f.recs);
        return rc;
    }
    if (rc) return rc;
    const uint64_t NR = F->n_recs;
    int8_t *dec = (int8_t *)malloc(n);
    uint64_t *cnt = (uint64_t *)calloc(n + 1, sizeof(uint64_t));
    uint32_t *rec_of = (uint32_t *)malloc((NR ? NR : 1) * sizeof(uint32_t));
    uint8_t *rhp = (uint8_t *)malloc(NR ? NR : 1);
    uint8_t *hp = NULL;
    entlist_t ent = {0};
    uint32_t n_limit = 0;
    if (!dec || !cnt || !rec_of || !rhp) rc = PF_ERR_NOMEM;
    for (uint32_t w = 0; w < n && !rc; w++) {
        dec[w] = -1;
        if (F->win_n_fetched[w] > PF_MAX_WIN_RECS) {
            fprintf(stderr, "[W::pomfret_amd] %s:%u-%u: %u records exceed the device limit of %u reads per window; "
                    "left undecided\n", p->gaps->names[J->contig], p->win_start[J->w0 + w], p->win_end[J->w0 + w],
                    F->win_n_fetched[w], PF_MAX_WIN_RECS);
            n_limit++;
        }
    }
    if (!rc && p->o.untagged && NR) {           /* the -u table replaces HP (1114-1122) */
        hp = (uint8_t *)malloc(NR);
        if (!hp) rc = PF_ERR_NOMEM;
        if (!rc) {
            const int64_t g = pf_tags_get(p->raw, (uint32_t)NR, F->qname_off, F->qname, 254, hp);
            if (g < 0) rc = (int)g;
        }
        if (!rc) rc = pf_batch_set_hp(db, hp, (uint32_t)NR);
    }
    if (!rc) {
        pf_window_out_t o;
        memset(&o, 0, sizeof o);
        o.decision = dec;
        o.read_hp = rhp;
        const double t0 = now_s();
        rc = pf_methphase_run(ctx, db, &o);
        st_fetch(p, 0, NULL, (now_s() - t0) * 1e3);
    }
    uint32_t R_ = 0;
    if (!rc) {
        R_ = pf_batch_n_reads(db);
        if (R_ > NR) rc = PF_ERR_INTERNAL;
    }
    if (!rc && R_) rc = pf_batch_read_recs(db, rec_of, (uint32_t)(NR ? NR : 1));
    if (!rc) {
        uint32_t i = 0;
        for (uint32_t w = 0; w < n && !rc; w++) {
            if (F->win_n_fetched[w] > PF_MAX_WIN_RECS) dec[w] = -1;
            const uint32_t rend = F->win_rec_off[w + 1];
            const uint64_t e0 = ent.n;
            for (; i < R_ && rec_of[i] < rend; i++) {
                if (dec[w] < 0 || p->o.mode == PF_MODE_REPORT) continue;
                const uint32_t rec = rec_of[i];
                rc = ent_push(&ent, F->qname + F->qname_off[rec], (size_t)(F->qname_off[rec + 1] - F->qname_off[rec]),
                              rhp[i]);
                if (rc) break;
            }
            cnt[w] = ent.n - e0;
        }
    }
    if (!rc) {
        uint64_t *toff = (uint64_t *)calloc(n + 1, sizeof(uint64_t));
        if (!toff) rc = PF_ERR_NOMEM;
        if (!rc) {
            for (uint32_t w = 0; w < n; w++) toff[w + 1] = toff[w] + cnt[w];
            static const uint64_t zero = 0;
            rc = job_store(J, n, dec, toff, ent.n, ent.off ? ent.off : &zero, ent.names, ent.hp, n_limit);
        }
        free(toff);
    }
    ent_free(&ent);
    pf_batch_free(db);
    pf_bam_dev_fetch_free(F);
    free(dec); free(cnt); free(rec_of); free(rhp); free(hp);
    return rc;
}

int pf_mp_run_job(pf_mp_plan_t *p, pf_ctx_t *ctx, uint32_t j) {
    job_t *J = job_of(p, PF_JOB_WINDOWS, j);
    if (!J || !ctx) return PF_ERR_ARG;
    if (p->o.untagged && !p->raw_merged) return PF_ERR_ARG;
    pf_bam_t *bam = NULL;
    int rc = pf_bam_open(p->bam_path, NULL, &bam);
    if (rc) return rc;
    if (!p->o.host_fetch) {
        rc = job_device_fetch(p, ctx, bam, J);
        pf_bam_close(bam);
        return rc;
    }
    fetch_t f;
    rc = job_fetch(p, bam, J, &f);
    if (!rc) rc = job_device(p, ctx, J, &f);
    if (f.recs) pf_bam_records_free(f.recs);
    pf_bam_close(bam);
    return rc;
}

/* ------------------------------------------------------------------ */
/* finish: merge, blocks, outputs                                       */

static int write_report(pf_mp_plan_t *p) {
    char *fn = (char *)malloc(strlen(p->out_prefix) + 32);
    if (!fn) return PF_ERR_NOMEM;
    sprintf(fn, "%s.report.tsv", p->out_prefix);
    FILE *fo = fopen(fn, "w");
    free(fn);
    if (!fo) return -1;
    float n_switch = 0, n_fail = 0, n_correct = 0;    /* main_methreport's counters (4962-4965) */
    int tot = 0;
    for (uint32_t c = 0; c < p->n_contigs; c++) {
        for (uint64_t w = p->win_off[c]; w < p->win_off[c + 1]; w++) {
            const int start = (int)p->win_start[w], end = (int)p->win_end[w];
            fprintf(fo, "%s\t%d\t%d\t", p->gaps->names[c], start, end);
            const int d = p->decision[w];
            if (d == 0) { n_correct++; fprintf(fo, "correct\n"); }
            else if (d == 1) { n_switch++; fprintf(fo, "switch\n"); }
            else { n_fail++; fprintf(fo, "fail\n"); }
            tot++;
            if (tot % 100 == 0)
                fprintf(stdout, "Parsed N=%d regions, currently at %s:%d-%d, correct/(correct+switch)=%.2f%%, "
                        "correct/N=%.2f%%\n", tot, p->gaps->names[c], start, end,
                        n_correct / (n_correct + n_switch) * 100.0, n_correct / (float)tot * 100.0);
        }
    }
    fprintf(stdout, "Total N=%d regions, correct/(correct+switch)=%.2f%%, correct/N=%.2f%%\n",
            tot, n_correct / (n_correct + n_switch) * 100.0, n_correct / (float)tot * 100.0);
    fprintf(stderr, "[M::%s] Total N=%d regions, correct/(correct+switch)=%.2f%%, correct/N=%.2f%%\n",
            "main_methreport", tot, n_correct / (n_correct + n_switch) * 100.0, n_correct / (float)tot * 100.0);
    fflush(stdout);
    p->report_counts[0] = n_correct; p->report_counts[1] = n_switch; p->report_counts[2] = n_fail;
    return fclose(fo) ? -1 : PF_OK;
}

/* the output BAM's compression threads: -T, else -t (cli.c:261-264) */
static int bam_threads(const pf_methphase_opts_t *o) {
    return o->bam_threads > 0 ? o->bam_threads : o->threads > 0 ? o->threads : 1;
}

/* the rescue of dropped-interval sites (recover_variant_phase_in_dropped_intervals)
 * and {prefix}.mp.vcf: only with --vcf (4706-4712) */
static int write_rescued_vcf(pf_mp_plan_t *p, char *fn, size_t L, int trace, double tw) {
    int rc = 0;
#define WTRACE(what) do { if (trace) { const double t_ = now_s(); fprintf(stderr, "[writers] %s %.3fs\n", what, t_ - tw); tw = t_; } } while (0)
    const uint32_t C = p->n_contigs;
    uint64_t *roff = (uint64_t *)calloc(C + 1, sizeof(uint64_t));
    uint32_t *rpos = NULL;
    uint8_t *rhap = NULL;
    uint64_t rn = 0, rcap = 0;
    pf_bam_t *bam = NULL;
    pf_qname_tags_t tm, tr;
    if (!rc && !roff) rc = PF_ERR_NOMEM;
    if (!rc) rc = pf_tags_view(p->qname_hp, &tm);
    if (!rc && p->o.untagged) rc = pf_tags_view(p->raw, &tr);
    /* every contig with dropped intervals at once: one work queue of
     * (contig, interval) items on the run's host threads */
    const pf_gaps_t *g = p->gaps;
    uint32_t nr = 0;
    const char **rn_names = (const char **)calloc(C ? C : 1, sizeof(char *));
    uint32_t *rn_nd = (uint32_t *)calloc(C ? C : 1, sizeof(uint32_t)), *rn_c = (uint32_t *)calloc(C ? C : 1, 4);
    const uint32_t **rn_ds = (const uint32_t **)calloc(C ? C : 1, sizeof(uint32_t *));
    const uint32_t **rn_de = (const uint32_t **)calloc(C ? C : 1, sizeof(uint32_t *));
    pf_known_table_t **kts = (pf_known_table_t **)calloc(C ? C : 1, sizeof(pf_known_table_t *));
    const pf_known_vars_t **kvs = (const pf_known_vars_t **)calloc(C ? C : 1, sizeof(pf_known_vars_t *));
    pf_rescue_map_t **maps = (pf_rescue_map_t **)calloc(C ? C : 1, sizeof(pf_rescue_map_t *));
    if (!rc && (!rn_names || !rn_nd || !rn_c || !rn_ds || !rn_de || !kts || !kvs || !maps)) rc = PF_ERR_NOMEM;
    /* one pass over the VCF for every contig's known table, with the
     * reference's attribution of lines to the phase-block file's contigs */
    pf_known_table_t **kall = NULL;
    int need = 0;
    for (uint32_t c = 0; c < C; c++) need |= g->drop_off[c + 1] > g->drop_off[c] && p->tid[c] >= 0;
    if (!rc && need) {
        kall = (pf_known_table_t **)calloc(C, sizeof(pf_known_table_t *));
        rc = kall ? pf_vcf_known_vars_multi(p->vcf_path, C, (const char *const *)g->names, kall) : PF_ERR_NOMEM;
    }
    for (uint32_t c = 0; c < C && !rc && need; c++) {
        const uint64_t nd = g->drop_off[c + 1] - g->drop_off[c];
        if (!nd || p->tid[c] < 0) continue;
        kts[nr] = kall[c];
        kall[c] = NULL;
        rn_names[nr] = g->names[c]; rn_nd[nr] = (uint32_t)nd; rn_c[nr] = c;
        rn_ds[nr] = g->drop_start + g->drop_off[c]; rn_de[nr] = g->drop_end + g->drop_off[c];
        kvs[nr] = &kts[nr]->vars;
        nr++;
    }
    for (uint32_t c = 0; kall && c < C; c++) pf_known_table_free(kall[c]);
    free(kall);
    WTRACE("known-variant tables");
    if (!rc && nr) rc = pf_bam_open(p->bam_path, NULL, &bam);
    if (!rc && nr)
        rc = pf_rescue_dropped_multi(bam, nr, rn_names, rn_nd, rn_ds, rn_de, kvs, &tm, p->o.untagged ? &tr : NULL,
                                     p->o.threads > 0 ? p->o.threads : 1, maps);
    for (uint32_t c = 0, i = 0; c < C && !rc; c++) {
        roff[c + 1] = rn;
        if (i >= nr || rn_c[i] != c) continue;
        const pf_rescue_map_t *m = maps[i++];
        if (!m->n) continue;
        if (rn + m->n > rcap) {
            while (rcap < rn + m->n) rcap = rcap ? 2 * rcap : 1024;
            uint32_t *a = (uint32_t *)realloc(rpos, rcap * sizeof(uint32_t));
            uint8_t *b = a ? (uint8_t *)realloc(rhap, rcap) : NULL;
            if (a) rpos = a;
            if (!a || !b) { rc = PF_ERR_NOMEM; break; }
            rhap = b;
        }
        memcpy(rpos + rn, m->pos, m->n * sizeof(uint32_t));
        memcpy(rhap + rn, m->hap_of_ref, m->n);
        rn += m->n;
        roff[c + 1] = rn;
    }
    for (uint32_t i = 0; i < nr; i++) {
        if (maps && maps[i]) pf_rescue_map_free(maps[i]);
        if (kts && kts[i]) pf_known_table_free(kts[i]);
    }
    free(rn_names); free(rn_nd); free(rn_c); free(rn_ds); free(rn_de); free(kts); free(kvs); free(maps);
    if (bam) pf_bam_close(bam);
    WTRACE("rescue (dropped intervals)");
    if (!rc) {
        pf_rescue_t res = {roff, rpos ? rpos : (const uint32_t *)roff, rhap ? rhap : (const uint8_t *)roff};
        snprintf(fn, L, "%s.mp.vcf", p->out_prefix);
        if (p->o.verbose >= 0) fprintf(stderr, "[M::main_blockjoin] writing vcf...\n");
        rc = pf_write_vcf(p->vcf_path, p->gaps, p->blocks, &res, fn, NULL);
        if (!rc && p->o.verbose >= 0) fprintf(stderr, "[M::main_blockjoin] vcf written.\n");
        WTRACE("vcf");
    }
    free(roff); free(rpos); free(rhap);
    return rc;
#undef WTRACE
}

static int write_methphase_outputs(pf_mp_plan_t *p) {
    const size_t L = strlen(p->out_prefix) + 32;
    char *fn = (char *)malloc(L);
    if (!fn) return PF_ERR_NOMEM;
    /* PF_MP_TRACE: the writers' steps on stderr (seconds) */
    const int trace = getenv("PF_MP_TRACE") != NULL;
    double tw = now_s();
#define WTRACE(what) do { if (trace) { const double t_ = now_s(); fprintf(stderr, "[writers] %s %.3fs\n", what, t_ - tw); tw = t_; } } while (0)
    snprintf(fn, L, "%s.mp.gtf", p->out_prefix);
    int rc = pf_write_gtf(p->gaps, p->blocks, fn);
    if (!rc && p->o.verbose >= 0) fprintf(stderr, "[M::main_blockjoin] gtf written.\n");
    if (!rc && p->o.write_tsv) {
        snprintf(fn, L, "%s.mp.tsv", p->out_prefix);
        rc = pf_write_tsv(p->gaps, p->blocks, fn);
        if (!rc && p->o.verbose >= 0) fprintf(stderr, "[M::main_blockjoin] tsv written.\n");
    }
    /* -U: {prefix}.mp.input_haptag.tsv (4494-4517), every record of the BAM */
    if (!rc && p->o.untagged && p->o.write_input_tagging) {
        snprintf(fn, L, "%s.mp.input_haptag.tsv", p->out_prefix);
        rc = pf_retag_bam(p->bam_path, NULL, NULL, fn, PF_RETAG_INPUT_HAPTAG, NULL, NULL, NULL, p->raw, -1, NULL);
    }
    WTRACE("gtf/tsv/input_haptag");
    /* the VCF only when --vcf was given (4706); the BAM whenever --write-bam
     * was (4714-4731), with or without a VCF */
    if (!rc && p->vcf_path) rc = write_rescued_vcf(p, fn, L, trace, tw);
    if (!rc && p->o.write_bam) {                    /* output_modify_bam + sam_index_build3 (4719-4731) */
        char *fb = (char *)malloc(L + 8);
        if (!fb) rc = PF_ERR_NOMEM;
        if (!rc) {
            snprintf(fn, L, "%s.mp.bam", p->out_prefix);
            snprintf(fb, L + 8, "%s.mp.bam.bai", p->out_prefix);
            rc = pf_retag_bam_threads(p->bam_path, fn, fb, NULL, PF_RETAG_METHPHASE, p->gaps, p->blocks, p->qname_hp,
                                      p->o.untagged ? p->raw : NULL, -1, bam_threads(&p->o), NULL);
            if (!rc && p->o.verbose >= 0) fprintf(stderr, "[M::main_blockjoin] bam written and indexed.\n");
        }
        free(fb);
    }
    free(fn);
    return rc;
#undef WTRACE
}

/* varhaptag (main_varhaptag, 4737-4836): the -u pre-pass on the devices,
 * then {out}.varhaptag.tsv and, with write_bam, the retagged {out} + .bai */
static int varhaptag_outputs(pf_mp_plan_t *p) {
    const size_t L = strlen(p->out_prefix) + 32;
    char *ft = (char *)malloc(L), *fb = (char *)malloc(L);
    int rc = (!ft || !fb) ? PF_ERR_NOMEM : 0;
    if (!rc) {
        snprintf(ft, L, "%s.varhaptag.tsv", p->out_prefix);
        snprintf(fb, L, "%s.bai", p->out_prefix);
        rc = pf_retag_bam_threads(p->bam_path, p->o.write_bam ? p->out_prefix : NULL, p->o.write_bam ? fb : NULL, ft,
                                  PF_RETAG_VARHAPTAG, NULL, NULL, NULL, p->raw, -1, bam_threads(&p->o), NULL);
    }
    free(ft); free(fb);
    return rc;
}

int pf_mp_finish(pf_mp_plan_t *p) {
    if (!p) return PF_ERR_ARG;
    if (p->finished) return PF_OK;
    const double t0 = now_s();
    free(p->decision);
    p->decision = (int8_t *)malloc(p->n_windows ? p->n_windows : 1);
    if (!p->decision) return PF_ERR_NOMEM;
    for (uint32_t w = 0; w < p->n_windows; w++) p->decision[w] = -1;
    p->n_limit = 0;
    /* jobs are runs of consecutive windows: visiting them by w0 visits the
     * windows in (contig, window) order, the order in which the reference's
     * per-contig tables fill (4396-4423) and then merge (4579-4595) */
    uint32_t *by_w0 = (uint32_t *)malloc((p->n_jobs ? p->n_jobs : 1) * sizeof(uint32_t));
    if (!by_w0) return PF_ERR_NOMEM;
    for (uint32_t j = 0; j < p->n_jobs; j++) by_w0[j] = j;
    for (uint32_t a = 1; a < p->n_jobs; a++) {            /* already sorted by construction */
        uint32_t x = by_w0[a], b = a;
        while (b > 0 && p->jobs[by_w0[b - 1]].w0 > p->jobs[x].w0) { by_w0[b] = by_w0[b - 1]; b--; }
        by_w0[b] = x;
    }
    int rc = PF_OK;
    for (uint32_t k = 0; k < p->n_jobs && !rc; k++) {
        const job_t *J = &p->jobs[by_w0[k]];
        if (!J->done) { rc = PF_ERR_ARG; break; }
        p->n_limit += J->n_limit;
        for (uint32_t w = J->w0; w < J->w1 && !rc; w++) {
            const uint32_t i = w - J->w0;
            p->decision[w] = J->dec[i];
            if (J->dec[i] < 0 || p->o.mode == PF_MODE_REPORT) continue;
            for (uint64_t e = J->tag_off[i]; e < J->tag_off[i + 1]; e++) {
                const int r = tags_put(p->qname_hp, J->names + J->name_off[e],
                                       (size_t)(J->name_off[e + 1] - J->name_off[e]), J->hp[e]);
                if (r < 0) { rc = r; break; }
            }
        }
    }
    free(by_w0);
    if (rc) return rc;
    if (p->o.mode == PF_MODE_REPORT) {
        if (p->out_prefix) rc = write_report(p);
    } else {
        rc = pf_phase_blocks(p->gaps, p->decision, &p->blocks);
        if (!rc && p->out_prefix) rc = write_methphase_outputs(p);
    }
    if (!rc) p->finished = 1;
    p->st.s_finish += now_s() - t0;
    return rc;
}

int pf_mp_report_counts(const pf_mp_plan_t *p, double *counts3) {
    if (!p || !counts3 || !p->finished) return PF_ERR_ARG;
    memcpy(counts3, p->report_counts, sizeof p->report_counts);
    return PF_OK;
}

/* The deferred coverage estimate (-u without -c, one process): the serial
 * pass's per-contig values from the -u pre-pass's fetches, the contigs the
 * pre-pass did not fetch (no variants) estimated on their own when a needed
 * contig comes after them, and the pass's quirks kept (a truncated record
 * zeroes every later contig; unplaced reads at the end zero the last contig
 * with reads; an index without n_no_coor: the serial host pass); then each
 * contig's parameters (4357-4390). */
static int finish_deferred_estimate(pf_mp_plan_t *p, pf_ctx_t *ctx) {
    if (!p->est_deferred) return PF_OK;
    const double t0 = now_s();
    pf_bam_t *bam = NULL;
    int rc = pf_bam_open(p->bam_path, NULL, &bam);
    if (rc) return rc;
    const int32_t nt = pf_bam_n_targets(bam);
    int32_t *covs = (int32_t *)calloc(nt > 0 ? nt : 1, sizeof(int32_t));
    int32_t *trunc = (int32_t *)calloc(nt > 0 ? nt : 1, sizeof(int32_t));
    uint8_t *have = (uint8_t *)calloc(nt > 0 ? nt : 1, 1);
    if (!covs || !trunc || !have) rc = PF_ERR_NOMEM;
    int32_t maxneed = -1;
    for (uint32_t c = 0; c < p->n_contigs && !rc; c++) {
        const int32_t t = p->tid[c];
        if (t < 0 || t >= nt) continue;
        if (p->uhave[c]) { covs[t] = p->ucov[c]; trunc[t] = p->utrunc[c]; have[t] = 1; }
        if (p->win_off[c + 1] > p->win_off[c] && t > maxneed) maxneed = t;
    }
    const int64_t n_unplaced = rc ? 0 : pf_bam_n_no_coor(bam);
    if (!rc && n_unplaced < 0) {
        rc = pf_bam_estimate_coverage(bam, covs, nt > 0 ? nt : 1);        /* as pf_bam_estimate_coverage_dev does */
    } else if (!rc) {
        int32_t last = -1;
        int stopped = 0;
        for (int32_t t = 0; t < nt && !rc; t++) {
            if (stopped) { covs[t] = 0; continue; }
            const int64_t nc = pf_bam_query_chunks(bam, t, 0, INT64_MAX, NULL, 0);
            if (nc < 0) { rc = (int)nc; break; }
            if (nc == 0) { covs[t] = 0; continue; }
            last = t;
            if (!have[t]) {
                if (t > maxneed) continue;                 /* neither used nor ahead of a contig that is */
                rc = pf_bam_estimate_contig_dev(ctx, bam, t, &covs[t], &trunc[t]);
            }
            if (trunc[t]) stopped = 1;
        }
        if (!rc && !stopped && n_unplaced > 0 && last >= 0) covs[last] = 0;
    }
    for (uint32_t c = 0; c < p->n_contigs && !rc; c++) {
        const int32_t t = p->tid[c];
        methphase_cfg(&p->cfg[c], &p->o, (t >= 0 && t < nt) ? covs[t] : 0);
    }
    free(covs); free(trunc); free(have);
    pf_bam_close(bam);
    p->st.s_estimate += now_s() - t0;
    return rc;
}

/* ------------------------------------------------------------------ */
/* in-process driver: one host thread per device                        */

/* Job queues of a run: one per affinity group (a device, or with
 * PF_FETCH_CACHE_SCOPE=ctx a context) holding the window jobs whose contig's
 * -u arena that group kept, plus a shared queue (the other jobs, and every job
 * of a run without kept arenas).  A worker takes from its group's queue,
 * then from the shared one, then steals from the other groups' (the jobs of
 * each queue in the plan's heaviest-first order). */
typedef struct {
    int n_groups;              /* affinity groups; queue n_groups is the shared one */
    uint32_t *list;            /* the jobs, queue by queue */
    uint32_t *off;             /* [n_groups + 2] */
    atomic_uint *pos;          /* [n_groups + 1] next index of each queue */
    int steal;                 /* 0: a worker never takes another group's jobs (PF_JOB_STEAL=0, tests) */
} jobq_t;

typedef struct {
    pf_mp_plan_t *p;
    pf_ctx_t *ctx;
    int device;
    int own_ctx;
    int kind;
    jobq_t *q;
    int group;                 /* its affinity group (-1: none) */
    int rc;
} dev_worker_t;

/* the worker's next job: 1 and *job, or 0 when every queue is drained */
static int next_job(dev_worker_t *W, uint32_t *job) {
    jobq_t *q = W->q;
    const int G = q->n_groups;
    for (int k = -1; k <= G; k++) {
        /* own group first, then the shared queue, then the others in turn */
        int g = k < 0 ? W->group : k == 0 ? G : (W->group + k) % (G > 0 ? G : 1);
        if (g < 0 || (k > 0 && (g == W->group || G == 0 || !q->steal))) continue;
        const uint32_t n = q->off[g + 1] - q->off[g];
        if (atomic_load(&q->pos[g]) >= n) continue;
        const uint32_t i = atomic_fetch_add(&q->pos[g], 1);
        if (i >= n) continue;
        *job = q->list[q->off[g] + i];
        if (k > 0) {
            pthread_mutex_lock(&W->p->st_mu);
            W->p->st.steals++;
            pthread_mutex_unlock(&W->p->st_mu);
        }
        return 1;
    }
    return 0;
}

typedef struct {
    const pf_mp_plan_t *p;
    pf_bam_t *bam;
    const job_t *J;
    fetch_t f;
} prefetch_t;

static void *prefetch_main(void *arg) {
    prefetch_t *a = (prefetch_t *)arg;
    job_fetch(a->p, a->bam, a->J, &a->f);
    return NULL;
}

static void *dev_main(void *arg) {
    dev_worker_t *W = (dev_worker_t *)arg;
    pf_mp_plan_t *p = W->p;
    int rc = PF_OK;
    if (!W->ctx) {
        rc = pf_ctx_create(W->device, &W->ctx);
        W->own_ctx = 1;
        if (rc) { W->rc = rc; return NULL; }
    }
    uint32_t jb;
    if (W->kind == PF_JOB_HAPTAG) {
        while (!rc && next_job(W, &jb)) rc = pf_mp_run_haptag_job(p, W->ctx, jb);
        W->rc = rc;
        return NULL;
    }
    /* window jobs: the fetch of the next job runs on a helper thread while
     * this thread drives the device on the current one */
    pf_bam_t *bam[2] = {NULL, NULL};
    rc = pf_bam_open(p->bam_path, NULL, &bam[0]);
    if (!rc) rc = pf_bam_open(p->bam_path, NULL, &bam[1]);
    if (!rc && !p->o.host_fetch) {              /* device fetch: host planning + reads, the rest on the GPU */
        while (!rc && next_job(W, &jb)) rc = job_device_fetch(p, W->ctx, bam[0], &p->jobs[jb]);
        pf_bam_close(bam[0]);
        pf_bam_close(bam[1]);
        W->rc = rc;
        return NULL;
    }
    prefetch_t cur, nxt;
    memset(&cur, 0, sizeof cur);
    memset(&nxt, 0, sizeof nxt);
    int have = 0, slot = 0;
    if (!rc && next_job(W, &jb)) {
        cur.p = p; cur.bam = bam[slot]; cur.J = &p->jobs[jb];
        job_fetch(p, cur.bam, cur.J, &cur.f);
        have = 1;
    }
    while (have && !rc) {
        pthread_t th;
        int spawned = 0;
        const int more = next_job(W, &jb);
        if (more) {
            nxt.p = p; nxt.bam = bam[slot ^ 1]; nxt.J = &p->jobs[jb];
            nxt.f.recs = NULL; nxt.f.rc = 0;
            spawned = pthread_create(&th, NULL, prefetch_main, &nxt) == 0;
            if (!spawned) job_fetch(p, nxt.bam, nxt.J, &nxt.f);
        }
        rc = job_device(p, W->ctx, (job_t *)cur.J, &cur.f);
        if (cur.f.recs) pf_bam_records_free(cur.f.recs);
        cur.f.recs = NULL;
        if (spawned) pthread_join(th, NULL);
        if (more) { cur = nxt; slot ^= 1; }
        else have = 0;
    }
    if (have && cur.f.recs) pf_bam_records_free(cur.f.recs);
    if (bam[0]) pf_bam_close(bam[0]);
    if (bam[1]) pf_bam_close(bam[1]);
    W->rc = rc;
    return NULL;
}

static int run_on_devices_(pf_mp_plan_t *p, const pf_methphase_opts_t *o, int kind);
static int run_on_devices(pf_mp_plan_t *p, const pf_methphase_opts_t *o, int kind) {
    const double t0 = now_s();
    const int rc = run_on_devices_(p, o, kind);
    *(kind == PF_JOB_HAPTAG ? &p->st.s_haptag : &p->st.s_windows) += now_s() - t0;
    return rc;
}

static int run_on_devices_(pf_mp_plan_t *p, const pf_methphase_opts_t *o, int kind) {
    const uint32_t n = kind == PF_JOB_HAPTAG ? p->n_ujobs : p->n_jobs;
    const uint32_t *ord = kind == PF_JOB_HAPTAG ? p->uorder : p->order;
    const job_t *J = kind == PF_JOB_HAPTAG ? p->ujobs : p->jobs;
    uint32_t *todo = (uint32_t *)malloc((n ? n : 1) * sizeof(uint32_t));
    if (!todo) return PF_ERR_NOMEM;
    uint32_t nt = 0;
    for (uint32_t i = 0; i < n; i++)
        if (o->world <= 1 || J[ord[i]].rank == o->rank) todo[nt++] = ord[i];
    int nd = o->n_ctxs > 0 ? o->n_ctxs : (o->n_devices > 0 ? o->n_devices : pf_device_count());
    if (nd <= 0) { free(todo); return PF_ERR_HIP; }
    dev_worker_t *W = (dev_worker_t *)calloc(nd, sizeof(dev_worker_t));
    pthread_t *th = (pthread_t *)calloc(nd, sizeof(pthread_t));
    /* affinity groups: window jobs of a run that kept the -u arenas go to the
     * device (or context) holding their contig's arena */
    jobq_t q;
    memset(&q, 0, sizeof q);
    int *gid = (int *)malloc(sizeof(int) * (size_t)nd);
    int *home = (int *)malloc(sizeof(int) * (size_t)(nt ? nt : 1));
    q.list = (uint32_t *)malloc(sizeof(uint32_t) * (nt ? nt : 1));
    q.off = (uint32_t *)calloc((size_t)nd + 2, sizeof(uint32_t));
    q.pos = (atomic_uint *)calloc((size_t)nd + 1, sizeof(atomic_uint));
    int rc = (!W || !th || !gid || !home || !q.list || !q.off || !q.pos) ? PF_ERR_NOMEM : PF_OK;
    const int affine = !rc && kind == PF_JOB_WINDOWS && p->keeps_arenas && o->n_ctxs > 0;
    {
        const char *e = getenv("PF_JOB_STEAL");
        q.steal = !(e && !strcmp(e, "0"));
    }
    for (int d = 0; d < nd && !rc; d++) {
        gid[d] = -1;
        if (!affine) continue;
        const int by_ctx = pf_fetch_cache_scope_ctx();
        for (int e = 0; e < d && gid[d] < 0; e++)
            if (!by_ctx && pf_ctx_device(o->ctxs[e]) == pf_ctx_device(o->ctxs[d])) gid[d] = gid[e];
        if (gid[d] < 0) gid[d] = q.n_groups++;
    }
    for (uint32_t i = 0; i < nt && !rc; i++) {
        home[i] = q.n_groups;                       /* the shared queue */
        if (affine) {
            const job_t *Jt = &J[todo[i]];
            const int h = pf_fetch_cache_home_range(o->ctxs, nd, p->bam_path, p->tid[Jt->contig], Jt->lo, Jt->hi);
            if (h >= 0) home[i] = gid[h];
        }
        q.off[home[i] + 1]++;
    }
    for (int g = 0; g <= q.n_groups && !rc; g++) q.off[g + 1] += q.off[g];
    if (!rc) {
        uint32_t *fill = (uint32_t *)calloc((size_t)q.n_groups + 1, sizeof(uint32_t));
        if (!fill) rc = PF_ERR_NOMEM;
        for (uint32_t i = 0; i < nt && !rc; i++) q.list[q.off[home[i]] + fill[home[i]]++] = todo[i];
        free(fill);
        for (int g = 0; g <= q.n_groups; g++) atomic_init(&q.pos[g], 0);
    }
    for (int d = 0; d < nd && !rc; d++) {
        W[d].p = p; W[d].kind = kind; W[d].q = &q; W[d].group = gid[d];
        W[d].ctx = o->n_ctxs > 0 ? o->ctxs[d] : NULL;
        W[d].device = o->devices ? o->devices[d] : d;
    }
    if (!rc && nd == 1) {
        dev_main(&W[0]);
    } else if (!rc) {
        for (int d = 0; d < nd; d++)
            if (pthread_create(&th[d], NULL, dev_main, &W[d])) { W[d].rc = PF_ERR_INTERNAL; th[d] = 0; }
        for (int d = 0; d < nd; d++) if (th[d]) pthread_join(th[d], NULL);
    }
    for (int d = 0; d < nd && W; d++) {
        if (!rc && W[d].rc) rc = W[d].rc;
        if (W[d].own_ctx && W[d].ctx) pf_ctx_destroy(W[d].ctx);
    }
    free(W); free(th); free(todo);
    free(gid); free(home); free(q.list); free(q.off); free((void *)q.pos);
    return rc;
}

int pf_mp_run_mine(pf_mp_plan_t *p, const pf_methphase_opts_t *run_opts, int kind) {
    if (!p || !run_opts) return PF_ERR_ARG;
    if (kind == PF_JOB_WINDOWS && p->o.untagged && !p->raw_merged) return PF_ERR_ARG;
    return run_on_devices(p, run_opts, kind);
}

static int methphase_main_(const pf_methphase_opts_t *o, pf_mp_plan_t **out);
void pf_fetch_cache_enable(pf_ctx_t *ctx, int on);   /* pf_ingest.hip */
int pf_ctx_device(const pf_ctx_t *ctx);              /* pf_api.hip */

/* the leading contexts of `ctxs` that are on distinct devices (the driver
 * lists its contexts device-major: one per GPU, then the second per GPU) */
static int distinct_device_prefix(pf_ctx_t *const *ctxs, int n) {
    int k = 0;
    for (; k < n; k++) {
        const int dev = pf_ctx_device(ctxs[k]);
        int seen = 0;
        for (int j = 0; j < k && !seen; j++) seen = pf_ctx_device(ctxs[j]) == dev;
        if (seen) break;
    }
    return k > 0 ? k : 1;
}

/* one set of contexts for the whole run (coverage pass, -u pre-pass, window
 * jobs): a context's streams, pinned staging and kernels are set up once, not
 * once per phase */
int pf_methphase_main(const pf_methphase_opts_t *o, pf_mp_plan_t **out) {
    if (!o || !out) return PF_ERR_ARG;
    *out = NULL;
    if (o->world > 1) return PF_ERR_ARG;           /* multi-process runs use the pf_mp_* steps */
    const int ng = o->n_ctxs > 0 ? 0 : (o->n_devices > 0 ? o->n_devices : pf_device_count());
    if (ng <= 0) return methphase_main_(o, out);
    /* PF_DEV_CONTEXTS contexts per GPU (default 2, at most 4), each on its own
     * host thread over the shared job queue: one job's K0/K12 fill the CUs
     * another job's K3 tail leaves idle (bench.py --split: 18.5 -> 17.0 ms on
     * the 1024-window mix).  Two contexts are four streams, the box's
     * GPU_MAX_HW_QUEUES; more would share hardware queues (4: 25 ms). */
    int per = 2;
    const char *e = getenv("PF_DEV_CONTEXTS");
    if (e && *e) per = atoi(e);
    if (per < 1) per = 1;
    if (per > 4) per = 4;
    const int nd = ng * per;
    pf_ctx_t **ctxs = (pf_ctx_t **)calloc((size_t)nd, sizeof(pf_ctx_t *));
    if (!ctxs) return PF_ERR_NOMEM;
    int rc = PF_OK;
    /* device-major within each round, so the first jobs spread over the GPUs */
    for (int d = 0; d < nd && !rc; d++) rc = pf_ctx_create(o->devices ? o->devices[d % ng] : d % ng, &ctxs[d]);
    if (!rc) {
        pf_methphase_opts_t oo = *o;
        oo.ctxs = ctxs;
        oo.n_ctxs = nd;
        rc = methphase_main_(&oo, out);
        if (*out) { (*out)->o.ctxs = NULL; (*out)->o.n_ctxs = 0; }
    }
    for (int d = 0; d < nd; d++) if (ctxs[d]) pf_ctx_destroy(ctxs[d]);
    free(ctxs);
    return rc;
}

static int methphase_main_(const pf_methphase_opts_t *o, pf_mp_plan_t **out) {
    if (o->mode == PF_MODE_VARHAPTAG) {
        if (!o->out_prefix) return PF_ERR_ARG;
        pf_methphase_opts_t v = *o;
        v.mode = PF_MODE_METHPHASE;
        v.untagged = 1;
        v.cov_for_selection = 1;                   /* no coverage estimate: no window runs */
        pf_mp_plan_t *p = NULL;
        int rc = pf_mp_plan(&v, &p);
        if (!rc) rc = run_on_devices(p, &v, PF_JOB_HAPTAG);
        if (!rc) rc = pf_mp_merge_raw(p);
        if (!rc) rc = varhaptag_outputs(p);
        if (rc) { pf_mp_free(p); return rc; }
        *out = p;
        return PF_OK;
    }
    pf_mp_plan_t *p = NULL;
    int rc = mp_plan(o, &p, 1);
    if (!rc && o->mode == PF_MODE_METHPHASE) {
        /* blockjoin_parallel's terminations (4450-4458, 4470-4477): counted on
         * the raw gaps, before merging */
        const pf_gaps_t *gs[2] = {o->untagged ? p->ug : NULL, p->gaps};
        for (int k = 0; k < 2 && !rc; k++) {
            if (!gs[k]) continue;
            if (gs[k]->raw_off[gs[k]->n_contigs] == 0) {
                if (k == 0)
                    fprintf(stderr, "[E::blockjoin_parallel] Nothing loaded from vcf (ref_n=%u), cannot haptag "
                                    "the input bam. Terminating.\n", gs[k]->n_contigs);
                else
                    fprintf(stderr, "[E::blockjoin_parallel] No intervals loaded, terminating.\n");
                rc = PF_ERR_ARG;
            }
        }
        if (rc) { pf_mp_free(p); p = NULL; }
    }
    /* the -u pre-pass's whole-contig arenas stay on the device for the window
     * jobs of the same context (device fetch only) */
    const int keep = !rc && o->untagged && !o->host_fetch && o->n_ctxs > 0;
    for (int d = 0; keep && d < o->n_ctxs; d++) pf_fetch_cache_enable(o->ctxs[d], 1);
    if (keep) p->keeps_arenas = 1;
    if (!rc && o->untagged) {
        /* the -u pre-pass on one context per device: its whole-contig fetches
         * are bound by the file reads, and a second context per GPU would only
         * pin a second contig-sized staging buffer (e2e_u CLI 2.1 -> 2.9 s);
         * the window jobs then run on every context and share the arenas */
        pf_methphase_opts_t ou = *o;
        if (o->n_ctxs > 1 && !pf_fetch_cache_scope_ctx()) ou.n_ctxs = distinct_device_prefix(o->ctxs, o->n_ctxs);
        rc = run_on_devices(p, &ou, PF_JOB_HAPTAG);
        if (!rc) rc = pf_mp_merge_raw(p);
    }
    if (!rc && p->est_deferred) rc = finish_deferred_estimate(p, o->ctxs[0]);
    if (!rc) rc = run_on_devices(p, o, PF_JOB_WINDOWS);
    for (int d = 0; keep && d < o->n_ctxs; d++) pf_fetch_cache_enable(o->ctxs[d], 0);
    if (!rc) rc = pf_mp_finish(p);
    if (rc) { pf_mp_free(p); return rc; }
    if (p->n_limit)
        fprintf(stderr, "[W::pomfret_amd] %u windows left undecided for exceeding a device limit\n", p->n_limit);
    *out = p;
    return PF_OK;
}
