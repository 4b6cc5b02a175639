/*
 * pomfret-amd -- command-line drop-in for `pomfret methphase` and `pomfret
 * report` (reference: main.c, cli.c parse_cli / sancheck_cliopt, and
 * blockjoin.c main_blockjoin 4643 / main_methreport 4901), running the
 * per-window hot path on the MI355X through libpomfret_amd.so.
 *
 *   pomfret-amd methphase -o out --vcf phased.vcf.gz [-c 60] [-u] [-t N] [--write-bam] [--gpus G] reads.bam
 *   pomfret-amd report    -o out --vcf phased.vcf.gz [-c C] [--chunk-size S --chunk-stride D] reads.bam
 *   pomfret-amd varhaptag -o out.bam in.vcf in.bam
 *
 * Options and defaults follow the reference's cliopt_t (cli.c:47-75) and
 * cliopt_haptag_t (cli.c:332-343); the -c arithmetic (cov/10, cov/4), the
 * order-dependent -n override and varhaptag's --write-bam (which there turns
 * the BAM output OFF, cli.c:416) are kept.  Added: --gpus G (GPUs driven by
 * this process; default all visible), --host-fetch (records inflated and
 * decoded on the host instead of the device fetch) and --job-windows W (windows per device
 * job).  Phase blocks come from --tsv, else --gtf, else --vcf (main_blockjoin
 * 4661-4666); with -u the VCF still supplies the variants and the contigs to
 * pre-haplotag.  -U writes {prefix}.mp.input_haptag.tsv (4494-4517).  --dbg's
 * {prefix}.mp.dbg.read2tag (2223-2248) lists a khash in bucket order, which
 * no other implementation reproduces: it is not written (a warning says so).
 */
#include <getopt.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <time.h>

#include "../../include/pomfret_amd.h"

static double now_s(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

static void help_main(void) {
    fprintf(stderr, "Usage: pomfret-amd <subcommand> [options]\n");
    fprintf(stderr, "Subcommands:\n");
    fprintf(stderr, "  methphase  Given aligned reads with methylation calls in bam\n");
    fprintf(stderr, "             and exiting phase blocks, try to use methylation to\n");
    fprintf(stderr, "             phase the unphased regions (on the GPU).\n");
    fprintf(stderr, "  varhaptag  Haplotag reads from phased variants (on the GPU).\n");
    fprintf(stderr, "  report     Given aligned reads in bam and a phased vcf, sample\n");
    fprintf(stderr, "             intervals within phase blocks, pretend they are phase gaps\n");
    fprintf(stderr, "             and report whether meth-phasing would generate correct \n");
    fprintf(stderr, "             phase block joining decisions.\n");
}

static void help_methphase(const char *prefix) {
    fprintf(stderr, "Usage: pomfret-amd methphase -o out_prefix --vcf phased.vcf[.gz] [...] reads.bam 2>log\n");
    fprintf(stderr, "Options:\n");
    fprintf(stderr, "  bam    [pos] Aligned reads. Must be sorted and has index. If reads are not\n");
    fprintf(stderr, "               haplotagged, supply -u and provide vcf (via --vcf).\n");
    fprintf(stderr, "  -h,--help [   ] Display this message.\n");
    fprintf(stderr, "  -c     [opt] Read coverage (total, not per-haplotap). Will infer if not supplied.\n");
    fprintf(stderr, "  -o     [opt] Name prefix of output files. [%s]\n", prefix);
    fprintf(stderr, "  --vcf  [opt] Input, sorted vcf file containing phased variants. Plain or gz'd.\n");
    fprintf(stderr, "  --gtf  [opt] Phase blocks as a GTF (e.g. whatshap stats --block-list). Overrides --vcf's.\n");
    fprintf(stderr, "  --tsv  [opt] Phase blocks as a 3-column tsv (chrom, start, end). Overrides --gtf and --vcf.\n");
    fprintf(stderr, "  -U,--write-input-tagging [opt] With -u, write {prefix}.mp.input_haptag.tsv.\n");
    fprintf(stderr, "  -u,--bam-is-untagged [opt] If present, will haplotag reads \n"
                    "               with phased variants in vcf first (on the GPU).\n");
    fprintf(stderr, "  -t     [opt] Host threads fetching reads, per GPU. [1]\n");
    fprintf(stderr, "  --output-tsv [opt] Also write {prefix}.mp.tsv.\n");
    fprintf(stderr, "  --write-bam  [opt] Also write {prefix}.mp.bam (+ .bai) with the new HP tags.\n");
    fprintf(stderr, "  -T,--bam-threads [opt] Compression threads of the output BAM. [-t]\n");
    fprintf(stderr, "  --gpus [opt] GPUs to use. [all visible]\n");
    fprintf(stderr, "  --host-fetch [opt] Inflate and decode BAM records (and the coverage pass) on the host instead of the GPU.\n");
}

enum { O_LO = 301, O_HI, O_GTF = 304, O_VCF = 306, O_MAPQ, O_TSV, O_WBAM, O_OTSV, O_BAMT, O_UNTAG, O_WIT,
       O_CSIZE, O_CSTRIDE, O_HELP = 400, O_DBG, O_GPUS = 500, O_JOBW, O_HFETCH };

static const struct option longopts[] = {
    {"lo", required_argument, 0, O_LO},          {"hi", required_argument, 0, O_HI},
    {"gtf", required_argument, 0, O_GTF},        {"vcf", required_argument, 0, O_VCF},
    {"mapq", required_argument, 0, O_MAPQ},      {"tsv", required_argument, 0, O_TSV},
    {"write-bam", no_argument, 0, O_WBAM},       {"output-tsv", no_argument, 0, O_OTSV},
    {"bam-threads", required_argument, 0, O_BAMT}, {"bam-is-untagged", no_argument, 0, O_UNTAG},
    {"write-input-tagging", no_argument, 0, O_WIT},
    {"chunk-size", required_argument, 0, O_CSIZE}, {"chunk-stride", required_argument, 0, O_CSTRIDE},
    {"help", no_argument, 0, O_HELP},            {"dbg", no_argument, 0, O_DBG},
    {"gpus", required_argument, 0, O_GPUS},      {"job-windows", required_argument, 0, O_JOBW},
    {"host-fetch", no_argument, 0, O_HFETCH},
    {0, 0, 0, 0}};

typedef struct {
    int help, threads, lo, hi, readlen, mapq, k, k_span, cov, cov_sel, n_cand, untagged, out_tsv, out_bam;
    int chunk_size, chunk_stride, gpus, job_windows, verbose, host_fetch, write_input_tagging, dbg, bam_threads;
    char *prefix, *vcf, *gtf, *tsv, *bam;
} cli_t;

static int parse(int argc, char **argv, cli_t *c) {
    memset(c, 0, sizeof *c);                          /* init_cliopt_t, cli.c:47-75 */
    c->threads = 1; c->lo = 100; c->hi = 156; c->readlen = 15000; c->mapq = 10; c->k = 3; c->k_span = 5000;
    c->cov_sel = -1; c->n_cand = 15; c->chunk_size = 50000; c->chunk_stride = 1000000;
    c->prefix = "pomfret";
    int o;
    optind = 1;
    while ((o = getopt_long(argc, argv, "vhuUo:k:L:l:c:n:t:T:", longopts, NULL)) >= 0) {
        switch (o) {
        case 'v': c->verbose++; break;
        case 'h': case O_HELP: c->help = 1; break;
        case 't': c->threads = atoi(optarg); break;
        case 'o': c->prefix = optarg; break;
        case 'k': c->k = atoi(optarg); break;
        case 'l': c->k_span = atoi(optarg); break;
        case 'L': c->readlen = atoi(optarg); break;
        case 'c': c->cov = atoi(optarg); c->cov_sel = c->cov / 10; c->n_cand = c->cov / 4; break;
        case 'n': c->n_cand = atoi(optarg); break;
        case O_LO: c->lo = atoi(optarg); break;
        case O_HI: c->hi = atoi(optarg); break;
        case O_GTF: c->gtf = optarg; break;
        case O_VCF: c->vcf = optarg; break;
        case O_MAPQ: c->mapq = atoi(optarg); break;
        case O_TSV: c->tsv = optarg; break;
        case O_WBAM: c->out_bam = 1; break;
        case O_OTSV: c->out_tsv = 1; break;
        case 'T': case O_BAMT: c->bam_threads = atoi(optarg); break;
        case 'u': case O_UNTAG: c->untagged = 1; break;
        case 'U': case O_WIT: c->write_input_tagging = 1; break;
        case O_CSIZE: c->chunk_size = atoi(optarg); break;
        case O_CSTRIDE: c->chunk_stride = atoi(optarg); break;
        case O_DBG: c->dbg = 1; break;
        case O_GPUS: c->gpus = atoi(optarg); break;
        case O_JOBW: c->job_windows = atoi(optarg); break;
        case O_HFETCH: c->host_fetch = 1; break;
        default:
            fprintf(stderr, "[E::parse_cli] unknown or incomplete option \"%s\"\n", argv[optind - 1]);
            return 1;
        }
    }
    for (int i = optind; i < argc; i++) {
        if (c->bam) { fprintf(stderr, "[E::parse_cli] multiple bam input is not supported.\n"); return 1; }
        c->bam = argv[i];
    }
    return 0;
}

static int sancheck(cli_t *c) {                       /* sancheck_cliopt, cli.c:111-222 */
    if (c->threads <= 0) c->threads = 1;
    if (c->lo < 0 || c->lo > 127) { fprintf(stderr, "[E::sancheck_cliopt] bad --lo (%d)\n", c->lo); return 1; }
    if (c->hi > 255 || c->hi <= 127) { fprintf(stderr, "[E::sancheck_cliopt] bad --hi (%d)\n", c->hi); return 1; }
    if (c->readlen < 0) c->readlen = 0;
    if (c->mapq < 0) c->mapq = 0;
    if (c->k <= 0) c->k = 1;
    if (c->k_span <= 0) c->k_span = 1;
    if (c->n_cand <= 0) c->n_cand = 1;
    if (!c->gtf && !c->tsv && !c->vcf) {
        fprintf(stderr, "[E::sancheck_cliopt] gtf, tsv and vcf cannot all be absent\n");
        return 1;
    }
    if (c->untagged && !c->vcf) {
        fprintf(stderr, "[E::sancheck_cliopt] input bam was flagged unhaplotagged, but vcf is missing.\n");
        return 1;
    }
    if (!c->bam) { fprintf(stderr, "[E::sancheck_cliopt] missing bam file\n"); return 1; }
    size_t l = c->prefix ? strlen(c->prefix) : 0;
    while (l > 0 && c->prefix[l - 1] == '/') c->prefix[--l] = 0;
    if (l == 0) { fprintf(stderr, "[E::sancheck_cliopt] no output prefix given\n"); return 1; }
    if (c->chunk_size <= 0 || c->chunk_stride <= 0) {
        fprintf(stderr, "[E::sancheck_cliopt] invalid chunk size or stride\n");
        return 1;
    }
    if ((c->gtf ? 1 : 0) + (c->tsv ? 1 : 0) + (c->vcf ? 1 : 0) > 1)
        fprintf(stderr, "[M::sancheck_cliopt] multiple phase block files. Will not resolve conflict, only total "
                        "override (order is always: tsv > gtf > vcf)\n");
    if (c->dbg)
        fprintf(stderr, "[W::pomfret-amd] --dbg: {prefix}.mp.dbg.read2tag (a hash table dump in bucket order) is "
                        "not written\n");
    return 0;
}

/* varhaptag: parse_cli_varhaptag (cli.c:386-446): -o out.bam, -t, -v,
 * --write-bam (disables the BAM), positional in.vcf then in.bam */
static int varhaptag(int argc, char **argv) {
    const char *out = "pomfret_varhaptag", *vcf = NULL, *bam = NULL;
    int threads = 1, verbose = 0, write_bam = 1, gpus = 0, o;
    optind = 1;
    while ((o = getopt_long(argc, argv, "ho:t:r:v", longopts, NULL)) >= 0) {
        switch (o) {
        case 'h': case O_HELP:
            fprintf(stderr, "Usage: pomfret-amd varhaptag [-t threads] -o out.bam in.vcf in.bam 2>log\n");
            return 1;
        case 'o': out = optarg; break;
        case 't': threads = atoi(optarg); break;
        case 'v': verbose = 1; break;
        case 'r': break;
        case O_WBAM: write_bam = 0; break;
        case O_GPUS: gpus = atoi(optarg); break;
        default:
            fprintf(stderr, "[E::parse_cli_varhaptag] unknown or incomplete option \"%s\"\n", argv[optind - 1]);
            return 1;
        }
    }
    for (int i = optind; i < argc; i++) {
        if (!vcf) vcf = argv[i];
        else if (!bam) bam = argv[i];
        else { fprintf(stderr, "[E::parse_cli_varhaptag] too many positional arguments\n"); return 1; }
    }
    if (!vcf || !bam) { fprintf(stderr, "[E::sancheck_cliopt_varhaptag] need a vcf and a bam\n"); return 1; }
    if (threads < 1) threads = 1;
    pf_methphase_opts_t op;
    memset(&op, 0, sizeof op);
    op.mode = PF_MODE_VARHAPTAG;
    op.bam_path = bam;
    op.vcf_path = vcf;
    op.out_prefix = out;
    op.write_bam = write_bam;
    op.threads = threads;
    op.n_devices = gpus;
    op.verbose = verbose;
    pf_mp_plan_t *p = NULL;
    const int rc = pf_methphase_main(&op, &p);
    if (rc) {
        fprintf(stderr, "[E::main] varhaptag failed: %s (%d)\n", pf_strerror(rc), rc);
        return 1;
    }
    pf_mp_free(p);
    return 0;
}

int main(int argc, char **argv) {
    fprintf(stderr, "[M::main] pomfret-amd (MI355X) ABI %d\n[M::main] CMD: ", pf_abi_version());
    for (int i = 0; i < argc; i++) fprintf(stderr, "%s ", argv[i]);
    fprintf(stderr, "\n");
    const double T = now_s();
    if (argc < 2 || !strcmp(argv[1], "-h") || !strcmp(argv[1], "--help") || !strcmp(argv[1], "help")) {
        help_main();
        return 1;
    }
    if (!strcmp(argv[1], "varhaptag")) return varhaptag(argc - 1, argv + 1);
    const int report = !strcmp(argv[1], "report");
    if (!report && strcmp(argv[1], "methphase")) {
        fprintf(stderr, "[E::main] unknown subcommand: %s\n", argv[1]);
        return 1;
    }
    cli_t c;
    if (argc == 2) { help_methphase("pomfret"); return 1; }
    if (parse(argc - 1, argv + 1, &c)) return 1;
    if (c.help) { help_methphase(c.prefix); return 1; }
    if (sancheck(&c)) return 1;
    if (report && !c.vcf) { fprintf(stderr, "[E::main] missing input: phasd vcf file.\n"); return 1; }

    pf_methphase_opts_t o;
    memset(&o, 0, sizeof o);
    o.mode = report ? PF_MODE_REPORT : PF_MODE_METHPHASE;
    o.bam_path = c.bam;
    o.vcf_path = c.vcf;
    o.out_prefix = c.prefix;
    o.cov_for_selection = c.cov_sel;
    o.n_cand = c.n_cand;
    o.cov = c.cov;
    o.k = c.k;
    o.k_span = c.k_span;
    o.load.min_mapq = c.mapq;
    o.load.min_len = c.readlen;
    o.load.qual_lo = c.lo;
    o.load.qual_hi = c.hi;
    o.untagged = c.untagged;
    o.write_tsv = c.out_tsv;
    o.write_bam = c.out_bam;
    o.chunk_size = c.chunk_size;
    o.chunk_stride = c.chunk_stride;
    o.threads = c.threads;
    o.bam_threads = c.bam_threads;                  /* -T; else -t (cli.c:261-264) */
    o.n_devices = c.gpus;
    o.job_windows = c.job_windows > 0 ? (uint32_t)c.job_windows : 0;
    o.host_fetch = c.host_fetch;
    o.verbose = c.verbose;
    if (!report && (c.tsv || c.gtf)) {         /* tsv > gtf > vcf (4661-4666) */
        o.interval_path = c.tsv ? c.tsv : c.gtf;
        o.interval_format = c.tsv ? PF_INTERVALS_TSV : PF_INTERVALS_GTF;
    }
    o.write_input_tagging = c.write_input_tagging;
    pf_mp_plan_t *p = NULL;
    const int rc = pf_methphase_main(&o, &p);
    if (rc) {
        fprintf(stderr, "[E::main] %s failed: %s (%d)\n", argv[1], pf_strerror(rc), rc);
        return 1;
    }
    const int8_t *dec;
    uint32_t n, n_limit;
    pf_mp_decisions(p, &dec, &n, &n_limit);
    uint32_t joined = 0;
    for (uint32_t i = 0; i < n; i++) joined += dec[i] >= 0;
    fprintf(stderr, "[M::main] %u of %u windows joined; %u read tags; done, used %.1fs\n", joined, n,
            (unsigned)pf_tags_size(pf_mp_qname_hp(p)), now_s() - T);
    if (c.verbose) {
        pf_mp_stats_t st;
        if (pf_mp_stats(p, &st) == PF_OK)
            fprintf(stderr, "[M::main] phases: plan %.3fs (coverage pass %.3fs), -u pre-pass %.3fs, windows %.3fs, "
                    "writers %.3fs; device inflate %.1f ms (-u) + %.1f ms (windows)\n", st.s_plan, st.s_estimate,
                    st.s_haptag, st.s_windows, st.s_finish, st.fetch_ms[1][1], st.fetch_ms[0][1]);
    }
    pf_mp_free(p);
    return 0;
}
