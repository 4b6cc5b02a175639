/*
 * pomfret_amd.h -- C ABI of the MI355X (gfx950) implementation of Pomfret's
 * per-window methylation-phasing hot path.
 *
 * Plain C, plain pointers and sizes; no HIP or torch types cross this
 * boundary.  The library (libpomfret_amd.so) owns its device buffers; callers
 * own every host buffer they pass in.  No entry point calls exit(): errors are
 * returned as negative PF_ERR_* codes ("no evidence" is decision = -1, not an
 * error), matching the reference's split between fatal exits and -1 decisions
 * (reference blockjoin.c:1059, 1150, 4266-4270, 4313-4320).
 *
 * Reference interfaces replaced (all line numbers: /root/reference/<file>):
 *
 *   pf_methphase_windows / pf_methphase_run
 *       replaces the per-window call haplotag_region_given_bam()
 *       (blockjoin.c:4217-4335) as driven by the kt_for worker
 *       blockjoin_one_chrom_callback() (blockjoin.c:4350-4426, dispatched at
 *       blockjoin.c:4560) and by the serial report loop (blockjoin.c:5054-5077).
 *       One call processes a whole batch of windows (gaps) from any number of
 *       contigs; decisions land in caller-owned arrays exactly where the
 *       reference writes ranges->decisions.a[i] (blockjoin.c:4406), and the
 *       per-read tags the worker stores for joined windows (blockjoin.c:4408-4423)
 *       are returned per read.
 *
 *   pf_haptag_reads
 *       replaces parse_variants_for_one_read() + haptag_one_read_with_variants()
 *       (blockjoin.c:1545-1840) as driven by pre_haplotagging_read_in_one_ref()
 *       (blockjoin.c:1841-1898), the --bam-is-untagged (-u) pre-pass.
 *
 *   pf_fisher_exact
 *       the two-sided Fisher exact test the reference borrows from htslib
 *       (kt_fisher_exact, called at blockjoin.c:3926).
 *
 * Input layout ("SoA"): what the reference's BAM window loader
 * (load_reads_given_interval, blockjoin.c:1043-1173) keeps per read after its
 * filters, flattened:
 *   - windows in any order; each window owns a contiguous run of reads;
 *   - reads of a window in BAM order (the order sam_itr_next returns them);
 *   - each read owns a contiguous run of 5mC calls in the order
 *     get_mod_poss_on_ref() produces them (blockjoin.c:605-792).
 */
#ifndef POMFRET_AMD_H
#define POMFRET_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PF_ABI_VERSION 1

/* error codes */
#define PF_OK               0
#define PF_ERR_ARG         -1   /* bad argument / inconsistent batch */
#define PF_ERR_HIP         -2   /* HIP runtime error (no device, launch failure) */
#define PF_ERR_NOMEM       -3   /* device or host allocation failed */
#define PF_ERR_UNSUPPORTED -4   /* configuration outside what this build implements */
#define PF_ERR_LIMIT       -5   /* input exceeds a documented hard limit */
#define PF_ERR_INTERNAL    -6

/* Methmer / tagging configuration.  Mirrors mmr_config_t (blockjoin.h:7-16)
 * plus the per-contig n_candidates_per_iter (blockjoin.c:4357-4390). */
typedef struct pf_cfg {
    int32_t k;                  /* methmer length, cli -k (default 3, cli.c:67)            */
    int32_t k_span;             /* methmer base-span limit, cli -l (default 5000)          */
    int32_t cov_for_selection;  /* site min meth AND unmeth calls (blockjoin.c:3270-3271)  */
    int32_t cov_for_runtime;    /* min hap0+hap1 methmer count to use a site (3669-3691)   */
    int32_t n_cand;             /* candidates scored per greedy iteration (4039-4045)      */
    int32_t hard_cov;           /* left-side per-haplotype read minimum, 15 (1161)         */
    int32_t flags;              /* PF_FLAG_*                                               */
    int32_t reserved;
} pf_cfg_t;

#define PF_FLAG_NONE 0

/* One batch of windows.  A "window" is one call of haplotag_region_given_bam:
 * the gap [win_start, win_end] (blockjoin.c:4397-4398) and the reads that
 * load_reads_given_interval fetched for [s-READBACK, e+READBACK] and kept. */
typedef struct pf_window_batch {
    uint32_t n_windows;
    uint32_t n_reads;
    uint64_t n_calls;
    const uint32_t *win_start;     /* [n_windows] gap start s (ranges->starts.a[i])         */
    const uint32_t *win_end;       /* [n_windows] gap end e   (ranges->ends.a[i])           */
    const uint32_t *win_read_off;  /* [n_windows+1] reads of window w: [off[w], off[w+1])   */
    const int32_t  *win_cov_sel;   /* [n_windows] or NULL -> cfg.cov_for_selection          */
    const int32_t  *win_cov_rt;    /* [n_windows] or NULL -> cfg.cov_for_runtime            */
    const int32_t  *win_n_cand;    /* [n_windows] or NULL -> cfg.n_cand                     */
    const uint32_t *read_start;    /* [n_reads] core.pos, 0-based (blockjoin.c:1124)        */
    const uint32_t *read_end;      /* [n_reads] bam_endpos, exclusive (blockjoin.c:1125)    */
    const uint8_t  *read_hp;       /* [n_reads] HP-1, 254 if untagged (910-923, 1114-1122)  */
    const uint64_t *read_call_off; /* [n_reads+1] calls of read r: [off[r], off[r+1])      */
    const uint32_t *call_pos;      /* [n_calls] reference position of the CpG's C           */
    const uint8_t  *call_cat;      /* [n_calls] 0 meth (q>=hi), 1 unmeth (q<lo), 2 nocall   */
} pf_window_batch_t;

/* Per-window results.  Every pointer except decision may be NULL. */
typedef struct pf_window_out {
    int8_t   *decision;      /* [n_windows] 0 cis, 1 trans, -1 no join (4313-4320)       */
    uint8_t  *read_hp;       /* [n_reads] rs->a[j].hp when the window returns; these are
                                the tags the worker stores when decision>=0 (4408-4423)   */
    int32_t  *dir_table;     /* [n_windows*2*4] 2x2 table buf[raw][new] per direction:
                                index (w*2+dir)*4 + raw*2 + new; dir 0 = forward
                                (left->right, scored on right strict reads), dir 1 =
                                backward (scored on left strict reads) (3881-3893)       */
    int32_t  *dir_join;      /* [n_windows*2] haplotag_region2 return: 0,1,-1 (4088)     */
    int32_t  *dir_which_way; /* [n_windows*2] evaluate_separation1 join_dir (-9 on fail) */
    double   *dir_fisher_p;  /* [n_windows*2] two-sided p (1.0 when not reached)          */
    float    *dir_score;     /* [n_windows*2] evaluate_separation1 return value           */
    uint32_t *win_n_sites;   /* [n_windows] methmer sites (ms->n); 0 => window skipped     */
    uint32_t *win_n_reads;   /* [n_windows] rs->n after the left-coverage check (1161)    */
} pf_window_out_t;

/* ------------------------------------------------------------------ */
/* Record-level input: the BAM records each window's region query returned,
 * decoded on the host (BGZF inflate and record split; htslib's part in the
 * reference) and kept as raw fields.  The read filters and the 5mC
 * extraction of load_reads_given_interval / fill_read_meth_record_from_bam_line
 * / get_mod_poss_on_ref (blockjoin.c:1043-1173, 794-908, 605-792) run on the
 * device (kernel K0), so the window batch above never exists on the host. */

/* Loader parameters: mmr_config_t's lo/hi/readlen_threshold/min_mapq
 * (blockjoin.h:7-16; cli defaults lo 100, hi 156, -L 15000, -q 10). */
typedef struct pf_load_cfg {
    int32_t min_mapq;     /* reads with core.qual < min_mapq are dropped (1082)        */
    int32_t min_len;      /* reads with l_qseq < min_len (or < 2) are dropped (1083)   */
    int32_t qual_lo;      /* ML < lo -> unmeth (1); passed as uint8_t (799, 876-878)   */
    int32_t qual_hi;      /* ML >= hi -> meth (0); otherwise no-call (2)               */
} pf_load_cfg_t;

typedef struct pf_aln_batch {
    uint32_t n_windows;
    uint32_t n_recs;
    const uint32_t *win_start;     /* [n_windows] gap start s                             */
    const uint32_t *win_end;       /* [n_windows] gap end e                               */
    const uint32_t *win_rec_off;   /* [n_windows+1] records of window w in BAM order      */
    const int32_t  *win_cov_sel;   /* [n_windows] or NULL -> cfg.cov_for_selection        */
    const int32_t  *win_cov_rt;    /* [n_windows] or NULL -> cfg.cov_for_runtime          */
    const int32_t  *win_n_cand;    /* [n_windows] or NULL -> cfg.n_cand                   */
    const uint16_t *flag;          /* [n_recs] core.flag                                  */
    const uint8_t  *mapq;          /* [n_recs] core.qual                                  */
    const uint32_t *pos;           /* [n_recs] core.pos (0-based)                         */
    const uint32_t *l_qseq;        /* [n_recs] core.l_qseq                                */
    const float    *de;            /* [n_recs] de:f value, -1 when absent (1079-1080)      */
    const uint8_t  *hp;            /* [n_recs] get_hp_from_aln (910-923) or the -u table  */
    const uint64_t *cigar_off;     /* [n_recs+1] into cigar                               */
    const uint32_t *cigar;         /* BAM encoding len<<4|op                              */
    const uint64_t *seq_off;       /* [n_recs+1] byte offsets into seq                    */
    const uint8_t  *seq;           /* BAM 4-bit packed SEQ                                */
    const uint64_t *mm_off;        /* [n_recs+1] MM:Z (or Mm:Z) text, no terminator       */
    const char     *mm;
    const uint64_t *ml_off;        /* [n_recs+1] ML:B:C values; empty = tag absent        */
    const uint8_t  *ml;
} pf_aln_batch_t;

/* ------------------------------------------------------------------ */
/* -u pre-pass: known phased variants of one contig and reads to tag.  */

/* variant ops as in blockjoin.c:28-31 */
#define PF_VAR_M 0
#define PF_VAR_X 1
#define PF_VAR_I 2
#define PF_VAR_D 3

typedef struct pf_known_vars {
    uint32_t n;
    const uint32_t *pos;       /* [n] 0-based, as insert_variant_from_vcf_line stores it (1432-1543) */
    const uint32_t *len;       /* [n] op length                                               */
    const uint8_t  *op;        /* [n] PF_VAR_X / PF_VAR_I / PF_VAR_D                          */
    const uint8_t  *haptag;    /* [n] haplotype carrying REF (GT[0])                          */
    const uint64_t *char_off;  /* [n+1] allele chars (seq_nt4 codes 0..4) of variant i        */
    const uint8_t  *chars;
} pf_known_vars_t;

/* Reads of ONE contig in BAM order, primary mapped only (flag filter of
 * blockjoin.c:1869-1870 already applied by the caller). */
typedef struct pf_read_aln_batch {
    uint32_t n_reads;
    const uint32_t *start;      /* [n] core.pos                                  */
    const uint32_t *end;        /* [n] bam_endpos                                */
    const uint64_t *cigar_off;  /* [n+1] into cigar                              */
    const uint32_t *cigar;      /* BAM encoding: len<<4 | op                     */
    const uint64_t *seq_off;    /* [n+1] byte offsets into seq (4-bit packed)    */
    const uint32_t *seq_len;    /* [n] l_qseq                                    */
    const uint8_t  *seq;        /* BAM 4-bit packed SEQ                          */
    const uint64_t *md_off;     /* [n+1] into md (no terminator needed)          */
    const char     *md;         /* MD:Z strings, concatenated                    */
} pf_read_aln_batch_t;

/* ------------------------------------------------------------------ */

typedef struct pf_ctx pf_ctx_t;        /* one device, one HIP stream          */
typedef struct pf_dbatch pf_dbatch_t;  /* a window batch resident in HBM      */

int  pf_abi_version(void);
int  pf_device_count(void);
const char *pf_strerror(int code);

/* Context bound to one device (one process per GPU). */
int  pf_ctx_create(int device, pf_ctx_t **out);
void pf_ctx_destroy(pf_ctx_t *ctx);

/* Upload a batch to HBM.  Validates it (offsets monotone, sizes, limits) and
 * keeps a device copy plus the few host-side arrays the decision epilogue
 * needs.  The caller's host arrays may be freed afterwards. */
int  pf_batch_upload(pf_ctx_t *ctx, const pf_cfg_t *cfg,
                     const pf_window_batch_t *batch, pf_dbatch_t **out);
void pf_batch_free(pf_dbatch_t *db);
uint32_t pf_batch_n_windows(const pf_dbatch_t *db);
/* Reads of the batch (record level: the kept records of the last finished
 * run -- K0 sizes the batch on the device -- bounded by the record count). */
uint32_t pf_batch_n_reads(const pf_dbatch_t *db);
/* Calls of the batch (record level: of the last finished run, 0 before). */
uint64_t pf_batch_n_calls(const pf_dbatch_t *db);

/* Run the hot path on a resident batch: all kernels, then the 2x2 tables and
 * tags come back to the host, where the Fisher test and the join decision
 * are applied.  Synchronous. */
int  pf_methphase_run(pf_ctx_t *ctx, pf_dbatch_t *db, pf_window_out_t *out);

/* Split, pipelined form of pf_methphase_run: pf_methphase_launch enqueues a
 * run and returns; pf_methphase_finish waits for the oldest unfinished run
 * and does its host epilogue (Fisher tests, decisions, tags).  Up to two runs
 * of a batch may be in flight, so the epilogue of one overlaps the kernels of
 * the next; a third launch before a finish returns PF_ERR_ARG. */
int  pf_methphase_launch(pf_ctx_t *ctx, pf_dbatch_t *db);
int  pf_methphase_finish(pf_ctx_t *ctx, pf_dbatch_t *db, pf_window_out_t *out);

/* Upload record-level input (pf_aln_batch_t).  The records stay resident in
 * HBM and every run of the batch starts with kernel K0, which applies the
 * loader's filters and extracts each kept read's 5mC calls on the device;
 * this call runs K0 once to size the batch.  The batch's reads are the kept
 * records in record order; pf_batch_read_recs maps them back. */
int  pf_batch_upload_aln(pf_ctx_t *ctx, const pf_cfg_t *cfg, const pf_load_cfg_t *lcfg,
                         const pf_aln_batch_t *aln, pf_dbatch_t **out);
/* rec_of_read[i] = record index of read i (n >= pf_batch_n_reads). */
int  pf_batch_read_recs(const pf_dbatch_t *db, uint32_t *rec_of_read, uint32_t n);
/* Parity/debug for K0: runs it and copies every read's calls sorted by
 * (pos, cat) as the methmer kernels consume them (call_off [R+1]), and the
 * first and last call of each read in get_mod_poss_on_ref's order.  Returns
 * the number of calls or < 0. */
int64_t pf_batch_debug_calls(pf_dbatch_t *db, uint64_t *call_off, uint32_t *pos, uint8_t *cat,
                             uint32_t *first, uint32_t *last, uint64_t cap);

/* K0 counters since upload (count pass + every run), out[0..7]: records
 * walked by the sequential path, records whose calls needed a sort, records
 * in implicit-canonical mode, records whose MM/ML could not be decoded,
 * emission chunks with a duplicate position.  n >= 8. */
/* test hook: a record-level batch's record arrays copied back (sizes[5] =
 * records, CIGAR ops, SEQ bytes (16-byte aligned slices), MM bytes, ML bytes;
 * flag == NULL fills sizes only) */
int  pf_batch_debug_recs(pf_dbatch_t *db, uint64_t *sizes, uint16_t *flag, uint8_t *mapq, uint32_t *pos,
                         uint32_t *l_qseq, float *de, uint8_t *hp, uint64_t *cigar_off, uint32_t *cigar,
                         uint64_t *seq_off, uint8_t *seq, uint64_t *mm_off, uint8_t *mm, uint64_t *ml_off,
                         uint8_t *ml);
int  pf_batch_load_counters(pf_dbatch_t *db, uint64_t *out, int n);

/* One-shot convenience: upload + run + free on `device`. */
int  pf_methphase_windows(int device, const pf_cfg_t *cfg,
                          const pf_window_batch_t *batch, pf_window_out_t *out);

/* Average device time (ms) of each kernel of the last run, measured with HIP
 * events on the library's stream.  names/ms arrays of length *n. */
int  pf_last_kernel_times(pf_ctx_t *ctx, const char **names, float *ms, int *n);

/* Per-(window,direction) counters of the last run, out[(w*2+dir)*8 + j]:
 * j=0 methmer lookups (in-range methmers of every scored candidate),
 * j=1 methmer insertions (reference reads + tagged reads), j=2 greedy
 * iterations that scored >= 1 candidate, j=3 reads visited by the candidate
 * scans, j=4 methmers of all reads, j=5 strict reference reads in the 2x2
 * table, j=6 reads, j=7 sites.  n >= 16*n_windows.  These feed the
 * algorithmic-byte model of DESIGN.md. */
int  pf_batch_stats(pf_dbatch_t *db, uint64_t *out, uint64_t n);
/* The greedy loop's slot-list source per (window, direction) of the last
 * run, out[w*2+dir]: 1 slot lists in LDS, 2 the candidate cache in LDS, 3
 * slot lists in HBM (the slim loop), 4 the general body (fallback kernel),
 * 5 the one-wave kernel (pf_k3_wave), 6 the candidate cache with the count
 * table in HBM (a problem a few KB past the main kernel's budget), 0 no
 * greedy run (no sites).  n >= 2*n_windows.  Tests assert which variant
 * PF_K3_CACHE / PF_K3_GCNT forced. */
int  pf_batch_k3_paths(pf_dbatch_t *db, uint8_t *out, uint64_t n);
/* K12's sites path per window of the last run, out[w]: 1 or 2 the fast
 * path (seen-twice bitmaps and rank counters) over one or two 512 kb
 * segments, 3 the dense path (per-chunk histograms in HBM: spans past 1 Mb,
 * or more repeated positions than a segment's counters), 0 no K12 sites pass
 * (no calls, or the left-coverage check of blockjoin.c:1161).  n >= n_windows.
 * Tests assert which path the wide headline windows took. */
int  pf_batch_k12_paths(pf_dbatch_t *db, uint8_t *out, uint64_t n);
/* The greedy launch this batch was given: out[0] the main kernel's dynamic
 * LDS per problem, out[1] its persistent workgroups (problems at once on the
 * device), out[2] pf_k3_heavy's dynamic LDS, out[3] its problems.  n >= 4. */
int  pf_batch_k3_budget(const pf_dbatch_t *db, uint32_t *out, uint64_t n);

/* The greedy problems (w<<1 | dir) this batch runs in pf_k3_heavy, the second
 * greedy kernel on the context's second stream: windows with at least 2,000
 * reads (1,100 when the batch's 90th-percentile window has <= 400 reads);
 * every other problem, heaviest first, runs in the main kernel.
 * PF_K3_HEAVY_X=x takes x times the median instead, PF_K3_HEAVY=n forces the
 * n heaviest problems.  Returns their count (<= cap copied). */
int  pf_batch_heavy(const pf_dbatch_t *db, uint32_t *probs, uint32_t cap);

/* Parity/debug: run K1 only and copy window w's sites (ms->sites_real_poss,
 * sites_starts, mmr_lens of direction dir); returns S or <0. */
int  pf_batch_debug_sites(pf_dbatch_t *db, uint32_t w, int dir, uint32_t *real,
                          uint32_t *starts, uint8_t *lens, uint32_t cap);
/* Parity/debug: run K1+K2 and copy every read's methmers of direction dir
 * (read_t.mmr_n, mmr_start_i, mmr keys back to back); returns #keys or <0. */
int64_t pf_batch_debug_methmers(pf_dbatch_t *db, int dir, uint32_t *mmr_n,
                                uint32_t *mmr_start, uint32_t *keys, uint64_t cap);

/* -u pre-pass: hp_out[r] in {0, 1, 254} for every read of one contig. */
int  pf_haptag_reads(pf_ctx_t *ctx, const pf_known_vars_t *known,
                     const pf_read_aln_batch_t *reads, uint8_t *hp_out);

/* Device self-test of what the kernels rely on for bit parity: the greedy
 * kernel's reciprocal-based division of 16-bit counts against the correctly
 * rounded fp32 division over all 2^32 operand pairs, and the DPP/permlane
 * wave scans and reductions against LDS references.  Writes the number of
 * mismatches (0 expected). */
int  pf_selftest(pf_ctx_t *ctx, uint64_t *mismatches);

/* Device BGZF inflate (the decompression of htslib's bgzf_read_block,
 * bgzf.c, which load_reads_given_interval reaches through sam_itr_next at
 * blockjoin.c:1076): every BGZF block of comp[0, comp_len) (whole blocks,
 * concatenated as in a BAM file) is inflated on the device, one wavefront per
 * block, and its CRC32 and ISIZE checked; the output (blocks back to back) is
 * copied to out.  block_status[i] (when given, i < status_cap) receives block
 * i's PF_INF_* code (pf_ingest.h; 0 = ok); kernel_ms the inflate kernel time.
 * PF_ERR_ARG for a malformed block table, an undersized out, or any block
 * that failed. */
int  pf_bgzf_inflate(pf_ctx_t *ctx, const uint8_t *comp, uint64_t comp_len, uint8_t *out, uint64_t out_cap,
                     uint64_t *out_len, uint32_t *block_status, uint32_t status_cap, float *kernel_ms);

/* ------------------------------------------------------------------ */
/* Window definition (host side).                                      */

/* Phase-block gaps of a phased VCF, per contig in VCF order.  raw_* are the
 * gaps as insert_vcf_line collects them (blockjoin.c:1348-1430, driven by
 * load_intervals_from_file, :1977-2170): [last POS of a block, PS of the next
 * block]; gap_* are the windows the methphase worker receives after
 * merge_close_intervals(readback) (:2190-2220, called with READBACK at
 * :4520-4521); drop_* the phased intervals that merging swallowed.  Slices of
 * contig c: [x_off[c], x_off[c+1]). */
typedef struct pf_gaps {
    uint32_t n_contigs;
    char **names;
    uint32_t *abs_start, *abs_end;     /* ranges_t.abs_start / abs_end */
    uint64_t *raw_off, *gap_off, *drop_off;
    uint32_t *raw_start, *raw_end;
    uint32_t *gap_start, *gap_end;
    uint32_t *drop_start, *drop_end;
} pf_gaps_t;

/* Parse a (bgzipped or plain) VCF.  Lines starting with '#' are skipped, as
 * load_intervals_from_file does (:2023-2026).  Returns PF_OK, PF_ERR_ARG for
 * the reference's fatal input error (a POS below the previous one,
 * :1383-1387), PF_ERR_NOMEM, or -1 when the file cannot be read. */
int  pf_vcf_gaps(const char *vcf_path, int32_t readback, pf_gaps_t **out);
/* The same loader for any phase-block file main_blockjoin accepts
 * (blockjoin.c:4661-4666: --tsv, then --gtf, then --vcf): PF_INTERVALS_VCF
 * (PS blocks, as pf_vcf_gaps), PF_INTERVALS_GTF (block = GTF columns 4/5) or
 * PF_INTERVALS_TSV (columns 2/3 of "chrom start end"), through insert_gtf_line
 * (:1305-1345): a gap is [end of a block, start of the next block], the first
 * block of each contig sets its abs_start (prev_end resets per new contig,
 * :2098).  Plain or gzipped. */
#define PF_INTERVALS_VCF 0
#define PF_INTERVALS_GTF 1
#define PF_INTERVALS_TSV 2
int  pf_interval_gaps(const char *path, int32_t format, int32_t readback, pf_gaps_t **out);
void pf_gaps_free(pf_gaps_t *gaps);

/* `pomfret report` chunk windows of one contig (main_methreport,
 * blockjoin.c:4963-4991) from its raw gaps: writes up to cap windows
 * [win_start, win_end) and returns how many there are (or < 0). */
int64_t pf_report_windows(uint32_t abs_start, const uint32_t *gap_start, const uint32_t *gap_end,
                          uint64_t n_gaps, uint32_t chunk_size, uint32_t chunk_stride,
                          uint32_t *win_start, uint32_t *win_end, uint64_t cap);

/* ------------------------------------------------------------------ */
/* Output epilogue (host side): decisions -> phase blocks -> GTF/TSV/VCF. */

/* Per contig (slices [x_off[c], x_off[c+1])): the raw gaps after
 * lift_decisions fused the joined ones (rawunphasedblocks, blockjoin.c:
 * 2250-2310), one decision and one cumulative flip per raw gap
 * (decisions_onraw / flips_onraw, :2312-2324), and the new phase blocks
 * [blk_start, blk_end) of generate_new_phase_blocks(use_raw=1) (:2326-2362). */
typedef struct pf_blocks {
    uint32_t n_contigs;
    uint64_t *raw_off, *dec_off, *blk_off;
    uint32_t *raw_start, *raw_end;
    int32_t *dec_onraw, *flip;
    uint32_t *blk_start, *blk_end;
} pf_blocks_t;

/* decision[] holds one join decision (-1 none, 0 cis, 1 trans; the
 * pf_window_out_t.decision of each window) per merged gap of g, contig by
 * contig in g's order (the windows gap_*[gap_off[c] ...]).  Replaces the
 * three calls at blockjoin.c:4685-4687. */
int  pf_phase_blocks(const pf_gaps_t *g, const int8_t *decision, pf_blocks_t **out);
void pf_blocks_free(pf_blocks_t *b);

/* output_gtf (:2721-2756) / output_tsv (:2696-2719) to a file path. */
int  pf_write_gtf(const pf_gaps_t *g, const pf_blocks_t *b, const char *path);
int  pf_write_tsv(const pf_gaps_t *g, const pf_blocks_t *b, const char *path);

/* Phase of the REF allele at variant sites inside dropped intervals
 * (st->varphase_in_dropped of recover_variant_phase_in_dropped_intervals,
 * :2618-2694), per contig of g: 0-based positions ascending in
 * [off[c], off[c+1]), hap_of_ref 0, 1 or 254 (unphased). */
typedef struct pf_rescue {
    const uint64_t *off;
    const uint32_t *pos;
    const uint8_t *hap_of_ref;
} pf_rescue_t;

/* output_modify_vcf (:2918-2988) / alter_vcf_line (:2758-2916): rewrite
 * vcf_in (bgzipped or plain) into vcf_out (plain text) with the new PS and
 * flipped GTs.  rescue may be NULL (no rescued sites).  counts (optional):
 * {lines rewritten, lines unphased by the rescue, lines read}.  Returns
 * PF_OK, PF_ERR_ARG for a #CHROM header without 10 columns, PF_ERR_NOMEM,
 * or -1 on an I/O error. */
int  pf_write_vcf(const char *vcf_in, const pf_gaps_t *g, const pf_blocks_t *b, const pf_rescue_t *rescue,
                  const char *vcf_out, int64_t *counts);

/* ------------------------------------------------------------------ */
/* BAM ingest on the host: BGZF + BAM + BAI reader and  */
/* the region fetch of load_reads_given_interval, feeding pf_aln_batch_t. */

typedef struct pf_bam pf_bam_t;

/* Open a BAM and its BAI (bai_path NULL: bam_path + ".bai", then the path
 * with ".bam" replaced by ".bai").  bam_path NULL opens the index alone
 * (pf_bam_index_stats only).  Replaces hts_open + sam_index_load +
 * sam_hdr_read of init_and_open_bamfile_t (blockjoin.c:565-585).  Returns
 * PF_OK, PF_ERR_ARG (not a BAM / BAI, truncated), PF_ERR_NOMEM, or -1 when a
 * file cannot be opened. */
int  pf_bam_open(const char *bam_path, const char *bai_path, pf_bam_t **out);
void pf_bam_close(pf_bam_t *bam);
/* The host BGZF reader's block decoder: 1 = libdeflate (loaded at run time,
 * as htslib links it), 0 = zlib (libdeflate absent, or PF_HOST_ZLIB set in
 * the environment before the first block).  Diagnostics only. */
int  pf_host_inflater(void);
int32_t pf_bam_n_targets(const pf_bam_t *bam);
const char *pf_bam_target_name(const pf_bam_t *bam, int32_t tid);
uint32_t pf_bam_target_len(const pf_bam_t *bam, int32_t tid);
int32_t pf_bam_tid(const pf_bam_t *bam, const char *name);   /* -1 when absent */
/* The index's per-reference metadata pseudo-bin: mapped / unmapped counts
 * (hts_idx_get_stat); PF_ERR_ARG when tid has none. */
int  pf_bam_index_stats(const pf_bam_t *bam, int32_t tid, uint64_t *n_mapped, uint64_t *n_unmapped);
const char *pf_bam_path(const pf_bam_t *bam);
/* The index's count of unplaced records (the optional n_no_coor after the
 * references); -1 when the index does not have one. */
int64_t pf_bam_n_no_coor(const pf_bam_t *bam);
/* The BAI chunks [u, v) (virtual offsets) of region [beg, end) of tid, sorted
 * by u, as hts_itr_query collects them (bins overlapping the region, chunks
 * ending before the linear-index offset dropped).  Writes min(n, cap) pairs
 * u, v to uv; returns n or a negative PF_ERR. */
int64_t pf_bam_query_chunks(const pf_bam_t *bam, int32_t tid, int64_t beg, int64_t end, uint64_t *uv, uint64_t cap);

/* The records of a set of windows of one contig, in window order and BAM
 * order inside a window, as pf_aln_batch_t (owned by this struct) plus the
 * qnames (for the first-wins tag table, blockjoin.c:4408-4423). */
typedef struct pf_bam_records {
    pf_aln_batch_t aln;
    const uint64_t *qname_off;     /* [n_recs+1] into qname, no terminators */
    const char *qname;
    const int32_t *hp_tag;         /* [n_recs] raw HP value, INT32_MIN when absent */
    uint64_t n_truncated;          /* windows whose fetch stopped at a record
                                      htslib refuses (CIGAR/SEQ length mismatch) */
} pf_bam_records_t;

/* For window w the records sam_itr_querys(chrom:b-(e+readback)) yields,
 * b = s-readback clipped at 0, as load_reads_given_interval builds the
 * region (1053-1054); HP as get_hp_from_aln (910-923: absent or 0 -> 254,
 * else HP-1); de as bam_aux2f or -1; MM from MM:Z / Mm:Z, ML from ML:B:C /
 * Ml:B:C (a tag of another type makes the record's MM empty: htslib's
 * bam_parse_basemod fails and the read carries no calls); the CIGAR from a
 * CG:B:I tag when the record holds the kSmN placeholder.  win_start/win_end
 * are copied into aln.  n_threads > 1 fetches windows in parallel (one file
 * handle per thread).  Returns PF_OK, PF_ERR_ARG (unknown contig, corrupt
 * file), PF_ERR_NOMEM, or -1 on an I/O error. */
int  pf_bam_fetch_windows(pf_bam_t *bam, const char *chrom, uint32_t n_windows, const uint32_t *win_start,
                          const uint32_t *win_end, uint32_t readback, int n_threads, pf_bam_records_t **out);
void pf_bam_records_free(pf_bam_records_t *recs);

/* Device fetch: the same records as pf_bam_fetch_windows, but the host only
 * plans the fetch from the BAI and reads the compressed bytes of the blocks
 * the windows' index chunks touch; the device inflates them (pf_bgzf_inflate's
 * kernels), walks the record chain, decodes every record (rec_decode,
 * bam_tag2cigar, bam_endpos, the aux tags), runs each window's chunk walk
 * (sam_itr_next, with the overlap rule pos + rlen > beg and the stops at
 * another tid, pos >= end, a truncated record or EOF), and gathers the
 * returned records into a record-level batch (pf_batch_upload_aln's layout)
 * -- the record fields never cross PCIe.  Windows with more than
 * max_win_recs records (0 = no limit) are left empty.  *out is the batch
 * (pf_methphase_run etc.), *fetch the qnames and statistics (free with
 * pf_bam_dev_fetch_free). */
typedef struct pf_bam_dev_fetch {
    uint32_t n_windows;
    uint64_t n_recs;               /* records in the batch                               */
    const uint32_t *win_rec_off;   /* [n_windows+1] the batch's records per window       */
    const uint32_t *win_n_fetched; /* [n_windows] records the fetch returned (before the limit) */
    const uint64_t *qname_off;     /* [n_recs+1] into qname                              */
    const char *qname;
    const int32_t *hp_tag;         /* [n_recs] raw HP value, INT32_MIN when absent       */
    uint64_t n_truncated;          /* windows ended at a CIGAR/SEQ length mismatch       */
    uint64_t comp_bytes, inflated_bytes, n_blocks, n_chain_recs;
    double ms_read, ms_inflate, ms_chain, ms_decode, ms_select, ms_build, ms_total;
    uint32_t attempts;             /* plans tried (a record past the planned blocks widens the plan) */
    const uint8_t *read_hp;        /* pf_haptag_bam: [n_recs] each read's tag (NULL otherwise)  */
    uint32_t from_arena;           /* 1: the blocks came from a kept -u arena (nothing read or inflated) */
} pf_bam_dev_fetch_t;
/* replace a record-level batch's per-record HP values (the -u table's tags,
 * blockjoin.c:1114-1122); n must equal its record count */
int  pf_batch_set_hp(pf_dbatch_t *db, const uint8_t *hp, uint32_t n);
int  pf_batch_upload_bam(pf_ctx_t *ctx, const pf_cfg_t *cfg, const pf_load_cfg_t *lcfg, pf_bam_t *bam,
                         const char *chrom, uint32_t n_windows, const uint32_t *win_start, const uint32_t *win_end,
                         uint32_t readback, uint32_t max_win_recs, pf_dbatch_t **out, pf_bam_dev_fetch_t **fetch);
void pf_bam_dev_fetch_free(pf_bam_dev_fetch_t *fetch);
/* The -u pre-pass with the device fetch: the reads pf_bam_fetch_contig_reads
 * returns (the whole contig, primary mapped, MD:Z required: PF_ERR_ARG
 * otherwise) inflated, selected and gathered on the device and haptagged there
 * by K4 against `known` (pf_haptag_reads' semantics).  *fetch holds n_recs
 * reads in BAM order: read_hp, qnames. */
int  pf_haptag_bam(pf_ctx_t *ctx, const pf_known_vars_t *known, pf_bam_t *bam, const char *chrom,
                   pf_bam_dev_fetch_t **fetch);
/* the same with the contig's coverage estimate (estimate_read_coverage_dirtyfast,
 * 951-1040) from the same whole-contig fetch: every record is selected, the
 * primary mapped ones are haplotagged; *truncated is set when a truncated
 * record ended the pass (the serial estimate stops there).  Used by the driver
 * for `methphase -u` without -c: one pass over each contig instead of two. */
int  pf_haptag_bam_cov(pf_ctx_t *ctx, const pf_known_vars_t *known, pf_bam_t *bam, const char *chrom,
                       pf_bam_dev_fetch_t **fetch_out, int32_t *cov, int32_t *truncated);
/* Both with the contig's position pieces given: n_bounds strictly increasing
 * positions > 0 split [0, HTS_POS_MAX) into n_bounds + 1 pieces (a read is
 * taken in the piece its start falls in; the reads, tags and order are the
 * one-piece fetch's).  fetch_ends (optional, fetch_ends[k] >= bounds[k]):
 * piece k fetches the region [bounds[k-1], fetch_ends[k]) -- reaching past
 * its bound over the windows that start in it -- while its reads stay those
 * starting before bounds[k].  With the fetch cache on (a -u pre-pass that
 * keeps its arenas) every piece's arena is kept, and a later window fetch of
 * the contig is served by the piece whose fetch region holds all its
 * windows.  cov / truncated NULL: no coverage estimate.  The driver places
 * the bounds between its windows' fetch regions where it can
 * (pf_pipeline.c). */
int  pf_haptag_bam_pieces(pf_ctx_t *ctx, const pf_known_vars_t *known, pf_bam_t *bam, const char *chrom,
                          uint32_t n_bounds, const int64_t *bounds, const int64_t *fetch_ends,
                          pf_bam_dev_fetch_t **fetch_out, int32_t *cov, int32_t *truncated);
/* The pieces the -u pre-pass fetches a contig in by default: K =
 * ceil(compressed bytes of the contig's index chunks / piece_bytes) (0: the
 * PF_FETCH_PIECE_BYTES variable or 4 GiB), each *step bases long. */
uint64_t pf_bam_contig_pieces(pf_bam_t *bam, int32_t tid, uint64_t piece_bytes, int64_t *step);


/* The -u pre-pass reads of one contig (pre_haplotagging_read_in_one_ref,
 * 1841-1898: sam_itr_querys over the whole contig, flags 4/256/2048
 * skipped), in BAM order, as pf_haptag_reads takes them, plus qnames for
 * its first-wins table.  A primary mapped record without MD:Z returns
 * PF_ERR_ARG (the reference asserts, 1594-1595). */
typedef struct pf_bam_reads {
    pf_read_aln_batch_t reads;
    const uint64_t *qname_off;     /* [n_reads+1] */
    const char *qname;
    uint64_t n_truncated;          /* 1 when the fetch stopped at a record htslib refuses */
} pf_bam_reads_t;
int  pf_bam_fetch_contig_reads(pf_bam_t *bam, const char *chrom, pf_bam_reads_t **out);
void pf_bam_reads_free(pf_bam_reads_t *reads);

/* Per-contig read coverage estimate for runs without -c
 * (estimate_read_coverage_dirtyfast, 951-1040): covs[tid] for
 * tid < pf_bam_n_targets (n >= that).  A full sequential pass over the BAM. */
int  pf_bam_estimate_coverage(pf_bam_t *bam, int32_t *covs, int32_t n);
/* BGZF inflate threads of the handle's sequential passes (the coverage
 * estimate and pf_bam_fetch_contig_reads): the reference's -t N, which sets
 * pomfret_n_bam_threads for bgzf_mt on every BAM it opens (cli.c:261-264,
 * blockjoin.c:576-578).  n <= 1: single-threaded (the default). */
void pf_bam_set_threads(pf_bam_t *bam, int n);
/* The same estimate with the BAM's records inflated, chained and decoded on
 * ctx's device (the device fetch, pieces of <= piece_bytes compressed bytes
 * per call; 0 = 4 GiB), contig by contig through the index; identical covs
 * for a coordinate-sorted, indexed BAM (the only kind the pipeline opens).
 * Falls back to pf_bam_estimate_coverage when the index has no unplaced-read
 * count (the last contig's estimate depends on it). */
int  pf_bam_estimate_coverage_dev(pf_ctx_t *ctx, pf_bam_t *bam, int32_t *covs, int32_t n, uint64_t piece_bytes);
/* one contig of that pass (0 without records; *truncated: the pass would stop here) */
int  pf_bam_estimate_contig_dev(pf_ctx_t *ctx, pf_bam_t *bam, int32_t tid, int32_t *cov, int32_t *truncated);


/* qname -> tag table across the boundary (first entry of a qname wins). */
typedef struct pf_qname_tags {
    uint32_t n;
    const uint64_t *off;           /* [n+1] into names */
    const char *names;
    const uint8_t *hp;
} pf_qname_tags_t;

/* VCF-writer rescue map of one contig: recover_variant_phase_in_dropped_
 * intervals (2618-2694) / recover_variant_phase_in_one_interval (2475-2616).
 * For each dropped interval [s, e] in order: the known positions in
 * [s-1, e+1); the records of region "chrom:(s-1)-(e+1)" whose qname is in
 * `methphased` (st->qname2haptag) and whose raw tag (`raw` table when given
 * -- the -u table -- else the HP tag) is not unphased; their variant
 * positions (CIGAR I, MD mismatches and closed ^-runs) voted by methphased
 * tag 0/1 at each known position: more hap0 -> REF on hap1, more hap1 ->
 * REF on hap0, else 254.  A known position sorted last among the interval's
 * entries gets no vote (the loop stops at n-1).  Positions ascending, last
 * write wins.  PF_ERR_ARG for an MD-less selected record (the reference
 * asserts) or an invalid MD character (it exits). */
typedef struct pf_rescue_map {
    uint32_t n;
    const uint32_t *pos;
    const uint8_t *hap_of_ref;
} pf_rescue_map_t;
int  pf_rescue_dropped(pf_bam_t *bam, const char *chrom, uint32_t n_drop, const uint32_t *drop_start,
                       const uint32_t *drop_end, const pf_known_vars_t *known, const pf_qname_tags_t *methphased,
                       const pf_qname_tags_t *raw, pf_rescue_map_t **out);
/* the same with the intervals spread over `threads` host threads (each with
 * its own file handle); the result is the serial pass's */
int  pf_rescue_dropped_mt(pf_bam_t *bam, const char *chrom, uint32_t n_drop, const uint32_t *drop_start,
                          const uint32_t *drop_end, const pf_known_vars_t *known, const pf_qname_tags_t *methphased,
                          const pf_qname_tags_t *raw, int threads, pf_rescue_map_t **out);
/* several contigs at once (the qname tables built once, every (contig,
 * interval) one work item); out[c] per contig, each the serial pass's */
int  pf_rescue_dropped_multi(pf_bam_t *bam, uint32_t n_contigs, const char *const *chroms, const uint32_t *n_drop,
                             const uint32_t *const *drop_start, const uint32_t *const *drop_end,
                             const pf_known_vars_t *const *known, const pf_qname_tags_t *methphased,
                             const pf_qname_tags_t *raw, int threads, pf_rescue_map_t **out);
void pf_rescue_map_free(pf_rescue_map_t *map);

/* -u known variants of one contig: insert_variant_from_vcf_line (1432-1543)
 * on every complete line whose CHROM equals `contig` (the variants the
 * reference collects for a contig before pre-haplotagging its reads,
 * 1937-1941, 2069-2080): GT "a|b" with a, b in {0,1}; SNP -> X at POS-1;
 * ref longer -> D at POS (len ref-alt, chars ref+1); alt longer -> I at
 * POS-1 (len alt-ref, chars alt+1); equal-length non-SNPs skipped; haptag =
 * GT[0].  Tokens split on runs of tabs as strtok_r does; '#' lines skipped
 * (:2023-2026).  Returns PF_OK, PF_ERR_NOMEM, or -1 when the file cannot be
 * read. */
typedef struct pf_known_table {
    pf_known_vars_t vars;
} pf_known_table_t;
int  pf_vcf_known_vars(const char *vcf_path, const char *contig, pf_known_table_t **out);
/* The tables recover_variant_phase_in_dropped_intervals builds for the run's
 * contigs (names: the phase-block file's contigs) in one pass over the VCF:
 * the var_storage branch of load_intervals_from_file (2150-2163), where a
 * line whose CHROM is not among `names` goes to the table the previous line
 * went to (skipped before the first match).  With the VCF's own contigs as
 * `names` (no --gtf / --tsv) out[c] equals pf_vcf_known_vars(names[c]).
 * out[0..n) are set on PF_OK (free each with pf_known_table_free). */
int  pf_vcf_known_vars_multi(const char *vcf_path, uint32_t n, const char *const *names, pf_known_table_t **out);
void pf_known_table_free(pf_known_table_t *t);

/* ------------------------------------------------------------------ */
/* qname -> haplotag tables (the reference's htstri_t: st->qname2haptag,  */
/* st->qname2haptag_raw), first entry of a qname wins.                    */

typedef struct pf_tags pf_tags_t;
pf_tags_t *pf_tags_new(void);
void     pf_tags_free(pf_tags_t *t);
uint64_t pf_tags_size(const pf_tags_t *t);
/* Insert every (names[off[i]:off[i+1]], hp[i]) whose qname is absent, in
 * order (kh_put + "if (absent)", blockjoin.c:4412-4421).  Returns the number
 * inserted or < 0. */
int64_t  pf_tags_put_first(pf_tags_t *t, uint32_t n, const uint64_t *off, const char *names, const uint8_t *hp);
/* hp_out[i] = tag of qname i, or dflt when absent; returns how many were found. */
int64_t  pf_tags_get(const pf_tags_t *t, uint32_t n, const uint64_t *off, const char *names, uint8_t dflt,
                     uint8_t *hp_out);
/* The entries in insertion order (valid until the next insertion). */
int      pf_tags_view(const pf_tags_t *t, pf_qname_tags_t *out);

/* ------------------------------------------------------------------ */
/* Pipeline driver: `pomfret methphase` (main_blockjoin, blockjoin.c:    */
/* 4643-4736) and `pomfret report` (main_methreport, 4901-5089) from     */
/* files, on one or more GPUs.                                           */

#define PF_READBACK 50000          /* blockjoin.c READBACK, the fetch margin of 1053-1054 */
#define PF_MODE_METHPHASE 0
#define PF_MODE_REPORT    1
#define PF_MODE_VARHAPTAG 2        /* pf_methphase_main only: out_prefix is the output BAM path */
#define PF_JOB_WINDOWS 0           /* a run of consecutive windows of one contig */
#define PF_JOB_HAPTAG  1           /* the -u pre-pass of one contig (1841-1898) */

typedef struct pf_methphase_opts {
    int32_t mode;                  /* PF_MODE_*                                                */
    const char *bam_path;          /* positional bam (sorted, indexed)                         */
    const char *vcf_path;          /* --vcf                                                    */
    const char *out_prefix;        /* -o; NULL: nothing written                                */
    /* methphase: cliopt->cov_for_selection / n_candidates_per_iter as the
     * CLI leaves them (-c C sets C/10 and C/4, -n sets n_cand; <= 0: per
     * contig from the coverage estimate, 4357-4374); cov_for_runtime <= 0
     * means 2*cov_for_selection (4655).  report: cov is -c (<= 0: the
     * estimate), parameters cov/10+1, 2x, cov/4+1 (5045-5051). */
    int32_t cov_for_selection, cov_for_runtime, n_cand, cov;
    int32_t k, k_span;             /* -k, -l (<= 0: 3, 5000)                                   */
    pf_load_cfg_t load;            /* -q, -L, --lo, --hi                                       */
    int32_t untagged;              /* -u, --bam-is-untagged                                    */
    int32_t write_tsv;             /* --output-tsv: {prefix}.mp.tsv                            */
    int32_t write_bam;             /* --write-bam: {prefix}.mp.bam + .bai (varhaptag: the BAM) */
    int32_t chunk_size, chunk_stride;  /* report: --chunk-size, --chunk-stride                 */
    int32_t threads;               /* host threads fetching one job's windows (-t)             */
    int32_t n_devices;             /* GPUs to drive from this process (0: all visible)         */
    const int32_t *devices;        /* their ids (NULL: 0..n_devices-1)                         */
    pf_ctx_t *const *ctxs;         /* or caller-owned contexts, one per device thread          */
    int32_t n_ctxs;
    int32_t rank, world;           /* multi-process runs: this process runs the jobs the static
                                      LPT partition gives `rank` (world <= 1: all of them)      */
    uint32_t job_windows;          /* max windows per job (0: 1024)                            */
    int32_t verbose;               /* < 0: no progress messages                                */
    int32_t host_fetch;            /* 1: records fetched and decoded on the host (pf_bam_fetch_windows
                                      + pf_batch_upload_aln); 0: the device fetch (pf_batch_upload_bam) */
    /* --tsv / --gtf phase blocks (main_blockjoin 4661-4666: tsv, then gtf,
     * then vcf).  NULL or PF_INTERVALS_VCF: the VCF's PS blocks.  With -u the
     * VCF still names the contigs whose reads are pre-haplotagged (4446) and
     * the file replaces the intervals (4460-4465); without vcf_path (methphase
     * only, no -u) no VCF is written (4706). */
    const char *interval_path;
    int32_t interval_format;       /* PF_INTERVALS_GTF or PF_INTERVALS_TSV                     */
    int32_t write_input_tagging;   /* -U (with -u): {prefix}.mp.input_haptag.tsv (4494-4517)  */
    int32_t bam_threads;           /* -T / --bam-threads: --write-bam's BGZF compression threads
                                      (<= 0: `threads`, as -t sets threads_bam, cli.c:261-264)  */
} pf_methphase_opts_t;

typedef struct pf_mp_plan pf_mp_plan_t;

/* Whole run in this process: plan, (-u) pre-pass jobs on the devices, window
 * jobs on the devices (one host thread per GPU; the next job's BAM fetch
 * overlaps the current job's kernels), merge and outputs:
 * {prefix}.mp.gtf, .mp.vcf (and .mp.tsv, .mp.bam + .mp.bam.bai), or
 * {prefix}.report.tsv plus the running totals on stdout, or (varhaptag) the
 * -u pre-pass alone with {out}.varhaptag.tsv and the retagged {out} + .bai.  On success *out holds the finished plan
 * (decisions, tables, blocks) until pf_mp_free. */
int  pf_methphase_main(const pf_methphase_opts_t *o, pf_mp_plan_t **out);

/* The same run split into steps, for one process per GPU: every rank builds
 * the same plan (deterministic), runs its jobs, exports their results; the
 * writer rank imports every rank's results and finishes. */
int  pf_mp_plan(const pf_methphase_opts_t *o, pf_mp_plan_t **out);
void pf_mp_free(pf_mp_plan_t *p);
uint32_t pf_mp_n_jobs(const pf_mp_plan_t *p, int kind);

typedef struct pf_mp_job_info {
    uint32_t contig;               /* index into the plan's gaps                    */
    const char *contig_name;
    uint32_t w0, w1;               /* windows [w0, w1) of pf_mp_windows             */
    int32_t rank;                  /* static LPT owner                              */
    uint32_t lpt_pos;              /* position in the longest-first order           */
    double cost;                   /* fetch span (bases) / contig length (-u)       */
    int32_t done;
    pf_cfg_t cfg;                  /* the contig's parameters (4357-4390)           */
} pf_mp_job_info_t;
int  pf_mp_job_info(const pf_mp_plan_t *p, int kind, uint32_t j, pf_mp_job_info_t *info);
/* All windows in (contig, window) order; contig c owns [off[c], off[c+1]). */
int  pf_mp_windows(const pf_mp_plan_t *p, const uint32_t **win_start, const uint32_t **win_end,
                   const uint64_t **contig_win_off, uint32_t *n_windows);

/* Run jobs of `kind` owned by run_opts->rank (all when world <= 1) on the
 * devices run_opts names (n_devices / devices / ctxs). */
int  pf_mp_run_mine(pf_mp_plan_t *p, const pf_methphase_opts_t *run_opts, int kind);
int  pf_mp_run_job(pf_mp_plan_t *p, pf_ctx_t *ctx, uint32_t j);          /* one window job */
int  pf_mp_run_haptag_job(pf_mp_plan_t *p, pf_ctx_t *ctx, uint32_t j);   /* one -u job     */
/* After every -u job has a result: the merged table (contig order, first
 * wins) that replaces HP in the window jobs (1114-1122). */
int  pf_mp_merge_raw(pf_mp_plan_t *p);

/* A job's result: decisions of its windows and the (qname, tag) entries of
 * its joined windows, window by window in read order (tag_off[w] ..
 * tag_off[w+1]); -u jobs: no windows, the contig's first-wins table in BAM
 * order.  get returns views into the plan; set copies. */
typedef struct pf_mp_job_result {
    uint32_t n_windows;
    const int8_t *decision;
    const uint64_t *tag_off;
    pf_qname_tags_t tags;
    uint32_t n_limit;              /* windows left undecided for a device limit */
} pf_mp_job_result_t;
int  pf_mp_get_job_result(const pf_mp_plan_t *p, int kind, uint32_t j, pf_mp_job_result_t *r);
int  pf_mp_set_job_result(pf_mp_plan_t *p, int kind, uint32_t j, const pf_mp_job_result_t *r);

/* Merge every job's result in (contig, window) order -- decisions, and the
 * joined windows' tags first-wins (4408-4423 then 4579-4595) -- then the
 * phase blocks and, with an output prefix, the files. */
int  pf_mp_finish(pf_mp_plan_t *p);
int  pf_mp_decisions(const pf_mp_plan_t *p, const int8_t **decision, uint32_t *n, uint32_t *n_limit);
const pf_gaps_t   *pf_mp_gaps(const pf_mp_plan_t *p);
const pf_blocks_t *pf_mp_blocks(const pf_mp_plan_t *p);
const pf_tags_t   *pf_mp_qname_hp(const pf_mp_plan_t *p);
const pf_tags_t   *pf_mp_raw_hp(const pf_mp_plan_t *p);     /* NULL without -u */
/* report: {correct, switch, fail} */
int  pf_mp_report_counts(const pf_mp_plan_t *p, double *counts3);
/* measurement hook: wall seconds per phase of the run and the device-fetch
 * sums (pf_bam_dev_fetch_t's ms_* and byte counts) of its jobs; index 0 =
 * window jobs, 1 = -u pre-pass jobs */
typedef struct pf_mp_stats {
    double s_plan;              /* VCF gaps, coverage estimate, job plan      */
    double s_estimate;          /* the coverage pass (inside s_plan)          */
    double s_haptag;            /* -u pre-pass jobs + the merge of their tables */
    double s_windows;           /* window jobs                                 */
    double s_finish;            /* first-wins merge, phase blocks, writers    */
    double fetch_ms[2][7];      /* read, inflate, chain, decode, select, build, total */
    uint64_t comp_bytes[2], inflated_bytes[2];
    double run_ms[2];           /* pf_methphase_run / K4 wall, summed over jobs */
    uint64_t n_fetch[2];        /* device fetches */
    /* window jobs of a run that keeps the -u pre-pass's arenas: fetches served
     * from a kept arena, fetches that read and inflated the file again (their
     * compressed bytes), and jobs a context took from another device's queue */
    uint64_t arena_hits, arena_misses, reread_bytes, steals;
} pf_mp_stats_t;
int  pf_mp_stats(const pf_mp_plan_t *p, pf_mp_stats_t *s);

/* ------------------------------------------------------------------ */
/* BAM output: --write-bam and varhaptag.                               */

#define PF_RETAG_METHPHASE 0       /* output_modify_bam (blockjoin.c:3022-3103)   */
#define PF_RETAG_VARHAPTAG 1       /* main_varhaptag (4737-4836)                  */
#define PF_RETAG_INPUT_HAPTAG 2    /* methphase -u -U: the TSV alone (4494-4517)  */

/* Every record of bam_in, in file order (sam_itr_querys "."), with HP set
 * to the new haplotag + 1 as bam_aux_update_int does it (an existing
 * integer HP keeps its size when the value fits, else it grows in place; a
 * missing HP is appended as the smallest integer type; a non-integer HP or
 * corrupt aux data leaves the record unchanged), written to bam_out (NULL:
 * none) with its BAI at bai_out (NULL: none; sam_index_build3 at 4723), and
 * for varhaptag one TSV line per record to tsv_out (NULL: none):
 * "#qname\thaptag_input\thaptag_new", then qname, HP-tag value, new + 1.
 *   PF_RETAG_METHPHASE: the raw tag is raw's (the -u table; absent:
 *     unphased) or the HP tag's (get_hp_from_aln); a qname in `methphased`
 *     (st->qname2haptag) takes its tag, a raw 0/1 otherwise; either is
 *     flipped when the phased interval the read starts in
 *     (check_if_in_phased_intervals over g's merged gaps) needs it -- the
 *     flip of blk's raw gap at the merged index - 1, carried over until the
 *     next interval is entered, across contigs too (get_flip_status_by_idx).
 *   PF_RETAG_VARHAPTAG: the new tag is raw's (absent: unphased).
 *   PF_RETAG_INPUT_HAPTAG: as VARHAPTAG with no BAM (bam_out must be NULL)
 *     and the -U header "#qname\treal_hp\ttagged_hp" ({prefix}.mp.input_haptag.tsv:
 *     the HP tag's value, the -u table's tag + 1 or 255).
 * level: zlib level (htslib's "w" mode: -1, Z_DEFAULT_COMPRESSION).
 * The iteration stops, as htslib's does, at a record whose CIGAR query
 * length differs from l_qseq.  *n_records: records processed. */
int  pf_retag_bam(const char *bam_in, const char *bam_out, const char *bai_out, const char *tsv_out, int mode,
                  const pf_gaps_t *g, const pf_blocks_t *blk, const pf_tags_t *methphased, const pf_tags_t *raw,
                  int level, uint64_t *n_records);
/* The same with `threads` BGZF compression threads for bam_out (-T /
 * --bam-threads: htslib's bgzf_mt for the output, cli.c:261-264, 3036):
 * blocks deflated in parallel, written in order; the BAM and BAI bytes do not
 * depend on the thread count. */
int  pf_retag_bam_threads(const char *bam_in, const char *bam_out, const char *bai_out, const char *tsv_out, int mode,
                          const pf_gaps_t *g, const pf_blocks_t *blk, const pf_tags_t *methphased,
                          const pf_tags_t *raw, int level, int threads, uint64_t *n_records);

/* Host helper: htslib kt_fisher_exact semantics. Returns the probability of
 * the observed table. */
double pf_fisher_exact(int n11, int n12, int n21, int n22,
                       double *left, double *right, double *two);

#ifdef __cplusplus
}
#endif
#endif /* POMFRET_AMD_H */
