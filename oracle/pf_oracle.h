/*
 * pf_oracle.h -- CPU oracle for the Pomfret methylation-phasing hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This is a plain-C restatement of the reference
 * algorithm (nanoporetech/pomfret v0.1-r14, /root/reference/blockjoin.c),
 * function by function, used as the checker for the HIP implementation and as
 * the CPU baseline leg of bench.py.  Nothing in pomfret_amd/ links or calls
 * it; only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * load it.
 *
 * PARITY PINNING: the reference itself cannot be built here (blockjoin.c
 * includes htslib headers; htslib is absent from this image and stand-ins are
 * not allowed), and the reference ships no test vectors for this path (its
 * example BAM is missing, .MISSING_LARGE_BLOBS).  The window-definition part
 * (VCF PS -> gaps) is pinned by the reference's example fixtures
 * (tests/test_oracle_fixtures.py); the methylation core is "parity unpinned":
 * it is checked only by line-by-line restatement of the reference source
 * (each function cites the lines it follows) and by hand-worked unit cases.
 */
#ifndef PF_ORACLE_H
#define PF_ORACLE_H
#include <stdint.h>
#include "../include/pomfret_amd.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Whole batch, n_threads pthreads over windows (kt_for analogue). */
int orc_methphase_windows(const pf_cfg_t *cfg, const pf_window_batch_t *b,
                          pf_window_out_t *out, int n_threads);

/* Per-(window,dir) greedy trace: for every successful iteration the tagged
 * read (window-local index), its tag and the float score bits.  `cap` entries
 * per (window,dir); counts[w*2+dir] = number recorded (may exceed cap). */
int orc_methphase_trace(const pf_cfg_t *cfg, const pf_window_batch_t *b,
                        uint32_t cap, uint32_t *read_ids, uint8_t *tags,
                        float *scores, uint32_t *counts);

/* Sites and methmers of one window (for unit tests). Returns S.  Arrays sized
 * by the caller: sites/starts/lens >= n_calls of the window. */
int orc_window_sites(const pf_cfg_t *cfg, const pf_window_batch_t *b, uint32_t w,
                     int dir, uint32_t *sites_real, uint32_t *sites_starts,
                     uint8_t *lens);

/* Methmers of every read of window w in direction dir.  mmr_n[r], start_i[r]
 * for the window's reads; keys written back to back (cap entries max).
 * Returns total keys or -1 if cap too small. */
long orc_window_methmers(const pf_cfg_t *cfg, const pf_window_batch_t *b,
                         uint32_t w, int dir, uint32_t *mmr_n, uint32_t *start_i,
                         uint32_t *keys, long cap);

/* htslib kt_fisher_exact restatement. */
double orc_fisher_exact(int n11, int n12, int n21, int n22,
                        double *left, double *right, double *two);

/* search_arr (blockjoin.c:391-421); exposed for unit tests. */
int orc_search_arr(const uint32_t *a, uint32_t l, uint32_t v, uint32_t *idx, int which_end);

/* -u pre-pass for one contig (reads in BAM order). */
int orc_haptag_reads(const pf_known_vars_t *known, const pf_read_aln_batch_t *reads,
                     uint8_t *hp_out);

/* Window definition from a (gz) VCF: per contig the raw gaps, then
 * merge_close_intervals(READBACK).  Results written as text lines to
 * out_path: "contig\tabs_start\tabs_end\n" then "raw\ts\te", "gap\ts\te",
 * "dropped\ts\te".  Returns number of contigs or <0. */
int orc_vcf_gaps(const char *vcf_path, int readback, const char *out_path);
/* fmt 0 VCF, 1 GTF, 2 TSV (load_intervals_from_file, blockjoin.c:1977-2176) */
int orc_interval_gaps(const char *path, int fmt, int readback, const char *out_path);

/* Window loader (pf_oracle_load.c): filters + 5mC extraction of every
 * record (load_reads_given_interval, blockjoin.c:1043-1173).  Writes the kept
 * reads as a pf_window_batch_t (calls in get_mod_poss_on_ref order) and
 * rec_read[r] = read index or UINT32_MAX.  Returns the number of kept reads,
 * -1 on a fatal CIGAR operation, -2 if call_cap is too small (*n_calls_out
 * holds the size needed). */
int orc_load_reads(const pf_load_cfg_t *lc, const pf_aln_batch_t *A, uint32_t *rec_read, uint32_t *win_read_off,
                   uint32_t *read_start, uint32_t *read_end, uint8_t *read_hp, uint64_t *call_off,
                   uint32_t *call_pos, uint8_t *call_cat, uint64_t call_cap, uint64_t *n_calls_out);

/* One window of a record-level batch loaded into a single-window batch `b`
 * (the arrays are owned by the struct; free with orc_window_free). */
typedef struct orc_window {
    pf_window_batch_t b;
    uint32_t win_start, win_end, win_read_off[2];
    uint32_t *read_start, *read_end, *call_pos;
    uint8_t *read_hp, *call_cat;
    uint64_t *read_call_off;
} orc_window_t;
int orc_load_window(const pf_load_cfg_t *lc, const pf_aln_batch_t *A, uint32_t w, orc_window_t *o);
void orc_window_free(orc_window_t *o);

/* Record-level path on the CPU: per window load (a3/a4) then the methphase
 * worker, n_threads pthreads over windows (the reference's per-window
 * structure, 4217-4335).  out->read_hp is not written.  Returns 0, or -1 on a
 * fatal CIGAR operation. */
int orc_methphase_aln(const pf_cfg_t *cfg, const pf_load_cfg_t *lc, const pf_aln_batch_t *A,
                      pf_window_out_t *out, int n_threads);

#ifdef __cplusplus
}
#endif
#endif
