/*
 * pf_load.h -- device-side layout of kernel K0 (the window loader on the GPU)
 * and of its pack step.
 *
 * K0 applies load_reads_given_interval's read filters (blockjoin.c:1079-1085),
 * decodes the 5mC calls of the MM/ML tags (fill_read_meth_record_from_bam_line,
 * 794-908) and maps them to the reference through the CIGAR, including the
 * implicit-canonical calls (get_mod_poss_on_ref, 605-792).  One wavefront per
 * BAM record.  Every run of a record-level batch sizes itself on the device:
 *   K0    decodes each record once; a kept record bump-allocates its call
 *         slice in the staging arena (exactly its trigger count, plus one
 *         position per two read bases for implicit-canonical reads) and adds
 *         itself to its window's kept/call totals;
 *   scan  one workgroup: window totals -> window read / call / site offsets
 *         (capacity checks; on overflow every window is emptied and the host
 *         grows the arrays and re-runs);
 *   pack  one workgroup per window: kept records -> read indices in record
 *         order (the reference's rs->a order), the batch's read arrays, and
 *         each read's calls copied from its staging slice to the window's
 *         contiguous run.
 * No count pass and no host round trip sit between the records and K12.
 */
#ifndef PF_LOAD_H
#define PF_LOAD_H
#include <stdint.h>

#define PF_K0_WAVES 4
#define PF_K0_TCAP 640            /* triggers per wave kept in LDS; longer lists use HBM scratch */
#define PF_K0_CB 128              /* read positions per implicit-mode chunk (4 per lane, half the wave) */
#define PF_K0_EC (PF_K0_CB / 2)   /* explicit / implicit calls per chunk (CpGs are >= 2 apart) */
#define PF_K0_SEQ_ALIGN 16        /* per-record SEQ slices are 16-byte aligned and padded */
#define PF_PACK_THREADS 1024
/* pf_k0_pack's pipelined copy pays in batches that fill the device with pack
 * workgroups (a 1024-window batch: 0.755 -> 0.628 ms); in the 512-window
 * batches of an 8-GPU rank its 256-call chunks lost (the N=8 step 12.63 ->
 * 13.0 ms), so smaller batches run pf_k0_pack_small (512-call chunks) */
#ifndef PF_PACK_PIPE_MIN
#define PF_PACK_PIPE_MIN 768u
#endif
#define PF_SCAN_THREADS 1024

/* status bits of K0 and the pack step (share the batch status word with
 * pf_device.h's) */
#define PF_ST_FATAL_CIGAR 32u     /* H/=/X/P/... reached in the CIGAR walk: exit(1) at 776-779 */
#define PF_ST_POS_LIMIT   64u     /* a call position >= 2^29 */
#define PF_ST_STAGE_OVF  128u     /* K0's call staging arena is too small (grow, re-run) */
#define PF_ST_CALL_OVF   256u     /* the batch call arrays are too small (grow, re-run) */
#define PF_ST_SITES_OVF  512u     /* the batch site arrays are too small (grow, re-run) */
#define PF_ST_MM_LIMIT  1024u     /* a record's MM tag has more than PF_K0_MAXT (8) C m entries */

/* counters (ctr[]) */
#define PF_K0C_SEQPATH  0         /* records walked by the sequential path */
#define PF_K0C_UNSORTED 1         /* records whose calls needed a sort */
#define PF_K0C_IMPLICIT 2         /* records in implicit-canonical mode */
#define PF_K0C_BADMM    3         /* records whose MM/ML could not be decoded */
#define PF_K0C_DUPCHUNK 4         /* emission chunks with a duplicate position */
#define PF_K0C_MULTICM  5         /* records with several C m entries (merged: duplex-style tags) */
#define PF_K0_NCTR 16             /* [8..15]: per-phase cycles of the diagnostic build */

/* I/O block header fields of the record-level path (byte offsets; the
 * header layout is in pf_api.hip) */
#define PF_IO_STAGE 48            /* u64 staging arena bump pointer (K0)   */
#define PF_IO_R     56            /* u32 kept reads (scan)                   */
#define PF_IO_N     64            /* u64 calls (scan)                        */
#define PF_IO_SITES 72            /* u64 site slots the windows need (scan)  */

/* K0's fields of one record, one 128-byte row per wave slot (slots in the
 * order[] order, longest reads first), so that a wave starts its record with
 * one coalesced load instead of one cache line per field array at a random
 * record index (round 4). */
struct pf_k0_hdr {
    uint64_t mm_off, ml_off, seq_off, cig_off, stage_off, scr_off;   /* words 0-11 */
    uint32_t mm_len, ml_len, ncig, stage_len;                        /* 12-15 */
    uint32_t scr_len, l_qseq, pos, rec;                              /* 16-19 */
    float de;                                                        /* 20 */
    uint32_t rec_win;                                                /* 21 */
    uint32_t flag_mapq;                                              /* 22: flag | mapq << 16 */
    uint32_t pad[9];
};

struct pf_load_dev {
    uint32_t n_recs, n_windows;
    uint32_t min_mapq, min_len;
    uint32_t lo, hi;                 /* uint8_t in the reference (799) */
    uint32_t force_seq;              /* test override: every record through the sequential path */
    uint32_t diag;                   /* measurement only (PF_K0_DIAG): 1 = trigger placement reads no SEQ word */
    const uint32_t *order;           /* [n_recs] record of each wave slot: longest reads first */
    const pf_k0_hdr *hdr;            /* [n_recs] K0's fields of each wave slot's record */
    const uint32_t *rec_win;         /* [n_recs] window of each record */
    const uint32_t *win_order;       /* [W] pack's workgroups: windows with the most records first */
    const uint32_t *win_rec_off;     /* [W+1] records of each window */
    const uint16_t *flag;
    const uint8_t *mapq;
    const uint32_t *pos, *l_qseq;
    const float *de;
    const uint8_t *hp;               /* [n_recs] get_hp_from_aln (910-923) or the -u table */
    const uint64_t *cigar_off;
    const uint32_t *cigar;
    const uint64_t *seq_off;         /* 16-byte aligned device offsets */
    const uint8_t *seq;
    const uint64_t *mm_off;
    const uint8_t *mm;
    const uint64_t *ml_off;
    const uint8_t *ml;
    const uint64_t *scr_off;         /* [n_recs+1] trigger-list scratch slices (u32 units); empty = LDS */
    uint32_t *scr;
    /* K0 output, per record */
    uint32_t *rec_n;                 /* calls of each kept record, PF_NONE when dropped */
    uint32_t *rec_out;               /* [8 n_recs] a kept record's row (one 32-byte store): start, end
                                        (bam_endpos), first and last call, staging offset (lo, hi), 0, 0 */
    uint32_t *stage_pos;             /* staging arena: per-record call slices */
    uint8_t *stage_cat;
    const uint64_t *stage_off;       /* [n_recs+1] static slices: each record's trigger bound */
    uint64_t stage_cap;              /* slots; [stage_off[n_recs], stage_cap) is bump-allocated */
    unsigned long long *stage_ctr;   /* bump pointer of that tail (I/O block header, zeroed per run) */
    uint32_t *win_kept, *win_calls;  /* [W] per-window totals (atomics, zeroed per run) */
    uint32_t *status;
    unsigned long long *ctr;         /* PF_K0_NCTR */
    uint32_t *multi_list;            /* [n_recs] wave slots of records with several C m entries (pf_k0_multi) */
    uint32_t *multi_ctr;             /* their count (I/O block header, zeroed per run) */
    /* scan + pack output: the batch's window / read / call arrays */
    uint8_t *io;                     /* I/O block (header totals, bump pointer) */
    uint64_t call_cap, sites_cap;
    uint32_t *win_read_off;          /* [W+1] device copy the kernels read */
    uint32_t *io_win_read_off;       /* [W+1] I/O block copy for the host epilogue */
    uint64_t *win_site_off;          /* [W] */
    uint32_t *win_site_cap;          /* [W] */
    const int32_t *win_par;          /* [W*4] cov_sel first */
    uint64_t *win_call_off;          /* [W+1] scratch */
    uint32_t *read_start, *read_end, *read_first, *read_last, *read_win;
    uint32_t *read_rec;              /* [R] record of each read (I/O block) */
    uint8_t *read_hp, *hp_raw;       /* read_hp: the kernels' copy; hp_raw: the I/O block's */
    uint64_t *read_call_off;         /* [R+1] */
    uint32_t *call_pos;
    uint8_t *call_cat;
};

#ifdef __cplusplus
/* placement of a record-level batch's large arrays (pf_aln_build, pf_api.hip):
 * fill() writes ld->cigar / mm / ml (sized by the batch's offsets) and the
 * SEQ slices (seq_off[r], 16-byte aligned, zero padded; seq_bytes total).
 * The pad nibble of an odd-length SEQ is written as 0 as well, so no nibble
 * past l_qseq is C or G: K0's SEQ counts have no per-word tail test. */
struct pf_ctx;
struct pf_dbatch;
typedef struct pf_aln_fill {
    int (*fill)(void *user, struct pf_ctx *ctx, pf_load_dev *ld, const uint64_t *seq_off, uint64_t seq_bytes);
    void *user;
} pf_aln_fill_t;
struct pf_cfg;
struct pf_load_cfg;
struct pf_aln_batch;
/* a record-level batch from the records' lengths and small fields (host
 * arrays of a; its cigar / seq / mm / ml pointers are not read) */
extern "C" int pf_aln_build(struct pf_ctx *ctx, const struct pf_cfg *cfg, const struct pf_load_cfg *lc,
                            const struct pf_aln_batch *a, const pf_aln_fill_t *fill, struct pf_dbatch **out);
#endif

#endif
