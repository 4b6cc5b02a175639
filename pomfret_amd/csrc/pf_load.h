/*
 * pf_load.h -- device-side layout of kernel K0 (the window loader on the GPU).
 *
 * K0 applies load_reads_given_interval's read filters (blockjoin.c:1079-1085),
 * decodes the 5mC calls of the MM/ML tags (fill_read_meth_record_from_bam_line,
 * 794-908) and maps them to the reference through the CIGAR, including the
 * implicit-canonical calls (get_mod_poss_on_ref, 605-792).  One wavefront per
 * BAM record.  Count mode sizes the batch at upload; write mode fills the
 * resident batch's read and call arrays on every run.
 */
#ifndef PF_LOAD_H
#define PF_LOAD_H
#include <stdint.h>

#define PF_K0_WAVES 4
#define PF_K0_TCAP 640            /* triggers per wave kept in LDS; longer lists use HBM scratch */
#define PF_K0_CB 128              /* read positions per implicit-mode chunk (4 per lane, half the wave) */
#define PF_K0_EC (PF_K0_CB / 2)   /* explicit / implicit calls per chunk (CpGs are >= 2 apart) */
#define PF_K0_SEQ_ALIGN 16        /* per-record SEQ slices are 16-byte aligned and padded */

/* status bits of K0 (share the batch status word with pf_device.h's) */
#define PF_ST_FATAL_CIGAR 32u     /* H/=/X/P/... reached in the CIGAR walk: exit(1) at 776-779 */
#define PF_ST_POS_LIMIT   64u     /* a call position >= 2^29 */

/* counters (ctr[]) */
#define PF_K0C_SEQPATH  0         /* records walked by the sequential path */
#define PF_K0C_UNSORTED 1         /* records whose calls needed a sort */
#define PF_K0C_IMPLICIT 2         /* records in implicit-canonical mode */
#define PF_K0C_BADMM    3         /* records whose MM/ML could not be decoded */
#define PF_K0C_DUPCHUNK 4         /* emission chunks with a duplicate position */
#define PF_K0_NCTR 16             /* [8..15]: per-phase cycles of the diagnostic build */

struct pf_load_dev {
    uint32_t n_recs;
    uint32_t min_mapq, min_len;
    uint32_t lo, hi;                 /* uint8_t in the reference (799) */
    uint32_t force_seq;              /* test override: every record through the sequential path */
    const uint32_t *order;           /* [n_recs] record of each wave slot: longest reads first */
    const uint16_t *flag;
    const uint8_t *mapq;
    const uint32_t *pos, *l_qseq;
    const float *de;
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
    /* count mode */
    uint32_t *rec_n;                 /* calls of each kept record, PF_NONE when dropped */
    uint32_t *rec_nd;                /* 5mC skip counts of the record's C+m entry (write-mode scratch sizing) */
    /* write mode */
    const uint32_t *rec_read;        /* read index of each record or PF_NONE */
    const uint64_t *read_call_off;
    uint32_t *call_pos;
    uint8_t *call_cat;
    uint32_t *read_start, *read_end, *read_first, *read_last;
    uint32_t *status;
    unsigned long long *ctr;         /* PF_K0_NCTR */
};

#endif
