// pf_ingest.h -- device-side BAM ingest (BGZF inflate, record chain, window
// fetch, field gather): shared between pf_inflate.hip, pf_ingest.hip and the
// host planner.
#pragma once
#include <stdint.h>

// one BGZF block of a fetch plan
typedef struct pf_bgzf_blk {
    uint64_t in_off;      // offset of the raw DEFLATE payload in the compressed buffer
    uint64_t out_off;     // offset of the block's output in the inflated arena
    uint32_t in_len;      // payload bytes
    uint32_t isize;       // output bytes (footer ISIZE, <= 65536)
    uint32_t crc;         // footer CRC32
    uint32_t run;         // run of consecutive blocks it belongs to
} pf_bgzf_blk;

// per-block status codes of the inflate/CRC kernels
#define PF_INF_OK 0u
#define PF_INF_ETYPE 1u        // BTYPE 11
#define PF_INF_ESTORED 2u      // stored block LEN/NLEN mismatch
#define PF_INF_ECODES 3u       // bad Huffman code set or an invalid code
#define PF_INF_EDIST 4u        // distance past the block's start
#define PF_INF_ESIZE 5u        // output differs from ISIZE
#define PF_INF_EINPUT 6u       // stream runs past the payload
#define PF_INF_ECRC 7u         // CRC32 mismatch
#define PF_INF_FALLBACK 100u   // (internal) a block left for inflate_blocks<true> (tools/ubench's two-pass decoder)

__global__ void pf_inflate(const uint8_t *in, const pf_bgzf_blk *blk, uint32_t nblk, uint8_t *arena,
                           uint32_t *status);

// ---- device fetch (pf_ingest.hip): runs of blocks, windows, chunks, records
typedef struct pf_run_dev {
    uint64_t a0, a1;          // the run's inflated bytes [a0, a1) in the arena
    uint64_t chain_start;     // first record start the chain walks from (min chunk start)
    uint64_t stop_pos;        // chain output: position after its last whole record
    uint32_t to_eof;          // the run ends at the file's end
    uint32_t rec0, n_rec;     // chain output: its records [rec0, rec0 + n_rec) of the record arrays
    uint32_t stop;            // chain output: PF_CHAIN_*
} pf_run_dev;
#define PF_CHAIN_END 0u        // stop_pos == a1
#define PF_CHAIN_CUT 1u        // a record (or its size field) runs past a1
#define PF_CHAIN_CORRUPT 2u    // block_size < 32 or > 2^30 at stop_pos

typedef struct pf_seg_dev {       // a piece of a run's record chain between known record starts
    uint64_t s, e;            // walk from s until e (the next known start, or the run's end a1)
    uint64_t a1;              // the run's end
    uint64_t stop_pos;        // count pass: position after its last whole record
    uint32_t run, last;       // its run; the run's last segment
    uint32_t n, stop;         // count pass: records, PF_CHAIN_*
    uint32_t rec0, live;      // write pass: first record index; 0 = past a corrupt segment
} pf_seg_dev;

typedef struct pf_chunk_dev {
    uint64_t u, v;            // arena positions of the chunk's virtual offsets
    uint32_t run, pad;
} pf_chunk_dev;

typedef struct pf_win_dev {
    int64_t beg, end;         // region [beg, end)
    uint32_t c0, c1;          // its chunks
    int32_t tid;
    uint16_t skip;            // write pass: window emptied (over the record limit)
    uint16_t reads;           // the -u pre-pass fetch: primary mapped records only, MD:Z required
    uint64_t out;             // write pass: first slot of its record list
} pf_win_dev;

// window status of the select pass
#define PF_WIN_OK 0u
#define PF_WIN_MORE 1u         // needs blocks past its run's end (host widens the plan)
#define PF_WIN_ERR 2u          // corrupt record / index offset inside a record / truncated file
#define PF_WIN_TRUNC 3u        // ended at a record whose CIGAR and SEQ lengths differ (counted, not an error)

// decoded records (SoA, indexed like the chain)
typedef struct pf_recs_dev {
    uint64_t *pos;            // arena position of the block_size field
    uint64_t *cig, *seq, *qn, *mm, *ml;     // arena positions
    uint32_t *bs, *l_qseq, *ncig, *rlen, *qn_len, *mm_len, *ml_len, *md_len, *nins;
    int32_t *tid, *rpos, *hp_tag;
    float *de;
    uint16_t *flag;
    uint8_t *mapq, *hp, *st;  // st: bit 0 corrupt, bit 1 truncated (CIGAR/SEQ length mismatch), bit 2 MD:Z present
    uint64_t *md;
} pf_recs_dev;
#define PF_REC_CORRUPT 1u
#define PF_REC_TRUNC 2u
#define PF_REC_MD 4u

__global__ void pf_chain(const uint8_t *arena, pf_seg_dev *segs, uint32_t n_segs, uint64_t *rec_pos);
__global__ void pf_recdec(const uint8_t *arena, uint32_t n_recs, pf_recs_dev R);
__global__ void pf_select(const pf_win_dev *wins, uint32_t n_wins, const pf_chunk_dev *chunks, const pf_run_dev *runs,
                          pf_recs_dev R, uint32_t write, uint32_t *win_n, uint32_t *win_st, uint32_t *out);
__global__ void pf_gather_small(const uint32_t *sel, uint64_t n, pf_recs_dev R, uint16_t *flag, uint8_t *mapq,
                                uint32_t *pos, uint32_t *l_qseq, float *de, uint8_t *hp, int32_t *hp_tag,
                                uint32_t *ncig, uint32_t *mm_len, uint32_t *ml_len, uint32_t *qn_len,
                                uint32_t *md_len, uint32_t *rlen, uint8_t *st, uint32_t *nins);
__global__ void pf_gather_big(const uint8_t *arena, const uint32_t *sel, uint64_t n, pf_recs_dev R,
                              const uint64_t *cig_off, uint32_t *cig, const uint64_t *seq_off, uint8_t *seq,
                              const uint64_t *mm_off, uint8_t *mm, const uint64_t *ml_off, uint8_t *ml,
                              const uint64_t *qn_off, uint8_t *qn, const uint64_t *md_off, uint8_t *md);

// -u reads for K4 (pf_haptag.hip): per-read host fields the cursor chain and
// scratch sizing need, and the reads' device arrays
typedef struct pf_k4_reads_host {
    const uint32_t *start, *end, *n_ins, *ncig, *md_len;
} pf_k4_reads_host;
typedef struct pf_k4_reads_dev {
    const uint32_t *start, *end;
    const uint64_t *cigar_off;
    const uint32_t *cigar;
    const uint64_t *seq_off;
    const uint32_t *seq_len;
    const uint8_t *seq;
    const uint64_t *md_off;
    const uint8_t *md;
} pf_k4_reads_dev;
#ifdef __cplusplus
struct pf_ctx;
struct pf_known_vars;
struct pf_read_aln_batch;
// prev_left: the reference's prev_i_left cursor (blockjoin.c:1716-1720) going
// in and coming out, so that a contig haptagged in pieces chains like one
// call (null: starts at 0)
int pf_haptag_core(struct pf_ctx *ctx, const struct pf_known_vars *K, uint32_t N, const pf_k4_reads_host &h,
                   const struct pf_read_aln_batch *Rb, const pf_k4_reads_dev *dv, uint8_t *hp_out,
                   uint32_t *prev_left = nullptr);
#endif
