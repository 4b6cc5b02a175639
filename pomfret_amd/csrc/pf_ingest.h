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

__global__ void pf_inflate(const uint8_t *in, const pf_bgzf_blk *blk, uint32_t nblk, uint8_t *arena,
                           uint32_t *status);
__global__ void pf_bgzf_crc(const uint8_t *arena, const pf_bgzf_blk *blk, uint32_t nblk, uint32_t *status);
