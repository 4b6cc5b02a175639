// MEASURED, NOT KEPT (round 5): pf_inflate.hip with long literal chains
// resolved by pointer jumping (INF_CHAIN; the first INF_CHAIN_WALK literals
// of a chain walked by readlane).  Build it into tools/ubench/inflate_ab as
// variant B to repeat the A/B.  profiles/r05/inflate_chain/: pure pointer
// jumping (walk 0) gave Huffman-only blocks 17.8 -> 25.5 GB/s but the
// synthetic genome BAM 21.7 -> 18.8 and BAM-like blocks 18.0 -> 16.1 (chains
// are short where matches interleave: ~10 LDS round trips per chain against a
// few scalar steps); with the walk in front, every data set is slower (the
// extra state spills).  The product keeps the readlane walk.
// pf_inflate.hip -- BGZF blocks inflated on the device (SURVEY.md 8 f1 moved
// to the GPU: host BGZF inflate bounds every run from files).
//
// A BAM file is a series of BGZF blocks, each an independent raw DEFLATE
// stream (RFC 1951) of <= 64 KiB output with its CRC32 and size in the
// footer.  htslib's bgzf_read_block inflates one block at a time and checks
// the CRC; here every block of a fetch plan is inflated at once, one
// wavefront per block, into a contiguous arena (block b's output at
// out_off[b], the prefix sum of the ISIZE fields), so the BAM byte stream of a
// run of consecutive blocks is contiguous in HBM.
//
// Decoder shape (wave64, gfx950):
//  * the whole wave runs the DEFLATE state machine in lockstep on uniform
//    values (bit buffer, output position) -- Huffman decoding is inherently
//    serial within a block, the parallelism is across blocks (thousands of
//    waves in flight);
//  * the compressed input is held lane-distributed: lane k of `cur` holds
//    dword k of the current 256-byte input window, `nxt` the next one,
//    prefetched one window ahead; the bit reader takes dwords with readlane;
//  * Huffman tables in LDS (per wave, ~4 KB): a 10-bit root table for
//    literal/length codes and an 8-bit one for distances (symbol | length << 9,
//    broadcast reads); a code longer than the root (rare) is found by all
//    code lengths tested at once, one per lane (the canonical walk's answer);
//    literal-pair root entries were tried and measured slower (few pairs fit
//    10 bits on BAM content, and the larger table costs a wave of occupancy);
//  * runs of literals and short matches are decoded speculatively: lane k
//    pre-decodes the symbol (and a match's distance) starting at bit offset k
//    of the buffered bits and the run follows the stream with readlanes;
//  * measured by SQ counters (tools/ubench/inflate_ab, BAM-like blocks): per
//    output byte 23 SALU + 21 VALU instructions and 0.5 LDS reads (35 + 25 +
//    0.9 before the speculative runs), the decode bound by scalar issue;
//  * output is assembled lane-distributed in 256-byte chunks aligned to the
//    arena (lane k holds bytes 4k..4k+3 of the chunk) and flushed with one
//    coalesced store per chunk; a match only records its bytes' sources, and
//    the chunk's flush loads every source in older output at once (after a
//    workgroup-scope fence that makes the flushed chunks visible) and resolves
//    in-chunk sources with ds_bpermute rounds;
//    11.5-13.6 GB/s of output on MI355X (8k-32k blocks);
//  * table construction is lane-parallel (counts by ballot, ranks by ballot
//    prefix, root fill one symbol per lane).
// Each block's CRC32 (reflected 0xEDB88320, zlib's crc32) is folded in at
// every chunk flush (VALU work beside the scalar decode) and checked with the
// ISIZE against the footer, as htslib does; any malformed stream, size or CRC
// mismatch sets the block's status word and the host fails the fetch.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "pf_ingest.h"

#define DEV static __device__ __forceinline__
#define INF_LROOT 10u
#define INF_DROOT 8u
#define INF_WAVES 4u
#ifndef INF_SPEC
#define INF_SPEC 1                      // literal runs decoded from every bit offset at once
#endif
#ifndef INF_SPECM
#define INF_SPECM 1                     // ... and short matches in the same run
#endif
#ifndef INF_CHAIN
#define INF_CHAIN 1                     // long literal chains resolved by pointer jumping, placed wave-wide
#endif
#ifndef INF_CHAIN_WALK
#define INF_CHAIN_WALK 4                // literals of a chain walked by readlane before the jump tables
#endif

DEV uint32_t uni(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }
DEV uint32_t rdl(uint32_t x, uint32_t l) { return (uint32_t)__builtin_amdgcn_readlane((int)x, (int)l); }
DEV uint32_t popc64(uint64_t m) { return (uint32_t)__popcll(m); }
DEV uint64_t uni64(uint64_t x) { return ((uint64_t)uni((uint32_t)(x >> 32)) << 32) | uni((uint32_t)x); }
DEV uint32_t bperm(uint32_t x, uint32_t src) {      // lane src's x (src < 64)
    return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src << 2), (int)x);
}
DEV uint32_t wave_shl1(uint32_t x) {                // lane i <- lane i + 1 (DPP wave_shl:1; lane 63 gets 0)
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x130, 0xF, 0xF, false);
}
DEV void wsync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

__constant__ uint8_t k_clord[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

struct InfLds {                         // one wave's tables
    uint16_t lroot[1u << INF_LROOT];
    union {
        uint16_t droot[1u << INF_DROOT];
        struct {                        // the code-length code: done with before droot is built
            uint16_t clroot[128];       // (max 7 bits: the root covers it)
            uint16_t cnt_cl[16], off_cl[16], fst_cl[16];
            uint16_t clsym[19];
        } cl;
    };
    uint16_t lsym[288];                 // symbols sorted by (length, value): canonical order
    uint16_t dsym[32];
    uint16_t cnt[2][16];                // codes per length (litlen, dist)
    uint16_t off[2][16];                // first sorted index of each length
    uint16_t fst[2][16];                // first canonical code of each length
    uint8_t lens[320];                  // code lengths: HLIT litlen then HDIST dist
    uint32_t ring[128];                 // input windows (bit reader)
};

// --------------------------------------------------------------------------
// bit reader over an LDS ring of two 256-byte input windows per wave: window
// j sits in slot j & 1; entering window j waits for its load (issued when
// window j-1 was entered) and issues window j+1's into the other slot with a
// direct global->LDS load, so the wait is a full window after the issue.
#define VMCNT0 0x0F70                   // s_waitcnt vmcnt(0) (gfx9 encoding, other counters at max)
struct Bits {
    uint64_t buf;
    uint32_t cnt;
    uint32_t rd;          // next dword (from the aligned base) to read
    uint32_t lim;         // dwords that may be read (payload + slack)
    uint32_t over;        // read past the payload
    const uint32_t *src;  // aligned base
    uint32_t *ring;       // 128 dwords of LDS
};

DEV void bits_issue(Bits &b, uint32_t j, uint32_t lane) {       // window j -> slot j & 1
    uint32_t k = j * 64 + lane;
    if (k >= b.lim) k = b.lim - 1;            // past the payload: any valid dword (never decoded)
    __builtin_amdgcn_global_load_lds((const void *)(b.src + k),
                                     (__attribute__((address_space(3))) void *)(b.ring + (j & 1u) * 64), 4, 0, 0);
}

DEV void bits_fill(Bits &b, uint32_t lane) {
    b.cnt = uni(b.cnt);
    b.buf = uni64(b.buf);
    b.rd = uni(b.rd);
    while (b.cnt <= 32) {
        if ((b.rd & 63u) == 0) {
            __builtin_amdgcn_s_waitcnt(VMCNT0);
            wsync();
            bits_issue(b, (b.rd >> 6) + 1, lane);
        }
        const uint32_t w = uni(b.ring[b.rd & 127u]);
        b.buf |= (uint64_t)w << b.cnt;
        b.cnt += 32;
        b.rd++;
        if (b.rd > b.lim) b.over = 1;
    }
}
DEV uint32_t bits_take(Bits &b, uint32_t n) {      // n < 32, after a fill covering it
    const uint32_t v = (uint32_t)b.buf & ((1u << n) - 1u);
    b.buf >>= n;
    b.cnt -= n;
    return v;
}
DEV uint32_t bits_get(Bits &b, uint32_t n) {       // n <= 32, after a fill covering it
    const uint32_t v = (uint32_t)b.buf & (n >= 32 ? 0xFFFFFFFFu : ((1u << n) - 1u));
    b.buf >>= n;
    b.cnt -= n;
    return v;
}

// --------------------------------------------------------------------------
// table construction.  lens[0..n) -> per-length counts, sorted symbols and a
// root table of `root` bits indexed by the bit-reversed code.  Returns 0 on
// success, 1 for an over-subscribed set or an incomplete one (zlib's
// inflate_table: incomplete only for a single length-1 code, never for the
// code-length code; an empty set builds a table every lookup of which fails).
template <typename E>
DEV uint32_t build_table(const uint8_t *lens, uint32_t n, uint32_t root, E *rt, uint16_t *sym,
                         uint16_t *cnt, uint16_t *off, uint16_t *fst, uint32_t lane, bool is_codes) {
    // counts per length (uniform, 15 ballots per 64 symbols)
    uint32_t c[16];
#pragma unroll
    for (uint32_t L = 0; L < 16; L++) c[L] = 0;
    for (uint32_t s0 = 0; s0 < n; s0 += 64) {
        const uint32_t s = s0 + lane;
        const uint32_t l = s < n ? lens[s] : 0u;
#pragma unroll
        for (uint32_t L = 1; L < 16; L++) c[L] += (uint32_t)__popcll(__ballot(l == L));
    }
    uint32_t maxl = 0;
    int32_t left = 1;
    bool bad = false;
#pragma unroll
    for (uint32_t L = 1; L < 16; L++) {
        left <<= 1;
        left -= (int32_t)c[L];
        if (left < 0) bad = true;
        if (c[L]) maxl = L;
    }
    if (bad) return 1;
    if (maxl != 0 && left > 0 && (is_codes || maxl != 1)) return 1;
    // offsets and first codes
    uint32_t o[16], first[16];
    o[0] = 0; o[1] = 0;
    first[0] = 0;
    uint32_t code = 0;
#pragma unroll
    for (uint32_t L = 1; L < 16; L++) {
        code = (code + (L > 1 ? c[L - 1] : 0u)) << 1;
        first[L] = code;
        if (L > 1) o[L] = o[L - 1] + c[L - 1];
    }
    if (lane < 16) { cnt[lane] = 0; off[lane] = 0; fst[lane] = 0; }
    wsync();
#pragma unroll
    for (uint32_t L = 1; L < 16; L++)
        if (lane == L) { cnt[lane] = (uint16_t)c[L]; off[lane] = (uint16_t)o[L]; fst[lane] = (uint16_t)first[L]; }
    // clear the root table
    const uint32_t rn = 1u << root;
    for (uint32_t i = lane; i < rn; i += 64) rt[i] = 0;
    wsync();
    // ranks within each length, in symbol order: sorted symbols + root entries
    uint32_t base[16];
#pragma unroll
    for (uint32_t L = 0; L < 16; L++) base[L] = 0;
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    for (uint32_t s0 = 0; s0 < n; s0 += 64) {
        const uint32_t s = s0 + lane;
        const uint32_t l = s < n ? lens[s] : 0u;
        uint32_t rank = 0, fc = 0, ol = 0;
#pragma unroll
        for (uint32_t L = 1; L < 16; L++) {
            const uint64_t m = __ballot(l == L);
            if (l == L) { rank = base[L] + (uint32_t)__popcll(m & lt); fc = first[L]; ol = o[L]; }
            base[L] += (uint32_t)__popcll(m);
        }
        if (l) {
            sym[ol + rank] = (uint16_t)s;
            if (l <= root) {
                const uint32_t cd = fc + rank;
                const uint32_t rev = __builtin_bitreverse32(cd) >> (32 - l);
                const E e = (E)(s | (l << 9));
                for (uint32_t k = 0; k < (1u << (root - l)); k++) rt[rev | (k << l)] = e;
            }
        }
    }
    wsync();
    return 0;
}

// canonical decode of a code longer than the root (or any code, from bit 0):
// lane L tests whether the next L bits, read as a code, fall in length L's
// range [fst[L], fst[L] + cnt[L]); the shortest such length is the code's
// (the serial canonical walk's answer, all lengths at once)
DEV uint32_t slow_decode(uint64_t bits, const uint16_t *cnt, const uint16_t *off, const uint16_t *fst,
                         const uint16_t *sym, uint32_t lane, uint32_t &len_out) {
    const uint32_t L = lane & 15u;
    const uint32_t c = cnt[L], f = fst[L], o = off[L];
    const uint32_t code = L ? __builtin_bitreverse32((uint32_t)bits) >> (32 - L) : 0u;
    const uint64_t m = __ballot(lane >= 1 && lane < 16 && code - f < c);
    if (!m) { len_out = 0; return 0xFFFFu; }
    const uint32_t Ls = (uint32_t)__builtin_ctzll(m);
    len_out = Ls;
    return sym[rdl(o + code - f, Ls)];
}

// --------------------------------------------------------------------------
// output: 256-byte chunks aligned to the arena, lane k holds bytes 4k..4k+3.
// A literal sets its byte; a match only records, per byte it covers, the
// source offset (block-relative).  At the chunk's flush every byte sourced
// from older output is loaded at once (one memory round trip per chunk, not
// per match), then bytes sourced inside the chunk are resolved in rounds of
// ds_bpermute (a source always precedes its byte, so every round resolves at
// least the earliest pending byte), and the chunk is stored.
// CRC32 (reflected 0xEDB88320, zlib's crc32) in raw form (init 0, no final
// xor): raw(A || B) = raw(A) * x^(8|B|) ^ raw(B) in GF(2)[x] mod P, and
// leading zero bytes leave a raw CRC unchanged.  crc32(M) = ~(raw(M) ^
// ~0 * x^(8|M|)).
DEV uint32_t gf_mul(uint32_t a, uint32_t b) {      // reflected, x^0 = 0x80000000 (zlib's multmodp)
    uint32_t p = 0;
#pragma unroll
    for (int i = 0; i < 32; i++) {
        p ^= (a & 0x80000000u) ? b : 0u;
        a <<= 1;
        b = (b & 1u) ? (b >> 1) ^ 0xEDB88320u : b >> 1;
    }
    return p;
}
DEV uint32_t x8n(uint64_t n, const uint32_t *x2n) {  // x^(8n) mod P; x2n[k] = x^(2^k)
    uint32_t p = 0x80000000u;
    uint64_t e = n << 3;
    for (uint32_t k = 0; e; k++, e >>= 1)
        if (e & 1u) p = gf_mul(p, x2n[k & 31u]);
    return p;
}

struct Out {               // positions are 32-bit, relative to base (scalar registers are scarce)
    uint8_t *base;        // the arena's 256-byte chunk holding the block's first byte
    uint32_t lo, hi;      // the block's output range [lo, hi), lo < 256
    uint32_t cb;          // current chunk
    uint32_t a;           // next output position
    uint32_t val;         // per lane: resolved bytes
    uint32_t pend;        // per lane: bit i set while byte i waits for its source
    uint32_t src[4];      // per lane: source position of pending byte i
    uint32_t any;         // uniform: the chunk has pending bytes
    uint32_t crc;         // uniform: raw CRC of the flushed chunks
    uint32_t ck;          // per lane: x^(8 * (252 - 4 lane)), its word's weight in a full chunk
    const uint32_t *tab;  // CRC table (LDS)
    const uint32_t *x2n;  // x^(2^k) (LDS)
};

// fold a chunk's resolved bytes into the block CRC: m = bytes of the chunk
// that belong to the block's stream (256, or the last chunk's length); bytes
// before the block's start are zero (leading zeros)
DEV void out_crc(Out &o, uint32_t lane, uint32_t m) {
    const uint32_t nv = m > 4 * lane ? (m - 4 * lane < 4 ? m - 4 * lane : 4u) : 0u;   // this lane's bytes
    uint32_t c = 0;
#pragma unroll
    for (uint32_t i = 0; i < 4; i++)
        if (i < nv) c = o.tab[(c ^ (o.val >> (8 * i))) & 0xFFu] ^ (c >> 8);
    uint32_t wgt = o.ck;
    if (m != 256) {                                     // weight of this lane's bytes: x^(8 (m - 4 lane - nv))
        const uint32_t e = nv ? m - 4 * lane - nv : 0u;
        wgt = x8n(e, o.x2n);
    }
    c = nv ? gf_mul(c, wgt) : 0u;
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1) c ^= (uint32_t)__shfl_xor((int)c, s, 64);
    o.crc = gf_mul(o.crc, m == 256 ? o.x2n[11] : x8n(m, o.x2n)) ^ uni(c);
}

DEV void out_flush(Out &o, uint32_t lane) {
    if (o.any) {
        // sources in flushed chunks: make their stores visible, load all at once
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        uint32_t add = 0, done = 0;
#pragma unroll
        for (uint32_t i = 0; i < 4; i++) {
            const uint32_t s = o.src[i];
            if (((o.pend >> i) & 1u) && s < o.cb) {
                add |= (uint32_t)o.base[s] << (8 * i);
                done |= 1u << i;
            }
        }
        o.val |= add;
        o.pend &= ~done;
        while (__ballot(o.pend != 0)) {
            const uint32_t v_all = o.val, r_all = ~o.pend & 0xFu;
            uint32_t nv = o.val, np = o.pend;
#pragma unroll
            for (uint32_t i = 0; i < 4; i++) {
                const bool pi = (o.pend >> i) & 1u;
                const uint32_t t = pi ? o.src[i] - o.cb : 4 * lane + i;
                const uint32_t w = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((t >> 2) << 2), (int)v_all);
                const uint32_t r = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((t >> 2) << 2), (int)r_all);
                if (pi && ((r >> (t & 3u)) & 1u)) {
                    nv |= ((w >> (8 * (t & 3u))) & 0xFFu) << (8 * i);
                    np &= ~(1u << i);
                }
            }
            o.val = nv;
            o.pend = np;
        }
    }
    out_crc(o, lane, o.a >= o.cb + 256 ? 256u : o.a - o.cb);
    const uint32_t addr = o.cb + 4 * lane;
    if (addr >= o.lo && addr + 4 <= o.hi && addr + 4 <= o.a) {
        *reinterpret_cast<uint32_t *>(o.base + addr) = o.val;
    } else {
#pragma unroll
        for (uint32_t i = 0; i < 4; i++) {
            const uint32_t q = addr + i;
            if (q >= o.lo && q < o.hi && q < o.a) o.base[q] = (uint8_t)(o.val >> (8 * i));
        }
    }
    o.cb += 256;
    o.val = 0;
    o.pend = 0;
    o.any = 0;
}

DEV void out_lit(Out &o, uint32_t v, uint32_t lane) {
    const uint32_t rel = o.a - o.cb;
    const uint32_t add = v << (8 * (rel & 3u));
    o.val |= lane == (rel >> 2) ? add : 0u;              // a select, not an exec-mask branch
    o.a++;
    if (rel == 255) out_flush(o, lane);
}

// n literal bytes (lane i holds byte i of the run, i < n) at the output
// position: one gather of 4-byte words per chunk the run touches (lane t's
// word covers chunk positions 4t..4t+3), a flush at each full chunk.  The
// bytes of the chunk at and past o.a are still zero (the chunk is built in
// order), so the words are OR-ed in.
DEV void out_lits(Out &o, uint32_t bl, uint32_t n, uint32_t lane) {
    const uint32_t s1 = wave_shl1(bl), s2 = wave_shl1(s1), s3 = wave_shl1(s2);
    const uint32_t wv = (bl & 0xFFu) | ((s1 & 0xFFu) << 8) | ((s2 & 0xFFu) << 16) | (s3 << 24);
    uint32_t done = 0;
    while (done < n) {
        const uint32_t r = o.a - o.cb;                   // chunk position of byte `done`
        const uint32_t take = min(n - done, 256u - r);
        const int sidx = (int)(4 * lane) - (int)r + (int)done;   // run byte at this lane's first position
        const uint32_t g = bperm(wv, (uint32_t)min(max(sidx, 0), 63));
        const uint32_t v = sidx >= 0 ? g : sidx >= -3 ? g << (8 * (uint32_t)(-sidx)) : 0u;
        // this lane's positions inside [r, r + take)
        const int lo = max(0, (int)r - (int)(4 * lane)), hi = min(4, (int)(r + take) - (int)(4 * lane));
        const uint32_t mhi = hi >= 4 ? 0xFFFFFFFFu : hi <= 0 ? 0u : (1u << (8 * hi)) - 1u;
        const uint32_t mlo = lo >= 4 ? 0u : ~((1u << (8 * lo)) - 1u);
        o.val |= v & mhi & mlo;
        o.a += take;
        done += take;
        if (o.a - o.cb == 256) out_flush(o, lane);
    }
}

// copy L bytes from distance D (D <= bytes already written, checked by the caller)
DEV void out_match(Out &o, uint32_t L, uint32_t D, uint32_t lane) {
    const uint32_t ms = o.a, me = o.a + L;
    while (o.a < me) {
        const uint32_t seg_end = me < o.cb + 256 ? me : o.cb + 256;
        uint32_t setp = 0;
        // (selects, not exec-mask branches: the scalar unit is the bottleneck)
        if (D < L) {                                     // overlapping copy: the source repeats with period D
#pragma unroll
            for (uint32_t i = 0; i < 4; i++) {
                const uint32_t q = o.cb + 4 * lane + i;
                const bool in = q >= o.a && q < seg_end;
                o.src[i] = in ? ms - D + (q - ms) % D : o.src[i];
                setp |= in ? 1u << i : 0u;
            }
        } else {
#pragma unroll
            for (uint32_t i = 0; i < 4; i++) {
                const uint32_t q = o.cb + 4 * lane + i;
                const bool in = q >= o.a && q < seg_end;
                o.src[i] = in ? q - D : o.src[i];
                setp |= in ? 1u << i : 0u;
            }
        }
        o.pend |= setp;
        o.any = 1;
        o.a = seg_end;
        if (seg_end == o.cb + 256) out_flush(o, lane);
    }
}

// --------------------------------------------------------------------------
#ifndef INF_WPE
#define INF_WPE 8                       // waves per SIMD the register allocation aims at
#endif
template <bool FALLBACK_ONLY>
DEV void inflate_blocks(const uint8_t *in, const pf_bgzf_blk *blk, uint32_t nblk, uint8_t *arena, uint32_t *status) {
    __shared__ InfLds lds_all[INF_WAVES];
    __shared__ uint32_t crc_tab[256], crc_x2n[32];
    if (FALLBACK_ONLY) {                            // (uniform per workgroup: skip the setup when nothing is flagged)
        const uint32_t b0 = blockIdx.x * INF_WAVES;
        bool any = false;
        for (uint32_t k = 0; k < INF_WAVES && b0 + k < nblk; k++) any |= status[b0 + k] == PF_INF_FALLBACK;
        if (!any) return;
    }
    for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x) {
        uint32_t c = i;
        for (int k = 0; k < 8; k++) c = (c & 1u) ? (c >> 1) ^ 0xEDB88320u : c >> 1;
        crc_tab[i] = c;
    }
    if (threadIdx.x == 0) {
        uint32_t p = 0x40000000u;                     // x^1
        for (int k = 0; k < 32; k++) { crc_x2n[k] = p; p = gf_mul(p, p); }
    }
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wv = uni(threadIdx.x >> 6);
    const uint32_t bi = blockIdx.x * INF_WAVES + wv;
    if (bi >= nblk) return;
    if (FALLBACK_ONLY && uni(status[bi]) != PF_INF_FALLBACK) return;
    InfLds &T = lds_all[wv];
    const pf_bgzf_blk B = blk[bi];
    const uint64_t in_off = B.in_off;
    const uint32_t in_len = B.in_len, isize = B.isize;

    Bits b;
    b.src = reinterpret_cast<const uint32_t *>(in + (in_off & ~3ull));
    b.lim = (uint32_t)(((in_off & 3u) + in_len + 3) >> 2) + 2;     // + slack: the reader peeks ahead
    b.rd = 0;
    b.over = 0;
    b.ring = T.ring;
    bits_issue(b, 0, lane);
    b.buf = 0;
    b.cnt = 0;
    bits_fill(b, lane);
    if ((in_off & 3u) != 0) bits_get(b, 8 * (uint32_t)(in_off & 3u));

    Out o;
    o.base = arena + (B.out_off & ~255ull);
    o.lo = (uint32_t)(B.out_off & 255u);
    o.hi = o.lo + isize;
    o.cb = 0;
    o.a = o.lo;
    o.val = 0;
    o.pend = 0;
    o.any = 0;
#pragma unroll
    for (uint32_t i = 0; i < 4; i++) o.src[i] = 0;
    o.crc = 0;
    o.tab = crc_tab;
    o.x2n = crc_x2n;
    o.ck = x8n(252 - 4 * lane, crc_x2n);

    uint32_t err = 0, final_blk = 0;
    while (!final_blk && !err) {
        err = uni(err);
        final_blk = uni(final_blk);
        bits_fill(b, lane);
        final_blk = bits_get(b, 1);
        const uint32_t type = bits_get(b, 2);
        if (type == 0) {                                   // stored
            bits_get(b, b.cnt & 7u);
            bits_fill(b, lane);
            const uint32_t len = bits_get(b, 16), nlen = bits_get(b, 16);
            if ((len ^ 0xFFFFu) != nlen) { err = PF_INF_ESTORED; break; }
            if (o.a + len > o.hi) { err = PF_INF_ESIZE; break; }
            for (uint32_t i = 0; i < len; i++) {
                bits_fill(b, lane);
                out_lit(o, bits_get(b, 8), lane);
            }
            if (b.over) { err = PF_INF_EINPUT; break; }
            continue;
        }
        if (type == 3) { err = PF_INF_ETYPE; break; }
        uint32_t nlit = 288, ndist = 32;
        if (type == 1) {                                   // fixed codes
            for (uint32_t s = lane; s < 320; s += 64)
                T.lens[s] = (uint8_t)(s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : s < 288 ? 8 : 5);
            wsync();
        } else {                                           // dynamic: code lengths first
            bits_fill(b, lane);
            nlit = bits_get(b, 5) + 257;
            ndist = bits_get(b, 5) + 1;
            const uint32_t ncl = bits_get(b, 4) + 4;
            if (nlit > 286 || ndist > 30) { err = PF_INF_ECODES; break; }
            uint64_t clbits = 0;                           // up to 19 x 3 bits
            bits_fill(b, lane);
            const uint32_t n1 = ncl < 10 ? ncl : 10;
            clbits = bits_get(b, 3 * n1);
            if (ncl > 10) { bits_fill(b, lane); clbits |= (uint64_t)bits_get(b, 3 * (ncl - 10)) << 30; }
            if (lane < 19) {
                uint32_t l = 0;
                for (uint32_t j = 0; j < ncl; j++)
                    if (k_clord[j] == lane) l = (uint32_t)(clbits >> (3 * j)) & 7u;
                T.lens[lane] = (uint8_t)l;
            }
            wsync();
            if (build_table(T.lens, 19, 7, T.cl.clroot, T.cl.clsym, T.cl.cnt_cl, T.cl.off_cl, T.cl.fst_cl, lane, true)) {
                err = PF_INF_ECODES;
                break;
            }
            // the litlen + dist code lengths (serial, uniform): litlen at
            // lens[0..nlit), dist at lens[288..288+ndist), the rest 0
            const uint32_t total = nlit + ndist;
            uint32_t i = 0, prev = 0;
            for (uint32_t q = lane; q < 320; q += 64) T.lens[q] = 0;
            wsync();
            while (i < total) {
                bits_fill(b, lane);
                const uint32_t e = uni(T.cl.clroot[(uint32_t)b.buf & 127u]);   // (no pairs in this table)
                const uint32_t l = e >> 9, s = e & 511u;
                if (l == 0) { err = PF_INF_ECODES; break; }
                bits_get(b, l);
                uint32_t rep = 1, val = s;
                if (s == 16) {
                    if (i == 0) { err = PF_INF_ECODES; break; }
                    rep = 3 + bits_get(b, 2);
                    val = prev;
                } else if (s == 17) {
                    rep = 3 + bits_get(b, 3);
                    val = 0;
                } else if (s == 18) {
                    rep = 11 + bits_get(b, 7);
                    val = 0;
                }
                if (i + rep > total) { err = PF_INF_ECODES; break; }
                if (val)
                    for (uint32_t j = lane; j < rep; j += 64) {
                        const uint32_t q = i + j;
                        T.lens[q < nlit ? q : 288 + q - nlit] = (uint8_t)val;
                    }
                i += rep;
                prev = val;
                if (b.over) { err = PF_INF_EINPUT; break; }
            }
            if (err) break;
            wsync();
            if (T.lens[256] == 0) { err = PF_INF_ECODES; break; }   // no end-of-block code
        }
        if (build_table(T.lens, nlit, INF_LROOT, T.lroot, T.lsym, T.cnt[0], T.off[0], T.fst[0], lane, false) ||
            build_table(T.lens + 288, ndist, INF_DROOT, T.droot, T.dsym, T.cnt[1], T.off[1], T.fst[1], lane, false)) {
            err = PF_INF_ECODES;
            break;
        }
        // ---- the block's symbols
        for (;;) {
            bits_fill(b, lane);
#if INF_SPEC
            // a run of literals: lane k looks up the root entry at bit offset
            // k of the buffered bits (a literal whose code lies inside them
            // is kept), then the run follows offsets 0, l0, l0 + l1, ... with
            // one readlane per literal; the first symbol that is not such a
            // literal goes to the general step below.  Matches with a length
            // code without extra bits join the run (INF_SPECM, +12.6 %).
            {
                const uint32_t ek = T.lroot[(uint32_t)(b.buf >> lane) & ((1u << INF_LROOT) - 1u)];
                const uint32_t lk = ek >> 9, sk = ek & 511u;
                const uint32_t lit = (lk != 0 && sk < 256 && lane + lk <= b.cnt) ? (sk | (lk << 8)) : 0u;
                uint32_t off = 0;
#if INF_SPECM
                // lane k also pre-decodes a length code without extra bits
                // (L | code length << 8) and a whole distance (D | its bits << 16)
                // at offset k, all in VALU; the run takes a match with three
                // readlanes
                const uint32_t mlen = (lk != 0 && sk >= 257 && sk <= 264 && lane + lk <= b.cnt)
                                          ? (sk - 254) | (lk << 8) : 0u;
                uint32_t dval = 0;
                {
                    const uint32_t dk = T.droot[(uint32_t)(b.buf >> lane) & ((1u << INF_DROOT) - 1u)];
                    const uint32_t dl = dk >> 9, ds = dk & 511u;
                    const uint32_t dx = ds < 4 ? 0u : (ds - 2) >> 1;
                    const uint32_t p = lane + dl;
                    if (dl != 0 && ds < 30 && p + dx <= b.cnt) {
                        const uint32_t ex = dx ? (uint32_t)(b.buf >> p) & ((1u << dx) - 1u) : 0u;
                        const uint32_t D = (ds < 4 ? 1 + ds : ((2 + (ds & 1u)) << dx) + 1) + ex;
                        dval = D | ((dl + dx) << 16);
                    }
                }
#endif
                if (o.hi - o.a >= 64) {                  // room for any run of literals (<= 64)
#if INF_CHAIN
                    // Literal chains past INF_CHAIN_WALK literals by pointer
                    // jumping (the scalar unit, shared by the CU's waves, bounds
                    // the decoder: ~12 scalar instructions per literal in the
                    // readlane walk; a chain resolved wave-wide costs ~10 LDS
                    // round trips, so short chains -- matches interleave with
                    // literals in BAM content -- keep the walk): J_b[k] = the
                    // offset 2^b literals after offset k (64: the chain ends),
                    // built on first use in this fill; lane i of a chain from
                    // `off` finds its literal's offset from the bits of i.
                    uint32_t j0 = 64u, j1 = 64u, j2 = 64u, j3 = 64u, j4 = 64u, j5 = 64u;
                    uint32_t jt = 0, walked = 0;
                    auto jump = [&](uint32_t J) { const uint32_t y = bperm(J, min(J, 63u)); return J < 64u ? y : 64u; };
                    while (off < 64) {
                        const uint32_t x = rdl(lit, off);
                        if (x && walked < INF_CHAIN_WALK) {
                            out_lit(o, x & 255u, lane);
                            off += x >> 8;
                            walked++;
                            continue;
                        }
                        if (x) {
                            if (jt == 0) {
                                j0 = lit ? lane + (lit >> 8) : 64u;
                                j1 = jump(j0); j2 = jump(j1); j3 = jump(j2);
                                jt = 1;
                            }
                            auto hop = [&](uint32_t q, uint32_t J, uint32_t bit) {
                                const uint32_t y = bperm(J, min(q, 63u));
                                return ((lane >> bit) & 1u) ? (q < 64u ? y : 64u) : q;
                            };
                            uint32_t q = hop(hop(hop(hop(off, j0, 0), j1, 1), j2, 2), j3, 3);
                            if (rdl(q, 15) < 64u) {             // a chain past 16 literals (short codes)
                                if (jt == 1) { j4 = jump(j3); j5 = jump(j4); jt = 2; }
                                q = hop(hop(q, j4, 4), j5, 5);
                            } else q = lane < 16 ? q : 64u;     // (lanes 16+ took only the hops of bits 0-3)
                            // the chain: the offsets below 64 holding a literal -- a prefix of
                            // the lanes (the step from a non-literal offset is 64)
                            const uint32_t lq = bperm(lit, min(q, 63u));
                            const uint32_t n = popc64(__ballot(q < 64u && lq != 0u));
                            const uint32_t e = rdl(q + (lq >> 8), n - 1);   // the offset after the chain
                            out_lits(o, lq, n, lane);
                            off = e;
                            if (off >= 64) break;
                        }
                        walked = 0;
#else
                    while (off < 64) {
                        const uint32_t x = rdl(lit, off);
                        if (x) {
                            out_lit(o, x & 255u, lane);
                            off += x >> 8;
                            continue;
                        }
#endif
#if INF_SPECM
                        const uint32_t m = rdl(mlen, off);
                        if (!m) break;
                        const uint32_t q = off + (m >> 8);
                        if (q >= 64) break;
                        const uint32_t dv = rdl(dval, q);
                        if (!dv) break;
                        const uint32_t L = m & 255u, D = dv & 0xFFFFu;
                        if (D > o.a - o.lo || o.a + L > o.hi) break;
                        out_match(o, L, D, lane);
                        off = q + (dv >> 16);
#else
                        break;
#endif
                    }
                } else {
                    while (off < 64) {
                        const uint32_t x = rdl(lit, off);
                        if (!x || o.a >= o.hi) break;    // (a full output is flagged by the general step)
                        out_lit(o, x & 255u, lane);
                        off += x >> 8;
                    }
                }
                if (off) {
                    b.buf = off >= 64 ? 0ull : b.buf >> off;
                    b.cnt -= off;
                    bits_fill(b, lane);
                }
            }
#endif
            uint32_t e = uni(T.lroot[(uint32_t)b.buf & ((1u << INF_LROOT) - 1u)]);
            uint32_t l = e >> 9, s = e & 511u;
            if (l == 0) {
                s = slow_decode(b.buf, T.cnt[0], T.off[0], T.fst[0], T.lsym, lane, l);
                s = uni(s);
                l = uni(l);
                if (l == 0) { err = PF_INF_ECODES; break; }
            }
            bits_get(b, l);
            if (s < 256) {
                if (o.a >= o.hi) { err = PF_INF_ESIZE; break; }
                out_lit(o, s, lane);
                continue;
            }
            if (s == 256) break;
            const uint32_t li = s - 257;
            if (li >= 29) { err = PF_INF_ECODES; break; }
            // length base / extra bits (RFC 1951 3.2.5) by arithmetic: a table
            // lookup would be a memory load on the decode chain
            uint32_t L;
            if (li < 8) L = 3 + li;                      // no extra bits (the short matches of BAM content)
            else if (li == 28) L = 258;
            else {
                const uint32_t lx = (li - 4) >> 2;
                L = ((4 + (li & 3u)) << lx) + 3 + bits_take(b, lx);
            }
            bits_fill(b, lane);
            e = uni(T.droot[(uint32_t)b.buf & ((1u << INF_DROOT) - 1u)]);
            l = e >> 9;
            s = e & 511u;
            if (l == 0) {
                s = slow_decode(b.buf, T.cnt[1], T.off[1], T.fst[1], T.dsym, lane, l);
                s = uni(s);
                l = uni(l);
                if (l == 0) { err = PF_INF_ECODES; break; }
            }
            bits_get(b, l);
            if (s >= 30) { err = PF_INF_ECODES; break; }
            uint32_t D;
            if (s < 4) D = 1 + s;
            else {
                const uint32_t dx = (s - 2) >> 1;
                D = ((2 + (s & 1u)) << dx) + 1 + bits_take(b, dx);
            }
            if (D > o.a - o.lo) { err = PF_INF_EDIST; break; }
            if (o.a + L > o.hi) { err = PF_INF_ESIZE; break; }
            out_match(o, L, D, lane);
            if (b.over) { err = PF_INF_EINPUT; break; }
        }
        if (b.over && !err) err = PF_INF_EINPUT;
    }
    if (!err && o.a != o.hi) err = PF_INF_ESIZE;
    // the partial last chunk (bytes below o.a only)
    if (o.a > o.cb) out_flush(o, lane);
    // CRC32 of the output against the footer (bgzf_uncompress's check)
    if (!err && ~(o.crc ^ gf_mul(0xFFFFFFFFu, x8n(isize, crc_x2n))) != B.crc) err = PF_INF_ECRC;
    if (lane == 0) status[bi] = err;
}

__global__ __launch_bounds__(64 * INF_WAVES) __attribute__((amdgpu_waves_per_eu(INF_WPE, INF_WPE))) void pf_inflate(
    const uint8_t *in, const pf_bgzf_blk *blk, uint32_t nblk, uint8_t *arena, uint32_t *status) {
    inflate_blocks<false>(in, blk, nblk, arena, status);
}

