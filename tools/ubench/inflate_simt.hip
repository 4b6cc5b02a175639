// inflate_simt.hip -- (experiment, not in the product build: measured slower
// than pf_inflate) BGZF inflate in two passes: one LANE per block for
// the Huffman decode, one workgroup per block for the LZ77 copies.
//
// pf_inflate (pf_inflate.hip) runs one wavefront per block with the whole
// wave stepping the DEFLATE state machine on uniform values: every symbol
// costs a chain of scalar instructions, and the scalar unit of a CU, shared
// by all its waves, bounds the rate (23 SALU per output byte, round 2).  Here
// the serial part -- the Huffman decode, inherently one symbol after another
// within a block -- runs one block per lane, in vector registers, 64 blocks
// per wave: the per-symbol chain is ~80 VALU instructions shared by 64
// blocks instead of ~40 scalar ones for one.  The decode emits tokens, not
// bytes; the byte work (match copies, CRC, the store) is data-parallel and
// goes to a second kernel where 256 threads own one block:
//
//  pf_inflate_tok  (64 threads = one wave per workgroup, lane i = block 64g+i)
//    * per-lane bit reader: a 64-bit buffer fed from the lane's own compressed
//      stream by 8-byte loads, one kept in flight ahead;
//    * per-lane Huffman tables in LDS, lane-interleaved (entry e of lane l at
//      [e * 64 + l], so a wave's 64 lookups fall in distinct dwords of at most
//      two banks' worth each): a 2^SI_LR root for literal/length codes and a
//      2^SI_DR root for distances (u16 = symbol | length << 9); a longer code
//      (rare) is decoded canonically from the block's per-length counts and
//      sorted symbols kept in a per-block global scratch (SiScr);
//    * tables are built per lane (counts packed 16 bits per length in four
//      u64s, root entries filled symbol by symbol); the dynamic headers of
//      zlib streams fall on the same symbol count in every block (a new
//      deflate block every 16383 symbols), so the 64 lanes of a wave build
//      together;
//    * tokens (u32): literal runs of 1-3 bytes (bit 31 clear, count in bits
//      24-25, bytes in 0-23) and matches (bit 31, length - 3 in bits 16-23,
//      distance - 1 in 0-15), queued four per lane and stored as one 16-byte
//      write; per 4096-byte output chunk the first token that covers it
//      (index | start offset << 17) for the second pass.
//  pf_inflate_lz   (256 threads per block)
//    * per 4096-byte chunk: the chunk's tokens, their starts by a block scan,
//      each byte's token by a max-scan of the token starts, the literal bytes
//      placed, match bytes whose source lies in an earlier chunk copied at
//      once from the LDS image of the block, the rest (sources inside the
//      chunk) resolved by pointer jumping (a byte's source always precedes
//      it: log2(chain) rounds);
//    * CRC32 of the block (256 slices combined in GF(2), zlib's polynomial)
//      against the footer, then the block image stored with 16-byte writes.
// Status codes are pf_inflate's (pf_ingest.h); a block that fails in the
// first pass is skipped by the second.  A block whose literal/length tree has
// more long codes than the LDS list holds (SI_LCAP; never seen on BAM data)
// is flagged PF_INF_FALLBACK and decoded by pf_inflate_fallback instead.
// the two-pass inflate's launch layout (was pf_ingest.h): token area of block
// i of a launch: u32 index ((out_off - out_base) & ~3) + 4 i
#ifndef PF_SI_META
#define PF_SI_META 20u                  // u32 per block of the meta array
#define PF_SI_SCR 1152u                 // bytes per block of the first pass's scratch
#endif
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "pf_ingest.h"

#define DEV static __device__ __forceinline__

#ifndef SI_LR
#define SI_LR 9u                       // literal/length root bits
#endif
#ifndef SI_DR
#define SI_DR 7u                       // distance root bits (>= 7: the code-length code is built there)
#endif
#ifndef SI_LCAP
#define SI_LCAP 128u                   // litlen symbols of codes longer than the root kept in LDS per lane
#endif
#ifndef SI_DCAP
#define SI_DCAP 32u                    // ... distance symbols (all of them)
#endif
#define SI_LN (1u << SI_LR)
#define SI_DN (1u << SI_DR)
#define SI_NLL (15u - SI_LR)           // long litlen code lengths SI_LR+1 .. 15
#define SI_NDL (15u - SI_DR)
#define SI_CH 4096u                    // output chunk of the second pass
#define SI_META 20u                    // u32 per block: token count, then the 16 chunk entries

struct SiScr {                         // per-block scratch of the first pass (global)
    uint8_t lens[320];                 // code lengths: litlen at 0..287, dist at 288..319
    uint8_t pad[832];                  // (keeps the per-block stride at PF_SI_SCR)
};

__constant__ uint8_t si_clord[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// --------------------------------------------------------------------------
// per-lane bit reader: a 64-bit buffer fed from a per-lane ring of 16-byte
// chunks in LDS (row r = chunk c with c % SI_RS == r, lane l's 16 bytes at
// [r * 256 + 4 l] dwords).  The ring is refilled by LDS-DMA (global_load_lds,
// 16 bytes per lane, one instruction per row: a masked lane keeps its slot),
// every SI_RP symbols, after a vmcnt(0) that retires the previous refill: a
// refill runs 16 * SI_RS - 96 bits ahead of the reader, so the HBM latency
// hides behind the symbols in between and no load result is ever waited for
// at the point of use (a register double buffer had the compiler wait for
// each load where the loop merges it).
#ifndef SI_RS
#define SI_RS 16u                      // ring rows (16 bytes per lane each)
#endif
#ifndef SI_RP
#define SI_RP 8u                       // symbols between refills (<= 48 bits each)
#endif
typedef __attribute__((address_space(3))) void lds_void;

struct LBits {
    const uint8_t *base;               // 16-byte aligned start of the lane's stream
    uint64_t buf;
    uint32_t cnt;                      // valid bits in buf
    uint32_t rd;                       // next dword of the stream to read
    uint32_t ld;                       // next 16-byte chunk to load into the ring
    uint32_t end;                      // rd past this: the stream over-ran its payload
    uint32_t nchunk;                   // chunks that may be loaded (payload + slack)
};

DEV uint32_t ring_read(const uint32_t *ring, uint32_t i) {
    // the compiler counts an LDS-DMA as a pending write to its array and
    // would wait vmcnt(0) before every read of it (draining the refill in
    // flight); the refill protocol already orders these reads
    uint32_t w;
    const uint32_t a = (uint32_t)(uintptr_t)(ring + i);
    asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(w) : "v"(a) : "memory");
    return w;
}

DEV void lb_fill(LBits &b, const uint32_t *ring, uint32_t lane) {   // afterwards cnt >= 33
    if (b.cnt <= 32) {
        const uint32_t w = ring_read(ring, ((b.rd >> 2) & (SI_RS - 1)) * 256 + lane * 4 + (b.rd & 3u));
        b.buf |= (uint64_t)w << b.cnt;
        b.cnt += 32;
        b.rd++;
    }
}

DEV uint32_t lb_take(LBits &b, uint32_t n) {     // n <= 32 bits, covered by cnt
    const uint32_t v = (uint32_t)(b.buf & (((uint64_t)1 << n) - 1));
    b.buf >>= n;
    b.cnt -= n;
    return v;
}

// wait for the previous refill, then load every free slot of the active
// lanes (chunks ld .. rd/4 + SI_RS - 1); rows visited twice in order so a
// lane's run of free slots wraps
DEV void lb_refill(LBits &b, uint32_t *ring, bool active) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    for (uint32_t pass = 0; pass < 2; pass++)
        for (uint32_t r = 0; r < SI_RS; r++) {
            if (active && (b.ld & (SI_RS - 1)) == r && b.ld < (b.rd >> 2) + SI_RS && b.ld < b.nchunk) {
                __builtin_amdgcn_global_load_lds((const void *)(b.base + 16ull * b.ld), (lds_void *)(ring + r * 256),
                                                 16, 0, 0);
                b.ld++;
            }
        }
}

// 16 u16 fields packed in four u64s, indexed by a per-lane value
DEV uint32_t get16(const uint64_t w[4], uint32_t i) {
    const uint32_t q = i >> 2;
    const uint64_t x = q == 0 ? w[0] : q == 1 ? w[1] : q == 2 ? w[2] : w[3];
    return (uint32_t)(x >> (16 * (i & 3u))) & 0xFFFFu;
}
DEV void add16(uint64_t w[4], uint32_t i, uint32_t v) {
    const uint32_t q = i >> 2;
    const uint64_t d = (uint64_t)v << (16 * (i & 3u));
    w[0] += q == 0 ? d : 0;
    w[1] += q == 1 ? d : 0;
    w[2] += q == 2 ? d : 0;
    w[3] += q == 3 ? d : 0;
}

// one lane's table: lens[0, n) (4-byte aligned) -> root table `row` (entry e
// at row[e * 64]); a code longer than the root leaves its prefix entry 0 and
// is decoded canonically: per length L > root, lim (first code + count) and
// base (first code - sorted index + the first long index) packed in
// lx[L - root - 1] (registers), its symbol at long index code - base in
// `lrow` (LDS, lane-interleaved, `cap` of them).  0 on success, 1 for an
// over-subscribed set or an incomplete one (zlib's inflate_table: incomplete
// only for a single length-1 code, never for the code-length code; an empty
// set builds a table every lookup of which fails), 2 for more than `cap` long
// codes (the block goes to pf_inflate instead).
template <uint32_t ROOT, uint32_t NL>
DEV uint32_t lane_build(const uint8_t *lens, uint32_t n, uint16_t *row, uint16_t *lrow, uint32_t cap,
                        uint32_t (&lx)[NL], bool is_codes) {
    const uint32_t *lw = reinterpret_cast<const uint32_t *>(lens);
    uint64_t cw[4] = {0, 0, 0, 0};
    for (uint32_t s4 = 0; s4 < n; s4 += 4) {
        const uint32_t w = lw[s4 >> 2];
#pragma unroll
        for (uint32_t j = 0; j < 4; j++)
            if (s4 + j < n) add16(cw, (w >> (8 * j)) & 0xFFu, 1u);
    }
    int32_t left = 1;
    uint32_t maxl = 0;
    bool bad = false;
    uint64_t fw[4] = {0, 0, 0, 0}, ow[4] = {0, 0, 0, 0};
    uint32_t code = 0, off = 0, prev_c = 0, off_long = 0;
#pragma unroll
    for (uint32_t L = 1; L < 16; L++) {
        const uint32_t c = get16(cw, L);
        left = 2 * left - (int32_t)c;
        bad |= left < 0;
        maxl = c ? L : maxl;
        code = (code + prev_c) << 1;
        off += L > 1 ? prev_c : 0u;
        add16(fw, L, code);
        add16(ow, L, off);
        if (L == ROOT + 1) off_long = off;
        prev_c = c;
    }
    if (bad) return 1;
    if (maxl != 0 && left > 0 && (is_codes || maxl != 1)) return 1;
#pragma unroll
    for (uint32_t i = 0; i < NL; i++) {
        const uint32_t L = ROOT + 1 + i;
        lx[i] = (get16(fw, L) + get16(cw, L)) | ((get16(fw, L) - get16(ow, L) + off_long) << 16);
    }
    const uint32_t rn = 1u << ROOT;
    if (left > 0)                                        // incomplete (or empty): unfilled entries must fail
        for (uint32_t i = 0; i < rn; i++) row[i * 64] = 0;
    uint64_t nc[4] = {fw[0], fw[1], fw[2], fw[3]};       // next code per length
    for (uint32_t s4 = 0; s4 < n; s4 += 4) {
        const uint32_t w = lw[s4 >> 2];
#pragma unroll
        for (uint32_t j = 0; j < 4; j++) {
            const uint32_t s = s4 + j, l = (w >> (8 * j)) & 0xFFu;
            if (s >= n || !l) continue;
            const uint32_t cd = get16(nc, l);
            add16(nc, l, 1u);
            const uint32_t rev = __builtin_bitreverse32(cd) >> (32 - l);
            if (l <= ROOT) {
                const uint16_t e = (uint16_t)(s | (l << 9));
                for (uint32_t k = rev; k < rn; k += 1u << l) row[k * 64] = e;
            } else {
                row[(rev & (rn - 1)) * 64] = 0;            // a long code's prefix: the canonical path
                const uint32_t li = get16(ow, l) + cd - get16(fw, l) - off_long;
                if (li >= cap) return 2;                   // more long codes than the LDS list holds
                lrow[li * 64] = (uint16_t)s;
            }
        }
    }
    return 0;
}

// canonical decode of a code longer than the root: the first length whose
// left-aligned code is below its limit (registers), then the symbol
template <uint32_t ROOT, uint32_t NL>
DEV uint32_t slow_sym(uint64_t buf, const uint32_t (&lx)[NL], const uint16_t *lrow, uint32_t &len) {
    const uint32_t r = __builtin_bitreverse32((uint32_t)buf);
    uint32_t idx = 0, L = 0;
#pragma unroll
    for (uint32_t i = NL; i-- > 0;) {                   // longest first: the last hit is the shortest length
        const uint32_t Li = ROOT + 1 + i;
        const uint32_t cd = r >> (32 - Li);
        const bool hit = cd < (lx[i] & 0xFFFFu);
        idx = hit ? cd - (lx[i] >> 16) : idx;
        L = hit ? Li : L;
    }
    len = L;
    if (!L) return 0xFFFFu;
    return lrow[idx * 64];                              // (idx < cap: a tree with more long codes is not decoded here)
}

enum { ST_HDR = 0, ST_SYM = 1, ST_STORED = 2, ST_DONE = 3 };

static_assert(sizeof(SiScr) == PF_SI_SCR, "scratch layout");
static_assert(SI_META == PF_SI_META, "meta layout");

__global__ __launch_bounds__(64) void pf_inflate_tok(const uint8_t *in, const pf_bgzf_blk *blk, uint32_t nblk,
                                                     uint64_t out_base, uint32_t *tok, uint32_t *meta,
                                                     uint8_t *scratch, uint32_t *status) {
    __shared__ uint16_t lt[SI_LN * 64];
    __shared__ uint16_t dt[SI_DN * 64];
    __shared__ uint16_t llt[SI_LCAP * 64];
    __shared__ uint16_t dlt[SI_DCAP * 64];
    const uint32_t lane = threadIdx.x;
    const uint32_t bi = blockIdx.x * 64 + lane;
    uint16_t *lrow = lt + lane, *drow = dt + lane, *llrow = llt + lane, *dlrow = dlt + lane;
    uint32_t llx[SI_NLL], dlx[SI_NDL];
    uint32_t state = ST_DONE, err = 0, isize = 0, bfinal = 0, rem = 0;
    __shared__ __attribute__((aligned(16))) uint32_t ring[SI_RS * 256];
    LBits b;
    pf_bgzf_blk B;
    SiScr *S = nullptr;
    uint32_t *tk = nullptr, *mt = nullptr;
    b.buf = 0;
    b.cnt = 0;
    b.rd = b.ld = b.end = b.nchunk = 0;
    b.base = in;
    uint32_t skip = 0;
    if (bi < nblk) {
        B = blk[bi];
        isize = B.isize;
        const uint64_t a = (uint64_t)(uintptr_t)(in + B.in_off);
        skip = (uint32_t)(a & 15u);
        b.base = in + (B.in_off - skip);
        b.rd = skip >> 2;
        b.end = ((skip + B.in_len + 3) >> 2) + 3;
        b.nchunk = (skip + B.in_len + 64) >> 4;
        S = reinterpret_cast<SiScr *>(scratch + (uint64_t)bi * sizeof(SiScr));
        tk = tok + (((B.out_off - out_base) & ~3ull) + 4ull * bi);
        mt = meta + (uint64_t)bi * SI_META;
        state = ST_HDR;
    }
    lb_refill(b, ring, bi < nblk);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (bi < nblk) {
        lb_fill(b, ring, lane);
        lb_take(b, 8 * (skip & 3u));
    }
    uint32_t out = 0, ntok = 0, tqn = 0, lacc = 0, ln = 0;
    uint32_t tq[7] = {0, 0, 0, 0, 0, 0, 0};

    // queue one token covering [p, p + n) of the block's output; eight
    // queued tokens go out as two 16-byte stores
    auto emit = [&](uint32_t t, uint32_t p, uint32_t n) {
        const uint32_t k = (p + n - 1) >> 12;
        if ((k << 12) >= p) mt[1 + k] = ntok | (((k << 12) - p) << 17);   // the first token of chunk k
        if (tqn == 7) {
            *reinterpret_cast<uint4 *>(tk + (ntok - 7)) = make_uint4(tq[0], tq[1], tq[2], tq[3]);
            *reinterpret_cast<uint4 *>(tk + (ntok - 3)) = make_uint4(tq[4], tq[5], tq[6], t);
            tqn = 0;
        } else {
#pragma unroll
            for (uint32_t j = 0; j < 7; j++) tq[j] = tqn == j ? t : tq[j];
            tqn++;
        }
        ntok++;
    };

    uint32_t it = 0;
#ifdef SI_PROF
    uint64_t p_ref = 0, p_hdr = 0, p_dec = 0, p_n = 0, p_t0 = __builtin_amdgcn_s_memtime(), pa = 0, pb = 0, pc = 0;
#define SI_TS(x) x = __builtin_amdgcn_s_memtime()
#else
#define SI_TS(x)
#endif
    while (__ballot(state != ST_DONE)) {
        SI_TS(pa);
        if (++it == SI_RP) {
            it = 0;
            lb_refill(b, ring, state != ST_DONE);
        }
        SI_TS(pb);
#ifdef SI_PROF
        p_ref += pb - pa;
        p_n++;
#endif
        if (state == ST_DONE) continue;
        if (b.rd > b.end) { err = PF_INF_EINPUT; state = ST_DONE; continue; }
        if (state == ST_HDR) {
            // ---- a deflate block header (lanes at a header build together)
            lb_fill(b, ring, lane);
            bfinal = lb_take(b, 1);
            const uint32_t type = lb_take(b, 2);
            if (type == 0) {                               // stored
                lb_take(b, b.cnt & 7u);
                lb_fill(b, ring, lane);
                const uint32_t len = lb_take(b, 16), nlen = lb_take(b, 16);
                if ((len ^ 0xFFFFu) != nlen) { err = PF_INF_ESTORED; state = ST_DONE; continue; }
                if (out + ln + len > isize) { err = PF_INF_ESIZE; state = ST_DONE; continue; }
                rem = len;
                state = len ? ST_STORED : (bfinal ? ST_DONE : ST_HDR);
                continue;
            }
            if (type == 3) { err = PF_INF_ETYPE; state = ST_DONE; continue; }
            uint32_t nlit = 288, ndist = 32;
            if (type == 1) {                               // fixed codes
                for (uint32_t s = 0; s < 320; s++)
                    S->lens[s] = (uint8_t)(s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : s < 288 ? 8 : 5);
            } else {                                       // dynamic: the code-length code first
                lb_fill(b, ring, lane);
                nlit = lb_take(b, 5) + 257;
                ndist = lb_take(b, 5) + 1;
                const uint32_t ncl = lb_take(b, 4) + 4;
                if (nlit > 286 || ndist > 30) { err = PF_INF_ECODES; state = ST_DONE; continue; }
                lb_fill(b, ring, lane);
                const uint32_t n1 = ncl < 10 ? ncl : 10;
                uint64_t clbits = lb_take(b, 3 * n1);
                if (ncl > 10) { lb_fill(b, ring, lane); clbits |= (uint64_t)lb_take(b, 3 * (ncl - 10)) << 30; }
                for (uint32_t j = 0; j < 19; j++)
                    S->lens[si_clord[j]] = (uint8_t)(j < ncl ? (uint32_t)(clbits >> (3 * j)) & 7u : 0u);
                uint32_t clx[8];
                if (lane_build<7, 8>(S->lens, 19, drow, nullptr, 0, clx, true)) {
                    err = PF_INF_ECODES;
                    state = ST_DONE;
                    continue;
                }
                const uint32_t total = nlit + ndist;
                uint32_t i = 0, prev = 0, nsym = 0;
                while (i < total) {
                    if ((nsym++ & 7u) == 0) lb_refill(b, ring, true);
                    lb_fill(b, ring, lane);
                    const uint32_t e = drow[((uint32_t)b.buf & 127u) * 64];
                    const uint32_t l = e >> 9, s = e & 511u;
                    if (l == 0) { err = PF_INF_ECODES; break; }
                    lb_take(b, l);
                    uint32_t rep = 1, val = s;
                    if (s == 16) {
                        if (i == 0) { err = PF_INF_ECODES; break; }
                        rep = 3 + lb_take(b, 2);
                        val = prev;
                    } else if (s == 17) {
                        rep = 3 + lb_take(b, 3);
                        val = 0;
                    } else if (s == 18) {
                        rep = 11 + lb_take(b, 7);
                        val = 0;
                    }
                    if (i + rep > total) { err = PF_INF_ECODES; break; }
                    for (uint32_t j = 0; j < rep; j++) {
                        const uint32_t q = i + j;
                        S->lens[q < nlit ? q : 288 + q - nlit] = (uint8_t)val;
                    }
                    i += rep;
                    prev = val;
                    if (b.rd > b.end) { err = PF_INF_EINPUT; break; }
                }
                if (err) { state = ST_DONE; continue; }
                if (S->lens[256] == 0) { err = PF_INF_ECODES; state = ST_DONE; continue; }   // no end-of-block code
            }
            uint32_t bl = lane_build<SI_LR, SI_NLL>(S->lens, nlit, lrow, llrow, SI_LCAP, llx, false);
            if (!bl) bl = lane_build<SI_DR, SI_NDL>(S->lens + 288, ndist, drow, dlrow, SI_DCAP, dlx, false);
            if (bl) {
                err = bl == 2 ? PF_INF_FALLBACK : PF_INF_ECODES;
                state = ST_DONE;
                continue;
            }
            state = ST_SYM;
            continue;
        }
        // ---- one symbol (or one stored byte) per lane
        SI_TS(pc);
#ifdef SI_PROF
        p_hdr += pc - pb;
#endif
        lb_fill(b, ring, lane);
        uint32_t s, L = 0, D = 0;
        if (state == ST_STORED) {
            s = lb_take(b, 8);
            if (--rem == 0) state = bfinal ? ST_DONE : ST_HDR;
        } else {
            const uint32_t e = lrow[((uint32_t)b.buf & (SI_LN - 1)) * 64];
            uint32_t l = e >> 9;
            s = e & 511u;
            if (l == 0) {
                s = slow_sym<SI_LR, SI_NLL>(b.buf, llx, llrow, l);
                if (l == 0) { err = PF_INF_ECODES; state = ST_DONE; continue; }
            }
            lb_take(b, l);
            if (s > 256) {
                const uint32_t li = s - 257;
                if (li >= 29) { err = PF_INF_ECODES; state = ST_DONE; continue; }
                if (li < 8) L = 3 + li;
                else if (li == 28) L = 258;
                else {
                    const uint32_t lx = (li - 4) >> 2;
                    L = ((4 + (li & 3u)) << lx) + 3 + lb_take(b, lx);
                }
                lb_fill(b, ring, lane);
                const uint32_t de = drow[((uint32_t)b.buf & (SI_DN - 1)) * 64];
                uint32_t dl = de >> 9, ds = de & 511u;
                if (dl == 0) {
                    ds = slow_sym<SI_DR, SI_NDL>(b.buf, dlx, dlrow, dl);
                    if (dl == 0) { err = PF_INF_ECODES; state = ST_DONE; continue; }
                }
                lb_take(b, dl);
                if (ds >= 30) { err = PF_INF_ECODES; state = ST_DONE; continue; }
                if (ds < 4) D = 1 + ds;
                else {
                    const uint32_t dx = (ds - 2) >> 1;
                    D = ((2 + (ds & 1u)) << dx) + 1 + lb_take(b, dx);
                }
            } else if (s == 256) {
                state = bfinal ? ST_DONE : ST_HDR;
            }
        }
#ifdef SI_PROF
        p_dec += __builtin_amdgcn_s_memtime() - pc;
#endif
        if (s < 256) {                                     // a literal (or a stored byte)
            if (out + ln >= isize) { err = PF_INF_ESIZE; state = ST_DONE; continue; }
            lacc |= s << (8 * ln);
            if (++ln == 3) {
                emit(lacc | (3u << 24), out, 3);
                out += 3;
                lacc = 0;
                ln = 0;
            }
        } else {                                           // end of block or a match: the pending literals first
            if (ln) {
                emit(lacc | (ln << 24), out, ln);
                out += ln;
                lacc = 0;
                ln = 0;
            }
            if (s > 256) {
                if (D > out) { err = PF_INF_EDIST; state = ST_DONE; continue; }
                if (out + L > isize) { err = PF_INF_ESIZE; state = ST_DONE; continue; }
                emit(0x80000000u | ((L - 3) << 16) | (D - 1), out, L);
                out += L;
            }
        }
    }
#ifdef SI_PROF
    const uint64_t p_tot = __builtin_amdgcn_s_memtime() - p_t0;
    if (lane == 0 && bi < nblk) { mt[17] = (uint32_t)p_n; mt[18] = (uint32_t)(p_tot >> 4); mt[19] = (uint32_t)(p_ref >> 4); }
    if (lane == 1 && bi < nblk) { mt[17] = (uint32_t)(p_hdr >> 4); mt[18] = (uint32_t)(p_dec >> 4); mt[19] = 0; }
#endif
    if (bi >= nblk) return;
    if (!err && ln) { emit(lacc | (ln << 24), out, ln); out += ln; }
    if (!err && out != isize) err = PF_INF_ESIZE;
    // the queued tokens
    const uint32_t q0 = ntok - tqn;
#pragma unroll
    for (uint32_t j = 0; j < 7; j++)
        if (j < tqn) tk[q0 + j] = tq[j];
    mt[0] = ntok;
    status[bi] = err;
}

// --------------------------------------------------------------------------
// second pass.  CRC32 in raw form (init 0, no final xor): raw(A || B) =
// raw(A) * x^(8|B|) ^ raw(B) in GF(2)[x] mod P; crc32(M) = ~(raw(M) ^ ~0 *
// x^(8|M|)) (pf_inflate.hip's combination).
DEV uint32_t gmul(uint32_t a, uint32_t b) {        // reflected, x^0 = 0x80000000 (zlib's multmodp)
    uint32_t p = 0;
#pragma unroll
    for (int i = 0; i < 32; i++) {
        p ^= (a & 0x80000000u) ? b : 0u;
        a <<= 1;
        b = (b & 1u) ? (b >> 1) ^ 0xEDB88320u : b >> 1;
    }
    return p;
}
DEV uint32_t gx8n(uint64_t n, const uint32_t *x2n) {  // x^(8n) mod P; x2n[k] = x^(2^k)
    uint32_t p = 0x80000000u;
    uint64_t e = n << 3;
    for (uint32_t k = 0; e; k++, e >>= 1)
        if (e & 1u) p = gmul(p, x2n[k & 31u]);
    return p;
}

#define LZ_T 256u
#define LZ_PER 16u                                 // chunk bytes per thread
#define LZ_TPT 17u                                 // chunk tokens per thread (<= 4097 tokens)

__global__ __launch_bounds__(LZ_T) void pf_inflate_lz(const pf_bgzf_blk *blk, uint32_t nblk, uint64_t out_base,
                                                      const uint32_t *tok, const uint32_t *meta, uint8_t *arena,
                                                      uint32_t *status) {
    __shared__ __attribute__((aligned(16))) uint8_t ob[65536 + 32];      // the block image (at arena alignment)
    __shared__ uint32_t tks[LZ_T * LZ_TPT];
    __shared__ uint16_t tss[LZ_T * LZ_TPT];        // token start in the chunk + 512
    __shared__ uint16_t own[SI_CH];                // byte -> token, then byte -> pending source
    __shared__ uint8_t rdy[SI_CH];
    __shared__ uint32_t crc_tab[256], x2n[32], wsum[LZ_T / 64];
    const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
    const uint32_t bi = blockIdx.x;
    if (bi >= nblk || status[bi]) return;
    const pf_bgzf_blk B = blk[bi];
    const uint32_t isize = B.isize;
    const uint32_t dl = (uint32_t)(B.out_off & 15u);                     // image byte j <-> arena[out_off - dl + j]
    const uint32_t *tk = tok + (((B.out_off - out_base) & ~3ull) + 4ull * bi);
    const uint32_t *mt = meta + (uint64_t)bi * SI_META;
    const uint32_t ntok = mt[0];
    for (uint32_t i = t; i < 256; i += LZ_T) {
        uint32_t c = i;
        for (int k = 0; k < 8; k++) c = (c & 1u) ? (c >> 1) ^ 0xEDB88320u : c >> 1;
        crc_tab[i] = c;
    }
    if (t == 0) {
        uint32_t p = 0x40000000u;                                          // x^1
        for (int k = 0; k < 32; k++) { x2n[k] = p; p = gmul(p, p); }
    }
    const uint64_t lt_mask = lane ? (~0ull >> (64 - lane)) : 0ull;

#ifdef SI_PROF
    uint64_t q_tok = 0, q_own = 0, q_val = 0, q_jmp = 0, q_rounds = 0, qa = 0, q0 = __builtin_amdgcn_s_memtime();
#define SQ_T(acc) { const uint64_t qn = __builtin_amdgcn_s_memtime(); acc += qn - qa; qa = qn; }
#else
#define SQ_T(acc)
#endif
    for (uint32_t c0 = 0; c0 < isize; c0 += SI_CH) {
#ifdef SI_PROF
        qa = __builtin_amdgcn_s_memtime();
#endif
        const uint32_t k = c0 >> 12;
        const uint32_t cl = isize - c0 < SI_CH ? isize - c0 : SI_CH;
        const uint32_t e0 = mt[1 + k];
        const uint32_t t0 = e0 & 0x1FFFFu, back = e0 >> 17;
        const uint32_t t1 = c0 + SI_CH < isize ? (mt[2 + k] & 0x1FFFFu) + 1 : ntok;
        const uint32_t m = t1 - t0;
        __syncthreads();                                                   // the previous chunk's readers are done
        for (uint32_t i = t; i < m; i += LZ_T) tks[i] = tk[t0 + i];
        for (uint32_t x = t; x < cl; x += LZ_T) own[x] = 0;
        __syncthreads();
        // token starts: lengths summed per thread, then a block exclusive scan
        const uint32_t a = t * LZ_TPT, z = a + LZ_TPT < m ? a + LZ_TPT : m;
        uint32_t sum = 0;
        for (uint32_t i = a; i < z; i++) {
            const uint32_t v = tks[i];
            sum += (v & 0x80000000u) ? ((v >> 16) & 255u) + 3 : (v >> 24) & 3u;
        }
        uint32_t inc = sum;
#pragma unroll
        for (uint32_t d = 1; d < 64; d <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)inc, d, 64);
            if (lane >= d) inc += y;
        }
        if (lane == 63) wsum[wv] = inc;
        __syncthreads();
        uint32_t pre = inc - sum;
        for (uint32_t w = 0; w < wv; w++) pre += wsum[w];
        int32_t st = (int32_t)pre - (int32_t)back;                         // chunk-relative start
        for (uint32_t i = a; i < z; i++) {
            const uint32_t v = tks[i];
            tss[i] = (uint16_t)(st + 512);
            if (i > 0 && st >= 0 && st < (int32_t)cl) own[st] = (uint16_t)i;
            st += (v & 0x80000000u) ? (int32_t)((v >> 16) & 255u) + 3 : (int32_t)((v >> 24) & 3u);
        }
        __syncthreads();
        SQ_T(q_tok);
        // each byte's token: the running max of the marks, per thread then across the block
        const uint32_t x0 = t * LZ_PER;
        uint32_t o[LZ_PER];
        uint32_t mx = 0;
#pragma unroll
        for (uint32_t j = 0; j < LZ_PER; j++) {
            const uint32_t x = x0 + j;
            mx = x < cl && own[x] > mx ? own[x] : mx;
            o[j] = mx;
        }
        uint32_t smx = mx;
#pragma unroll
        for (uint32_t d = 1; d < 64; d <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)smx, d, 64);
            if (lane >= d) smx = y > smx ? y : smx;
        }
        __syncthreads();
        if (lane == 63) wsum[wv] = smx;
        __syncthreads();
        uint32_t carry = (uint32_t)__shfl_up((int)smx, 1, 64);
        if (lane == 0) carry = 0;
        for (uint32_t w = 0; w < wv; w++) carry = wsum[w] > carry ? wsum[w] : carry;
        SQ_T(q_own);
        // values, or the source of a byte copied from this chunk
        uint32_t pend = 0;
#pragma unroll
        for (uint32_t j = 0; j < LZ_PER; j++) {
            const uint32_t x = x0 + j;
            if (x >= cl) continue;
            const uint32_t i = o[j] > carry ? o[j] : carry;
            const uint32_t v = tks[i];
            const int32_t s = (int32_t)tss[i] - 512;
            const uint32_t P = c0 + x;
            if (!(v & 0x80000000u)) {
                ob[dl + P] = (uint8_t)(v >> (8 * (x - s)));
                rdy[x] = 1;
                continue;
            }
            const uint32_t Lm = ((v >> 16) & 255u) + 3, D = (v & 0xFFFFu) + 1;
            const uint32_t A = (uint32_t)((int32_t)c0 + s);
            const uint32_t src = D >= Lm ? P - D : A - D + (P - A) % D;
            if (src < c0) {
                ob[dl + P] = ob[dl + src];
                rdy[x] = 1;
            } else {
                own[x] = (uint16_t)(src - c0);
                rdy[x] = 0;
                pend |= 1u << j;
            }
        }
        SQ_T(q_val);
        // sources inside the chunk: pointer jumping
        while (__syncthreads_or(pend != 0)) {
#ifdef SI_PROF
            q_rounds++;
#endif
            uint32_t got = 0, nv[LZ_PER], ns[LZ_PER];
#pragma unroll
            for (uint32_t j = 0; j < LZ_PER; j++) {
                nv[j] = 0;
                ns[j] = 0;
                if (!((pend >> j) & 1u)) continue;
                const uint32_t y = own[x0 + j];
                if (rdy[y]) { nv[j] = ob[dl + c0 + y]; got |= 1u << j; }
                else ns[j] = own[y];
            }
            __syncthreads();
#pragma unroll
            for (uint32_t j = 0; j < LZ_PER; j++) {
                if (!((pend >> j) & 1u)) continue;
                if ((got >> j) & 1u) { ob[dl + c0 + x0 + j] = (uint8_t)nv[j]; rdy[x0 + j] = 1; }
                else own[x0 + j] = (uint16_t)ns[j];
            }
            pend &= ~got;
        }
    }
#ifdef SI_PROF
    {
        const uint64_t qn = __builtin_amdgcn_s_memtime();
        q_jmp += 0;
        if (t == 0 && (bi & 63u) >= 2) {            // per block (x16 clocks): chunks total, tokens + owners, values | rounds
            uint32_t *pm = const_cast<uint32_t *>(mt);
            pm[17] = (uint32_t)((qn - q0) >> 4);
            pm[18] = (uint32_t)((q_tok + q_own) >> 4);
            pm[19] = (uint32_t)((q_val >> 4) & 0xFFFFFFu) | ((uint32_t)(q_rounds < 255 ? q_rounds : 255) << 24);
        }
    }
#endif
    __syncthreads();
    // CRC32 of the image: 256 slices of 256 bytes combined
    {
        const uint32_t a = t * 256u, z = a + 256u < isize ? a + 256u : isize;
        uint32_t c = 0;
        for (uint32_t p = a; p < z; p++) c = crc_tab[(c ^ ob[dl + p]) & 0xFFu] ^ (c >> 8);
        c = a < z ? gmul(c, gx8n(isize - z, x2n)) : 0u;
#pragma unroll
        for (int s = 32; s >= 1; s >>= 1) c ^= (uint32_t)__shfl_xor((int)c, s, 64);
        __syncthreads();
        if (lane == 0) wsum[wv] = c;
        __syncthreads();
        uint32_t crc = 0;
        for (uint32_t w = 0; w < LZ_T / 64; w++) crc ^= wsum[w];
        if (~(crc ^ gmul(0xFFFFFFFFu, gx8n(isize, x2n))) != B.crc) {
            if (t == 0) status[bi] = PF_INF_ECRC;
            return;
        }
    }
    // the image to the arena: whole 16-byte words, byte stores at the two ends
    uint8_t *base = arena + (B.out_off - dl);
    const uint32_t end = dl + isize, nw = (end + 15) >> 4;
    for (uint32_t w = t; w < nw; w += LZ_T) {
        const uint32_t j = w << 4;
        if (j >= dl && j + 16 <= end) {
            *reinterpret_cast<uint4 *>(base + j) = *reinterpret_cast<const uint4 *>(ob + j);
        } else {
            for (uint32_t q = j; q < j + 16; q++)
                if (q >= dl && q < end) base[q] = ob[q];
        }
    }
    (void)lt_mask;
}
