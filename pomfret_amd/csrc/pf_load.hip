// pf_load.hip -- K0: the window loader of the methphase path on the GPU.
//
// One wavefront per BAM record (4 per workgroup, ~9 KB of LDS per wave so 16
// waves share a CU).  Reference semantics, all /root/reference/blockjoin.c:
//   filters               load_reads_given_interval 1079-1085
//   5mC calls at CpG      fill_read_meth_record_from_bam_line 832-882
//   reference positions   get_mod_poss_on_ref 605-792
//   keep rule             add_read_record_from_bam_line 932-936 (>= 1 call
//                         at CpG and a CIGAR)
// plus htslib's MM/ML decoding (bam_parse_basemod / bam_mods_at_next_pos),
// restated from the SAM tag specification (see oracle/pf_oracle_load.c for
// the definitions on malformed input, which this kernel shares).
//
// Phases of one record (all wave-parallel):
//  1. MM: the tag text is staged in LDS (word loads); ballots over 64-byte
//     steps find the entries, the C+m entry's skip counts are parsed one lane
//     per comma and turned into ranks with a wave scan.
//  2. SEQ: stream the 4-bit SEQ in 1024-base chunks (16 bases per lane, next
//     chunk prefetched), count the C's (forward) or G's (reverse, ranks from
//     the end) per lane, and resolve each rank to its read position with a
//     64-entry LDS search and a select-k-th-bit; the CpG context test and the
//     ML category follow.  Result: the trigger list T (position<<2 | category),
//     ascending.
//  3. CIGAR: 64 operations per step (prefix sums of read advance and reference
//     offset); the triggers each op consumes -- the reference's
//     `while (i_read+length >= next_trigger)` (663) takes every trigger up to
//     and INCLUDING the op's end -- are mapped 64 at a time by an LDS search
//     over the op ends, and pushed with the de-duplication against the previous
//     push (`calls.a[n-1] == pos`, 704-706).  Implicit-mode reads also scan
//     their SEQ in 256-position chunks for the CpGs the reference's canonical
//     scan visits (666-700, 727-761) and merge both lists in push order.
//  4. The calls are written at the read's offset; a read whose calls are not
//     strictly increasing (rare) is sorted in place by (pos, cat), the order
//     the methmer kernels consume.
// A record whose leading soft clip swallows every trigger (the stale-trigger
// case of 629-652) is walked by lane 0 with a literal restatement of the loop.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "pf_device.h"
#include "pf_load.h"

#define DEV static __device__ __forceinline__
#define NT_C 2u
#ifndef PF_K0_SEQ_REREAD
#define PF_K0_SEQ_REREAD 0                 // SEQ pass: trigger words re-read (1: +4.6 GB HBM reads on the mix, no faster) or taken by ds_bpermute (0)
#endif

// Diagnostic build only (-DPF_K0_PROFILE): cycles per phase summed over the
// records into ctr[8 + phase] (s_memtime, one fenced asm statement).
#ifdef PF_K0_PROFILE
DEV unsigned long long k0_now() {
    unsigned long long t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
#define K0_STAMP(i) do { const unsigned long long t_ = k0_now(); \
    if (d.ctr && lane == 0) atomicAdd(&d.ctr[8 + (i)], t_ - k0_t); k0_t = t_; } while (0)
#define K0_T0 unsigned long long k0_t = k0_now()
#else
#define K0_STAMP(i) do { } while (0)
#define K0_T0 do { } while (0)
#endif
#define NT_G 4u
// Out-of-line code (pf_k0_load is ~77 KB inlined, past the 64 KB instruction
// cache two CUs share): bit 0 the record path of HBM trigger lists (long
// records), bit 1 the cold paths (SWAR parse, lane-0 walk, implicit chunks)
#ifndef PF_K0_NOINL
#define PF_K0_NOINL 0
#endif
#if PF_K0_NOINL & 1
#define DEV_HBM static __device__ __attribute__((noinline))
#else
#define DEV_HBM DEV
#endif
#if PF_K0_NOINL & 2
#define DEV_COLD static __device__ __attribute__((noinline))
#else
#define DEV_COLD DEV
#endif
// SEQ-pass trigger placement (round 6): 1 = the block's trigger range by a
// wave-parallel search (2 round trips instead of ~10 dependent ones) and each
// trigger's word pair by two 8-wide LDS reads with packed compares (group,
// then pair) instead of a 6-step binary search; 0 = round 5
#ifndef PF_K0_PLACE
#define PF_K0_PLACE 1
#endif
// CIGAR walk (round 6): 1 = each trigger's operation by two 8-wide LDS reads
// (the tile's group ends, then the group) instead of a 6-step binary search
#ifndef PF_K0_WALK2
#define PF_K0_WALK2 1
#endif
// SEQ pass (round 6): 1 = the placement writes the CpG triggers compacted
// (forward reads from the bottom of the list, reverse reads from the top)
// instead of a compaction pass over the whole list afterwards
#ifndef PF_K0_FUSEC
#define PF_K0_FUSEC 1
#endif
// SEQ count without a per-word tail test (round 6): every nibble past the
// record's SEQ is 0 in the slice, the odd-length pad nibble included (both
// producers clear it: pf_load.h), and 0 is never a target
#ifndef PF_K0_PADFIX
#define PF_K0_PADFIX 1
#endif
// SEQ placement (round 6): 1 = a trigger takes its own word only (4
// ds_bpermute per row); the neighbour word, needed for the context base of a
// trigger at the word's last (forward) / first (reverse) base, is fetched
// afterwards for those triggers alone (1 in 16); 0 = every trigger takes its
// word and the neighbour pair (6 ds_bpermute and 2 readlanes per row)
#ifndef PF_K0_NBRARE
#define PF_K0_NBRARE 1
#endif
// MM ranks (round 6): 1 = one text load per lane and row, the neighbour
// words' non-digit flags by DPP; 0 = three loads per lane and row
#ifndef PF_K0_RANKDPP
#define PF_K0_RANKDPP 1
#endif
// pack (round 6): 1 = each wave's next 512-call chunk loaded before the
// current chunk is stored
#ifndef PF_PACK_PIPE
#define PF_PACK_PIPE 1
#endif
#ifndef PF_PACK_U
#define PF_PACK_U 4                        // calls per lane per chunk of the pipelined pack
#endif
// MM entries (round 6): 1 = a one-code header ("C+m?") parsed from one
// 4-byte window instead of byte by byte
#ifndef PF_K0_HDRFAST
#define PF_K0_HDRFAST 1
#endif
// emission (round 6): 1 = when the kept calls are lanes 0..n-1, each call's
// predecessor by DPP wave_shr:1 instead of a ds_bpermute from the previous
// kept lane
#ifndef PF_K0_EMITDPP
#define PF_K0_EMITDPP 1
#endif
#ifndef PF_K0_WPE
#define PF_K0_WPE 8                        // pf_k0_load's waves per SIMD (register budget: 512 / WPE VGPRs)
#endif

DEV uint32_t uni(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }
DEV uint64_t lanemask_lt(uint32_t lane) { return lane ? (~0ull >> (64 - lane)) : 0ull; }
DEV uint32_t popc(uint64_t m) { return (uint32_t)__popcll(m); }
// set bits of b below this lane (popc(b & lanemask_lt(lane)) in two mbcnt)
DEV uint32_t below_cnt(uint64_t b) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u));
}
DEV uint32_t rdl(uint32_t x, uint32_t l) { return (uint32_t)__builtin_amdgcn_readlane((int)x, (int)l); }

DEV void wsync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// Inclusive wave prefix sum with DPP: row_shr 1/2/4/8 inside each 16-lane
// row, then row_bcast:15 / row_bcast:31 carry the row totals upwards (the same
// sequence pf_selftest checks for the greedy kernel).
DEV uint32_t dpp_shr_add(uint32_t x, const int ctrl) {
    uint32_t y;
    switch (ctrl) {
    case 1: y = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, true); break;
    case 2: y = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, true); break;
    case 4: y = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, true); break;
    case 8: y = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, true); break;
    case 15: y = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false); break;
    default: y = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false); break;
    }
    return x + y;
}
DEV uint32_t wscan(uint32_t x, uint32_t) {
    x = dpp_shr_add(x, 1);
    x = dpp_shr_add(x, 2);
    x = dpp_shr_add(x, 4);
    x = dpp_shr_add(x, 8);
    x = dpp_shr_add(x, 15);
    x = dpp_shr_add(x, 31);
    return x;
}
DEV uint64_t wscan64(uint64_t x, uint32_t lane) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint64_t y = __shfl_up(x, o, 64);
        if (lane >= (uint32_t)o) x += y;
    }
    return x;
}
DEV uint64_t rdl64(uint64_t x, uint32_t l) {
    return ((uint64_t)rdl((uint32_t)(x >> 32), l) << 32) | rdl((uint32_t)x, l);
}

DEV uint32_t nib(const uint8_t *s, uint32_t i) { return (s[i >> 1] >> ((~i & 1u) << 2)) & 0xFu; }
// base i (0..15) of 16 packed bases held as a little-endian u64
DEV uint32_t nibw(uint64_t w, uint32_t i) { return (uint32_t)(w >> (8u * (i >> 1) + ((i & 1u) ? 0u : 4u))) & 0xFu; }
DEV uint32_t match16(uint64_t w, uint32_t tb, uint32_t nv) {
    uint32_t m = 0;
#pragma unroll
    for (uint32_t i = 0; i < 16; i++) m |= (nibw(w, i) == tb && i < nv) ? (1u << i) : 0u;
    return m;
}
DEV uint32_t select_bit(uint32_t m, uint32_t k) {
    for (uint32_t i = 0; i < k; i++) m &= m - 1;
    return (uint32_t)__builtin_ctz(m);
}
DEV bool is_digit(uint32_t c) { return c >= '0' && c <= '9'; }
DEV bool is_alpha(uint32_t c) { return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z'); }

// first index o in [0, n) with a[o] >= v (LE = false) or a[o] > v (LE = true)
template <bool LE>
DEV uint32_t lb64(const uint32_t *a, uint32_t n, uint32_t v) {
    uint32_t lo = 0;
    while (n > 0) {
        const uint32_t h = n >> 1;
        const uint32_t x = a[lo + h];
        if (LE ? x <= v : x < v) { lo += h + 1; n -= h + 1; } else n = h;
    }
    return lo;
}

struct K0Merge {                      // implicit-mode chunk lists
    uint32_t eP[PF_K0_EC], eV[PF_K0_EC];
    uint32_t iP[PF_K0_EC], iV[PF_K0_EC];
    uint32_t mV[2 * PF_K0_EC];
    uint8_t eC[PF_K0_EC];
    uint8_t mC[2 * PF_K0_EC];         // cat | 0x80 for implicit calls
};
struct K0Seq {
    uint16_t sb[8 * 64];              // SEQ block: rank base of each (row, word pair)
    uint8_t sc[8 * 64];               //            target count of the pair's first word
};
struct K0W {                          // LDS of one wave (5 KB: 8 waves per SIMD)
    uint32_t T[PF_K0_TCAP];           // ranks, then triggers (p<<2 | cat)
    uint32_t opE[64], opOff[64], opA[64];
    uint8_t opT[64];
    union {
        K0Seq s;                      // phase 2
        K0Merge mg;                   // phase 3: implicit-mode lists, emission spill
    } u;
};

// emission state, uniform across the wave
struct K0Out {
    uint32_t n, first, last;
    uint32_t sorted, lim;
    uint32_t *pos;                    // write mode: the read's slice of call_pos / call_cat
    uint8_t *cat;
};

// ---------------------------------------------------------------------------
// Phase 1: MM/ML -> ranks of the called C's (original orientation).  The MM
// text is read as aligned words straight from HBM/L2 (the device copy is
// padded, so the last word may run past the text): lane k of a 64-word row
// holds text bytes 4k - mis .. 4k - mis + 3.  ';' and ',' are found four bytes
// per lane by per-byte flags; each comma's skip count is converted from the 7
// bytes after it (the lane's word and the next) by a SWAR decimal parse, and
// a count that may run past that window takes a byte loop.
struct K0Tgt { uint32_t nd, nc, mi, th, te; uint64_t ml; };
// The MM entries that give 5mC calls: every entry with canonical base C and
// the code m among its codes, whatever its strand (htslib matches the
// canonical base against the read's base and reports the strand as a field:
// a C-m entry counts the same C's as C+m).  The first is kept in registers;
// the others (rare: a duplex-style or repeated C m entry) go to the wave's
// LDS, PF_K0_TW words each (no private array: dynamic indexing would put it
// in scratch on every record).  Up to PF_K0_MAXT; more sets PF_ST_MM_LIMIT.
#define PF_K0_MAXT 8
#define PF_K0_TW 7
struct K0Tgts { K0Tgt t0; uint32_t n, over; uint32_t *xt; };
DEV void k0_tgt_put(uint32_t *xt, uint32_t e, const K0Tgt &t, uint32_t lane) {   // e >= 1, uniform
    if (lane == 0) {
        uint32_t *q = xt + PF_K0_TW * (e - 1);
        q[0] = t.nd; q[1] = t.nc; q[2] = t.mi; q[3] = t.th; q[4] = t.te; q[5] = (uint32_t)t.ml;
        q[6] = (uint32_t)(t.ml >> 32);
    }
}
DEV K0Tgt k0_tgt_get(const K0Tgts &T, uint32_t e) {  // e uniform
    if (e == 0) return T.t0;
    const uint32_t *q = T.xt + PF_K0_TW * (e - 1);
    K0Tgt t;
    t.nd = q[0]; t.nc = q[1]; t.mi = q[2]; t.th = q[3]; t.te = q[4];
    t.ml = ((uint64_t)q[6] << 32) | q[5];
    return t;
}

DEV uint32_t bytes_eq(uint32_t w, uint32_t c) {      // 0x80 in each byte of w equal to c
    const uint32_t t = w ^ (c * 0x01010101u);
    return ~(((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t) & 0x80808080u;
}
DEV uint32_t bytes_in(int32_t b, uint32_t lo, uint32_t hi) {   // bytes with text index in [lo, hi)
    const int32_t s = min(max((int32_t)lo - b, 0), 4), e = min(max((int32_t)hi - b, 0), 4);
    const uint32_t ml = s >= 4 ? 0u : 0x80808080u << (8 * s);
    const uint32_t mh = e <= 0 ? 0u : 0x80808080u >> (8 * (4 - e));
    return ml & mh;
}
DEV uint32_t wsum_small(uint32_t c) {                // wave sum of per-lane values 0..7
    return popc(__ballot(c & 1u)) + 2u * popc(__ballot(c & 2u)) + 4u * popc(__ballot(c & 4u));
}
DEV uint64_t nondigit_bytes(uint64_t y) {            // 0x80 in each byte of y outside '0'..'9'
    const uint64_t hi = (y & 0xF0F0F0F0F0F0F0F0ull) ^ 0x3030303030303030ull;
    const uint64_t hz = ~(((hi & 0x7F7F7F7F7F7F7F7Full) + 0x7F7F7F7F7F7F7F7Full) | hi) & 0x8080808080808080ull;
    const uint64_t ge10 = ((y & 0x0F0F0F0F0F0F0F0Full) + 0x7676767676767676ull) & 0x8080808080808080ull;
    return (~hz & 0x8080808080808080ull) | ge10;
}
DEV uint32_t swar_dec(uint64_t y, uint32_t n) {      // bytes 0..n-1 of y (n in 1..7) as decimal digits
    uint64_t z = (y & ((1ull << (8 * n)) - 1)) << (8 * (8 - n));   // leading zeros pad to 8 digits
    z = ((z & 0x0F0F0F0F0F0F0F0Full) * 2561u) >> 8;
    z = ((z & 0x00FF00FF00FF00FFull) * 6553601u) >> 16;
    return (uint32_t)(((z & 0x0000FFFF0000FFFFull) * 42949672960001ull) >> 32);
}

// One pass over the text with the next row in flight: every ';' of a row
// closes an entry (its comma count is a difference of the row's comma scan),
// and the next entry's header is parsed right away from the row registers
// (readlane; a header past the next row -- never in real data -- reads
// memory).  Round 2 rescanned from each entry's start and read every header
// byte from memory: one dependent round trip per row and per header byte.
struct K0Hdr { uint32_t base, strand, nc, h; int mi; };

template <bool MULTI>
DEV bool k0_mm_entries(const uint32_t *gw, const uint8_t *mm, uint32_t mis, uint32_t mlen, uint32_t mln,
                       uint32_t lane, K0Tgts &T) {
    T.n = 0;
    T.over = 0;
    T.t0.nd = 0;
    if (mlen == 0) return true;
    const uint32_t wend = mis + mlen;
    const uint32_t kmaxw = (wend - 1) / 4 + 1;       // the padded text holds this word
    auto ld = [&](uint32_t k) { return gw[min(k, kmaxw)]; };
    uint32_t k0 = 0;
    // rows in flight four deep (a 2 KB text -- dorado's h + m entries of a
    // 30 kb read -- costs one memory round trip, not eight)
    uint32_t w = ld(lane), pw = ld(64 + lane), pw2 = ld(128 + lane), pw3 = ld(192 + lane);
    auto byte_at = [&](uint32_t x) -> uint32_t {      // text byte x < mlen (uniform x)
        const uint32_t kx = (mis + x) >> 2, sh = 8 * ((mis + x) & 3u);
        if (kx - k0 < 64) return (rdl(w, kx - k0) >> sh) & 0xFFu;
        if (kx - k0 < 128) return (rdl(pw, kx - k0 - 64) >> sh) & 0xFFu;
        return mm[x];
    };
    K0Hdr H;
#if PF_K0_HDRFAST
    auto dword_at = [&](uint32_t kx) -> uint32_t {    // text dword kx (uniform)
        if (kx - k0 < 64) return rdl(w, kx - k0);
        if (kx - k0 < 128) return rdl(pw, kx - k0 - 64);
        return gw[min(kx, kmaxw)];
    };
#endif
    auto header = [&](uint32_t i) {                   // base, strand, codes, '.'/'?' (the entry's ';' stops every loop)
#if PF_K0_HDRFAST
        // one code ("C+m?", "C+h.", "C+m,"): bytes i..i+3 at once; anything
        // else (several codes, a ChEBI number, a header at the text's end)
        // takes the byte loop below, which gives the same fields
        if (i + 3 < mlen) {
            const uint32_t x = mis + i, kx = x >> 2, sh = 8u * (x & 3u);
            const uint32_t lo = dword_at(kx);
            const uint32_t b4 = sh ? (lo >> sh) | (dword_at(kx + 1) << (32u - sh)) : lo;
            const uint32_t c2 = (b4 >> 16) & 0xFFu, c3 = b4 >> 24;
            if (is_alpha(c2) && !is_alpha(c3)) {
                H.base = b4 & 0xFFu;
                H.strand = (b4 >> 8) & 0xFFu;
                H.nc = 1;
                H.mi = c2 == 'm' ? 0 : -1;
                H.h = i + 3 + ((c3 == '.' || c3 == '?') ? 1u : 0u);
                return;
            }
        }
#endif
        H.base = byte_at(i);
        H.strand = i + 1 < mlen ? byte_at(i + 1) : 0u;
        uint32_t h = i + 2, nc = 0;
        int mi = -1;
        uint32_t c = h < mlen ? byte_at(h) : 0u;
        if (is_digit(c)) {
            while (h < mlen && is_digit(byte_at(h))) h++;
            nc = 1;
        } else {
            while (h < mlen && is_alpha(c = byte_at(h))) {
                if (c == 'm' && mi < 0) mi = (int)nc;
                nc++;
                h++;
            }
        }
        if (h < mlen && ((c = byte_at(h)) == '.' || c == '?')) h++;
        H.h = h; H.nc = nc; H.mi = mi;
    };
    uint64_t ml_cur = 0;
    // entry [i, e) with `commas` commas
    auto close = [&](uint32_t i, uint32_t e, uint32_t commas) -> bool {
        if (e - i < 3) return false;
        if (H.strand != '+' && H.strand != '-') return false;
        if (H.nc == 0) return false;
        if (H.base == ',') commas--;                  // count the skip list's commas only
        if (H.base == 'C' && H.mi >= 0 && commas > 0) {
            if (mln && ml_cur + (uint64_t)commas * H.nc > mln) return false;
            if (!MULTI && T.n) { T.n = 2; return true; }   // the main pass hands the record over
            if (T.n == PF_K0_MAXT) { T.over = 1; return true; }
            K0Tgt t;
            t.nd = commas; t.nc = H.nc; t.mi = (uint32_t)H.mi; t.th = H.h; t.te = e; t.ml = ml_cur;
            if (T.n == 0) T.t0 = t;
            else if constexpr (MULTI) k0_tgt_put(T.xt, T.n, t, lane);
            T.n++;
        }
        ml_cur += (uint64_t)commas * H.nc;
        return true;
    };
    uint32_t i = 0, ci = 0, cg = 0;                   // entry start, commas before it, before the row
    header(0);
    for (;;) {
        const int32_t b = (int32_t)(4 * (k0 + lane)) - (int32_t)mis;
        const uint32_t vm = bytes_in(b, 0, mlen);
        const uint32_t sm = bytes_eq(w, ';') & vm, cm = bytes_eq(w, ',') & vm;
        const uint32_t ncl = (uint32_t)__builtin_popcount(cm);
        const uint32_t cin = wscan(ncl, lane);
        for (uint64_t bs = __ballot(sm != 0); bs; bs &= bs - 1) {
            const uint32_t l0 = (uint32_t)__ffsll((long long)bs) - 1;
            const uint32_t sml = rdl(sm, l0), cml = rdl(cm, l0), cb0 = cg + rdl(cin, l0) - rdl(ncl, l0);
            for (uint32_t m = sml; m; m &= m - 1) {
                const uint32_t sb = (uint32_t)__builtin_ctz(m) >> 3;
                const uint32_t e = 4 * (k0 + l0) - mis + sb;
                const uint32_t ce = cb0 + (uint32_t)__builtin_popcount(cml & ((1u << (8 * sb)) - 1u));
                if (!close(i, e, ce - ci)) return false;
                i = e + 1;
                ci = ce;
                if (i < mlen) header(i);
            }
        }
        cg += rdl(cin, 63);
        if (4 * (k0 + 64) >= wend) break;
        k0 += 64;
        w = pw;
        pw = pw2;
        pw2 = pw3;
        pw3 = ld(k0 + 192 + lane);
    }
    if (i < mlen && !close(i, mlen, cg - ci)) return false;   // an entry without its ';'
    if (mln && ml_cur > mln) return false;
    return true;
}

// Ranks in TB, reversed for reverse reads (TB[nd-1-j] holds skip j's rank) so
// that TB is in forward read order for the SEQ pass.
//
// Digit-weight form (round 3): rank d = sum of skips 0..d + d, and the sum
// of the skip counts before a byte is the sum over the digits before it of
// digit x 10^(digits left in its number).  Every lane weighs its 4 bytes (the
// digits left come from a 12-byte non-digit mask: the lane's word and the
// next two), one wave scan gives the sum before each lane, and comma k writes
// rank k-1 = (sum before the comma) + k-1; the last rank is the total +
// nd-1.  No per-number parse and no per-comma loop: ~1/4 of the
// instructions of the per-comma SWAR parse, which stays as the fallback for
// counts of 8+ digits (never in real data).  Malformed text is rejected as
// the oracle does (pf_oracle_load.c:81-89): a comma not followed by a digit,
// a byte other than digit or comma before the last comma; bytes after the
// last count's digits are ignored.
DEV uint32_t nondigit4(uint32_t y) {                 // 0x80 in each byte of y outside '0'..'9'
    const uint32_t hi = (y & 0xF0F0F0F0u) ^ 0x30303030u;
    const uint32_t hz = ~(((hi & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | hi) & 0x80808080u;
    const uint32_t ge10 = ((y & 0x0F0F0F0Fu) + 0x76767676u) & 0x80808080u;
    return (~hz & 0x80808080u) | ge10;
}
DEV uint32_t pack4(uint32_t f) {                     // 0x80 byte flags -> 4-bit mask
    uint32_t x = f >> 7;                              // bits 0, 8, 16, 24
    x |= x >> 7;                                      // + 1 (from 8), 9, 17 (from 24)
    x |= x >> 14;                                     // + 2 (from 16), 3 (from 17)
    return x & 0xFu;
}
// digit x 10^e table (index digit << 3 | e, digits 0..9), in the wave's
// spare LDS during the MM phase
DEV uint32_t k0_dw(uint32_t i) {                     // (i >> 3) x 10^(i & 7), branch-free
    const uint32_t e = i & 7u;
    return (i >> 3) * ((e & 1u) ? 10u : 1u) * ((e & 2u) ? 100u : 1u) * ((e & 4u) ? 10000u : 1u);
}
DEV void k0_dw_table(uint32_t *tbl, uint32_t lane) {
    tbl[lane] = k0_dw(lane);
    if (lane < 16u) tbl[64u + lane] = k0_dw(64u + lane);
}

template <typename TP>
DEV_COLD bool k0_mm_ranks_swar(const uint32_t *gw, const uint8_t *mm, uint32_t mis, const K0Tgt &t, bool rev, TP TB,
                          uint32_t lane);

template <typename TP>
DEV bool k0_mm_ranks(const uint32_t *gw, const uint8_t *mm, uint32_t mis, const K0Tgt &t, bool rev, TP TB,
                     const uint32_t *tbl, uint32_t lane) {
    if (mm[t.th] != ',') return false;
    const uint32_t lo = t.th;
    uint32_t hi = t.te;                               // shrinks to the first stray byte
    const uint32_t wend = mis + t.te;
    uint64_t carry = 0;                               // digit sum of the rows before
    uint32_t kk = 0;                                  // commas before the row
    const uint32_t k0s = (mis + lo) >> 2;
    // unconditional loads (a static vmcnt for the row in flight): word
    // indices clamp to the last one the padded text holds; bytes past hi are
    // masked below
    const uint32_t kmaxw = (wend - 1) / 4 + 2;
    auto ld = [&](uint32_t k) { return gw[min(k, kmaxw)]; };
#if PF_K0_RANKDPP
    // one load per lane and row, two rows in flight; the next two words'
    // non-digit flags come from lanes + 1, + 2 (DPP wave_shl:1), the row's
    // last lanes taking the next row's first two
    uint32_t w = ld(k0s + lane), pw = ld(k0s + lane + 64);
    uint32_t nd0 = pack4(nondigit4(w));
#else
    uint32_t w = ld(k0s + lane), wn = ld(k0s + lane + 1), wn2 = ld(k0s + lane + 2);
#endif
    for (uint32_t k0 = k0s; 4 * k0 < wend; k0 += 64) {
        const uint32_t k = k0 + lane;
#if PF_K0_RANKDPP
        const uint32_t ppw = ld(k + 128);             // two rows ahead, in flight
        const uint32_t ndn = pack4(nondigit4(pw));
        const uint32_t nd1 = (uint32_t)__builtin_amdgcn_update_dpp((int)rdl(ndn, 0), (int)nd0, 0x130, 0xF, 0xF, false);
        const uint32_t nd2 = (uint32_t)__builtin_amdgcn_update_dpp((int)rdl(ndn, 1), (int)nd1, 0x130, 0xF, 0xF, false);
        const uint32_t ndm = nd0 | (nd1 << 4) | (nd2 << 8);
#else
        const uint32_t pw = ld(k + 64), pwn = ld(k + 65), pwn2 = ld(k + 66);   // the next row, in flight
        const uint32_t ndm = pack4(nondigit4(w)) | (pack4(nondigit4(wn)) << 4) | (pack4(nondigit4(wn2)) << 8);
#endif
        const int32_t b = (int32_t)(4 * k) - (int32_t)mis;
        const uint32_t nlo = (uint32_t)min(max((int32_t)lo - b, 0), 4);
        const uint32_t cw = pack4(bytes_eq(w, ','));
        uint32_t M, vb, cb;
        for (;;) {
            const uint32_t nin = (uint32_t)min(max((int32_t)hi - b, 0), 12);
            M = ndm | (~0u << nin);                   // non-digit or out of range; bit 12 a sentinel
            vb = (0xFu << nlo) & ~(~0u << min(nin, 4u)) & 0xFu;
            cb = cw & vb;
            const uint32_t jb = vb & M & ~cb;         // stray bytes
            const uint64_t bj = __ballot(jb != 0);
            if (!bj) break;
            const uint32_t l0 = (uint32_t)__ffsll((long long)bj) - 1;
            hi = rdl((uint32_t)(b + (int32_t)__builtin_ctz(jb | 0x10u)), l0);
        }
        const uint32_t D = ~M & 0xFFFu;               // digit bytes over the 12-byte window
        uint32_t x8 = D & (D >> 1);
        x8 &= x8 >> 2;
        x8 &= x8 >> 4;                                // bit j: bytes j..j+7 all digits
        const uint32_t db = D & vb;                   // the word's digits
        const bool badc = (cb & (M >> 1)) != 0;       // a comma not followed by a digit
        if (__ballot((x8 & db) != 0 || badc)) {       // rare: one ballot for both
            if (__ballot((x8 & db) != 0)) return k0_mm_ranks_swar(gw, mm, mis, t, rev, TB, lane);
            return false;
        }
        uint32_t c[4];
#pragma unroll
        for (uint32_t j = 0; j < 4; j++) {            // branch-free: every lane weighs all 4 bytes
            const uint32_t e = ((uint32_t)__builtin_ctz(M >> j) - 1u) & 7u;   // digits after byte j (bit 12 set)
            const uint32_t ix = ((db >> j) & 1u) ? ((((w >> (8 * j)) & 0xFu) << 3) | e) : 0u;
            c[j] = tbl[ix];
        }
        const uint32_t p1 = c[0], p2 = p1 + c[1], p3 = p2 + c[2], ls = p3 + c[3];   // < 4e7: fits 32 bits
        const uint32_t nc = (uint32_t)__builtin_popcount(cb);   // <= 2: commas are followed by digits
        const uint32_t sincl = wscan(ls, lane), cincl = wscan(nc, lane);
        const uint64_t part = carry + (sincl - ls);
        const uint32_t kl = kk + cincl - nc;          // index of the lane's first comma
        auto pre = [&](uint32_t j) { return j == 0 ? 0u : j == 1 ? p1 : j == 2 ? p2 : p3; };
        bool ovf = false;
        if (nc > 0 && kl > 0) {                       // comma k writes rank k-1
            const uint64_t rank = part + pre((uint32_t)__builtin_ctz(cb)) + (kl - 1);
            ovf |= rank > 0xFFFFFFFFull;
            TB[rev ? t.nd - kl : kl - 1] = (uint32_t)rank;
        }
        if (nc > 1) {
            const uint64_t rank = part + pre((uint32_t)__builtin_ctz(cb & (cb - 1))) + kl;
            ovf |= rank > 0xFFFFFFFFull;
            TB[rev ? t.nd - 1 - kl : kl] = (uint32_t)rank;
        }
        if (__ballot(ovf)) return false;
        carry += (uint64_t)rdl(sincl, 63);
        kk += rdl(cincl, 63);
#if PF_K0_RANKDPP
        w = pw; pw = ppw; nd0 = ndn;
#else
        w = pw; wn = pwn; wn2 = pwn2;
#endif
    }
    if (kk != t.nd) return false;                     // commas after a stray byte
    const uint64_t last = carry + (t.nd - 1);
    if (last > 0xFFFFFFFFull) return false;
    if (lane == 0) TB[rev ? 0u : t.nd - 1] = (uint32_t)last;
    return true;
}

// Per-comma SWAR parse (rounds 1-2): the fallback for counts of 8+ digits.
template <typename TP>
DEV_COLD bool k0_mm_ranks_swar(const uint32_t *gw, const uint8_t *mm, uint32_t mis, const K0Tgt &t, bool rev, TP TB,
                     uint32_t lane) {
    if (mm[t.th] != ',') return false;
    const uint32_t wend = mis + t.te;
    uint64_t carry = 0;
    uint32_t idx = 0;
    bool bad = false;
    for (uint32_t k0 = (mis + t.th) >> 2; 4 * k0 < wend; k0 += 64) {
        const uint32_t k = k0 + lane;
        const int32_t b = (int32_t)(4 * k) - (int32_t)mis;
        const uint32_t w = 4 * k < wend ? gw[k] : 0u;
        const uint32_t wn = 4 * k + 4 < wend ? gw[k + 1] : 0u;
        const uint32_t cm = bytes_eq(w, ',') & bytes_in(b, t.th, t.te);
        const uint32_t nl = (uint32_t)__builtin_popcount(cm);
        const uint32_t ie = wscan(nl, lane);
        const uint32_t gi0 = idx + ie - nl;
        const uint64_t x = ((uint64_t)wn << 32) | w;
        uint32_t vq[4] = {0, 0, 0, 0};
        uint64_t lsum = 0;
        bool ok = true;
        uint32_t m = cm;
#pragma unroll
        for (uint32_t q = 0; q < 4; q++) {
            if (!__ballot(q < nl)) break;
            if (q < nl) {
                const uint32_t pb = (uint32_t)__builtin_ctz(m) >> 3;
                m &= m - 1;
                const uint32_t xc = (uint32_t)(b + (int32_t)pb);          // the comma's text index
                const uint32_t win = 7 - pb, lim = t.te - xc - 1;        // bytes seen / bytes before te
                const uint64_t y = x >> (8 * (pb + 1));
                const uint32_t n = (uint32_t)__builtin_ctzll(nondigit_bytes(y)) >> 3;   // <= win: y's top bytes are 0
                const bool last = gi0 + q + 1 >= t.nd;
                uint64_t v;
                if (n < win || lim <= win) {
                    const uint32_t nv = n < lim ? n : lim;
                    v = nv ? swar_dec(y, nv) : 0u;
                    ok = ok && nv > 0;
                    if (!last) ok = ok && nv < lim && (uint32_t)((y >> (8 * nv)) & 0xFFu) == ',';
                } else {                              // a count of 7+ digits: byte loop
                    uint32_t kk = xc + 1;
                    v = 0;
                    while (kk < t.te && is_digit(mm[kk])) { v = v * 10u + (uint64_t)(mm[kk] - '0'); kk++; }
                    ok = ok && v <= 0xFFFFFFFFull;
                    if (!last) ok = ok && kk < t.te && mm[kk] == ',';
                }
                vq[q] = (uint32_t)v;
                lsum += (uint32_t)v;
            }
        }
        const uint64_t incl = (__ballot(lsum >= (1ull << 24)) ? wscan64(lsum, lane) : (uint64_t)wscan((uint32_t)lsum, lane)) +
                              carry;
        uint64_t run = incl - lsum;
#pragma unroll
        for (uint32_t q = 0; q < 4; q++) {
            if (q < nl) {
                run += vq[q];
                const uint64_t rank = run + gi0 + q;
                if (rank > 0xFFFFFFFFull) ok = false;
                else TB[rev ? t.nd - 1 - (gi0 + q) : gi0 + q] = (uint32_t)rank;
            }
        }
        if (__ballot(!ok)) { bad = true; break; }
        carry = rdl64(incl, 63);
        idx += rdl(ie, 63);
    }
    return !bad;
}

// Phase 2: ranks -> triggers (p<<2 | cat) in ascending p, in place in TB.
// On entry TB holds rank | ML value << 24 in forward read order (reversed for
// reverse reads, whose ranks count from the end).  Returns the trigger count
// (0 when a skip count runs past the read); `implicit` set when a 5mC call
// sits outside CpG context (852-858).
DEV uint64_t nibswap(uint64_t w) {                   // base i -> bits 4i..4i+3
    return ((w & 0x0F0F0F0F0F0F0F0Full) << 4) | ((w >> 4) & 0x0F0F0F0F0F0F0F0Full);
}
// bit 4i+3 set iff nibble i of x == 0: a nibble's low 3 bits + 7 carry into
// its bit 3 unless they are 0 (no carry leaves the nibble), so bit 3 of the
// sum | x is 0 exactly for a zero nibble (5 ops per 32 bits)
DEV uint64_t zero_nibbles_hi(uint64_t x) {
    const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
    const uint32_t zl = ~(((lo & 0x77777777u) + 0x77777777u) | lo) & 0x88888888u;
    const uint32_t zh = ~(((hi & 0x77777777u) + 0x77777777u) | hi) & 0x88888888u;
    return ((uint64_t)zh << 32) | zl;
}
DEV uint64_t zero_nibbles(uint64_t x) { return zero_nibbles_hi(x) >> 3; }   // bit 4i set iff nibble i of x == 0
// index of the k-th (k < popcount) set nibble flag (bits 4i) of m, branch-free
DEV uint32_t sel_nibble(uint64_t m, uint32_t k) {
    uint32_t lo = (uint32_t)m, base = 0;
    uint32_t c = (uint32_t)__builtin_popcount(lo);
    if (k >= c) { k -= c; lo = (uint32_t)(m >> 32); base = 8; }
    c = (uint32_t)__builtin_popcount(lo & 0xFFFFu);
    if (k >= c) { k -= c; lo >>= 16; base += 4; }
    c = (uint32_t)__builtin_popcount(lo & 0xFFu);
    if (k >= c) { k -= c; lo >>= 8; base += 2; }
    c = (uint32_t)__builtin_popcount(lo & 0xFu);
    if (k >= c) base += 1;
    return base;
}
// how many of the 8 u16 values of q (each < 2^15) are <= f: the sign bits of
// the packed differences q - (f + 1)
typedef short k0_s16x2 __attribute__((ext_vector_type(2)));
DEV uint32_t le8_u16(uint4 q, uint32_t f) {
    const uint32_t F1 = (f + 1u) * 0x10001u;
    auto neg = [&](uint32_t x) {
        const k0_s16x2 a = __builtin_bit_cast(k0_s16x2, x), b = __builtin_bit_cast(k0_s16x2, F1);
        return __builtin_bit_cast(uint32_t, (k0_s16x2)(a - b)) & 0x80008000u;
    };
    return (uint32_t)__builtin_popcount(neg(q.x)) + (uint32_t)__builtin_popcount(neg(q.y)) +
           (uint32_t)__builtin_popcount(neg(q.z)) + (uint32_t)__builtin_popcount(neg(q.w));
}
// u16 element e (0..7) of q
DEV uint32_t u16_at(uint4 q, uint32_t e) {
    const uint32_t d = e < 2 ? q.x : e < 4 ? q.y : e < 6 ? q.z : q.w;
    return (e & 1u) ? d >> 16 : d & 0xFFFFu;
}
DEV uint64_t valid_nibbles(uint32_t nv) { return nv >= 16 ? 0x1111111111111111ull : ((1ull << (4 * nv)) - 1) & 0x1111111111111111ull; }

template <typename TP>
DEV uint32_t k0_seq_pass(const pf_load_dev &d, K0W &L, const uint8_t *seq, uint32_t len, bool rev, const K0Tgt &t,
                         TP TB, uint32_t lane, bool &implicit, uint32_t &tb_off) {
    // Blocks of 1024 16-base words (16384 bases), read by 8 coalesced
    // wave-instructions of 1 KiB (lane L holds words 2L, 2L+1 of each 128-word
    // row i).  Target counts per word pair, one scan per row, and each pair's
    // forward rank base (within the block) and first-word count go to LDS.  The
    // block's triggers are then placed one per lane: row by the 8 row prefixes,
    // pair by an LDS search, word by the first-word count, base by a select in
    // the re-read word.  Reverse reads walk the blocks from the end (their
    // ranks count from the end) and turn the rank into a forward one; each
    // trigger replaces its rank in TB.
    constexpr uint32_t ROWS = 8, RW = 128, BW = ROWS * RW;
    const uint64_t pat = (rev ? (uint64_t)NT_G : (uint64_t)NT_C) * 0x1111111111111111ull;
    const uint4 *sq4 = reinterpret_cast<const uint4 *>(seq);
    const uint32_t nwords = (len + 15) / 16;
    const uint32_t nblk = (nwords + BW - 1) / BW;
    const uint32_t nd = t.nd;
    auto slot = [&](uint32_t j) { return rev ? nd - 1 - j : j; };   // rank order -> TB index
    uint32_t carry = 0, ti = 0, nout = 0;             // nout: CpG triggers written (PF_K0_FUSEC)
    bool imp = false;
    tb_off = 0;
    for (uint32_t bb = 0; bb < nblk && ti < nd; bb++) {
        const uint32_t b = rev ? nblk - 1 - bb : bb;
        uint4 v[ROWS];
#pragma unroll
        for (uint32_t i = 0; i < ROWS; i++) {
            const uint32_t w = b * BW + i * RW + 2 * lane;
            v[i] = w < nwords ? sq4[w >> 1] : make_uint4(0, 0, 0, 0);
        }
        uint32_t pref[ROWS];
        uint32_t run = 0;
        // target counts per lane (word pair) of two rows at a time, one wave
        // scan for both in 16-bit halves (a row counts at most 64 x 32 = 2048
        // targets, so the low half never carries)
        auto count = [&](uint32_t i, uint32_t &c0) {
            const uint32_t w = b * BW + i * RW + 2 * lane;
            const uint64_t xs[2] = {((uint64_t)v[i].y << 32) | v[i].x, ((uint64_t)v[i].w << 32) | v[i].z};
            uint32_t c[2];
#pragma unroll
            for (uint32_t h = 0; h < 2; h++) {
#if PF_K0_PADFIX
                (void)w;
                c[h] = (uint32_t)__popcll(zero_nibbles_hi(xs[h] ^ pat));   // past the read: 0 nibbles, no targets
#else
                c[h] = 0;
                if (w + h < nwords) {
                    if ((w + h) * 16 + 16 > len)
                        c[h] = (uint32_t)__popcll(zero_nibbles(nibswap(xs[h]) ^ pat) & valid_nibbles(len - (w + h) * 16));
                    else c[h] = (uint32_t)__popcll(zero_nibbles_hi(xs[h] ^ pat));
                }
#endif
            }
            c0 = c[0];
            return c[0] + c[1];
        };
#pragma unroll
        for (uint32_t i = 0; i < ROWS; i += 2) {
            uint32_t c0a, c0b;
            const uint32_t ca = count(i, c0a), cb = count(i + 1, c0b);
            L.u.s.sc[i * 64 + lane] = (uint8_t)c0a;
            L.u.s.sc[(i + 1) * 64 + lane] = (uint8_t)c0b;
            const uint32_t inc = wscan(ca | (cb << 16), lane);
            const uint32_t tot = rdl(inc, 63);
            pref[i] = run;
            const uint32_t ba = run + (inc & 0xFFFFu) - ca;
            L.u.s.sb[i * 64 + lane] = (uint16_t)ba;
            run += tot & 0xFFFFu;
            pref[i + 1] = run;
            const uint32_t bb2 = run + (inc >> 16) - cb;
            L.u.s.sb[(i + 1) * 64 + lane] = (uint16_t)bb2;
            run += tot >> 16;
#if PF_K0_PLACE
            if ((lane & 7u) == 0) {                   // group bases: every 8th pair's (opA is free until the walk)
                uint16_t *gb = reinterpret_cast<uint16_t *>(L.opA);
                gb[i * 8 + (lane >> 3)] = (uint16_t)ba;
                gb[(i + 1) * 8 + (lane >> 3)] = (uint16_t)bb2;
            }
#endif
        }
        const uint32_t btot = run;
        // the block's triggers: ranks < carry + btot, from ti on
        uint32_t tend = ti;
#if PF_K0_PLACE
        {
            // the answer lies in [lo, lo + n]: strided probes narrow it to a
            // stride, then one probe per lane (ranks increase with j)
            const uint32_t lim = carry + btot;
            uint32_t lo = ti, n = nd - ti;
            while (n > 64) {
                const uint32_t sd = (n + 63) / 64, off = lane * sd;
                const bool in = off < n && (TB[slot(min(lo + off, nd - 1))] & 0xFFFFFFu) < lim;
                const uint32_t c = popc(__ballot(in));
                if (c == 0) { n = 0; break; }
                const uint32_t nlo = lo + (c - 1) * sd + 1;
                n = min(c * sd, n) - (c - 1) * sd - 1;
                lo = nlo;
            }
            const bool in = lane < n && (TB[slot(min(lo + lane, nd - 1))] & 0xFFFFFFu) < lim;   // (nd > ti >= 0)
            tend = uni(lo + popc(__ballot(in)));
        }
#else
        {
            uint32_t n = nd - ti;
            while (n > 0) {
                const uint32_t h = n >> 1;
                if ((TB[slot(tend + h)] & 0xFFFFFFu) < carry + btot) { tend += h + 1; n -= h + 1; } else n = h;
            }
            tend = uni(tend);
        }
#endif
        wsync();
        // PF_K0_DIAG=5 (measurement only): the count and the trigger-range
        // search without the placement
        for (uint32_t j0 = ti; j0 < (d.diag == 5u ? ti : tend); j0 += 64) {
            const uint32_t j = j0 + lane;
            const bool act = j < tend;
            uint32_t e = 0, i = 8, Lw = 0, hw = 0, k = 0;
            uint32_t key = 0xFFFFFFFFu;
            if (act) {
                e = TB[slot(j)];
                const uint32_t rr = (e & 0xFFFFFFu) - carry;
                const uint32_t f = rev ? btot - 1 - rr : rr;    // forward rank inside the block
                i = 0;
#pragma unroll
                for (uint32_t q = 1; q < ROWS; q++) i += pref[q] <= f ? 1u : 0u;
                const uint16_t *sbi = L.u.s.sb + i * 64;
#if PF_K0_PLACE
                // last pair with base <= f: its group of 8 (the row's group
                // bases; the first is the row's own base, <= f), then the pair
                const uint4 G = *reinterpret_cast<const uint4 *>(reinterpret_cast<const uint16_t *>(L.opA) + i * 8);
                const uint32_t g = le8_u16(G, f) - 1u;
                const uint4 P = *reinterpret_cast<const uint4 *>(sbi + 8 * g);
                const uint32_t c = le8_u16(P, f) - 1u;
                Lw = 8 * g + c;
                k = f - u16_at(P, c);
#else
                uint32_t lo = 0, n = 64;                        // last pair with base <= f
                while (n > 0) { const uint32_t h = n >> 1; if (sbi[lo + h] <= f) { lo += h + 1; n -= h + 1; } else n = h; }
                Lw = lo - 1;
                k = f - sbi[Lw];
#endif
                const uint32_t c0 = L.u.s.sc[i * 64 + Lw];
                if (k >= c0) { k -= c0; hw = 1; }
            }
#if PF_K0_SEQ_REREAD
            // The trigger's word and its neighbour word (the context base at a
            // word edge) are read again from SEQ: the block was just loaded, so
            // the two 8-byte loads per trigger hit the caches.
            bool edge = false;
            uint2 xv = make_uint2(0, 0), nv = make_uint2(0, 0);
            uint32_t w = 0;
            if (act) {
                w = b * BW + i * RW + 2 * Lw + hw;
                const uint32_t wn = rev ? (w > 0 ? w - 1 : 0u) : (w + 1 < nwords ? w + 1 : w);
                const uint2 *sq2 = reinterpret_cast<const uint2 *>(seq);
                xv = sq2[w];
                nv = sq2[wn];
            }
            if (act) {
                const uint64_t xw = d.diag == 1u ? 0x2222222222222222ull : nibswap(((uint64_t)xv.y << 32) | xv.x);
                const uint64_t xn = nibswap(((uint64_t)nv.y << 32) | nv.x);
#elif PF_K0_NBRARE
            // The trigger's word comes from the registers of the lane that
            // loaded it (ds_bpermute): lane Lw of row i holds words 2Lw (x, y)
            // and 2Lw+1 (z, w).
            uint32_t x0 = 0, x1 = 0;
#pragma unroll
            for (uint32_t q = 0; q < ROWS; q++) {
                const bool mine = i == q;
                if (!__ballot(mine)) continue;
                const int sl = (int)((mine ? Lw : lane) << 2);
                const uint32_t a0 = (uint32_t)__builtin_amdgcn_ds_bpermute(sl, (int)v[q].x);
                const uint32_t a1 = (uint32_t)__builtin_amdgcn_ds_bpermute(sl, (int)v[q].y);
                const uint32_t a2 = (uint32_t)__builtin_amdgcn_ds_bpermute(sl, (int)v[q].z);
                const uint32_t a3 = (uint32_t)__builtin_amdgcn_ds_bpermute(sl, (int)v[q].w);
                if (mine) {
                    x0 = hw ? a2 : a0;
                    x1 = hw ? a3 : a1;
                }
            }
            const uint32_t w = b * BW + i * RW + 2 * Lw + hw;
            const uint64_t xw = d.diag == 1u ? 0x2222222222222222ull : nibswap(((uint64_t)x1 << 32) | x0);
            const uint32_t bi = act ? sel_nibble(zero_nibbles(xw ^ pat), k) : 0u;
            // The context base: inside the word, or -- for the word's last base
            // (forward) / first base (reverse) -- the neighbour word's first /
            // last base: the pair's other word, the next / previous pair (lane
            // Lw +- 1), the next / previous row's edge pair, or past the
            // block's edge a byte of SEQ.
            const bool atedge = act && (rev ? bi == 0 : bi == 15);
            uint32_t cb = (uint32_t)(xw >> (4 * ((rev ? bi - 1u : bi + 1u) & 15u))) & 15u;   // edge lanes: below
            if (__ballot(atedge)) {
                const uint32_t p = w * 16 + bi;
                const bool inpair = rev ? hw != 0 : hw == 0;     // the pair's other word
                uint32_t n0 = 0;
#pragma unroll
                for (uint32_t q = 0; q < ROWS; q++) {
                    const bool mine = atedge && i == q;
                    if (!__ballot(mine)) continue;
                    // the word holding the context base: forward the next word's
                    // first base (byte 0 high nibble), reverse the previous
                    // word's last base (byte 7 low nibble)
                    const uint32_t nl = inpair ? Lw : rev ? Lw - 1u : Lw + 1u;   // out of the row: 64 or ~0
                    const int snl = (int)(((mine && nl < 64u) ? nl : lane) << 2);
                    // forward: the low dword of word 2nl+1 (z, the pair's other
                    // word) or of word 2nl (x, the next pair); reverse: the high
                    // dword of word 2nl (y) or 2nl+1 (w).  ds_bpermute's source
                    // operand is one VGPR for all lanes, so both are taken.
                    const uint32_t e0 = (uint32_t)__builtin_amdgcn_ds_bpermute(snl, (int)(rev ? v[q].y : v[q].z));
                    const uint32_t e1 = (uint32_t)__builtin_amdgcn_ds_bpermute(snl, (int)(rev ? v[q].w : v[q].x));
                    uint32_t r = 0;
                    bool redge = true;                          // past the block
                    if (!rev && q + 1 < ROWS) { r = rdl(v[q + 1 < ROWS ? q + 1 : q].x, 0); redge = false; }
                    if (rev && q > 0) { r = rdl(v[q > 0 ? q - 1 : q].w, 63); redge = false; }
                    if (mine) {
                        if (inpair) n0 = e0;
                        else if (nl < 64u) n0 = e1;
                        else if (!redge) n0 = r;
                        else n0 = 0xFFFFFFFFu;                  // marker: read SEQ
                    }
                }
                if (atedge) {
                    // forward: byte 0 of the next word, high nibble; reverse:
                    // byte 7 of the previous word (byte 3 of its high dword),
                    // low nibble
                    if (n0 == 0xFFFFFFFFu) cb = p > 0 && p < len - 1 ? (rev ? nib(seq, p - 1) : nib(seq, p + 1)) : 0u;
                    else cb = rev ? (n0 >> 24) & 15u : (n0 >> 4) & 15u;
                }
            }
            if (act) {
#else
            // The trigger's word and its neighbour word (the context base at a
            // word edge) come from the registers of the lane that loaded them
            // (ds_bpermute), not from a second read of SEQ: lane Lw of row i
            // holds words 2Lw (x, y) and 2Lw+1 (z, w).
            uint32_t x0 = 0, x1 = 0, n0 = 0, n1 = 0;
            bool edge = false;
#pragma unroll
            for (uint32_t q = 0; q < ROWS; q++) {
                const bool mine = i == q;
                if (!__ballot(mine)) continue;
                const int sl = (int)((mine ? Lw : lane) << 2);
                const uint32_t a0 = (uint32_t)__builtin_amdgcn_ds_bpermute(sl, (int)v[q].x);
                const uint32_t a1 = (uint32_t)__builtin_amdgcn_ds_bpermute(sl, (int)v[q].y);
                const uint32_t a2 = (uint32_t)__builtin_amdgcn_ds_bpermute(sl, (int)v[q].z);
                const uint32_t a3 = (uint32_t)__builtin_amdgcn_ds_bpermute(sl, (int)v[q].w);
                // neighbour pair: forward reads need the next word, reverse the previous one
                const uint32_t nl = rev ? (Lw > 0 ? Lw - 1 : 0u) : (Lw < 63 ? Lw + 1 : 63u);
                const int snl = (int)((mine ? nl : lane) << 2);
                const uint32_t b0 = (uint32_t)__builtin_amdgcn_ds_bpermute(snl, (int)(rev ? v[q].z : v[q].x));
                const uint32_t b1 = (uint32_t)__builtin_amdgcn_ds_bpermute(snl, (int)(rev ? v[q].w : v[q].y));
                // across a row boundary: the next row's first word / the previous row's last word
                uint32_t r0 = 0, r1 = 0;
                bool redge = true;
                if (!rev && q + 1 < ROWS) { r0 = rdl(v[q + 1 < ROWS ? q + 1 : q].x, 0); r1 = rdl(v[q + 1 < ROWS ? q + 1 : q].y, 0); redge = false; }
                if (rev && q > 0) { r0 = rdl(v[q > 0 ? q - 1 : q].z, 63); r1 = rdl(v[q > 0 ? q - 1 : q].w, 63); redge = false; }
                if (mine) {
                    x0 = hw ? a2 : a0;
                    x1 = hw ? a3 : a1;
                    if (!rev) {
                        if (!hw) { n0 = a2; n1 = a3; }
                        else if (Lw < 63) { n0 = b0; n1 = b1; }
                        else { n0 = r0; n1 = r1; edge = redge; }
                    } else {
                        if (hw) { n0 = a0; n1 = a1; }
                        else if (Lw > 0) { n0 = b0; n1 = b1; }
                        else { n0 = r0; n1 = r1; edge = redge; }
                    }
                }
            }
            if (act) {
                const uint32_t w = b * BW + i * RW + 2 * Lw + hw;
                const uint64_t xw = d.diag == 1u ? 0x2222222222222222ull : nibswap(((uint64_t)x1 << 32) | x0);
                const uint64_t xn = nibswap(((uint64_t)n1 << 32) | n0);
#endif
#if !PF_K0_NBRARE || PF_K0_SEQ_REREAD
                const uint32_t bi = sel_nibble(zero_nibbles(xw ^ pat), k);
#endif
                const uint32_t p = w * 16 + bi;
                if (p > 0 && p < len - 1) {
                    bool ctx;
#if PF_K0_NBRARE && !PF_K0_SEQ_REREAD
                    ctx = cb == (rev ? NT_C : NT_G);
#else
                    if (!rev) ctx = (bi < 15 ? (uint32_t)(xw >> (4 * (bi + 1))) & 15u
                                             : edge ? nib(seq, p + 1) : (uint32_t)xn & 15u) == NT_G;
                    else ctx = (bi > 0 ? (uint32_t)(xw >> (4 * (bi - 1))) & 15u
                                       : edge ? nib(seq, p - 1) : (uint32_t)(xn >> 60) & 15u) == NT_C;
#endif
                    if (ctx) {
                        const uint32_t q = e >> 24;
                        key = (p << 2) | (q < d.lo ? 1u : q >= d.hi ? 0u : 2u);
                    } else imp = true;
                }
            }
#if PF_K0_FUSEC
            // the CpG triggers in rank order, compacted as they are placed: a
            // forward read's list grows from TB[0], a reverse read's (ranks
            // from the end) from TB[nd - 1] down, so either ends in ascending
            // position; every write lands on a slot this batch or an earlier
            // one has read (x <= j)
            const uint64_t kb = __ballot(act && key != 0xFFFFFFFFu);
            if (act && key != 0xFFFFFFFFu) {
                const uint32_t x = nout + below_cnt(kb);
                TB[rev ? nd - 1 - x : x] = key;
            }
            nout += popc(kb);
#else
            if (act) TB[slot(j)] = key;
#endif
        }
        wsync();
        ti = tend;
        carry += btot;
    }
    implicit = __ballot(imp) != 0;
    if (ti < nd) return 0;                            // skip counts beyond the read
    wsync();
#if PF_K0_FUSEC
    tb_off = rev ? nd - nout : 0u;
#else
    // compaction in place (order kept)
    for (uint32_t c0 = 0; c0 < nd; c0 += 64) {
        const uint32_t jj = c0 + lane;
        const uint32_t key = jj < nd ? TB[jj] : 0xFFFFFFFFu;
        const uint64_t pb = __ballot(key != 0xFFFFFFFFu);
        if (key != 0xFFFFFFFFu) TB[nout + popc(pb & lanemask_lt(lane))] = key;
        nout += popc(pb);
    }
    wsync();
#endif
    return nout;
}

// ---------------------------------------------------------------------------
// emission (uniform)
template <int MODE>
DEV void k0_emit_one(K0Out &o, uint32_t v, uint32_t cat, bool implicit) {
    if (o.n && o.last == v) {                         // 681, 704-706, 742
        if (!implicit && MODE) o.cat[o.n - 1] = (uint8_t)cat;
        return;
    }
    if (MODE) { o.pos[o.n] = v; o.cat[o.n] = (uint8_t)cat; }
    if (o.n == 0) o.first = v;
    else if (v < o.last) o.sorted = 0;
    if (v >= (1u << 29)) o.lim = 1;
    o.last = v;
    o.n++;
}

DEV void k0_bcast(K0Out &o, const K0Out &s) {
    o.n = uni(s.n); o.first = uni(s.first); o.last = uni(s.last);
    o.sorted = uni(s.sorted); o.lim = uni(s.lim);
}

// Emit up to 64 calls held one per lane (lanes with `keep`, in lane order,
// `imp` marking implicit calls): parallel unless one repeats the previous
// push's position, then lane 0 replays them through k0_emit_one.
template <int MODE>
DEV void k0_emit_lanes(const pf_load_dev &d, K0Out &o, bool keep, uint32_t v, uint32_t cat, bool imp,
                       uint32_t lane, uint32_t *sv, uint8_t *sc) {
    const uint64_t bk = __ballot(keep);
    if (!bk) return;
    const uint32_t cnt = popc(bk);
    const uint32_t idx = below_cnt(bk);                // kept lanes below this one
    uint32_t vprev;
#if PF_K0_EMITDPP
    if ((bk & (bk + 1u)) == 0) {
        // the kept lanes are lanes 0..cnt-1 (the walk's usual case): the
        // previous call is the previous lane's (DPP wave_shr:1), lane 0's the
        // last one pushed
        vprev = (uint32_t)__builtin_amdgcn_update_dpp((int)o.last, (int)v, 0x138, 0xF, 0xF, false);
    } else
#endif
    {
        const uint64_t below = bk & lanemask_lt(lane);
        const uint32_t pl = below ? 63u - (uint32_t)__clzll(below) : lane;
        const uint32_t vprev_l = (uint32_t)__shfl((int)v, (int)pl, 64);
        vprev = below ? vprev_l : o.last;
    }
    const bool has_prev = idx > 0 || o.n > 0;
    // one ballot for the three rare cases: a repeated position, a position
    // below its predecessor, a position past 2^29
    if (__ballot(keep && ((has_prev && v <= vprev) || v >= (1u << 29)))) {
        if (__ballot(keep && has_prev && v == vprev)) {
            if (d.ctr && lane == 0) atomicAdd(&d.ctr[PF_K0C_DUPCHUNK], 1ull);
            if (keep) { sv[idx] = v; sc[idx] = (uint8_t)(cat | (imp ? 0x80u : 0u)); }
            wsync();
            K0Out s = o;
            if (lane == 0)
                for (uint32_t q = 0; q < cnt; q++) k0_emit_one<MODE>(s, sv[q], sc[q] & 3u, (sc[q] & 0x80u) != 0);
            k0_bcast(o, s);
            wsync();
            return;
        }
        if (__ballot(keep && has_prev && v < vprev)) o.sorted = 0;
        if (__ballot(keep && v >= (1u << 29))) o.lim = 1;
    }
    if (MODE && keep) { o.pos[o.n + idx] = v; o.cat[o.n + idx] = (uint8_t)cat; }
    const uint32_t fl = (uint32_t)__ffsll((long long)bk) - 1, ll = 63u - (uint32_t)__clzll(bk);
    if (o.n == 0) o.first = rdl(v, fl);
    o.last = rdl(v, ll);
    o.n += cnt;
}

// Lane 0 walks the record with the reference loop itself (605-792): used for
// the stale-trigger case of a leading soft clip, and by tests for everything.
template <int MODE, typename TP>
DEV_COLD void k0_walk_seq(const uint32_t *cig, uint32_t ncig, uint32_t qs, bool rev, TP TB, uint32_t nT,
                     const uint8_t *seqi, uint32_t len, K0Out &o, bool &fatal) {
    const uint32_t cgoffset = rev ? 0xFFFFFFFFu : 0u;
    uint32_t i_read = 0, i_ref = qs, it = 0;
    uint32_t nt = TB[0] >> 2, nq = TB[0] & 3u;
    uint32_t ic = 0;
    if ((cig[0] & 15u) == 4u) {
        i_read = cig[0] >> 4;
        while (nt < i_read) {
            it++;
            if (it < nT) { nt = TB[it] >> 2; nq = TB[it] & 3u; } else break;
        }
        if (nt == i_read) {
            k0_emit_one<MODE>(o, i_ref + cgoffset, nq, false);
            it++;
            if (it < nT) { nt = TB[it] >> 2; nq = TB[it] & 3u; }
        }
        i_ref -= cig[0] >> 4;
        ic = 1;
    }
    uint32_t offset = 0;
    for (; ic < ncig; ic++) {
        const uint32_t op = cig[ic] & 15u, length = cig[ic] >> 4;
        if (op <= 1) {
            uint32_t pc = i_read;
            while (i_read + length >= nt) {
                if (op == 0 && nt != 0xFFFFFFFFu) {
                    if (seqi) {
                        const uint32_t a = nt - 1, b = i_read + length, until = a < b ? a : b;
                        for (uint32_t u = pc; u < until; u++)
                            if (u < len - 1 && nib(seqi, u) == NT_C && nib(seqi, u + 1) == NT_G) {
                                k0_emit_one<MODE>(o, i_ref + u + offset, 1, true);
                                u++;
                            }
                    }
                    k0_emit_one<MODE>(o, i_ref + nt + cgoffset + offset, nq, false);
                    pc = cgoffset == 0 ? nt + 1 : nt + 2;
                }
                it++;
                if (it >= nT) { nt = 0xFFFFFFFFu; break; }
                nt = TB[it] >> 2;
                nq = TB[it] & 3u;
            }
            if (op == 0) {
                if (seqi) {
                    const uint32_t until = i_read + length;
                    for (uint32_t u = pc; u < until; u++)
                        if (u < len - 1 && nib(seqi, u) == NT_C && nib(seqi, u + 1) == NT_G) {
                            k0_emit_one<MODE>(o, i_ref + u + offset, 1, true);
                            u++;
                        }
                }
                i_read += length;
            } else {
                i_read += length;
                offset -= length;
            }
        } else if (op == 2) {
            offset += length;
        } else if (op == 3 || op == 4) {
            break;
        } else {
            fatal = true;
            return;
        }
    }
}

// lower bound of x in the trigger positions (TB entries >> 2)
template <typename TP>
DEV uint32_t k0_tlb(TP TB, uint32_t n, uint32_t x) {
    uint32_t lo = 0;
    while (n > 0) {
        const uint32_t h = n >> 1;
        if ((TB[lo + h] >> 2) < x) { lo += h + 1; n -= h + 1; } else n = h;
    }
    return lo;
}

// Implicit mode: one chunk of read positions [c0, c0 + CB) of a CIGAR tile.
// Explicit triggers with p <= a_end and CpGs in [a_cur, a_end) that the
// reference's scan visits, merged in push order, then emitted.
template <int MODE, typename TP>
DEV_COLD void k0_chunk_implicit(const pf_load_dev &d, K0W &L, uint32_t nv, uint32_t c0, uint32_t a_cur, uint32_t a_end,
                           uint32_t i_ref, uint32_t cgoffset, bool rev, TP TB, uint32_t nT, uint32_t &tc,
                           const uint8_t *seq, uint32_t len, uint32_t lane, K0Out &o) {
    K0Merge &M = L.u.mg;
    const uint32_t c1 = c0 + PF_K0_CB;
    uint32_t ne = 0;
    for (;;) {
        const uint32_t k = tc + lane;
        const uint32_t key = k < nT ? TB[k] : 0xFFFFFFFFu;
        const uint32_t p = key >> 2;
        const bool in = k < nT && p < c1 && p <= a_end;
        const uint64_t bi = __ballot(in);
        if (!bi) break;
        bool keep = false;
        uint32_t v = 0;
        if (in) {
            const uint32_t oi = lb64<false>(L.opE, nv, p);
            keep = L.opT[oi] == 0;
            v = i_ref + p + cgoffset + L.opOff[oi];
        }
        const uint64_t bk = __ballot(keep);
        if (keep) {
            const uint32_t x = ne + popc(bk & lanemask_lt(lane));
            M.eP[x] = p;
            M.eV[x] = v;
            M.eC[x] = (uint8_t)(key & 3u);
        }
        ne += popc(bk);
        tc += popc(bi);
        if (popc(bi) < 64) break;
    }
    uint32_t ni = 0;
    if (c0 < a_end) {
        const uint32_t lo = a_cur > c0 ? a_cur : c0;
        const uint32_t hi = a_end < c1 ? a_end : c1;
        const uint32_t b0 = c0 + 4u * lane;            // 4 positions per lane
        uint32_t cm = 0;
        if (b0 < hi && b0 + 4 > lo && b0 < len) {
            const uint32_t w0 = *reinterpret_cast<const uint32_t *>(seq + (b0 >> 1) - ((b0 >> 1) & 3u));
            const uint32_t w1 = *reinterpret_cast<const uint32_t *>(seq + (b0 >> 1) - ((b0 >> 1) & 3u) + 4);
            const uint64_t w = (((uint64_t)w1 << 32) | w0) >> (8u * ((b0 >> 1) & 3u));
#pragma unroll
            for (uint32_t i = 0; i < 4; i++) {
                const uint32_t p = b0 + i;
                if (p >= lo && p < hi && p + 1 < len && nibw(w, i) == NT_C && nibw(w, i + 1) == NT_G) cm |= 1u << i;
            }
        }
        uint32_t kept = 0;
        uint32_t vv[2], pp[2];
        for (uint32_t mm = cm; mm; mm &= mm - 1) {
            const uint32_t p = b0 + (uint32_t)__builtin_ctz(mm);
            const uint32_t oi = lb64<true>(L.opE, nv, p);
            if (oi >= nv || L.opT[oi] != 0) continue;
            const uint32_t ao = L.opA[oi];
            // excluded: the positions [t-1, t+1+rev) around a trigger t the same op consumed
            uint32_t x = k0_tlb(TB, nT, p ? p - 1 : 0u);
            bool ex = false;
            for (; x < nT && (TB[x] >> 2) <= p + 1; x++) {
                const uint32_t tp = TB[x] >> 2;
                if (tp == p + 1 || (tp == p && p > ao) || (rev && tp + 1 == p && tp > ao)) ex = true;
            }
            if (ex) continue;
            pp[kept] = p;
            vv[kept] = i_ref + p + L.opOff[oi];
            kept++;
        }
        const uint32_t inc = wscan(kept, lane);
        for (uint32_t i = 0; i < kept; i++) {
            M.iP[inc - kept + i] = pp[i];
            M.iV[inc - kept + i] = vv[i];
        }
        ni = rdl(inc, 63);
    }
    wsync();
    const uint32_t nm = ne + ni;
    if (nm == 0) return;
    for (uint32_t q = lane; q < ne; q += 64) {
        const uint32_t r = q + lb64<false>(M.iP, ni, M.eP[q]);
        M.mV[r] = M.eV[q];
        M.mC[r] = M.eC[q];
    }
    for (uint32_t q = lane; q < ni; q += 64) {
        const uint32_t r = q + lb64<true>(M.eP, ne, M.iP[q]);
        M.mV[r] = M.iV[q];
        M.mC[r] = 0x80 | 1u;
    }
    wsync();
    for (uint32_t q0 = 0; q0 < nm; q0 += 64) {
        const uint32_t q = q0 + lane;
        const bool keep = q < nm;
        const uint32_t v = keep ? M.mV[q] : 0u, c = keep ? M.mC[q] : 0u;
        wsync();
        k0_emit_lanes<MODE>(d, o, keep, v, c & 3u, (c & 0x80u) != 0, lane, M.eP, M.eC);
        wsync();
    }
}

// Wave-parallel walk (phase 3).  Returns false when the CIGAR reaches a
// fatal operation.
// bam_endpos rides along: each lane sums the reference-consuming lengths of
// the operations it loads (M/D/N/=/X), every tile of the CIGAR, including the
// tiles past the last trigger (round 2 re-read the whole CIGAR afterwards).
DEV uint32_t k0_refc(uint32_t c) {
    const uint32_t op = c & 15u;
    return (op == 0 || op == 2 || op == 3 || op == 7 || op == 8) ? c >> 4 : 0u;
}

template <int MODE, typename TP>
DEV bool k0_walk(const pf_load_dev &d, K0W &L, const uint32_t *cig, uint32_t ncig, uint32_t qs, bool rev, TP TB,
                 uint32_t nT, const uint8_t *seq, uint32_t len, bool implicit, uint32_t lane, K0Out &o,
                 uint32_t &racc) {
    const uint32_t cgoffset = rev ? 0xFFFFFFFFu : 0u;
    uint32_t a_cur = 0, off_cur = 0, j = 0, tc = 0, i_ref = qs;
    if ((cig[0] & 15u) == 4u) {                       // prologue (629-652)
        const uint32_t sclip = cig[0] >> 4;
        tc = k0_tlb(TB, nT, sclip + 1);
        if (tc > 0 && (TB[tc - 1] >> 2) == sclip) k0_emit_one<MODE>(o, qs + cgoffset, TB[tc - 1] & 3u, false);
        i_ref = qs - sclip;
        a_cur = sclip;
        j = 1;
    }
    bool trunc = false;
    // the next tile in flight (three in flight measured in round 6: no faster)
    auto ld_tile = [&](uint32_t t) { return t + lane < ncig ? cig[t + lane] : 4u; };
    uint32_t cn = ld_tile(j);
    auto next_tile = [&]() { cn = j + 64 < ncig ? ld_tile(j + 64) : 4u; };   // cn is tile j + 64 then
    while (j < ncig && !trunc && (tc < nT || implicit)) {
        // ---- 64 CIGAR operations: read starts, reference offsets, ends
        const uint32_t g = j + lane;
        const uint32_t c = cn;
        next_tile();
        racc += k0_refc(c);                           // past the end: 4u (S), nothing
        const uint32_t op = c & 15u, ln = c >> 4;
        const uint64_t stop = __ballot(op == 3u || op == 4u);     // past the end acts as a stop
        const uint64_t bad = __ballot(op > 4u && g < ncig);
        const uint32_t fs = stop ? (uint32_t)__ffsll((long long)stop) - 1 : 64u;
        const uint32_t fb = bad ? (uint32_t)__ffsll((long long)bad) - 1 : 64u;
        if (fb < fs) return false;                    // exit(1) at 776-779
        const uint32_t nv = fs;
        trunc = fs < 64;
        const bool valid = lane < nv;
        const uint32_t rl = valid && op <= 1u ? ln : 0u;
        const uint32_t dl = !valid ? 0u : op == 2u ? ln : op == 1u ? 0u - ln : 0u;
        const uint32_t rin = wscan(rl, lane), din = wscan(dl, lane);
        const uint32_t a = a_cur + rin - rl, off = off_cur + din - dl;
        const uint32_t oe = valid ? a + rl : 0xFFFFFFFFu;
        L.opE[lane] = oe;
        L.opA[lane] = a;
        L.opOff[lane] = off;
        L.opT[lane] = (uint8_t)op;
#if PF_K0_WALK2
        // the 8 groups' last ends (explicit mode only: the implicit chunks use
        // the merge lists this shares)
        if (!implicit && (lane & 7u) == 7u) L.u.mg.eP[lane >> 3] = oe;
#endif
        const uint32_t a_end = a_cur + rdl(rin, 63);
        const uint32_t off_end = off_cur + rdl(din, 63);
        wsync();
        if (!implicit) {
            // the triggers this tile consumes (p <= a_end), 64 at a time
            for (;;) {
                const uint32_t k = tc + lane;
                const uint32_t key = k < nT ? TB[k] : 0xFFFFFFFFu;
                const uint32_t p = key >> 2;
                const bool in = k < nT && p <= a_end;
                const uint64_t bi = __ballot(in);
                if (!bi) break;
                bool keep = false;
                uint32_t v = 0;
                if (in) {
#if PF_K0_WALK2
                    // first operation with end >= p (ends past nv are ~0): the
                    // groups whose last end is < p, then within the group
                    auto lt8 = [&](uint4 x, uint4 y) {
                        return (x.x < p ? 1u : 0u) + (x.y < p ? 1u : 0u) + (x.z < p ? 1u : 0u) + (x.w < p ? 1u : 0u) +
                               (y.x < p ? 1u : 0u) + (y.y < p ? 1u : 0u) + (y.z < p ? 1u : 0u) + (y.w < p ? 1u : 0u);
                    };
                    const uint4 *gl = reinterpret_cast<const uint4 *>(L.u.mg.eP);
                    const uint32_t g = lt8(gl[0], gl[1]);              // < 8: the last end of the tile is >= p
                    const uint4 *ge = reinterpret_cast<const uint4 *>(L.opE + 8 * g);
                    const uint32_t oi = 8 * g + lt8(ge[0], ge[1]);
#else
                    const uint32_t oi = lb64<false>(L.opE, nv, p);
#endif
                    keep = L.opT[oi] == 0;
                    v = i_ref + p + cgoffset + L.opOff[oi];
                }
                k0_emit_lanes<MODE>(d, o, keep, v, key & 3u, false, lane, L.u.mg.mV, L.u.mg.mC);
                tc += popc(bi);
                if (popc(bi) < 64) break;
            }
        } else {
            for (uint32_t c0 = a_cur & ~3u; c0 <= a_end && (c0 < a_end || tc < nT); c0 += PF_K0_CB)
                k0_chunk_implicit<MODE>(d, L, nv, c0, a_cur, a_end, i_ref, cgoffset, rev, TB, nT, tc, seq, len,
                                        lane, o);
        }
        wsync();
        a_cur = a_end;
        off_cur = off_end;
        j += 64;
    }
    // fatal operations past the last consumed trigger are still reached
    // by the reference's loop (it walks every op up to N/S); the end position
    // counts every operation (the tile at j is already in flight in cn)
    for (; j < ncig; j += 64) {
        const uint32_t g = j + lane;
        const uint32_t c = cn;
        next_tile();
        racc += k0_refc(c);
        if (trunc) continue;
        const uint32_t op = c & 15u;
        const uint64_t stop = __ballot(op == 3u || op == 4u);
        const uint64_t bad = __ballot(op > 4u && g < ncig);
        const uint32_t fs = stop ? (uint32_t)__ffsll((long long)stop) - 1 : 64u;
        const uint32_t fb = bad ? (uint32_t)__ffsll((long long)bad) - 1 : 64u;
        if (fb < fs) return false;
        trunc = fs < 64;
    }
    return true;
}

// a record's fields, read from its wave slot's row (pf_k0_hdr) with one
// coalesced load and moved to scalar registers
struct K0Rec {
    uint32_t r, len, flag, mapq, pos, win, mlen, mln, ncig, slen, scr_len;
    float de;
    uint64_t mm_off, ml_off, seq_off, cig_off, s_lo, scr_off;
};
DEV K0Rec k0_rec(const pf_load_dev &d, uint32_t slot, uint32_t lane) {
    const uint32_t *hw = reinterpret_cast<const uint32_t *>(d.hdr + slot);
    const uint32_t v = hw[lane & 31u];
    auto w32 = [&](uint32_t k) { return rdl(v, k); };
    auto w64 = [&](uint32_t k) { return ((uint64_t)rdl(v, k + 1) << 32) | rdl(v, k); };
    K0Rec R;
    R.mm_off = w64(0); R.ml_off = w64(2); R.seq_off = w64(4); R.cig_off = w64(6); R.s_lo = w64(8); R.scr_off = w64(10);
    R.mlen = w32(12); R.mln = w32(13); R.ncig = w32(14); R.slen = w32(15);
    R.scr_len = w32(16); R.len = w32(17); R.pos = w32(18); R.r = w32(19);
    R.de = __uint_as_float(w32(20)); R.win = w32(21);
    const uint32_t fm = w32(22);
    R.flag = fm & 0xFFFFu; R.mapq = fm >> 16;
    return R;
}

// Several C m entries (a duplex-style tag, or C+m twice): every entry's rank
// list (the same C's counted: the ranks compare), each call's ML value in its
// top byte, merged in rank order -- at one C the entries' calls in MM order,
// as bam_mods_at_next_pos reports them and fill_read_meth_record_from_bam_line
// pushes them (846-880) -- and cut to one call per C, the last entry's: the
// one get_mod_poss_on_ref keeps (704-706 overwrite the quality of an equal
// position; nothing else between the duplicates depends on them).  The lists
// and the merge live in a tail slice of the staging arena (2 x the calls);
// TB receives the merged list in the single-entry layout.  Rare (no config
// has such tags): one wave, binary searches per call.
template <typename TP>
DEV bool k0_merge_targets(const pf_load_dev &d, K0W &L, const K0Tgts &T, uint32_t N, bool rev, TP TB,
                          const uint32_t *gw, const uint8_t *mmg, uint32_t mis, const uint8_t *ml, uint32_t mln,
                          uint32_t lane, uint32_t &nd_out, bool &past, bool &ovf) {
    nd_out = 0;
    ovf = false;
    unsigned long long t0 = 0;
    if (lane == 0) t0 = atomicAdd(d.stage_ctr, 2ull * N);
    const uint64_t cb = d.stage_off[d.n_recs] + (((uint64_t)uni((uint32_t)(t0 >> 32)) << 32) | uni((uint32_t)t0));
    if (cb + 2ull * N > d.stage_cap) {
        if (lane == 0) atomicOr(d.status, PF_ST_STAGE_OVF);
        ovf = true;
        return false;
    }
    uint32_t *tmp = d.stage_pos + cb, *mrg = tmp + N;
    k0_dw_table(L.u.mg.mV, lane);
    wsync();
    bool pst = false;
    for (uint32_t e = 0, oe = 0; e < T.n; e++) {
        const K0Tgt te = k0_tgt_get(T, e);
        uint32_t *TBe = tmp + oe;
        if (!k0_mm_ranks(gw, mmg, mis, te, rev, TBe, L.u.mg.mV, lane)) return false;
        wsync();
        for (uint32_t j = lane; j < te.nd; j += 64) {
            const uint32_t q = mln ? (uint32_t)ml[te.ml + (uint64_t)j * te.nc + te.mi] : 255u;
            const uint32_t sj = rev ? te.nd - 1 - j : j;
            const uint32_t rk = TBe[sj];
            pst |= rk >= (1u << 24);
            TBe[sj] = (rk & 0xFFFFFFu) | (q << 24);
        }
        wsync();
        oe += te.nd;
    }
    past = __ballot(pst) != 0;
    if (past) return true;
    // merged index: j plus, in every other list, the calls of a smaller rank
    // (and of an equal rank in the earlier entries)
    for (uint32_t e = 0, oe = 0; e < T.n; e++) {
        const uint32_t ne = k0_tgt_get(T, e).nd;
        for (uint32_t j = lane; j < ne; j += 64) {
            const uint32_t v = tmp[oe + (rev ? ne - 1 - j : j)], rk = v & 0xFFFFFFu;
            uint32_t pos = j;
            for (uint32_t f = 0, of = 0; f < T.n; f++) {
                const uint32_t nf = k0_tgt_get(T, f).nd;
                if (f != e) {
                    uint32_t lo = 0, hi = nf;              // first index whose rank is > (f < e) or >= rk
                    while (lo < hi) {
                        const uint32_t mid = (lo + hi) >> 1;
                        const uint32_t x = tmp[of + (rev ? nf - 1 - mid : mid)] & 0xFFFFFFu;
                        if (f < e ? x <= rk : x < rk) lo = mid + 1;
                        else hi = mid;
                    }
                    pos += lo;
                }
                of += nf;
            }
            mrg[pos] = v;
        }
        oe += ne;
    }
    wsync();
    // one call per C: the last of equal ranks
    uint32_t kept = 0;
    for (uint32_t k0 = 0; k0 < N; k0 += 64) {
        const uint32_t k = k0 + lane;
        const bool keep = k < N && (k + 1 == N || (mrg[k] & 0xFFFFFFu) != (mrg[k + 1] & 0xFFFFFFu));
        kept += popc(__ballot(keep));
    }
    for (uint32_t k0 = 0, base = 0; k0 < N; k0 += 64) {
        const uint32_t k = k0 + lane;
        const uint32_t v = k < N ? mrg[k] : 0u;
        const bool keep = k < N && (k + 1 == N || (v & 0xFFFFFFu) != (mrg[k + 1] & 0xFFFFFFu));
        const uint64_t b = __ballot(keep);
        if (keep) {
            const uint32_t j = base + popc(b & lanemask_lt(lane));
            TB[rev ? kept - 1 - j : j] = v;
        }
        base += popc(b);
    }
    wsync();
    nd_out = kept;
    return true;
}

template <bool MULTI, typename TP>
DEV void k0_record(const pf_load_dev &d, K0W &L, const K0Rec &R, uint32_t lane, TP TB, uint32_t cap, const K0Tgts &T,
                   bool okm) {
    K0Tgt t = T.t0;
    bool multi = false;
    uint32_t ndsum = t.nd;
    if constexpr (MULTI) {                            // the main pass only sees records of one C m entry
        multi = T.n > 1;
        for (uint32_t e = 1; e < T.n; e++) ndsum += k0_tgt_get(T, e).nd;
    }
    const uint32_t r = R.r;
    const uint32_t len = R.len;
    const bool rev = (R.flag & 16u) != 0;
    const uint8_t *mmg = d.mm + R.mm_off;
    const uint8_t *ml = d.ml + R.ml_off;
    const uint32_t mln = R.mln;
    const uint8_t *seq = d.seq + R.seq_off;
    const uint32_t *cig = d.cigar + R.cig_off;
    const uint32_t ncig = R.ncig;

    bool okmm = okm;
    uint32_t nT = 0, mlq0 = 0xFFFFFFFFu, mlq1 = 0xFFFFFFFFu;
    bool implicit = false;
    K0_T0;
    {
        const uint32_t mis = (uint32_t)(reinterpret_cast<uintptr_t>(mmg) & 3u);
        const uint32_t *gw = reinterpret_cast<const uint32_t *>(mmg - mis);
        if (okmm && ndsum > cap) okmm = false;      // only a malformed tag lists more calls than its size allows
        if (okmm && t.nd && !multi) {
            // the first 512 ML values (8 per lane, packed) are loaded before
            // the rank pass and arrive while it runs
            if (mln) {
                uint32_t q[8];
#pragma unroll
                for (uint32_t u = 0; u < 8; u++) {
                    const uint32_t j = min(lane + 64u * u, t.nd - 1);   // in the entry's ML slice (checked)
                    q[u] = ml[t.ml + (uint64_t)j * t.nc + t.mi];
                }
                mlq0 = q[0] | (q[1] << 8) | (q[2] << 16) | (q[3] << 24);
                mlq1 = q[4] | (q[5] << 8) | (q[6] << 16) | (q[7] << 24);
            }
            k0_dw_table(L.u.mg.mV, lane);
            wsync();
            okmm = k0_mm_ranks(gw, mmg, mis, t, rev, TB, L.u.mg.mV, lane);
        }
    }
    wsync();
    bool past = false;
    if constexpr (MULTI) {
        if (okmm && multi) {
            if (d.ctr && lane == 0) atomicAdd(&d.ctr[PF_K0C_MULTICM], 1ull);
            bool ovf = false;
            uint32_t ndm = 0;
            const uint32_t mis = (uint32_t)(reinterpret_cast<uintptr_t>(mmg) & 3u);
            okmm = k0_merge_targets(d, L, T, ndsum, rev, TB, reinterpret_cast<const uint32_t *>(mmg - mis), mmg, mis,
                                    ml, mln, lane, ndm, past, ovf);
            if (ovf) { if (lane == 0) d.rec_n[r] = PF_NONE; return; }
            t.nd = ndm;
        }
    }
    if (!multi && okmm && t.nd) {                        // the C+m entry's ML values ride in the ranks' top byte
        uint32_t u = 0;
        for (uint32_t j = lane; j < t.nd; j += 64, u++) {
            const uint32_t q = !mln ? 255u : u < 8 ? ((u < 4 ? mlq0 : mlq1) >> (8 * (u & 3))) & 0xFFu
                                                   : (uint32_t)ml[t.ml + (uint64_t)j * t.nc + t.mi];
            const uint32_t sj = rev ? t.nd - 1 - j : j;
            const uint32_t rk = TB[sj];
            past |= rk >= (1u << 24);                 // l_qseq < 2^24: such a rank is past the read's C's
            TB[sj] = (rk & 0xFFFFFFu) | (q << 24);
        }
        past = __ballot(past) != 0;
        wsync();
    }
    K0_STAMP(0);
    if (d.diag == 2u) { if (lane == 0) d.rec_n[r] = PF_NONE; return; }
    uint32_t tb_off = 0;
    if (okmm && t.nd && !past) nT = k0_seq_pass(d, L, seq, len, rev, t, TB, lane, implicit, tb_off);
    TB = TB + uni(tb_off);                            // the compacted triggers start here
    K0_STAMP(1);
    if (d.diag == 3u || d.diag == 5u) { if (lane == 0) d.rec_n[r] = PF_NONE; return; }
    if (!okmm && d.ctr && lane == 0) atomicAdd(&d.ctr[PF_K0C_BADMM], 1ull);
    nT = uni(nT);

    if (ncig == 0 || nT == 0) {                       // get_mod_poss_on_ref returns 0: read dropped
        if (lane == 0) d.rec_n[r] = PF_NONE;
        return;
    }
    // The record's call slice in the staging arena: its static slice (the
    // upload's trigger bound; each trigger pushes at most once), or, for an
    // implicit-canonical read -- which also pushes the CpGs the canonical scan
    // adds, CpG C's being >= 2 read bases apart -- a slice bump-allocated from
    // the arena's tail.  A full tail flags the batch: the bump pointer keeps
    // counting, so it ends at the size the run needs, and the host grows the
    // arena to that and re-runs.
    const uint64_t s_lo = R.s_lo, s_hi = R.s_lo + R.slen;
    uint64_t cb = s_lo;
    if (implicit || (uint64_t)nT > s_hi - s_lo) {
        const uint64_t need = (uint64_t)nT + (uint64_t)(len + 1) / 2;
        unsigned long long t = 0;
        if (lane == 0) t = atomicAdd(d.stage_ctr, (unsigned long long)need);
        cb = d.stage_off[d.n_recs] + (((uint64_t)uni((uint32_t)(t >> 32)) << 32) | uni((uint32_t)t));
        if (cb + need > d.stage_cap) {
            if (lane == 0) { atomicOr(d.status, PF_ST_STAGE_OVF); d.rec_n[r] = PF_NONE; }
            return;
        }
    }
    K0Out o;
    o.n = 0; o.first = 0; o.last = 0; o.sorted = 1; o.lim = 0;
    o.pos = d.stage_pos + cb;
    o.cat = d.stage_cat + cb;
    if (implicit && d.ctr && lane == 0) atomicAdd(&d.ctr[PF_K0C_IMPLICIT], 1ull);

    const uint32_t qs = R.pos;
    const bool stale = (cig[0] & 15u) == 4u && (TB[nT - 1] >> 2) <= (cig[0] >> 4);
    bool fatal = false, walked = false;
    uint32_t racc = 0;                                // this lane's share of bam_endpos (the wave walk)
    if (stale || d.force_seq) {
        if (d.ctr && lane == 0) atomicAdd(&d.ctr[PF_K0C_SEQPATH], 1ull);
        K0Out s = o;
        bool f = false;
        if (lane == 0) k0_walk_seq<1>(cig, ncig, qs, rev, TB, nT, implicit ? seq : nullptr, len, s, f);
        k0_bcast(o, s);
        fatal = uni(f ? 1u : 0u) != 0;
    } else {
        fatal = !k0_walk<1>(d, L, cig, ncig, qs, rev, TB, nT, seq, len, implicit, lane, o, racc);
        walked = true;
    }
    K0_STAMP(2);
    if (fatal) {
        if (lane == 0) { atomicOr(d.status, PF_ST_FATAL_CIGAR); d.rec_n[r] = PF_NONE; }
        return;
    }
    if (o.lim && lane == 0) atomicOr(d.status, PF_ST_POS_LIMIT);
    // ---- the calls in (pos, cat) order, then the record's scalars
    if (!o.sorted && o.n > 1) {
        if (d.ctr && lane == 0) atomicAdd(&d.ctr[PF_K0C_UNSORTED], 1ull);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        if (lane == 0) {                              // insertion sort by (pos, cat): rare, short
            for (uint32_t i = 1; i < o.n; i++) {
                const uint32_t v = o.pos[i];
                const uint8_t cc = o.cat[i];
                uint32_t k = i;
                while (k > 0 && (o.pos[k - 1] > v || (o.pos[k - 1] == v && o.cat[k - 1] > cc))) {
                    o.pos[k] = o.pos[k - 1];
                    o.cat[k] = o.cat[k - 1];
                    k--;
                }
                o.pos[k] = v;
                o.cat[k] = cc;
            }
        }
    }
    // bam_endpos: reference-consuming operations of the whole CIGAR (summed
    // by the wave walk; the lane-0 walk's records sum them here)
    uint32_t rlen = racc;
    if (!walked)
        for (uint32_t c = lane; c < ncig; c += 64) rlen += k0_refc(cig[c]);
    rlen = rdl(wscan(rlen, lane), 63);
    if (lane < 8) {                                   // the record's row: one 32-byte store
        const uint32_t v = lane == 0 ? qs : lane == 1 ? qs + rlen : lane == 2 ? o.first : lane == 3 ? o.last
                         : lane == 4 ? (uint32_t)cb : lane == 5 ? (uint32_t)(cb >> 32) : 0u;
        d.rec_out[8ull * r + lane] = v;
    }
    if (lane == 63) {
        d.rec_n[r] = o.n;
        const uint32_t w = R.win;
        atomicAdd(&d.win_kept[w], 1u);
        atomicAdd(&d.win_calls[w], o.n);
    }
    K0_STAMP(3);
}

// a record whose trigger list is past the wave's LDS list: its HBM slice
template <bool MULTI>
DEV_HBM void k0_record_hbm(const pf_load_dev &d, K0W &L, const K0Rec &R, uint32_t lane, const K0Tgts &T, bool okm) {
    k0_record<MULTI>(d, L, R, lane, d.scr + R.scr_off, R.scr_len, T, okm);
}

// One record on the wave: filters, the MM entries, the rest.  The main pass
// hands a record with several C m entries to pf_k0_multi (rare; its merge
// would cost the common path registers) and leaves its rec_n to it.
template <bool MULTI>
DEV void k0_one(const pf_load_dev &d, K0W &L, uint32_t slot, uint32_t lane) {
    const K0Rec R = k0_rec(d, slot, lane);
    const uint32_t r = R.r;
    // filters (1079-1085)
    const uint32_t flag = R.flag;
    const bool drop = (flag & 4u) || (flag & 256u) || (flag & 2048u) || R.mapq < d.min_mapq ||
                      R.len < 2u || R.len < d.min_len || (double)R.de > 0.1;
    if (drop) {
        if (lane == 0) d.rec_n[r] = PF_NONE;
        return;
    }
    // PF_K0_DIAG=4/2/3 (measurement only, results invalid): stop after the
    // filters / the MM phase / the SEQ pass, so that phase costs are kernel-time
    // differences (the s_memtime build's counter atomics distort them)
    if (d.diag == 4u) { if (lane == 0) d.rec_n[r] = PF_NONE; return; }
    // The tag's entries first: the C m entries' skip counts decide where the
    // trigger list lives -- the wave's LDS list when it fits (640), else the
    // record's HBM slice, which the upload sizes from the ML length (an upper
    // bound: dorado's h + m entries make it twice the m list, so round 2 sent
    // ~45 % of 60x records to HBM, with every rank, key and binary search of
    // their trigger lists an L2 round trip).
    const uint8_t *mmg = d.mm + R.mm_off;
    const uint32_t mis = (uint32_t)(reinterpret_cast<uintptr_t>(mmg) & 3u);
    K0Tgts T;
    T.xt = L.opE;                                     // free until the CIGAR walk (PF_K0_TW x 7 <= 64 words)
    const bool okm = k0_mm_entries<MULTI>(reinterpret_cast<const uint32_t *>(mmg - mis), mmg, mis, R.mlen, R.mln, lane, T);
    if (T.over) {                                     // more C m entries than this build merges
        if (lane == 0) { atomicOr(d.status, PF_ST_MM_LIMIT); d.rec_n[r] = PF_NONE; }
        return;
    }
    if (!MULTI && okm && T.n > 1) {
        if (lane == 0) d.multi_list[atomicAdd(d.multi_ctr, 1u)] = slot;
        return;
    }
    uint32_t ndsum = T.t0.nd;
    if constexpr (MULTI)
        for (uint32_t e = 1; e < T.n; e++) ndsum += k0_tgt_get(T, e).nd;
    if (R.scr_len == 0 || !okm || uni(ndsum) <= (uint32_t)PF_K0_TCAP)
        k0_record<MULTI>(d, L, R, lane, L.T, (uint32_t)PF_K0_TCAP, T, okm);
    else k0_record_hbm<MULTI>(d, L, R, lane, T, okm);
}

__global__ __launch_bounds__(PF_K0_WAVES * 64) __attribute__((amdgpu_waves_per_eu(PF_K0_WPE))) void pf_k0_load(pf_load_dev d) {
    __shared__ K0W lds[PF_K0_WAVES];
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wv = uni(threadIdx.x >> 6);
    const uint32_t slot = blockIdx.x * PF_K0_WAVES + wv;
    if (slot >= d.n_recs) return;
    k0_one<false>(d, lds[wv], slot, lane);
}

// The records pf_k0_load handed over (several C m entries): one wave each,
// grid-stride over its list.
__global__ __launch_bounds__(PF_K0_WAVES * 64) void pf_k0_multi(pf_load_dev d) {
    __shared__ K0W lds[PF_K0_WAVES];
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wv = uni(threadIdx.x >> 6);
    const uint32_t n = *d.multi_ctr;
    for (uint32_t i = blockIdx.x * PF_K0_WAVES + wv; i < n; i += gridDim.x * PF_K0_WAVES)
        k0_one<true>(d, lds[wv], d.multi_list[i], lane);
}

// ---------------------------------------------------------------------------
// scan: window totals -> offsets of the batch's reads, calls and site slots
// (one workgroup).  Site slots per window: calls / (2 cov_sel) + 1 (a site
// needs >= cov_sel meth and >= cov_sel unmeth calls).  When K0's arena or
// the batch arrays are too small every window is emptied (no later kernel
// touches the arrays) and the needs go to the I/O header.
template <uint32_t NT, typename T>
DEV T blk_excl_scan(T v, T *sh, T &total) {
    static_assert(NT % 64 == 0 && NT <= 4096, "block of whole waves");
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wid = tid >> 6;
    constexpr uint32_t NW = NT / 64;
    T x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const T y = __shfl_up(x, o, 64);
        if (lane >= (uint32_t)o) x += y;
    }
    if (lane == 63) sh[wid] = x;
    __syncthreads();
    if (wid == 0) {
        T s = lane < NW ? sh[lane] : (T)0;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const T y = __shfl_up(s, o, 64);
            if (lane >= (uint32_t)o) s += y;
        }
        if (lane < NW) sh[NW + lane] = s;
    }
    __syncthreads();
    const T base = wid ? sh[NW + wid - 1] : (T)0;
    total = sh[2 * NW - 1];
    __syncthreads();
    return base + x - v;
}

__global__ __launch_bounds__(PF_SCAN_THREADS) void pf_k0_scan(pf_load_dev d) {
    __shared__ uint64_t sh[2 * (PF_SCAN_THREADS / 64)];
    __shared__ uint32_t sh32[2 * (PF_SCAN_THREADS / 64)];
    const uint32_t tid = threadIdx.x, W = d.n_windows;
    uint32_t rc = 0;
    uint64_t cc = 0, sc = 0;
    for (uint32_t w0 = 0; w0 < W; w0 += PF_SCAN_THREADS) {
        const uint32_t w = w0 + tid;
        const uint32_t kept = w < W ? d.win_kept[w] : 0u;
        const uint64_t calls = w < W ? (uint64_t)d.win_calls[w] : 0ull;
        const int32_t sel = w < W ? max(d.win_par[4ull * w], 1) : 1;
        const uint64_t slots = w < W ? calls / (2ull * (uint64_t)sel) + 1ull : 0ull;
        uint32_t tk;
        uint64_t tcl, ts;
        const uint32_t ek = blk_excl_scan<PF_SCAN_THREADS, uint32_t>(kept, sh32, tk);
        const uint64_t ec = blk_excl_scan<PF_SCAN_THREADS, uint64_t>(calls, sh, tcl);
        const uint64_t es = blk_excl_scan<PF_SCAN_THREADS, uint64_t>(slots, sh, ts);
        if (w < W) {
            d.win_read_off[w] = rc + ek;
            d.win_call_off[w] = cc + ec;
            d.win_site_off[w] = sc + es;
            d.win_site_cap[w] = (uint32_t)min(slots, (uint64_t)0xFFFFFFF0u);
        }
        rc += tk;
        cc += tcl;
        sc += ts;
    }
    const uint32_t st = __hip_atomic_load(d.status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const bool c_ovf = cc > d.call_cap, s_ovf = sc > d.sites_cap;
    const bool empty = c_ovf || s_ovf || (st & (PF_ST_STAGE_OVF | PF_ST_FATAL_CIGAR | PF_ST_POS_LIMIT));
    if (tid == 0) {
        d.win_read_off[W] = rc;
        d.win_call_off[W] = cc;
        *reinterpret_cast<uint32_t *>(d.io + PF_IO_R) = rc;
        *reinterpret_cast<uint64_t *>(d.io + PF_IO_N) = cc;
        *reinterpret_cast<uint64_t *>(d.io + PF_IO_SITES) = sc;
        if (c_ovf) atomicOr(d.status, PF_ST_CALL_OVF);
        if (s_ovf) atomicOr(d.status, PF_ST_SITES_OVF);
    }
    __syncthreads();
    for (uint32_t w = tid; w <= W; w += PF_SCAN_THREADS) {
        if (empty) {
            d.win_read_off[w] = 0;
            if (w < W) d.win_site_cap[w] = 0;
        }
        d.io_win_read_off[w] = d.win_read_off[w];
    }
}

// ---------------------------------------------------------------------------
// pack: one workgroup per window.  Kept records become reads in record
// order; their scalars move to the read arrays and their calls from the
// staging slices to the window's contiguous run (one wave per read).
template <bool PIPE>
DEV void k0_pack(pf_load_dev d) {
    constexpr uint32_t NT = PF_PACK_THREADS, NW = NT / 64;
    __shared__ uint32_t sh32[2 * NW];
    __shared__ uint32_t l_n[NT];
    __shared__ uint64_t l_src[NT], l_dst[NT];
    const uint32_t w = d.win_order[blockIdx.x], tid = threadIdx.x, lane = tid & 63u, wid = tid >> 6;
    const uint32_t rb = d.win_read_off[w], re = d.win_read_off[w + 1];
    const bool last = w + 1 == d.n_windows;
    if (re == rb) {
        if (last && tid == 0) d.read_call_off[re] = re ? d.win_call_off[d.n_windows] : 0ull;
        return;
    }
    const uint32_t rec0 = d.win_rec_off[w], rec1 = d.win_rec_off[w + 1];
    uint32_t kc = 0, ccarry = 0;
    const uint64_t cb = d.win_call_off[w];
    for (uint32_t i0 = rec0; i0 < rec1; i0 += NT) {
        const uint32_t r = i0 + tid;
        const uint32_t n = r < rec1 ? d.rec_n[r] : PF_NONE;
        const bool keep = n != PF_NONE;
        uint32_t tk, tc;
        const uint32_t ek = blk_excl_scan<NT, uint32_t>(keep ? 1u : 0u, sh32, tk);
        // per-window calls fit u32 (the window totals are u32 atomics)
        const uint32_t ec = blk_excl_scan<NT, uint32_t>(keep ? n : 0u, sh32, tc);
        if (keep) {
            const uint32_t ri = rb + kc + ek;
            const uint64_t co = cb + ccarry + ec;
            const uint4 ro = reinterpret_cast<const uint4 *>(d.rec_out)[2ull * r];
            const uint2 rc = reinterpret_cast<const uint2 *>(d.rec_out)[4ull * r + 2];
            d.read_start[ri] = ro.x;
            d.read_end[ri] = ro.y;
            d.read_first[ri] = ro.z;
            d.read_last[ri] = ro.w;
            d.read_win[ri] = w;
            d.read_rec[ri] = r;
            const uint8_t h = d.hp[r];
            d.read_hp[ri] = h;
            d.hp_raw[ri] = h;
            d.read_call_off[ri] = co;
            l_n[ek] = n;
            l_src[ek] = ((uint64_t)rc.y << 32) | rc.x;
            l_dst[ek] = co;
        }
        __syncthreads();
        if constexpr (PIPE) {
        // one wave per read, 256-call chunks (4 calls per lane); the next
        // chunk's loads are issued before this chunk's stores, so a wave's
        // chunks overlap one memory round trip with the next (two chunks in
        // registers: the kernel keeps 8 waves per SIMD)
        {
            constexpr uint32_t U = PF_PACK_U;
            uint32_t j = wid, c0 = 0;
            uint32_t pv[U];
            uint8_t cv[U];
            auto load = [&](uint32_t jj, uint32_t cc, uint32_t *p8, uint8_t *q8) {
                const uint32_t cn = l_n[jj];
                const uint64_t s = l_src[jj];
#pragma unroll
                for (uint32_t u = 0; u < U; u++) {
                    const uint32_t c = cc + u * 64 + lane;
                    p8[u] = c < cn ? d.stage_pos[s + c] : 0u;
                    q8[u] = c < cn ? d.stage_cat[s + c] : (uint8_t)0;
                }
            };
            if (j < tk) load(j, 0, pv, cv);
            while (j < tk) {
                uint32_t jn = j, cn0 = c0 + U * 64;
                if (cn0 >= l_n[j]) { jn = j + NW; cn0 = 0; }
                uint32_t pn[U];
                uint8_t qn[U];
                if (jn < tk) load(jn, cn0, pn, qn);
                const uint32_t cn = l_n[j];
                const uint64_t t = l_dst[j];
#pragma unroll
                for (uint32_t u = 0; u < U; u++) {
                    const uint32_t c = c0 + u * 64 + lane;
                    if (c < cn) { d.call_pos[t + c] = pv[u]; d.call_cat[t + c] = cv[u]; }
                }
#pragma unroll
                for (uint32_t u = 0; u < U; u++) { pv[u] = pn[u]; cv[u] = qn[u]; }
                j = jn;
                c0 = cn0;
            }
        }
        } else {
        // one wave per read, 8 calls per lane in flight (loads before stores)
        for (uint32_t j = wid; j < tk; j += NW) {
            const uint32_t cn = l_n[j];
            const uint64_t s = l_src[j], t = l_dst[j];
            for (uint32_t c0 = 0; c0 < cn; c0 += 8 * 64) {
                uint32_t pv[8];
                uint8_t cv[8];
#pragma unroll
                for (uint32_t u = 0; u < 8; u++) {
                    const uint32_t c = c0 + u * 64 + lane;
                    pv[u] = c < cn ? d.stage_pos[s + c] : 0u;
                    cv[u] = c < cn ? d.stage_cat[s + c] : (uint8_t)0;
                }
#pragma unroll
                for (uint32_t u = 0; u < 8; u++) {
                    const uint32_t c = c0 + u * 64 + lane;
                    if (c < cn) { d.call_pos[t + c] = pv[u]; d.call_cat[t + c] = cv[u]; }
                }
            }
        }
        }
        __syncthreads();
        kc += tk;
        ccarry += tc;
    }
    if (last && tid == 0) d.read_call_off[re] = d.win_call_off[d.n_windows];
}
// a batch of PF_PACK_PIPE_MIN+ windows takes the pipelined copy (two
// workgroups per CU held by the register budget), a smaller one the plain one
__global__ __launch_bounds__(PF_PACK_THREADS) __attribute__((amdgpu_waves_per_eu(8))) void pf_k0_pack(pf_load_dev d) {
    k0_pack<PF_PACK_PIPE != 0>(d);
}
__global__ __launch_bounds__(PF_PACK_THREADS) void pf_k0_pack_small(pf_load_dev d) { k0_pack<false>(d); }
