// pf_load.hip -- K0: the window loader of the methphase path on the GPU.
//
// One wavefront per BAM record (4 per workgroup).  Reference semantics, all
// /root/reference/blockjoin.c:
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
//  1. MM: find the C+m entry with ballots over 64-byte chunks, parse its skip
//     counts (one lane per comma) and turn them into ranks with a wave scan.
//  2. SEQ: stream the 4-bit SEQ in 1024-base chunks (16 bases per lane), count
//     the C's (forward) or G's (reverse, ranks from the end) per lane, and
//     resolve each rank to its read position with a 64-entry LDS search and a
//     select-k-th-bit; the CpG context test and the ML category follow.  The
//     result is the trigger list T (position<<2 | category), ascending.
//  3. CIGAR: walk 64 operations per step (prefix sums of read advance and
//     reference offset), and per 512-position chunk map the triggers that the
//     reference's `while (i_read+length >= next_trigger)` loop assigns to each
//     op (an op consumes every trigger up to and INCLUDING its end) and, for
//     implicit-mode reads, the CpGs of the SEQ inside M ops that the
//     reference's canonical scan visits.  Both lists are merged in the
//     reference's push order and de-duplicated against the previous push
//     (the `calls.a[n-1] == pos` tests at 681, 704, 742).
//  4. The calls are written at the read's offset; a read whose calls are not
//     strictly increasing (rare) is sorted in place by (pos, cat), which is the
//     order the methmer kernels consume.
// A record whose leading soft clip swallows every trigger (the stale-trigger
// case of 629-652) is walked by lane 0 with a literal restatement of the loop.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "pf_device.h"
#include "pf_load.h"

#define DEV static __device__ __forceinline__
#define NT_C 2u
#define NT_G 4u

DEV uint32_t uni(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }
DEV uint64_t lanemask_lt(uint32_t lane) { return lane ? (~0ull >> (64 - lane)) : 0ull; }
DEV uint32_t popc(uint64_t m) { return (uint32_t)__popcll(m); }

DEV void wsync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

DEV uint32_t wscan(uint32_t x, uint32_t lane) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= (uint32_t)o) x += y;
    }
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
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, (int)l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(x >> 32), (int)l);
    return ((uint64_t)hi << 32) | lo;
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

struct K0W {                          // LDS of one wave (~17 KB)
    uint32_t T[PF_K0_TCAP];           // ranks, then triggers (p<<2 | cat)
    uint32_t lc[64];                  // per-lane rank bases of a SEQ chunk
    uint32_t opE[64], opOff[64], opA[64];
    uint32_t eP[PF_K0_EC], eV[PF_K0_EC];
    uint32_t iP[PF_K0_EC], iV[PF_K0_EC];
    uint32_t mV[2 * PF_K0_EC];
    uint8_t opT[64];
    uint8_t eC[PF_K0_EC];
    uint8_t mC[2 * PF_K0_EC];         // cat | 0x80 for implicit calls
};

// emission state, uniform across the wave
struct K0Out {
    uint32_t n, first, last;
    uint32_t sorted, lim;
    uint32_t *pos;                    // write mode: the read's slice of call_pos / call_cat
    uint8_t *cat;
};

// ---------------------------------------------------------------------------
// Phase 1: MM/ML -> ranks of the called C's (original orientation) in TB.
// Returns the number of ranks; *ok = 0 when the tags cannot be decoded.
struct K0Tgt { uint32_t nd, nc, mi, th, te; uint64_t ml; };

DEV bool k0_mm_entries(const uint8_t *mm, uint32_t mlen, uint32_t mln, uint32_t lane, K0Tgt &t) {
    uint32_t i = 0;
    uint64_t ml_cur = 0;
    bool found = false;
    t.nd = 0;
    while (i < mlen) {
        uint32_t e = mlen, commas = 0;
        for (uint32_t c = i; c < mlen; c += 64) {
            const uint32_t q = c + lane;
            const uint32_t ch = q < mlen ? mm[q] : 0u;
            const uint64_t semi = __ballot(q < mlen && ch == ';');
            uint64_t com = __ballot(q < mlen && ch == ',');
            if (semi) {
                const uint32_t s = (uint32_t)__ffsll((long long)semi) - 1;
                e = c + s;
                commas += popc(com & lanemask_lt(s));
                break;
            }
            commas += popc(com);
        }
        e = uni(e);
        commas = uni(commas);
        if (e - i < 3) return false;
        const uint32_t base = mm[i], strand = mm[i + 1];
        if (strand != '+' && strand != '-') return false;
        uint32_t h = i + 2, nc = 0;
        int mi = -1;
        if (is_digit(mm[h])) {
            while (h < e && is_digit(mm[h])) h++;
            nc = 1;
        } else {
            while (h < e && is_alpha(mm[h])) {
                if (mm[h] == 'm' && mi < 0) mi = (int)nc;
                nc++;
                h++;
            }
        }
        if (nc == 0) return false;
        if (base == ',') commas--;                    // count the skip list's commas only
        if (h < e && (mm[h] == '.' || mm[h] == '?')) h++;
        if (!found && base == 'C' && strand == '+' && mi >= 0 && commas > 0) {
            found = true;
            if (mln && ml_cur + (uint64_t)commas * nc > mln) return false;
            t.nd = commas; t.nc = nc; t.mi = (uint32_t)mi; t.th = h; t.te = e; t.ml = ml_cur;
        }
        ml_cur += (uint64_t)commas * nc;
        i = e + 1;
    }
    if (mln && ml_cur > mln) return false;
    return true;
}

template <typename TP>
DEV bool k0_mm_ranks(const uint8_t *mm, const K0Tgt &t, TP TB, uint32_t lane) {
    if (mm[t.th] != ',') return false;
    uint64_t carry = 0;
    uint32_t idx = 0;
    bool bad = false;
    for (uint32_t c = t.th; c < t.te; c += 64) {
        const uint32_t q = c + lane;
        const bool is_c = q < t.te && mm[q] == ',';
        const uint64_t com = __ballot(is_c);
        const uint32_t gi = idx + popc(com & lanemask_lt(lane));
        uint64_t v = 0;
        bool ok = true;
        if (is_c) {
            uint32_t k = q + 1;
            while (k < t.te && is_digit(mm[k])) { v = v * 10u + (uint64_t)(mm[k] - '0'); k++; }
            ok = k > q + 1 && v <= 0xFFFFFFFFull;
            if (gi + 1 < t.nd) ok = ok && k < t.te && mm[k] == ',';
        }
        const uint64_t incl = wscan64(is_c ? v : 0ull, lane) + carry;
        const uint64_t rank = incl + gi;
        if (is_c) {
            if (rank > 0xFFFFFFFFull) ok = false;
            if (ok) TB[gi] = (uint32_t)rank;
        }
        if (__ballot(is_c && !ok)) { bad = true; break; }
        carry = rdl64(incl, 63);
        idx += popc(com);
    }
    return !bad;
}

// Phase 2: ranks -> triggers (p<<2 | cat) in ascending p, in place in TB.
// Returns the trigger count (0 on failure); *implicit set when a 5mC call sits
// outside CpG context (852-858).
template <typename TP>
DEV uint32_t k0_seq_pass(const pf_load_dev &d, const uint8_t *seq, uint32_t len, bool rev, const uint8_t *ml,
                         uint32_t mln, const K0Tgt &t, TP TB, uint32_t *lc, uint32_t lane, bool &implicit) {
    const uint32_t tb = rev ? NT_G : NT_C;
    uint32_t carry = 0, ti = 0, nout = 0;
    bool imp = false;
    const uint32_t nch = (len + 1023) / 1024;
    for (uint32_t ci = 0; ci < nch && ti < t.nd; ci++) {
        const uint32_t c0 = (rev ? nch - 1 - ci : ci) * 1024u;
        const uint32_t b0 = c0 + 16u * lane;
        const uint32_t nv = b0 < len ? (len - b0 < 16u ? len - b0 : 16u) : 0u;
        const uint64_t w = nv ? *reinterpret_cast<const uint64_t *>(seq + (b0 >> 1)) : 0ull;
        const uint32_t m = match16(w, tb, nv);
        const uint32_t cnt = (uint32_t)__builtin_popcount(m);
        const uint32_t incl = wscan(cnt, lane);
        const uint32_t tot = uni(__shfl(incl, 63, 64));
        lc[lane] = rev ? carry + tot - incl : carry + incl - cnt;
        wsync();
        for (;;) {
            const uint32_t j = ti + lane;
            const uint32_t rk = j < t.nd ? TB[j] : 0xFFFFFFFFu;
            const bool inr = j < t.nd && rk < carry + tot;
            const uint64_t bal = __ballot(inr);
            if (!bal) break;
            const uint32_t nb = popc(bal);
            // owning lane: last lane with lc <= rk (forward), first (reverse)
            uint32_t L = 0;
            if (rev) {
                uint32_t lo = 0, n = 64;
                while (n > 0) { const uint32_t h = n >> 1; if (lc[lo + h] > rk) { lo += h + 1; n -= h + 1; } else n = h; }
                L = lo;
            } else {
                uint32_t lo = 0, n = 64;
                while (n > 0) { const uint32_t h = n >> 1; if (lc[lo + h] <= rk) { lo += h + 1; n -= h + 1; } else n = h; }
                L = lo - 1;
            }
            L = inr ? L : lane;
            const uint64_t wl = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(w >> 32), (int)L, 64) << 32) |
                                (uint32_t)__shfl((int)(uint32_t)w, (int)L, 64);
            const uint32_t ml_ = (uint32_t)__shfl((int)m, (int)L, 64);
            bool pass = false, hit = false;
            uint32_t key = 0;
            if (inr) {
                const uint32_t k = rk - lc[L];
                const uint32_t cL = (uint32_t)__builtin_popcount(ml_);
                const uint32_t bit = select_bit(ml_, rev ? cL - 1 - k : k);
                const uint32_t p = c0 + 16u * L + bit;
                const uint32_t q = mln ? ml[t.ml + (uint64_t)j * t.nc + t.mi] : 255u;
                if (p > 0 && p < len - 1) {
                    const bool ctx = nibw(wl, bit) == NT_C ? nib(seq, p + 1) == NT_G : nib(seq, p - 1) == NT_C;
                    pass = ctx;
                    hit = !ctx;
                }
                const uint32_t cat = q < d.lo ? 1u : q >= d.hi ? 0u : 2u;
                key = (p << 2) | cat;
            }
            const uint64_t pb = __ballot(pass);
            if (pass) TB[nout + popc(pb & lanemask_lt(lane))] = key;
            if (__ballot(hit)) imp = true;
            nout += popc(pb);
            ti += nb;
            wsync();
            if (nb < 64) break;
        }
        carry += tot;
        wsync();
    }
    implicit = imp;
    if (ti < t.nd) return 0;                          // skip counts beyond the read
    if (rev) {                                        // produced in descending p
        for (uint32_t a = lane; a < nout / 2; a += 64) {
            const uint32_t x = TB[a], y = TB[nout - 1 - a];
            TB[a] = y;
            TB[nout - 1 - a] = x;
        }
        wsync();
    }
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

// Lane 0 walks the record with the reference loop itself (605-792): used for
// the stale-trigger case of a leading soft clip, and by tests for everything.
template <int MODE, typename TP>
DEV void k0_walk_seq(const uint32_t *cig, uint32_t ncig, uint32_t qs, bool rev, TP TB, uint32_t nT,
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

// Wave-parallel walk (phase 3).  Returns false when the CIGAR reaches a
// fatal operation.
template <int MODE, typename TP>
DEV bool k0_walk(const pf_load_dev &d, K0W &L, const uint32_t *cig, uint32_t ncig, uint32_t qs, bool rev, TP TB,
                 uint32_t nT, const uint8_t *seq, uint32_t len, bool implicit, uint32_t lane, K0Out &o) {
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
    while (j < ncig && !trunc) {
        // ---- 64 CIGAR operations: read starts, reference offsets, ends
        const uint32_t g = j + lane;
        const uint32_t c = g < ncig ? cig[g] : (4u);   // past the end acts as a stop
        const uint32_t op = c & 15u, ln = c >> 4;
        const uint64_t stop = __ballot(op == 3u || op == 4u);
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
        L.opE[lane] = valid ? a + rl : 0xFFFFFFFFu;
        L.opA[lane] = a;
        L.opOff[lane] = off;
        L.opT[lane] = (uint8_t)op;
        const uint32_t a_end = a_cur + uni(__shfl(rin, 63, 64));
        const uint32_t off_end = off_cur + uni(__shfl(din, 63, 64));
        wsync();
        // ---- chunks of read positions: explicit p in (a_cur, a_end], implicit p in [a_cur, a_end)
        for (uint32_t c0 = a_cur & ~7u; c0 <= a_end && (c0 < a_end || tc < nT); c0 += PF_K0_CB) {
            const uint32_t c1 = c0 + PF_K0_CB;
            // explicit triggers of the chunk
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
                    L.eP[x] = p;
                    L.eV[x] = v;
                    L.eC[x] = (uint8_t)(key & 3u);
                }
                ne += popc(bk);
                tc += popc(bi);
                if (popc(bi) < 64) break;
            }
            // implicit canonicals of the chunk (8 positions per lane)
            uint32_t ni = 0;
            if (implicit && c0 < a_end) {
                const uint32_t lo = a_cur > c0 ? a_cur : c0;
                const uint32_t hi = a_end < c1 ? a_end : c1;
                const uint32_t b0 = c0 + 8u * lane;
                uint32_t cm = 0;
                if (b0 < hi && b0 + 8 > lo && b0 < len) {
                    const uint32_t w0 = *reinterpret_cast<const uint32_t *>(seq + (b0 >> 1));
                    const uint32_t w1 = *reinterpret_cast<const uint32_t *>(seq + (b0 >> 1) + 4);
                    const uint64_t w = ((uint64_t)w1 << 32) | w0;
#pragma unroll
                    for (uint32_t i = 0; i < 8; i++) {
                        const uint32_t p = b0 + i;
                        if (p >= lo && p < hi && p + 1 < len && nibw(w, i) == NT_C && nibw(w, i + 1) == NT_G)
                            cm |= 1u << i;
                    }
                }
                // keep the CpGs the reference's scan visits: inside an M op,
                // not within a consumed trigger's exclusion window
                uint32_t kept = 0;
                uint32_t vv[4], pp[4];
                for (uint32_t mm = cm; mm; mm &= mm - 1) {
                    const uint32_t p = b0 + (uint32_t)__builtin_ctz(mm);
                    const uint32_t oi = lb64<true>(L.opE, nv, p);
                    if (oi >= nv || L.opT[oi] != 0) continue;
                    const uint32_t ao = L.opA[oi];
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
                    L.iP[inc - kept + i] = pp[i];
                    L.iV[inc - kept + i] = vv[i];
                }
                ni = uni(__shfl(inc, 63, 64));
            }
            wsync();
            // ---- merge in push order (by position; explicit first on ties) and emit
            const uint32_t nm = ne + ni;
            if (nm == 0) continue;
            if (ni == 0) {
                for (uint32_t q = lane; q < ne; q += 64) { L.mV[q] = L.eV[q]; L.mC[q] = L.eC[q]; }
            } else {
                for (uint32_t q = lane; q < ne; q += 64) {
                    const uint32_t r = q + lb64<false>(L.iP, ni, L.eP[q]);
                    L.mV[r] = L.eV[q];
                    L.mC[r] = L.eC[q];
                }
                for (uint32_t q = lane; q < ni; q += 64) {
                    const uint32_t r = q + lb64<true>(L.eP, ne, L.iP[q]);
                    L.mV[r] = L.iV[q];
                    L.mC[r] = 0x80 | 1u;
                }
            }
            wsync();
            bool dup = false;
            for (uint32_t q0 = 0; q0 < nm; q0 += 64) {
                const uint32_t q = q0 + lane;
                const uint32_t prev = q == 0 ? o.last : L.mV[q - 1];
                if (__ballot(q < nm && (q > 0 || o.n > 0) && L.mV[q] == prev)) dup = true;
            }
            if (dup) {                                // rare: sequential emission with qual replacement
                if (d.ctr && lane == 0) atomicAdd(&d.ctr[PF_K0C_DUPCHUNK], 1ull);
                K0Out s = o;
                if (lane == 0)
                    for (uint32_t q = 0; q < nm; q++)
                        k0_emit_one<MODE>(s, L.mV[q], L.mC[q] & 3u, (L.mC[q] & 0x80) != 0);
                o.n = uni(s.n); o.first = uni(s.first); o.last = uni(s.last);
                o.sorted = uni(s.sorted); o.lim = uni(s.lim);
            } else {
                bool uns = false, lim = false;
                for (uint32_t q0 = 0; q0 < nm; q0 += 64) {
                    const uint32_t q = q0 + lane;
                    if (q < nm) {
                        const uint32_t v = L.mV[q];
                        if (MODE) { o.pos[o.n + q] = v; o.cat[o.n + q] = L.mC[q] & 3u; }
                        const uint32_t prev = q == 0 ? o.last : L.mV[q - 1];
                        if ((q > 0 || o.n > 0) && v < prev) uns = true;
                        if (v >= (1u << 29)) lim = true;
                    }
                }
                if (__ballot(uns)) o.sorted = 0;
                if (__ballot(lim)) o.lim = 1;
                if (o.n == 0) o.first = L.mV[0];
                o.last = L.mV[nm - 1];
                o.n += nm;
            }
            wsync();
        }
        a_cur = a_end;
        off_cur = off_end;
        j += 64;
    }
    return true;
}

template <int MODE, typename TP>
DEV void k0_record(const pf_load_dev &d, K0W &L, uint32_t r, uint32_t lane, TP TB, uint32_t cap) {
    const uint32_t len = d.l_qseq[r];
    const bool rev = (d.flag[r] & 16u) != 0;
    const uint8_t *mm = d.mm + d.mm_off[r];
    const uint32_t mlen = (uint32_t)(d.mm_off[r + 1] - d.mm_off[r]);
    const uint8_t *ml = d.ml + d.ml_off[r];
    const uint32_t mln = (uint32_t)(d.ml_off[r + 1] - d.ml_off[r]);
    const uint8_t *seq = d.seq + d.seq_off[r];
    const uint32_t *cig = d.cigar + d.cigar_off[r];
    const uint32_t ncig = (uint32_t)(d.cigar_off[r + 1] - d.cigar_off[r]);

    K0Tgt t;
    bool okmm = k0_mm_entries(mm, mlen, mln, lane, t);
    uint32_t nT = 0;
    bool implicit = false;
    if (okmm && t.nd > cap) okmm = false;           // only a malformed tag lists more calls than its size allows
    if (okmm && t.nd) okmm = k0_mm_ranks(mm, t, TB, lane);
    if (okmm && t.nd) nT = k0_seq_pass(d, seq, len, rev, ml, mln, t, TB, L.lc, lane, implicit);
    if (!okmm && d.ctr && lane == 0) atomicAdd(&d.ctr[PF_K0C_BADMM], 1ull);
    nT = uni(nT);

    if (ncig == 0 || nT == 0) {                       // get_mod_poss_on_ref returns 0: read dropped
        if (MODE == 0 && lane == 0) d.rec_n[r] = PF_NONE;
        return;
    }
    const uint32_t ri = MODE ? d.rec_read[r] : 0;
    K0Out o;
    o.n = 0; o.first = 0; o.last = 0; o.sorted = 1; o.lim = 0;
    o.pos = MODE ? d.call_pos + d.read_call_off[ri] : nullptr;
    o.cat = MODE ? d.call_cat + d.read_call_off[ri] : nullptr;
    if (implicit && d.ctr && lane == 0) atomicAdd(&d.ctr[PF_K0C_IMPLICIT], 1ull);

    const uint32_t qs = d.pos[r];
    const bool stale = (cig[0] & 15u) == 4u && (TB[nT - 1] >> 2) <= (cig[0] >> 4);
    bool fatal = false;
    if (stale || d.force_seq) {
        if (d.ctr && lane == 0) atomicAdd(&d.ctr[PF_K0C_SEQPATH], 1ull);
        K0Out s = o;
        bool f = false;
        if (lane == 0) k0_walk_seq<MODE>(cig, ncig, qs, rev, TB, nT, implicit ? seq : nullptr, len, s, f);
        o.n = uni(s.n); o.first = uni(s.first); o.last = uni(s.last);
        o.sorted = uni(s.sorted); o.lim = uni(s.lim);
        fatal = uni(f ? 1u : 0u) != 0;
    } else {
        fatal = !k0_walk<MODE>(d, L, cig, ncig, qs, rev, TB, nT, seq, len, implicit, lane, o);
    }
    if (fatal) {
        if (lane == 0) atomicOr(d.status, PF_ST_FATAL_CIGAR);
        if (MODE == 0 && lane == 0) d.rec_n[r] = PF_NONE;
        return;
    }
    if (o.lim && lane == 0) atomicOr(d.status, PF_ST_POS_LIMIT);
    if (MODE == 0) {
        if (lane == 0) d.rec_n[r] = o.n;
        return;
    }
    // ---- write mode: sort if needed, then the read's scalars
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
    // bam_endpos: reference-consuming operations of the whole CIGAR
    uint32_t rlen = 0;
    for (uint32_t c = lane; c < ncig; c += 64) {
        const uint32_t op = cig[c] & 15u;
        if (op == 0 || op == 2 || op == 3 || op == 7 || op == 8) rlen += cig[c] >> 4;
    }
    rlen = wscan(rlen, lane);
    if (lane == 63) {
        d.read_start[ri] = qs;
        d.read_end[ri] = qs + rlen;
        d.read_first[ri] = o.first;
        d.read_last[ri] = o.last;
    }
}

template <int MODE>
__global__ __launch_bounds__(PF_K0_WAVES * 64) void pf_k0_load(pf_load_dev d) {
    __shared__ K0W lds[PF_K0_WAVES];
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wv = uni(threadIdx.x >> 6);
    const uint32_t r = blockIdx.x * PF_K0_WAVES + wv;
    if (r >= d.n_recs) return;
    K0W &L = lds[wv];
    if (MODE == 1 && d.rec_read[r] == PF_NONE) return;
    // filters (1079-1085)
    const uint32_t flag = d.flag[r];
    const bool drop = (flag & 4u) || (flag & 256u) || (flag & 2048u) || (uint32_t)d.mapq[r] < d.min_mapq ||
                      d.l_qseq[r] < 2u || d.l_qseq[r] < d.min_len || (double)d.de[r] > 0.1;
    if (drop) {
        if (MODE == 0 && lane == 0) d.rec_n[r] = PF_NONE;
        return;
    }
    const uint64_t s0 = d.scr_off[r], s1 = d.scr_off[r + 1];
    if (s1 == s0) k0_record<MODE>(d, L, r, lane, L.T, (uint32_t)PF_K0_TCAP);
    else k0_record<MODE>(d, L, r, lane, d.scr + s0, (uint32_t)(s1 - s0));
}

template __global__ void pf_k0_load<0>(pf_load_dev d);
template __global__ void pf_k0_load<1>(pf_load_dev d);
