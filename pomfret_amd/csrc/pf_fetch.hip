// pf_fetch.hip -- the region fetch of load_reads_given_interval on the device
// (blockjoin.c:1053-1076 through htslib's sam_itr_querys / sam_itr_next),
// over BGZF runs already inflated into the arena (pf_inflate.hip).
//
// The host (pf_ingest.hip) plans the fetch from the BAI exactly as
// pf_bam_fetch_windows does (the same chunk lists, pf_bam_query_chunks), reads
// the compressed bytes of the blocks those chunks touch (plus an extension for
// records that run past a chunk's last block) and ships them; here:
//   pf_chain    one lane per run: the record chain (block_size hops) from the
//               run's first chunk start -- every chunk start of the run is on
//               it (count pass, then write pass);
//   pf_recdec   one wavefront per record: the fields bam_read1 / rec_decode
//               validates, the CG:B:I long-CIGAR swap (bam_tag2cigar), query
//               and reference length of the CIGAR (lane-parallel), and one aux
//               walk for de, HP, MM/Mm, ML/Ml, CG and MD with the host
//               reader's semantics (pf_bam.c aux_find: the walk stops at the
//               first malformed tag; Z strings are scanned lane-parallel);
//   pf_select   one wavefront per window: the chunk walk of hts_itr_next with
//               its `done` offset -- records read while their start is before
//               the chunk's end, the fetch ending at EOF, a record of another
//               tid, pos >= end or a truncated record; a record is returned
//               when pos + rlen > beg (count pass, then write pass);
//   pf_gather_small / pf_gather_big   the returned records' fields into the
//               record-level batch layout K0 reads (pf_load.h): small fields
//               to SoA arrays, CIGAR / SEQ (16-byte aligned slices) / MM / ML /
//               qname copied out of the arena.
// Positions are arena byte offsets; a virtual offset's comparison order is
// the arena order (runs are laid out in file order, and the offset htslib
// reports after a block's last byte -- the next block's start -- is the same
// arena position).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "pf_ingest.h"

#define DEV static __device__ __forceinline__

DEV uint32_t uni(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }
DEV uint64_t uni64(uint64_t x) { return ((uint64_t)uni((uint32_t)(x >> 32)) << 32) | uni((uint32_t)x); }
DEV uint64_t lanemask_lt(uint32_t lane) { return lane ? (~0ull >> (64 - lane)) : 0ull; }

// unaligned little-endian loads from the arena (padded: reads may run 8 bytes past)
DEV uint32_t ld32u(const uint8_t *a, uint64_t p) {
    const uint64_t q = p & ~3ull;
    const uint32_t s = (uint32_t)(p & 3u) * 8u;
    const uint32_t w0 = *reinterpret_cast<const uint32_t *>(a + q);
    if (!s) return w0;
    const uint32_t w1 = *reinterpret_cast<const uint32_t *>(a + q + 4);
    return (w0 >> s) | (w1 << (32 - s));
}
DEV uint32_t ld16u(const uint8_t *a, uint64_t p) { return ld32u(a, p) & 0xFFFFu; }

// ---------------------------------------------------------------------------
// The record chain, split at the chunk starts the index already knows to be
// record boundaries: one lane per segment walks block_size hops from its
// start; a segment other than its run's last must land exactly on the next
// start (else the chain is treated as corrupt there).  Count pass (rec_pos
// null): n, stop, stop_pos per segment; write pass: positions from rec0.
__global__ __launch_bounds__(64) void pf_chain(const uint8_t *arena, pf_seg_dev *segs, uint32_t n_segs,
                                               uint64_t *rec_pos) {
    const uint32_t i = blockIdx.x * 64 + threadIdx.x;
    if (i >= n_segs) return;
    const pf_seg_dev S = segs[i];
    if (rec_pos && !S.live) return;
    uint64_t p = S.s;
    uint32_t n = 0, stop = PF_CHAIN_END;
    while (p < S.e) {
        if (p + 4 > S.a1) { stop = PF_CHAIN_CUT; break; }
        const uint32_t bs = ld32u(arena, p);
        if (bs < 32 || bs > (1u << 30)) { stop = PF_CHAIN_CORRUPT; break; }
        if (p + 4 + bs > S.a1) { stop = PF_CHAIN_CUT; break; }
        if (rec_pos) rec_pos[S.rec0 + n] = p;
        n++;
        p += 4 + (uint64_t)bs;
    }
    if (!S.last && stop == PF_CHAIN_END && p != S.e) stop = PF_CHAIN_CORRUPT;   // overshot a known boundary
    if (!rec_pos) {
        segs[i].n = n;
        segs[i].stop = stop;
        segs[i].stop_pos = p;
    }
}

// ---------------------------------------------------------------------------
// record decode
DEV bool wave_find_nul(const uint8_t *a, uint64_t from, uint64_t end, uint32_t lane, uint64_t &at) {
    for (uint64_t q0 = from; q0 < end; q0 += 64) {
        const uint64_t q = q0 + lane;
        const bool z = q < end && a[q] == 0;
        const uint64_t m = __ballot(z);
        if (m) { at = q0 + (uint64_t)__ffsll((long long)m) - 1; return true; }
    }
    return false;
}

// aux field size past its 3-byte header (pf_bam.c aux_size); 0 = malformed
DEV uint64_t aux_size(const uint8_t *a, uint64_t p, uint64_t end, uint32_t lane) {
    const uint32_t t = a[p + 2];
    const uint64_t v = p + 3;
    switch (t) {
    case 'A': case 'c': case 'C': return 1;
    case 's': case 'S': return 2;
    case 'i': case 'I': case 'f': return 4;
    case 'd': return 8;
    case 'Z': case 'H': {
        uint64_t at;
        if (!wave_find_nul(a, v, end, lane, at)) return 0;
        return uni64(at) - v + 1;
    }
    case 'B': {
        if (v + 5 > end) return 0;
        const uint32_t cnt = ld32u(a, v + 1);
        uint64_t es;
        switch (a[v]) {
        case 'c': case 'C': es = 1; break;
        case 's': case 'S': es = 2; break;
        case 'i': case 'I': case 'f': es = 4; break;
        default: return 0;
        }
        return 5 + (uint64_t)cnt * es;
    }
    default: return 0;
    }
}

DEV bool aux_int(const uint8_t *a, uint64_t p, int64_t &out) {
    const uint64_t v = p + 3;
    switch (a[p + 2]) {
    case 'c': out = (int8_t)a[v]; return true;
    case 'C': out = a[v]; return true;
    case 's': out = (int16_t)ld16u(a, v); return true;
    case 'S': out = ld16u(a, v); return true;
    case 'i': out = (int32_t)ld32u(a, v); return true;
    case 'I': out = ld32u(a, v); return true;
    default: return false;
    }
}

DEV double aux_f(const uint8_t *a, uint64_t p) {           // bam_aux2f
    const uint64_t v = p + 3;
    int64_t x;
    if (a[p + 2] == 'd') {
        const uint64_t bits = (uint64_t)ld32u(a, v) | ((uint64_t)ld32u(a, v + 4) << 32);
        return __longlong_as_double((long long)bits);
    }
    if (a[p + 2] == 'f') return (double)__uint_as_float(ld32u(a, v));
    if (aux_int(a, p, x)) return (double)x;
    return 0.0;
}

#define TAG(x, y) ((uint32_t)(x) | ((uint32_t)(y) << 8))

__global__ __launch_bounds__(256) void pf_recdec(const uint8_t *arena, uint32_t n_recs, pf_recs_dev R) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t r = uni(blockIdx.x * 4 + (threadIdx.x >> 6));
    if (r >= n_recs) return;
    const uint8_t *a = arena;
    const uint64_t p = uni64(R.pos[r]);
    const uint32_t bs = ld32u(a, p);
    const uint64_t d = p + 4, dend = d + bs;
    const int32_t tid = (int32_t)ld32u(a, d), pos = (int32_t)ld32u(a, d + 4);
    const uint32_t lrn = a[d + 8], mapq = a[d + 9];
    uint32_t ncig = ld16u(a, d + 12);
    const uint32_t flag = ld16u(a, d + 14);
    const int32_t lseq = (int32_t)ld32u(a, d + 16);
    uint8_t st = 0;
    uint64_t cig = d + 32 + lrn;
    const uint64_t seq = cig + 4ull * ncig;
    uint64_t aux = seq + ((uint64_t)lseq + 1) / 2 + (uint64_t)lseq;
    if (lseq < 0 || lrn == 0 || aux > dend) st |= PF_REC_CORRUPT;
    // qname: strnlen over l_read_name bytes
    uint32_t qlen = lrn;
    {
        uint64_t at;
        if (!(st & PF_REC_CORRUPT) && wave_find_nul(a, d + 32, d + 32 + lrn, lane, at)) qlen = (uint32_t)(uni64(at) - (d + 32));
    }
    // aux walk: first occurrence of each wanted tag before any malformed one
    uint64_t t_de = 0, t_hp = 0, t_mm = 0, t_mm2 = 0, t_ml = 0, t_ml2 = 0, t_cg = 0, t_md = 0;
    uint64_t mm_z = 0, mm2_z = 0, md_z = 0;       // Z sizes (incl. NUL)
    if (!(st & PF_REC_CORRUPT)) {
        uint64_t q = aux;
        while (q + 3 <= dend) {
            const uint64_t s = aux_size(a, q, dend, lane);
            if (s == 0 || q + 3 + s > dend) break;
            const uint32_t tg = TAG(a[q], a[q + 1]);
            if (tg == TAG('d', 'e') && !t_de) t_de = q + 1;
            else if (tg == TAG('H', 'P') && !t_hp) t_hp = q + 1;
            else if (tg == TAG('M', 'M') && !t_mm) { t_mm = q + 1; mm_z = s; }
            else if (tg == TAG('M', 'm') && !t_mm2) { t_mm2 = q + 1; mm2_z = s; }
            else if (tg == TAG('M', 'L') && !t_ml) t_ml = q + 1;
            else if (tg == TAG('M', 'l') && !t_ml2) t_ml2 = q + 1;
            else if (tg == TAG('C', 'G') && !t_cg) t_cg = q + 1;
            else if (tg == TAG('M', 'D') && !t_md) { t_md = q + 1; md_z = s; }
            q = uni64(q + 3 + s);
        }
    }
    // (tag positions are stored + 1 so that 0 means absent)
    // bam_tag2cigar: the kSmN placeholder with a CG:B:I / B:i tag
    if (!(st & PF_REC_CORRUPT) && ncig > 0 && tid >= 0 && pos >= 0) {
        const uint32_t c0 = ld32u(a, cig);
        if ((c0 & 15u) == 4u && (c0 >> 4) == (uint32_t)lseq && t_cg) {
            const uint64_t t = t_cg - 1;
            if (a[t + 2] == 'B' && (a[t + 3] == 'I' || a[t + 3] == 'i')) {
                const uint32_t n = ld32u(a, t + 4);
                if (n >= ncig && n < (1u << 29)) { cig = t + 8; ncig = n; }
            }
        }
    }
    // CIGAR query and reference lengths (lane-parallel)
    uint64_t rl = 0, ql = 0;
    uint32_t nins = 0;
    if (!(st & PF_REC_CORRUPT)) {
        for (uint32_t c = lane; c < ncig; c += 64) {
            const uint32_t v = ld32u(a, cig + 4ull * c), op = v & 15u, ln = v >> 4;
            if (op == 0 || op == 2 || op == 3 || op == 7 || op == 8) rl += ln;
            if (op == 0 || op == 1 || op == 4 || op == 7 || op == 8) ql += ln;
            nins += op == 1 ? 1u : 0u;
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) nins += (uint32_t)__shfl_xor((int)nins, o, 64);
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            rl += (uint64_t)__shfl_xor((long long)rl, o, 64);
            ql += (uint64_t)__shfl_xor((long long)ql, o, 64);
        }
        if (ncig > 0 && lseq > 0 && !(flag & 4u) && ql != (uint64_t)lseq) st |= PF_REC_TRUNC;
    }
    if ((flag & 4u) || ncig == 0) rl = 0;
    if (rl == 0) rl = 1;
    float de = -1.f;
    if (t_de) de = (float)aux_f(a, t_de - 1);
    int32_t hp_tag = INT32_MIN;
    uint32_t hp = 254;
    if (t_hp) {
        int64_t v = 0;
        if (!aux_int(a, t_hp - 1, v)) v = 0;
        hp_tag = v < INT32_MIN ? INT32_MIN + 1 : v > INT32_MAX ? INT32_MAX : (int32_t)v;
        hp = (v >= 1 && v <= 255) ? (uint32_t)(v - 1) : 254u;
    }
    uint64_t mm = t_mm ? t_mm : t_mm2, mmz = t_mm ? mm_z : mm2_z;
    const uint64_t ml = t_ml ? t_ml : t_ml2;
    bool ok = true;
    if (mm && a[mm - 1 + 2] != 'Z') ok = false;
    if (ml && (a[ml - 1 + 2] != 'B' || a[ml - 1 + 3] != 'C')) ok = false;
    uint32_t mm_len = 0, ml_len = 0;
    uint64_t mm_pos = 0, ml_pos = 0;
    if (ok && mm) {
        mm_pos = mm - 1 + 3;
        mm_len = (uint32_t)(mmz - 1);
        if (ml) { ml_len = ld32u(a, ml - 1 + 4); ml_pos = ml - 1 + 8; }
    }
    if (t_md && a[t_md - 1 + 2] == 'Z') st |= PF_REC_MD;
    if (lane == 0) {
        R.bs[r] = bs;
        R.tid[r] = tid;
        R.rpos[r] = pos;
        R.flag[r] = (uint16_t)flag;
        R.mapq[r] = (uint8_t)mapq;
        R.l_qseq[r] = (uint32_t)lseq;
        R.ncig[r] = ncig;
        R.nins[r] = nins;
        R.cig[r] = cig;
        R.seq[r] = seq;
        R.qn[r] = d + 32;
        R.qn_len[r] = qlen;
        R.rlen[r] = (uint32_t)(rl > 0xFFFFFFFFull ? 0xFFFFFFFFull : rl);
        R.st[r] = st;
        R.de[r] = de;
        R.hp[r] = (uint8_t)hp;
        R.hp_tag[r] = hp_tag;
        R.mm[r] = mm_pos;
        R.mm_len[r] = mm_len;
        R.ml[r] = ml_pos;
        R.ml_len[r] = ml_len;
        R.md[r] = t_md ? t_md - 1 + 3 : 0;
        R.md_len[r] = (t_md && (st & PF_REC_MD)) ? (uint32_t)(md_z - 1) : 0u;
    }
}

// ---------------------------------------------------------------------------
// window selection.  write == 0: count (win_n, win_st); write == 1: the
// record indices into out[win.out ...].
__global__ __launch_bounds__(256) void pf_select(const pf_win_dev *wins, uint32_t n_wins, const pf_chunk_dev *chunks,
                                                 const pf_run_dev *runs, pf_recs_dev R, uint32_t write,
                                                 uint32_t *win_n, uint32_t *win_st, uint32_t *out) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t w = uni(blockIdx.x * 4 + (threadIdx.x >> 6));
    if (w >= n_wins) return;
    const pf_win_dev W = wins[w];
    if (write && W.skip) return;
    uint64_t done = 0;
    uint32_t cnt = 0, status = PF_WIN_OK;
    uint32_t nxt = UINT32_MAX, nxt_run = UINT32_MAX;    // the chain record after the last one read
    bool stop = false;
    for (uint32_t c = W.c0; c < W.c1 && !stop; c++) {
        const pf_chunk_dev C = chunks[c];
        const uint64_t at = C.u > done ? C.u : done;
        if (at >= C.v) continue;
        const pf_run_dev Rn = runs[C.run];
        const uint32_t rend = Rn.rec0 + Rn.n_rec;
        // the chain record starting at `at`: among the 64 after the last one
        // read (consecutive chunks of a long query), else a lower bound over
        // the run's chain
        uint32_t lo = UINT32_MAX;
        if (C.run == nxt_run) {
            const uint32_t k = nxt + lane;
            const uint64_t hit = __ballot(k < rend && R.pos[k] == at);
            if (hit) lo = nxt + (uint32_t)__ffsll((long long)hit) - 1;
        }
        if (lo == UINT32_MAX) {
            lo = Rn.rec0;
            uint32_t n = Rn.n_rec;
            while (n > 0) {
                const uint32_t h = n >> 1;
                if (R.pos[lo + h] < at) { lo += h + 1; n -= h + 1; } else n = h;
            }
        }
        lo = uni(lo);
        uint32_t idx = lo;
        if (idx < rend ? R.pos[idx] != at : at != Rn.stop_pos) { status = PF_WIN_ERR; break; }
        for (;;) {
            const uint32_t k = idx + lane;
            const bool valid = k < rend;
            const uint64_t sp = valid ? R.pos[k] : Rn.stop_pos;
            const bool in = valid && sp < C.v;                          // tell < v
            const uint8_t rst = in ? R.st[k] : 0;
            const int32_t tid = in ? R.tid[k] : 0, rp = in ? R.rpos[k] : 0;
            const bool halt = in && ((rst & (PF_REC_CORRUPT | PF_REC_TRUNC)) || tid != W.tid || (int64_t)rp >= W.end);
            const uint64_t mh = __ballot(halt), mi = __ballot(in);
            const uint32_t fh = mh ? (uint32_t)__ffsll((long long)mh) - 1 : 64u;
            // -u reads (pre_haplotagging_read_in_one_ref, 1869-1871): primary mapped only
            const bool take = in && lane < fh && (int64_t)rp + (int64_t)(in ? R.rlen[k] : 0) > W.beg &&
                              (!W.reads || !(R.flag[k] & (4u | 256u | 2048u)));
            if (W.reads && __ballot(take && !(rst & PF_REC_MD))) { status = PF_WIN_ERR; stop = true; break; }
            const uint64_t mt = __ballot(take);
            if (write && take) out[W.out + cnt + (uint32_t)__popcll(mt & lanemask_lt(lane))] = k;
            cnt += (uint32_t)__popcll(mt);
            if (mh) {
                const uint8_t hs = (uint8_t)__shfl((int)rst, (int)fh, 64);
                if (hs & PF_REC_CORRUPT) status = PF_WIN_ERR;
                else if (hs & PF_REC_TRUNC) status = PF_WIN_TRUNC;     // bam_read1's -4: the fetch ends
                stop = true;                                           // truncated / other tid / pos >= end
                break;
            }
            const uint32_t ni = (uint32_t)__popcll(mi);                 // records read in this step
            if (ni) {
                const uint32_t l = ni - 1;
                const uint64_t e = valid ? R.pos[k] + 4 + R.bs[k] : 0ull;
                const uint32_t elo = (uint32_t)__shfl((int)(uint32_t)e, (int)l, 64);
                const uint32_t ehi = (uint32_t)__shfl((int)(uint32_t)(e >> 32), (int)l, 64);
                done = uni64(((uint64_t)ehi << 32) | elo);
            }
            if (ni < 64) {
                // the chunk ends before lane ni: either a record starting at or
                // after v, or the chain's end
                const uint32_t ke = idx + ni;
                nxt = ke;
                nxt_run = C.run;
                if (ke >= rend) {
                    if (Rn.stop_pos < C.v) {                           // the chunk wants more records
                        if (Rn.stop == PF_CHAIN_CORRUPT) status = PF_WIN_ERR;
                        else if (Rn.to_eof) status = Rn.stop == PF_CHAIN_END ? PF_WIN_OK : PF_WIN_ERR;
                        else status = PF_WIN_MORE;
                        stop = true;                                   // EOF ends the fetch (g == 0)
                    }
                }
                break;
            }
            idx += 64;
        }
        status = uni(status);
        stop = uni(stop ? 1u : 0u) != 0;
    }
    if (!write && lane == 0) {
        win_n[w] = cnt;
        win_st[w] = status;
    }
}

// ---------------------------------------------------------------------------
// gather: small fields of the selected records (one thread each)
__global__ __launch_bounds__(256) void pf_gather_small(const uint32_t *sel, uint64_t n, pf_recs_dev R, uint16_t *flag,
                                                       uint8_t *mapq, uint32_t *pos, uint32_t *l_qseq, float *de,
                                                       uint8_t *hp, int32_t *hp_tag, uint32_t *ncig, uint32_t *mm_len,
                                                       uint32_t *ml_len, uint32_t *qn_len, uint32_t *md_len,
                                                       uint32_t *rlen, uint8_t *st, uint32_t *nins) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint32_t k = sel[i];
    flag[i] = R.flag[k];
    mapq[i] = R.mapq[k];
    pos[i] = (uint32_t)R.rpos[k];
    l_qseq[i] = R.l_qseq[k];
    de[i] = R.de[k];
    hp[i] = R.hp[k];
    hp_tag[i] = R.hp_tag[k];
    ncig[i] = R.ncig[k];
    mm_len[i] = R.mm_len[k];
    ml_len[i] = R.ml_len[k];
    qn_len[i] = R.qn_len[k];
    md_len[i] = R.md_len[k];
    rlen[i] = R.rlen[k];
    st[i] = R.st[k];
    nins[i] = R.nins[k];
}

// byte copy (any alignment), one wave
DEV void wcopy(uint8_t *dst, const uint8_t *a, uint64_t src, uint64_t n, uint32_t lane) {
    for (uint64_t j = lane; j < n; j += 64) dst[j] = a[src + j];
}
// dword copy to a 4-byte aligned destination from any source alignment; the
// last dword's bytes past n come from the source too (padded arena)
DEV void wcopy32(uint32_t *dst, const uint8_t *a, uint64_t src, uint64_t nw, uint32_t lane) {
    for (uint64_t j = lane; j < nw; j += 64) dst[j] = ld32u(a, src + 4 * j);
}

// the large arrays of the selected records (one wave each) at the batch's
// offsets; SEQ slices are zero padded to their aligned size, an odd length's
// pad nibble included (K0's counts rely on it: pf_load.h)
__global__ __launch_bounds__(256) void pf_gather_big(const uint8_t *arena, const uint32_t *sel, uint64_t n, pf_recs_dev R,
                                                     const uint64_t *cig_off, uint32_t *cig, const uint64_t *seq_off,
                                                     uint8_t *seq, const uint64_t *mm_off, uint8_t *mm,
                                                     const uint64_t *ml_off, uint8_t *ml, const uint64_t *qn_off,
                                                     uint8_t *qn, const uint64_t *md_off, uint8_t *md) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t i = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= n) return;
    const uint32_t k = sel[i];
    if (cig) wcopy32(cig + cig_off[i], arena, R.cig[k], R.ncig[k], lane);
    if (seq) {
        // whole bytes, then an odd length's last base with its pad nibble cleared
        const uint64_t lq = R.l_qseq[k], full = lq / 2, sb = (lq + 1) / 2, s0 = seq_off[i], s1 = seq_off[i + 1];
        uint8_t *dst = seq + s0;
        const uint64_t nw = (s0 & 3u) ? 0 : full / 4;        // unaligned slices (the -u reads): bytes
        wcopy32(reinterpret_cast<uint32_t *>(dst), arena, R.seq[k], nw, lane);
        for (uint64_t j = 4 * nw + lane; j < s1 - s0; j += 64)
            dst[j] = j < full ? arena[R.seq[k] + j] : j < sb ? (uint8_t)(arena[R.seq[k] + j] & 0xF0u) : 0;
    }
    if (mm && mm_off[i + 1] > mm_off[i]) wcopy(mm + mm_off[i], arena, R.mm[k], mm_off[i + 1] - mm_off[i], lane);
    if (ml && ml_off[i + 1] > ml_off[i]) wcopy(ml + ml_off[i], arena, R.ml[k], ml_off[i + 1] - ml_off[i], lane);
    if (qn) wcopy(qn + qn_off[i], arena, R.qn[k], qn_off[i + 1] - qn_off[i], lane);
    if (md && md_off[i + 1] > md_off[i]) wcopy(md + md_off[i], arena, R.md[k], md_off[i + 1] - md_off[i], lane);
}
