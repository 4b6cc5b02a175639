// pf_haptag.hip -- --bam-is-untagged (-u) pre-pass on gfx950.
//
// Replaces parse_variants_for_one_read + haptag_one_read_with_variants
// (/root/reference/blockjoin.c:1545-1840) driven by
// pre_haplotagging_read_in_one_ref (blockjoin.c:1841-1898).
//
// Two device kernels, same results:
//   pf_k4_haptag (default): one wavefront per read, lane-parallel CIGAR / MD
//     passes and a neighbour-rule vote (described above the kernel below);
//   pf_k4_thread (PF_K4_IMPL=thread): one thread per read, the serial walk:
//     1. CIGAR: insertions become read variants (I) at the current reference
//        position, chars from SEQ (:1564-1589);
//     2. MD: mismatches (X, base from SEQ) and '^' deletions (D, chars from
//        MD), advancing the query cursor past insertions only after numeric
//        runs (:1604-1673);
//     3. the known phased variants of the read's span (VCF order slice
//        [i_left, j_end), sorted in place by (pos, idx)) merged with its own
//        variants by the piggy-back key pos<<33 | is_read<<32 | idx
//        (:1727-1738), then the vote (:1749-1832).
// At 20,000 reads of ~12 kb (one 4 Mb contig at 60x) the wave kernel takes
// 0.19 ms against 1.35 ms (profiles/r02/k4_*).
// The known-variant cursor (prev_i_left, :1716-1720) is a serial chain over the
// reads of a contig; the host resolves it once (O(reads + variants)) and hands
// every read its slice bounds.
#include <hip/hip_runtime.h>
#include "pf_ingest.h"
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <vector>
#include "../../include/pomfret_amd.h"

#define HAPTAG_UNPHASED 254

struct pf_haptag_dev {
    uint32_t n_reads, n_known;
    const uint32_t *kpos, *klen;
    const uint8_t *kop, *khap;
    const uint64_t *kchar_off;
    const uint8_t *kchars;
    const uint32_t *start, *end;
    const uint64_t *cigar_off;
    const uint32_t *cigar;
    const uint64_t *seq_off;
    const uint32_t *seq_len;
    const uint8_t *seq;
    const uint64_t *md_off;
    const uint8_t *md;
    const uint32_t *i_left, *j_end;
    const uint64_t *scr_off;     // per read: scratch slice (u32 units, even)
    uint64_t *scr;
    uint8_t *hp_out;
    uint32_t *err;
    unsigned long long *prof;    // PF_K4_PROF=1: per-phase cycles of the wave kernel (measurement only)
};

// read variant record: pos, len, op, src offset (query pos for I/X, MD offset for D)
struct RVar { uint32_t pos, len, src; uint32_t op; };

static __device__ __forceinline__ uint8_t nt4_of_char(uint8_t c) {
    switch (c) {
    case 'A': case 'a': return 0;
    case 'C': case 'c': return 1;
    case 'G': case 'g': return 2;
    case 'T': case 't': case 'U': case 'u': return 3;
    default: return 4;
    }
}
// seq_nt16_str = "=ACMGRSVTWYHKDBN" mapped through seq_nt4_table
static __device__ __forceinline__ uint8_t nt4_of_nib(uint32_t nib) {
    return nib == 1 ? 0 : nib == 2 ? 1 : nib == 4 ? 2 : nib == 8 ? 3 : 4;
}
static __device__ __forceinline__ uint8_t seq_code(const uint8_t *seq, uint32_t lq, uint32_t i) {
    if (i >= lq) return 4;
    return nt4_of_nib((seq[i >> 1] >> ((~i & 1) << 2)) & 0xf);
}
static __device__ __forceinline__ int md_op(uint8_t c) {
    if (c >= '0' && c <= '9') return 0;
    if (c == '^') return 1;
    switch (c) {
    case 'A': case 'C': case 'G': case 'T': case 'U': case 'N':
    case 'a': case 'c': case 'g': case 't': case 'u': case 'n': return 2;
    }
    return 4;
}

__global__ __launch_bounds__(64) void pf_k4_thread(pf_haptag_dev d) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= d.n_reads) return;
    if (d.n_known == 0) { d.hp_out[r] = HAPTAG_UNPHASED; return; }
    const uint32_t *cig = d.cigar + d.cigar_off[r];
    const uint32_t ncig = (uint32_t)(d.cigar_off[r + 1] - d.cigar_off[r]);
    const uint8_t *seq = d.seq + d.seq_off[r];
    const uint32_t lq = d.seq_len[r];
    const uint8_t *md = d.md + d.md_off[r];
    const int mdl = (int)(d.md_off[r + 1] - d.md_off[r]);
    const uint32_t ks = d.i_left[r], ke = d.j_end[r];
    const uint32_t nk = ke - ks;
    uint32_t n_ins = 0;
    for (uint32_t i = 0; i < ncig; i++) n_ins += (cig[i] & 0xf) == 1;
    // scratch layout: [keys: nk + n_ins + mdl + 1 u64][vars: n_ins + mdl + 1 RVar]
    uint64_t *keys = reinterpret_cast<uint64_t *>(reinterpret_cast<uint32_t *>(d.scr) + d.scr_off[r]);
    const uint32_t vcap = n_ins + (uint32_t)mdl + 1;
    RVar *vars = reinterpret_cast<RVar *>(keys + nk + vcap);
    uint32_t nv = 0;

    // 1. CIGAR: insertions (I variants) and the leading soft clip
    uint32_t ref_pos = d.start[r], self_pos = 0, self_start = 0;
    for (uint32_t i = 0; i < ncig; i++) {
        const uint32_t op = cig[i] & 0xf, l = cig[i] >> 4;
        if (op == 3) ref_pos += l;
        else if (op == 4) { if (i == 0) self_start = l; self_pos += l; }
        else if (op == 0 || op == 7 || op == 8) { ref_pos += l; self_pos += l; }
        else if (op == 1) { vars[nv++] = RVar{ref_pos, l, self_pos, (uint32_t)PF_VAR_I}; self_pos += l; }
        else if (op == 2) ref_pos += l;
    }
    const uint32_t n_i = nv;
    // 2. MD walk
    uint32_t ins_idx = 0;
    int prev_md_i = 0, prev_t, t;
    self_pos = self_start;
    ref_pos = d.start[r];
    bool bad = mdl <= 0;
    if (!bad) {
        prev_t = md_op(md[0]);
        if (prev_t == 2) {
            vars[nv++] = RVar{ref_pos, 1, self_pos, (uint32_t)PF_VAR_X};
            ref_pos++; self_pos++;
            prev_t = -1;
        }
        if (prev_t >= 4) bad = true;
        for (int i = 1; !bad && i < mdl; i++) {
            t = md_op(md[i]);
            if (t == 4) { bad = true; break; }
            if (t != prev_t) {
                if (prev_t == 0) {
                    int l = 0;
                    for (int j = prev_md_i; j < i; j++) l = l * 10 + (md[j] - '0');
                    ref_pos += l; self_pos += l;
                    while (ins_idx < n_i && self_pos > vars[ins_idx].src) {
                        self_pos += vars[ins_idx].len;
                        ins_idx++;
                    }
                } else if (prev_t == 1) {
                    if (t == 0) {
                        const uint32_t l = (uint32_t)(i - prev_md_i - 1);
                        vars[nv++] = RVar{ref_pos, l, (uint32_t)(prev_md_i + 1), (uint32_t)PF_VAR_D};
                        ref_pos += l;
                        prev_t = t;
                        prev_md_i = i;
                    }
                    continue;
                }
                if (t == 2) {
                    vars[nv++] = RVar{ref_pos, 1, self_pos, (uint32_t)PF_VAR_X};
                    ref_pos++; self_pos++;
                    prev_t = -1;
                    prev_md_i = i;
                } else {
                    prev_t = t;
                    prev_md_i = i;
                }
            }
        }
    }
    if (bad) { d.hp_out[r] = HAPTAG_UNPHASED; atomicOr(d.err, 1u); return; }

    // 3. piggy-back keys: known slice sorted by (pos, idx) (insertion sort: VCF
    //    order is sorted up to the DEL pos+1 shift), read variants = merge of the
    //    position-sorted I list and MD list (keys carry the read list index)
    uint64_t *kk = keys;                 // known keys  [nk]
    for (uint32_t i = 0; i < nk; i++) {
        const uint64_t key = ((uint64_t)d.kpos[ks + i]) << 33 | (ks + i);
        uint32_t j = i;
        while (j > 0 && kk[j - 1] > key) { kk[j] = kk[j - 1]; j--; }
        kk[j] = key;
    }
    uint64_t *rk = keys + nk;            // read keys [nv], merged I/MD lists
    {
        uint32_t a = 0, b = n_i, o = 0;
        const uint64_t TB = 1ull << 32;
        while (a < n_i || b < nv) {
            uint64_t ka = a < n_i ? (((uint64_t)vars[a].pos) << 33 | TB | a) : ~0ull;
            uint64_t kb = b < nv ? (((uint64_t)vars[b].pos) << 33 | TB | b) : ~0ull;
            if (ka <= kb) { rk[o++] = ka; a++; } else { rk[o++] = kb; b++; }
        }
    }
    // merged sequence accessor over kk (known) and rk (read)
    // materialise the merge after rk (space: vcap u64 reserved after nk + vcap)
    // -> reuse: merge into a local walk with two cursors and a 1-element history
    const uint64_t typebit = 1ull << 32;
    int hp_cnt[2] = {0, 0};
    uint32_t ia = 0, ib = 0;             // cursors into kk, rk
    auto peek = [&](uint32_t a, uint32_t b, uint64_t &v) -> bool {
        if (a >= nk && b >= nv) return false;
        const uint64_t x = a < nk ? kk[a] : ~0ull, y = b < nv ? rk[b] : ~0ull;
        v = x <= y ? x : y;
        return true;
    };
    auto advance = [&](uint32_t &a, uint32_t &b) {
        const uint64_t x = a < nk ? kk[a] : ~0ull, y = b < nv ? rk[b] : ~0ull;
        if (x <= y) a++; else b++;
    };
    bool has_prev = false;
    uint64_t prev = 0, cur, nxt;
    while (peek(ia, ib, cur)) {
        // element i = cur; element i+1 = next in merge order
        uint32_t ja = ia, jb = ib;
        advance(ja, jb);
        const bool has_next = peek(ja, jb, nxt);
        if (cur & typebit) {                                   // read-only variant
            prev = cur; has_prev = true; ia = ja; ib = jb;
            continue;
        }
        const uint32_t ref_p = (uint32_t)(cur >> 33), ref_i = (uint32_t)cur;
        if (!has_next) {                                       // last entry: REF vote
            hp_cnt[d.khap[ref_i] & 1]++;
            break;
        }
        const uint32_t self_p = (uint32_t)(nxt >> 33), self_i = (uint32_t)nxt;
        if (ref_p != self_p) {
            bool skip_due_del = false;
            if (has_prev && (prev & typebit)) {
                const RVar &lv = vars[(uint32_t)prev];
                if (lv.op == PF_VAR_D && (uint32_t)(prev >> 33) + lv.len >= ref_p) skip_due_del = true;
            }
            if (!skip_due_del) hp_cnt[d.khap[ref_i] & 1]++;
            prev = cur; has_prev = true; ia = ja; ib = jb;
        } else {
            if (!(nxt & typebit)) {
                // two known entries at one position: multi-allelic, skip both
            } else {
                const RVar &sv = vars[self_i];
                bool ok = d.klen[ref_i] == sv.len;
                if (ok) {
                    const uint8_t *kc = d.kchars + d.kchar_off[ref_i];
                    for (uint32_t j = 0; j < sv.len && ok; j++) {
                        uint8_t c;
                        if (sv.op == PF_VAR_D) c = nt4_of_char(md[sv.src + j]);
                        else c = seq_code(seq, lq, sv.src + j);
                        ok = kc[j] == c;
                    }
                }
                if (ok) hp_cnt[(d.khap[ref_i] ^ 1) & 1]++;
            }
            // i += 2
            prev = nxt; has_prev = true;
            advance(ja, jb);
            ia = ja; ib = jb;
        }
    }
    const int c0 = hp_cnt[0], c1 = hp_cnt[1];
    const float mx = (float)(c0 > c1 ? c0 : c1);
    const int mn = c0 < c1 ? c0 : c1;
    const float ratio = mn == 0 ? 0.f : mx / (float)mn;
    uint8_t h;
    if ((c0 > 3 && c1 > 3 && ratio < 5.f) || c0 == c1) h = HAPTAG_UNPHASED;
    else h = c0 > c1 ? 0 : 1;
    d.hp_out[r] = h;
}

// ------------------------------------------------------------------------
// pf_k4_haptag: one wavefront per read (default).  The three serial walks of
// the per-thread kernel above become wave-wide passes:
//   A. CIGAR, 64 ops a step: per-op reference / query advances, DPP prefix
//      sums -> each insertion's (ref pos, query pos) compacted by ballot into
//      the read's I list, with the running insertion length L(m) and the
//      threshold T(m) = src(m) - L(m).  The MD walk's cursor rule "after a
//      numeric run, skip every insertion whose query position is below the
//      cursor" (:1634-1638) consumes insertion m exactly when the cursor
//      WITHOUT insertions exceeds T(m) (T is non-decreasing), so the number
//      consumed after a run is a lower_bound over T;
//   B. MD, 64 chars a step: ballots of digits / '^' / letters give every
//      char the state of the serial machine (inside a '^' run iff the last
//      '^' is after the last digit), the closing digit of each '^' run emits a
//      D, letters outside runs emit an X, the last digit of a run carries its
//      value; DPP prefix sums give each event its reference position and its
//      query cursor (plus the insertions consumed at the last run end, taken
//      from that lane by a shuffle).  Events are compacted in MD order;
//   C. the known slice [i_left, j_end) is rank-sorted by (pos, idx) (no
//      insertion sort), and every known entry decides its own vote from its
//      neighbours in the merged order (binary searches in the I and MD
//      lists), reproducing the serial pairing: inside a run of knowns at one
//      position the 1st, 3rd, ... are visited, a visited known followed by a
//      known at its position skips both, the last visited known of a run
//      meets the first read variant at that position (ALT check) or, when the
//      next entry sits elsewhere, votes REF unless the previous entry is a
//      read deletion reaching it (:1749-1832).  Votes are summed over the wave.
// Per-read scratch (u32): ipos/ilen/isrc/T [ncig] + Lp [ncig + 1], epos/elen/
// esrc/eop [mdl], sorted known pos/idx [nk] -- written and read by the same
// wave (L2-resident).
#define K4W_WAVES 4

static __device__ __forceinline__ uint32_t k4_uni(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }
static __device__ __forceinline__ uint64_t k4_lt(uint32_t lane) { return lane ? (~0ull >> (64 - lane)) : 0ull; }
static __device__ __forceinline__ uint32_t k4_rdl(uint32_t x, uint32_t l) { return (uint32_t)__builtin_amdgcn_readlane((int)x, (int)l); }
static __device__ __forceinline__ void k4_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}
static __device__ __forceinline__ uint32_t k4_shr_add(uint32_t x, const int ctrl) {
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
// inclusive wave prefix sum (row_shr within 16-lane rows, row_bcast carries)
static __device__ __forceinline__ uint32_t k4_scan(uint32_t x) {
    x = k4_shr_add(x, 1);
    x = k4_shr_add(x, 2);
    x = k4_shr_add(x, 4);
    x = k4_shr_add(x, 8);
    x = k4_shr_add(x, 15);
    x = k4_shr_add(x, 31);
    return x;
}
// highest set bit's absolute index (j0 + bit), or `carry` for an empty mask
static __device__ __forceinline__ int k4_last(uint64_t m, int j0, int carry) {
    return m ? j0 + 63 - (int)__clzll((long long)m) : carry;
}
// first index of a[0..n) with a[i] >= key
static __device__ __forceinline__ uint32_t k4_lower(const uint32_t *a, uint32_t n, uint32_t key) {
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (a[mid] < key) lo = mid + 1; else hi = mid;
    }
    return lo;
}

__global__ __launch_bounds__(64 * K4W_WAVES) void pf_k4_haptag(pf_haptag_dev d) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t r = k4_uni(blockIdx.x * K4W_WAVES + (threadIdx.x >> 6));
    if (r >= d.n_reads) return;
    if (d.n_known == 0) { if (lane == 0) d.hp_out[r] = HAPTAG_UNPHASED; return; }
    const uint64_t c0 = d.cigar_off[r];
    const uint32_t ncig = k4_uni((uint32_t)(d.cigar_off[r + 1] - c0));
    const uint32_t *cig = d.cigar + c0;
    const uint8_t *seq = d.seq + d.seq_off[r];
    const uint32_t lq = d.seq_len[r];
    const uint64_t m0 = d.md_off[r];
    const uint32_t mdl = k4_uni((uint32_t)(d.md_off[r + 1] - m0));
    const uint8_t *md = d.md + m0;
    const uint32_t ks = k4_uni(d.i_left[r]), nk = k4_uni(d.j_end[r] - ks);
    const uint32_t start = k4_uni(d.start[r]);
    uint32_t *S = reinterpret_cast<uint32_t *>(d.scr) + d.scr_off[r];
    uint32_t *ipos = S, *ilen = S + ncig, *isrc = S + 2 * ncig, *iT = S + 3 * ncig, *iLp = S + 4 * ncig;
    uint32_t *epos = S + 5 * ncig + 1, *elen = epos + mdl, *esrc = elen + mdl, *eop = esrc + mdl;
    uint32_t *kp = eop + mdl, *ki = kp + nk;

    unsigned long long t_prev = d.prof ? clock64() : 0ull;
#define K4_STAMP(i) do { if (d.prof) { const unsigned long long t_ = clock64(); \
        if (lane == 0) atomicAdd(&d.prof[i], t_ - t_prev); t_prev = t_; } } while (0)
    // A. CIGAR -> I list
    const uint32_t self_start = ncig && (cig[0] & 0xf) == 4 ? k4_uni(cig[0] >> 4) : 0u;
    uint32_t n_i = 0, cr = 0, cq = 0, cl = 0;
    for (uint32_t b = 0; b < ncig; b += 64) {
        const uint32_t c = b + lane;
        const uint32_t w = c < ncig ? cig[c] : 0u;
        const uint32_t op = w & 0xf, l = w >> 4;
        const bool valid = c < ncig;
        const uint32_t rl = valid && (op == 0 || op == 2 || op == 3 || op == 7 || op == 8) ? l : 0u;
        const uint32_t ql = valid && (op == 0 || op == 1 || op == 4 || op == 7 || op == 8) ? l : 0u;
        const bool isI = valid && op == 1;
        const uint32_t il = isI ? l : 0u;
        const uint32_t sr = k4_scan(rl), sq = k4_scan(ql), sl = k4_scan(il);
        const uint64_t im = __ballot(isI);
        if (isI) {
            const uint32_t k = n_i + (uint32_t)__popcll(im & k4_lt(lane));
            const uint32_t src = cq + sq - ql, Lx = cl + sl - il;
            ipos[k] = start + cr + sr - rl;
            ilen[k] = l;
            isrc[k] = src;
            iT[k] = src - Lx;
            iLp[k] = Lx;
        }
        n_i += (uint32_t)__popcll(im);
        cr += k4_rdl(sr, 63); cq += k4_rdl(sq, 63); cl += k4_rdl(sl, 63);
    }
    if (lane == 0) iLp[n_i] = cl;
    k4_sync();
    K4_STAMP(0);

    // B. MD -> X / D events
    bool bad = mdl == 0;
    uint32_t nE = 0, c_ref = 0, c_base = 0, c_cnt = 0;
    int c_dig = -1, c_car = -1, c_nd = -1, c_ds = -1;
    for (uint32_t b = 0; b < mdl && !bad; b += 64) {
        const uint32_t j = b + lane;
        const bool valid = j < mdl;
        const uint8_t ch = valid ? md[j] : (uint8_t)'0';
        const int t = valid ? md_op(ch) : 5;
        if (__ballot(t == 4)) { bad = true; break; }
        const uint64_t Dm = __ballot(t == 0), Cm = __ballot(t == 1), Lm = __ballot(t == 2);
        const uint64_t lt = k4_lt(lane);
        const int jb = (int)b;
        const int ld = k4_last(Dm & lt, jb, c_dig), lc = k4_last(Cm & lt, jb, c_car);
        const bool in_del = lc > ld;             // state after the chars before j
        const bool isX = t == 2 && !in_del;
        const bool isDc = t == 0 && in_del;
        const uint8_t nx = j + 1 < mdl ? md[j + 1] : (uint8_t)'0';
        const bool isNE = t == 0 && j + 1 < mdl && md_op(nx) != 0;
        const bool open0 = c_car > c_dig;        // a '^' run is open where this step starts
        uint32_t dlen = 0, dstart = 0;
        if (isDc) {
            // the '^' that opened the run: the first one after the last digit
            // (later '^' inside the run are part of it, :1641-1652)
            if (ld < jb && open0) {
                dstart = (uint32_t)c_ds;
            } else {
                const uint64_t above = ld >= jb ? ~((2ull << (ld - jb)) - 1ull) : ~0ull;
                dstart = (uint32_t)(jb + __ffsll((long long)(Cm & lt & above)) - 1);
            }
            dlen = j - dstart - 1;
        }
        uint32_t val = 0;
        if (isNE) {
            const int rs = k4_last((Cm | Lm) & lt, jb, c_nd) + 1;
            for (int q = rs; q <= (int)j; q++) val = val * 10u + (uint32_t)(md[q] - '0');
        }
        const uint32_t a_ref = (isX ? 1u : 0u) + dlen + val, a_base = (isX ? 1u : 0u) + val;
        const uint32_t s_ref = k4_scan(a_ref), s_base = k4_scan(a_base);
        const uint32_t ref_at = start + c_ref + s_ref - a_ref;
        const uint32_t base_at = self_start + c_base + s_base - a_base;
        uint32_t cnt = 0;
        if (isNE) cnt = k4_lower(iT, n_i, base_at + val);      // #{m : T(m) < cursor after the run}
        const uint64_t NEm = __ballot(isNE);
        // insertions consumed at the last run end before j
        const uint64_t ne_lt = NEm & lt;
        const int src_lane = ne_lt ? 63 - (int)__clzll((long long)ne_lt) : 0;
        const uint32_t cnt_sh = (uint32_t)__shfl((int)cnt, src_lane, 64);
        const uint32_t cnt_last = ne_lt ? cnt_sh : c_cnt;
        const uint64_t Em = __ballot(isX || isDc);
        if (isX || isDc) {
            const uint32_t k = nE + (uint32_t)__popcll(Em & lt);
            epos[k] = ref_at;
            if (isX) {
                elen[k] = 1; esrc[k] = base_at + iLp[cnt_last]; eop[k] = PF_VAR_X;
            } else {
                elen[k] = dlen; esrc[k] = dstart + 1; eop[k] = PF_VAR_D;
            }
        }
        nE += (uint32_t)__popcll(Em);
        c_ref += k4_rdl(s_ref, 63);
        c_base += k4_rdl(s_base, 63);
        if (NEm) c_cnt = k4_rdl(cnt, 63 - (uint32_t)__clzll((long long)NEm));
        {
            const int ldt = k4_last(Dm, jb, -1);
            if (ldt >= jb || !open0) {
                const uint64_t above = ldt >= jb ? ~((2ull << (ldt - jb)) - 1ull) : ~0ull;
                const uint64_t m = Cm & above;
                c_ds = m ? jb + __ffsll((long long)m) - 1 : -1;
            }
        }
        c_dig = k4_last(Dm, jb, c_dig);
        c_car = k4_last(Cm, jb, c_car);
        c_nd = k4_last(Cm | Lm, jb, c_nd);
    }
    if (bad) {
        if (lane == 0) { d.hp_out[r] = HAPTAG_UNPHASED; atomicOr(d.err, 1u); }
        return;
    }

    K4_STAMP(1);
    // C. known slice sorted by (pos, idx)
    for (uint32_t a = lane; a < nk; a += 64) {
        const uint32_t pa = d.kpos[ks + a];
        uint32_t rank = 0;
        for (uint32_t q = 0; q < nk; q++) {
            const uint32_t pq = d.kpos[ks + q];
            rank += pq < pa || (pq == pa && q < a);
        }
        kp[rank] = pa;
        ki[rank] = ks + a;
    }
    k4_sync();
    K4_STAMP(2);
    uint32_t v0 = 0, v1 = 0;
    for (uint32_t t = lane; t < nk; t += 64) {
        const uint32_t p = kp[t];
        uint32_t gs = t, ge = t + 1;
        while (gs > 0 && kp[gs - 1] == p) gs--;
        while (ge < nk && kp[ge] == p) ge++;
        if (((t - gs) & 1) || t + 1 < ge) continue;      // consumed, or a known pair at p
        const uint32_t kx = ki[t];
        const uint32_t h = d.khap[kx];
        const uint32_t rI = k4_lower(ipos, n_i, p), rE = k4_lower(epos, nE, p);
        const bool hasI = rI < n_i, hasE = rE < nE;
        const bool nr_I = hasI && (!hasE || ipos[rI] <= epos[rE]);
        const bool has_nr = hasI || hasE;
        const uint32_t nr_pos = nr_I ? ipos[rI] : (hasE ? epos[rE] : 0u);
        if (!has_nr && t + 1 >= nk) { if (h & 1) v1++; else v0++; continue; }   // last entry
        if (has_nr && nr_pos == p) {
            // ALT check against the first read variant at p
            uint32_t len, src, op;
            if (nr_I) { len = ilen[rI]; src = isrc[rI]; op = PF_VAR_I; }
            else { len = elen[rE]; src = esrc[rE]; op = eop[rE]; }
            bool ok = d.klen[kx] == len;
            const uint8_t *kc = d.kchars + d.kchar_off[kx];
            for (uint32_t q = 0; q < len && ok; q++) {
                const uint8_t cq = op == PF_VAR_D ? nt4_of_char(md[src + q]) : seq_code(seq, lq, src + q);
                ok = kc[q] == cq;
            }
            if (ok) { if ((h ^ 1) & 1) v1++; else v0++; }
            continue;
        }
        bool skip = false;
        if (ge - gs == 1) {
            // previous entry: the known before (pos < p) or the last read variant below p
            const bool pI = rI > 0, pE = rE > 0;
            if (pI || pE) {
                const bool prev_E = pE && (!pI || epos[rE - 1] >= ipos[rI - 1]);
                const uint32_t rp = prev_E ? epos[rE - 1] : ipos[rI - 1];
                const bool prev_read = t == 0 || rp >= kp[t - 1];
                if (prev_read && prev_E && eop[rE - 1] == PF_VAR_D && rp + elen[rE - 1] >= p) skip = true;
            }
        }
        if (!skip) { if (h & 1) v1++; else v0++; }
    }
    const uint32_t s0 = k4_rdl(k4_scan(v0), 63), s1 = k4_rdl(k4_scan(v1), 63);
    if (lane == 0) {
        const int n0 = (int)s0, n1 = (int)s1;
        const float mx = (float)(n0 > n1 ? n0 : n1);
        const int mn = n0 < n1 ? n0 : n1;
        const float ratio = mn == 0 ? 0.f : mx / (float)mn;
        uint8_t hh;
        if ((n0 > 3 && n1 > 3 && ratio < 5.f) || n0 == n1) hh = HAPTAG_UNPHASED;
        else hh = n0 > n1 ? 0 : 1;
        d.hp_out[r] = hh;
    }
    K4_STAMP(3);
    if (d.prof && lane == 0) atomicAdd(&d.prof[4], 1ull);
}

// ------------------------------------------------------------------------
// host side
struct pf_ctx;
extern "C" int pf_ctx_device(const pf_ctx *c);
extern "C" hipStream_t pf_ctx_stream(const pf_ctx *c);
extern "C" void pf_ctx_set_haptag_ms(pf_ctx *c, float ms, const char *name);

#define HCHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "[E::pomfret_amd] %s: %s\n", #x, hipGetErrorString(e_)); rc = PF_ERR_HIP; goto done; } } while (0)

template <typename T>
static hipError_t put(std::vector<void *> &al, T **dst, const T *src, size_t n) {
    void *p = nullptr;
    hipError_t e = hipMalloc(&p, std::max<size_t>(n, 1) * sizeof(T));
    if (e != hipSuccess) return e;
    al.push_back(p);
    *dst = (T *)p;
    if (n && src) e = hipMemcpy(p, src, n * sizeof(T), hipMemcpyHostToDevice);
    return e;
}

// K4 over reads whose arrays may already be on the device: per read the host
// needs start, end, the number of CIGAR insertions, the CIGAR length and the
// MD length (the cursor chain and the scratch slices); dv supplies the reads'
// device arrays (cigar_off .. md) or is null (copied from Rb's host arrays).
int pf_haptag_core(pf_ctx_t *ctx, const pf_known_vars_t *K, uint32_t N, const pf_k4_reads_host &h,
                   const pf_read_aln_batch_t *Rb, const pf_k4_reads_dev *dv, uint8_t *hp_out, uint32_t *prev_left) {
    if (N == 0) return PF_OK;
    const uint32_t V = K->n;
    if (V == 0) { memset(hp_out, HAPTAG_UNPHASED, N); return PF_OK; }
    int rc = PF_OK;
    bool thread_impl = false;
    std::vector<void *> al;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    pf_haptag_dev d;
    memset(&d, 0, sizeof(d));
    // known-variant cursor chain (blockjoin.c:1716-1720) and slice ends (:1728-1729)
    std::vector<uint32_t> il(N), je(N);
    std::vector<uint64_t> so(N + 1);
    {
        uint32_t prev = prev_left ? *prev_left : 0;
        uint64_t acc = 0;
        for (uint32_t r = 0; r < N; r++) {
            uint32_t i = prev;
            while (i < V && K->pos[i] < h.start[r]) i++;
            prev = i == 0 ? 0 : i - 1;
            uint32_t j = i;
            while (j < V && K->pos[j] < h.end[r]) j++;
            il[r] = i; je[r] = j;
            const uint64_t mdl = h.md_len[r], ncig = h.ncig[r];
            const uint64_t vcap = h.n_ins[r] + mdl + 1;
            // u32 units: per-thread kernel keys (nk + vcap u64) + RVar (16 B each);
            // wave kernel I lists (5 ncig + 1), MD events (4 mdl), sorted knowns (2 nk)
            const uint64_t need_t = 2 * ((j - i) + vcap + 2 * vcap);
            const uint64_t need_w = 5 * ncig + 1 + 4 * mdl + 2 * (uint64_t)(j - i);
            so[r] = acc;
            acc += (std::max(need_t, need_w) + 1) & ~1ull;
        }
        so[N] = acc;
        if (prev_left) *prev_left = prev;
    }
    {
        const int dev = pf_ctx_device(ctx);
        hipStream_t st = pf_ctx_stream(ctx);
        HCHK(hipSetDevice(dev));
        d.n_reads = N; d.n_known = V;
        HCHK(put(al, (uint32_t **)&d.kpos, K->pos, V));
        HCHK(put(al, (uint32_t **)&d.klen, K->len, V));
        HCHK(put(al, (uint8_t **)&d.kop, K->op, V));
        HCHK(put(al, (uint8_t **)&d.khap, K->haptag, V));
        HCHK(put(al, (uint64_t **)&d.kchar_off, K->char_off, V + 1));
        HCHK(put(al, (uint8_t **)&d.kchars, K->chars, K->char_off[V]));
        if (dv) {
            d.start = dv->start; d.end = dv->end; d.cigar_off = dv->cigar_off; d.cigar = dv->cigar;
            d.seq_off = dv->seq_off; d.seq_len = dv->seq_len; d.seq = dv->seq; d.md_off = dv->md_off; d.md = dv->md;
        } else {
            const uint64_t ncig = Rb->cigar_off[N], nseq = Rb->seq_off[N], nmd = Rb->md_off[N];
            HCHK(put(al, (uint32_t **)&d.start, Rb->start, N));
            HCHK(put(al, (uint32_t **)&d.end, Rb->end, N));
            HCHK(put(al, (uint64_t **)&d.cigar_off, Rb->cigar_off, N + 1));
            HCHK(put(al, (uint32_t **)&d.cigar, Rb->cigar, ncig));
            HCHK(put(al, (uint64_t **)&d.seq_off, Rb->seq_off, N + 1));
            HCHK(put(al, (uint32_t **)&d.seq_len, Rb->seq_len, N));
            HCHK(put(al, (uint8_t **)&d.seq, Rb->seq, nseq));
            HCHK(put(al, (uint64_t **)&d.md_off, Rb->md_off, N + 1));
            HCHK(put(al, (uint8_t **)&d.md, (const uint8_t *)Rb->md, nmd));
        }
        HCHK(put(al, (uint32_t **)&d.i_left, il.data(), N));
        HCHK(put(al, (uint32_t **)&d.j_end, je.data(), N));
        HCHK(put(al, (uint64_t **)&d.scr_off, so.data(), N + 1));
        HCHK(put(al, &d.scr, (const uint64_t *)nullptr, so[N] / 2));
        HCHK(put(al, &d.hp_out, (const uint8_t *)nullptr, N));
        HCHK(put(al, &d.err, (const uint32_t *)nullptr, 1));
        HCHK(hipMemsetAsync(d.err, 0, 4, st));
        const char *pe = getenv("PF_K4_PROF");
        if (pe && *pe == '1') {
            HCHK(put(al, &d.prof, (const unsigned long long *)nullptr, 8));
            HCHK(hipMemsetAsync(d.prof, 0, 64, st));
        }
        HCHK(hipEventCreate(&e0));
        HCHK(hipEventCreate(&e1));
        HCHK(hipEventRecord(e0, st));
        // PF_K4_IMPL=thread: the per-thread walk (A/B reference for the wave kernel)
        const char *impl = getenv("PF_K4_IMPL");
        thread_impl = impl && !strcmp(impl, "thread");
        if (thread_impl)
            hipLaunchKernelGGL(pf_k4_thread, dim3((N + 63) / 64), dim3(64), 0, st, d);
        else
            hipLaunchKernelGGL(pf_k4_haptag, dim3((N + K4W_WAVES - 1) / K4W_WAVES), dim3(64 * K4W_WAVES), 0, st, d);
        HCHK(hipGetLastError());
        HCHK(hipEventRecord(e1, st));
        HCHK(hipMemcpyAsync(hp_out, d.hp_out, N, hipMemcpyDeviceToHost, st));
        uint32_t err = 0;
        HCHK(hipMemcpyAsync(&err, d.err, 4, hipMemcpyDeviceToHost, st));
        HCHK(hipStreamSynchronize(st));
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, e0, e1) == hipSuccess)
            pf_ctx_set_haptag_ms(ctx, ms, thread_impl ? "pf_k4_thread" : "pf_k4_haptag");
        else
            (void)hipGetLastError();       // a failed timing query must not fail a later launch check
        if (d.prof) {
            unsigned long long pr[8];
            HCHK(hipMemcpy(pr, d.prof, sizeof(pr), hipMemcpyDeviceToHost));
            fprintf(stderr, "[pf_k4 prof] waves %llu cycles/wave: cigar %.0f md %.0f sort %.0f vote %.0f\n", pr[4],
                    (double)pr[0] / pr[4], (double)pr[1] / pr[4], (double)pr[2] / pr[4], (double)pr[3] / pr[4]);
        }
        if (err) rc = PF_ERR_ARG;      // malformed MD (fatal exit in the reference, :1621-1624)
    }
done:
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    for (void *p : al) (void)hipFree(p);
    return rc;
}

extern "C" int pf_haptag_reads(pf_ctx_t *ctx, const pf_known_vars_t *K, const pf_read_aln_batch_t *Rb,
                               uint8_t *hp_out) {
    if (!ctx || !K || !Rb || !hp_out) return PF_ERR_ARG;
    const uint32_t N = Rb->n_reads;
    if (N == 0) return PF_OK;
    std::vector<uint32_t> nins(N), ncig(N), mdl(N);
    for (uint32_t r = 0; r < N; r++) {
        uint32_t n = 0;
        for (uint64_t c = Rb->cigar_off[r]; c < Rb->cigar_off[r + 1]; c++) n += (Rb->cigar[c] & 0xf) == 1;
        nins[r] = n;
        ncig[r] = (uint32_t)(Rb->cigar_off[r + 1] - Rb->cigar_off[r]);
        mdl[r] = (uint32_t)(Rb->md_off[r + 1] - Rb->md_off[r]);
    }
    pf_k4_reads_host h{Rb->start, Rb->end, nins.data(), ncig.data(), mdl.data()};
    return pf_haptag_core(ctx, K, N, h, Rb, nullptr, hp_out);
}
