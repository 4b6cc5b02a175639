// pf_haptag.hip -- --bam-is-untagged (-u) pre-pass on gfx950.
//
// Replaces parse_variants_for_one_read + haptag_one_read_with_variants
// (/root/reference/blockjoin.c:1545-1840) driven by
// pre_haplotagging_read_in_one_ref (blockjoin.c:1841-1898).
//
// Device kernel pf_k4_haptag: one thread per read (this round; the walk is a
// serial state machine).  Per read it
//   1. walks the CIGAR: insertions become read variants (I) at the current
//      reference position, chars from SEQ (:1564-1589);
//   2. walks the MD tag: mismatches (X, base from SEQ) and '^' deletions (D,
//      chars from MD), advancing the query cursor past insertions only after
//      numeric runs (:1604-1673);
//   3. merges the known phased variants of its span (VCF order slice
//      [i_left, j_end), sorted in place by (pos, idx)) with its own variants
//      by the reference's piggy-back key pos<<33 | is_read<<32 | idx (:1727-1738)
//      and votes (:1749-1832).
// The known-variant cursor (prev_i_left, :1716-1720) is a serial chain over the
// reads of a contig; the host resolves it once (O(reads + variants)) and hands
// every read its slice bounds.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
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
    const uint64_t *scr_off;     // per read: scratch entries (u64 merged keys + var records)
    uint64_t *scr;
    uint8_t *hp_out;
    uint32_t *err;
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

__global__ __launch_bounds__(64) void pf_k4_haptag(pf_haptag_dev d) {
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
    uint64_t *keys = d.scr + d.scr_off[r];
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
// host side
struct pf_ctx;
extern "C" int pf_ctx_device(const pf_ctx *c);
extern "C" hipStream_t pf_ctx_stream(const pf_ctx *c);
extern "C" void pf_ctx_set_haptag_ms(pf_ctx *c, float ms);

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

extern "C" int pf_haptag_reads(pf_ctx_t *ctx, const pf_known_vars_t *K, const pf_read_aln_batch_t *Rb,
                               uint8_t *hp_out) {
    if (!ctx || !K || !Rb || !hp_out) return PF_ERR_ARG;
    const uint32_t N = Rb->n_reads, V = K->n;
    if (N == 0) return PF_OK;
    if (V == 0) { memset(hp_out, HAPTAG_UNPHASED, N); return PF_OK; }
    int rc = PF_OK;
    std::vector<void *> al;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    pf_haptag_dev d;
    memset(&d, 0, sizeof(d));
    // known-variant cursor chain (blockjoin.c:1716-1720) and slice ends (:1728-1729)
    std::vector<uint32_t> il(N), je(N);
    std::vector<uint64_t> so(N + 1);
    {
        uint32_t prev = 0;
        uint64_t acc = 0;
        for (uint32_t r = 0; r < N; r++) {
            uint32_t i = prev;
            while (i < V && K->pos[i] < Rb->start[r]) i++;
            prev = i == 0 ? 0 : i - 1;
            uint32_t j = i;
            while (j < V && K->pos[j] < Rb->end[r]) j++;
            il[r] = i; je[r] = j;
            uint32_t n_ins = 0;
            for (uint64_t c = Rb->cigar_off[r]; c < Rb->cigar_off[r + 1]; c++) n_ins += (Rb->cigar[c] & 0xf) == 1;
            const uint64_t mdl = Rb->md_off[r + 1] - Rb->md_off[r];
            const uint64_t vcap = n_ins + mdl + 1;
            so[r] = acc;
            acc += (j - i) + vcap + 2 * vcap;     // keys (nk + vcap) + RVar (16 B = 2 u64 each)
        }
        so[N] = acc;
    }
    {
        const int dev = pf_ctx_device(ctx);
        hipStream_t st = pf_ctx_stream(ctx);
        const uint64_t ncig = Rb->cigar_off[N], nseq = Rb->seq_off[N], nmd = Rb->md_off[N];
        HCHK(hipSetDevice(dev));
        d.n_reads = N; d.n_known = V;
        HCHK(put(al, (uint32_t **)&d.kpos, K->pos, V));
        HCHK(put(al, (uint32_t **)&d.klen, K->len, V));
        HCHK(put(al, (uint8_t **)&d.kop, K->op, V));
        HCHK(put(al, (uint8_t **)&d.khap, K->haptag, V));
        HCHK(put(al, (uint64_t **)&d.kchar_off, K->char_off, V + 1));
        HCHK(put(al, (uint8_t **)&d.kchars, K->chars, K->char_off[V]));
        HCHK(put(al, (uint32_t **)&d.start, Rb->start, N));
        HCHK(put(al, (uint32_t **)&d.end, Rb->end, N));
        HCHK(put(al, (uint64_t **)&d.cigar_off, Rb->cigar_off, N + 1));
        HCHK(put(al, (uint32_t **)&d.cigar, Rb->cigar, ncig));
        HCHK(put(al, (uint64_t **)&d.seq_off, Rb->seq_off, N + 1));
        HCHK(put(al, (uint32_t **)&d.seq_len, Rb->seq_len, N));
        HCHK(put(al, (uint8_t **)&d.seq, Rb->seq, nseq));
        HCHK(put(al, (uint64_t **)&d.md_off, Rb->md_off, N + 1));
        HCHK(put(al, (uint8_t **)&d.md, (const uint8_t *)Rb->md, nmd));
        HCHK(put(al, (uint32_t **)&d.i_left, il.data(), N));
        HCHK(put(al, (uint32_t **)&d.j_end, je.data(), N));
        HCHK(put(al, (uint64_t **)&d.scr_off, so.data(), N + 1));
        HCHK(put(al, &d.scr, (const uint64_t *)nullptr, so[N]));
        HCHK(put(al, &d.hp_out, (const uint8_t *)nullptr, N));
        HCHK(put(al, &d.err, (const uint32_t *)nullptr, 1));
        HCHK(hipMemsetAsync(d.err, 0, 4, st));
        HCHK(hipEventCreate(&e0));
        HCHK(hipEventCreate(&e1));
        HCHK(hipEventRecord(e0, st));
        // 64-thread workgroups: one wave per CU for small batches spreads the
        // (divergent, latency-bound) per-read walks over more CUs
        hipLaunchKernelGGL(pf_k4_haptag, dim3((N + 63) / 64), dim3(64), 0, st, d);
        HCHK(hipGetLastError());
        HCHK(hipEventRecord(e1, st));
        HCHK(hipMemcpyAsync(hp_out, d.hp_out, N, hipMemcpyDeviceToHost, st));
        uint32_t err = 0;
        HCHK(hipMemcpyAsync(&err, d.err, 4, hipMemcpyDeviceToHost, st));
        HCHK(hipStreamSynchronize(st));
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, e0, e1) == hipSuccess) pf_ctx_set_haptag_ms(ctx, ms);
        if (err) rc = PF_ERR_ARG;      // malformed MD (fatal exit in the reference, :1621-1624)
    }
done:
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    for (void *p : al) (void)hipFree(p);
    return rc;
}
