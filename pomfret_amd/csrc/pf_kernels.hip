// pf_kernels.hip -- gfx950 kernels of the methphase hot path.
//
// Launches per batch (reference call stack in SURVEY.md section 3.1):
//
//   pf_k12_sites_methmers  one 1024-thread workgroup per window.
//       Sites: the left-coverage check of load_reads_given_interval
//       (blockjoin.c:1161-1163), get_methmer_sites_and_ranges (:3202-3354) for
//       both directions (LDS hash of per-position meth/unmeth counts, site
//       ranks from a bitmap prefix popcount, the u16 wrap at 4096 emulated) and
//       the revbuf end-order (:1126, :1140).  Methmers: get_mmr_of_read
//       (:3357-3451) for every (read, direction) by one wavefront, restated as
//       an "entry walk" over the site arrays staged in LDS; the merged site/call
//       buffer the reference radix-sorts per read is never materialised.
//   pf_k2_methmers  fallback for the reads K12 hands over (site-entry bound
//       above its wave buffer, windows whose sites do not fit LDS).
//   pf_k3_greedy    one 256-thread workgroup per (window, direction), heaviest
//       first.  haplotag_region1 (:3958-4080) and the 2x2 table of
//       evaluate_separation (:3940-3956).  The per-site methmer key lists of
//       the reference (linear search, :3453-3515) become a dense per-site slot
//       dictionary built once per problem, so a lookup is one LDS load.  The
//       candidate scores are exact fp64 sums of the fp32 terms; the sequential
//       fp32 sums of the reference (:3619-3636) are only evaluated when the
//       rounding-error intervals cannot decide the pick.
//   pf_k3_fallback  the same greedy loop with every variant (tables or slot
//       lists in HBM, n_cand > 64, chunked record rows) for the problems the
//       main kernel defers.
//
// Bit-exactness notes: fp32 division is IEEE (no fast-math; the reciprocal
// path is checked over all 2^32 operand pairs), the fallback fold is strictly
// sequential in methmer order, and candidate selection reproduces the stable
// merge sort + walk-from-end of predict_tags_of_reads (:3729-3766) as "max
// score, ties to the later candidate".
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "pf_device.h"

#define DEV static __device__ __forceinline__

// Diagnostic build only (-DPF_K3_PROFILE): per-phase s_memtime cycle shares of
// the greedy loop, written to d.prof.  The real kernel executes no stamp.
#ifdef PF_K3_PROFILE
// one asm statement fenced by scheduling barriers, so no code moves across a
// stamp and each segment owns exactly its instructions (~40 cycles per stamp)
DEV unsigned long long k3_stamp_now() {
    unsigned long long t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
#define K3_STAMP(i) do { const unsigned long long t_ = k3_stamp_now(); \
    prof_acc[i] += t_ - prof_last; prof_last = t_; } while (0)
// the chip-wide constant-rate clock (100 MHz), for the problems' start/end times
DEV unsigned long long k3_realtime() {
    unsigned long long t;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory");
    return t;
}
#define K3_COUNT(i, v) do { prof_acc[i] += (v); } while (0)
#define K12_STAMP(i) do { if (threadIdx.x == 0) { const unsigned long long t_ = k3_stamp_now(); \
    d.prof[64ull * d.W + (uint64_t)w * 16 + (i)] = t_ - k12_t0; k12_t0 = t_; } } while (0)
#define K2_STAMP(i) do { if (k2acc) { const unsigned long long t_ = k3_stamp_now(); \
    k2acc[i] += t_ - k2acc[9]; k2acc[9] = t_; } } while (0)
#else
#define K12_STAMP(i) do { } while (0)
#define K2_STAMP(i) do { } while (0)
#define K3_STAMP(i) do { } while (0)
#define K3_COUNT(i, v) do { } while (0)
#endif

#ifdef PF_ASM_MARK
#define K3_MARK(s) asm volatile("; MARK " s)
#else
#define K3_MARK(s) do { } while (0)
#endif

// ------------------------------------------------------------------------
// small helpers
// a value every lane holds alike (LDS-broadcast control words, wave index),
// moved to an SGPR so the compiler sees it as uniform: scalar branches instead
// of exec-mask structurisation
DEV uint32_t uni(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }
DEV int uni_i(int x) { return __builtin_amdgcn_readfirstlane(x); }

DEV uint64_t lanemask_lt(uint32_t lane) { return lane ? (~0ull >> (64 - lane)) : 0ull; }

DEV void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Same, ordering global memory as well (record rows may live in HBM when the
// problem does not fit LDS).
DEV void wave_sync_mem() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

DEV uint32_t wave_incl_scan(uint32_t x, uint32_t lane) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        uint32_t y = __shfl_up(x, o, 64);
        if (lane >= (uint32_t)o) x += y;
    }
    return x;
}

DEV uint32_t wave_max_u32(uint32_t x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) { uint32_t y = __shfl_xor(x, o, 64); x = y > x ? y : x; }
    return x;
}

// Wave max with DPP row ops (quad perms, half-row and row mirrors) and four
// readlanes: no LDS round trip, unlike the shuffle butterfly above.
DEV uint32_t dpp_max_step(uint32_t x, const int ctrl_sel) {
    uint32_t y;
    switch (ctrl_sel) {
    case 0: y = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xB1, 0xF, 0xF, false); break;  // quad_perm [1,0,3,2]
    case 1: y = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x4E, 0xF, 0xF, false); break;  // quad_perm [2,3,0,1]
    case 2: y = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x141, 0xF, 0xF, false); break; // row_half_mirror
    default: y = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x140, 0xF, 0xF, false); break; // row_mirror
    }
    return y > x ? y : x;
}
DEV uint32_t wave_max_dpp(uint32_t x) {
    x = dpp_max_step(x, 0);
    x = dpp_max_step(x, 1);
    x = dpp_max_step(x, 2);
    x = dpp_max_step(x, 3);
    const uint32_t a = (uint32_t)__builtin_amdgcn_readlane((int)x, 0), b = (uint32_t)__builtin_amdgcn_readlane((int)x, 16);
    const uint32_t c = (uint32_t)__builtin_amdgcn_readlane((int)x, 32), e = (uint32_t)__builtin_amdgcn_readlane((int)x, 48);
    const uint32_t ab = a > b ? a : b, ce = c > e ? c : e;
    return ab > ce ? ab : ce;
}
// lane i <- lane i + 1 (DPP wave_shl:1; lane 63 gets 0): no LDS round trip,
// unlike a ds_bpermute shuffle
DEV uint32_t wave_shl1(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x130, 0xF, 0xF, false);
}
// (float)cnt/sum of query_counts_of_mmrs (blockjoin.c:3508-3509) for 16-bit
// counts (0 <= a <= 65535, 1 <= b <= 65535), correctly
// rounded: one Newton correction of the hardware reciprocal.  Exact here since
// a/b is never within 2^-40 (relative) of an fp32 rounding midpoint when
// b < 2^16, while the corrected quotient is within ~2^-46; checked on the
// device over all 2^32 (a, b) pairs by pf_selftest (tests/test_parity_gpu.py).
DEV float div_u16_y(float fa, float fb, float y) {
    const float q0 = fa * y;
    const float r = __builtin_fmaf(-q0, fb, fa);
    return __builtin_fmaf(r, y, q0);
}
DEV float div_u16(uint32_t a, uint32_t b) {
    const float fb = (float)b;
    return div_u16_y((float)a, fb, __builtin_amdgcn_rcpf(fb));
}
// per-site divisor cache of the greedy kernel: (h0, h1, 1/h0, 1/h1) with a
// zero hap total stored as (1, 0) so that 0/h evaluates to 0 without a branch
DEV float4 site_rec(uint32_t v) {
    const uint32_t h0 = v & 0xffffu, h1 = v >> 16;
    const float f0 = (float)(h0 ? h0 : 1u), f1 = (float)(h1 ? h1 : 1u);
    return make_float4(f0, f1, h0 ? __builtin_amdgcn_rcpf(f0) : 0.f, h1 ? __builtin_amdgcn_rcpf(f1) : 0.f);
}

// Inclusive wave prefix sum with DPP: row_shr 1/2/4/8 inside each 16-lane row,
// then row_bcast:15 / row_bcast:31 carry the row totals upwards.
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
DEV uint32_t wave_incl_scan_dpp(uint32_t x) {
    x = dpp_shr_add(x, 1);
    x = dpp_shr_add(x, 2);
    x = dpp_shr_add(x, 4);
    x = dpp_shr_add(x, 8);
    x = dpp_shr_add(x, 15);
    x = dpp_shr_add(x, 31);
    return x;
}
// Sum over the lanes congruent modulo ncp (a power of two): row rotations for
// strides below 16, the gfx950 permlane16/32 swaps for 16 and 32.
template <int N>
DEV uint32_t ror_add(uint32_t x) {
    return x + (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x120 + N, 0xF, 0xF, false);
}
DEV uint32_t wave_group_sum(uint32_t x, uint32_t ncp) {
    if (ncp < 2) x = ror_add<1>(x);
    if (ncp < 4) x = ror_add<2>(x);
    if (ncp < 8) x = ror_add<4>(x);
    if (ncp < 16) x = ror_add<8>(x);
    if (ncp < 32) { const auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false); x = r[0] + r[1]; }
    if (ncp < 64) { const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false); x = r[0] + r[1]; }
    return x;
}

// wave_group_sum for doubles: the same lane pattern on both 32-bit halves
template <int N>
DEV double ror_add_d(double x) {
    const long long b = __double_as_longlong(x);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)b, 0x120 + N, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)(b >> 32), 0x120 + N, 0xF, 0xF, false);
    return x + __longlong_as_double((long long)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo));
}
DEV double swap16_add_d(double x) {
    const long long b = __double_as_longlong(x);
    const auto lo = __builtin_amdgcn_permlane16_swap((uint32_t)b, (uint32_t)b, false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap((uint32_t)(b >> 32), (uint32_t)(b >> 32), false, false);
    const double a = __longlong_as_double((long long)(((uint64_t)hi[0] << 32) | lo[0]));
    const double c = __longlong_as_double((long long)(((uint64_t)hi[1] << 32) | lo[1]));
    return a + c;
}
DEV double swap32_add_d(double x) {
    const long long b = __double_as_longlong(x);
    const auto lo = __builtin_amdgcn_permlane32_swap((uint32_t)b, (uint32_t)b, false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap((uint32_t)(b >> 32), (uint32_t)(b >> 32), false, false);
    const double a = __longlong_as_double((long long)(((uint64_t)hi[0] << 32) | lo[0]));
    const double c = __longlong_as_double((long long)(((uint64_t)hi[1] << 32) | lo[1]));
    return a + c;
}
DEV double wave_group_sum_d(double x, uint32_t ncp) {
    if (ncp < 2) x = ror_add_d<1>(x);
    if (ncp < 4) x = ror_add_d<2>(x);
    if (ncp < 8) x = ror_add_d<4>(x);
    if (ncp < 16) x = ror_add_d<8>(x);
    if (ncp < 32) x = swap16_add_d(x);
    if (ncp < 64) x = swap32_add_d(x);
    return x;
}

DEV uint32_t rdl(uint32_t x, uint32_t l) { return (uint32_t)__builtin_amdgcn_readlane((int)x, (int)l); }

DEV uint64_t wave_max_u64(uint64_t x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        uint64_t y = __shfl_xor(x, o, 64);
        x = y > x ? y : x;
    }
    return x;
}

// exclusive block scan; sh must hold NT/64+1 words; returns exclusive prefix,
// *total = block sum.  Contains barriers: call from all threads.
template <int NT>
DEV uint32_t block_excl_scan(uint32_t v, uint32_t *sh, uint32_t *total) {
    const uint32_t tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    constexpr int NW = NT / 64;
    uint32_t x = wave_incl_scan(v, lane);
    if (lane == 63) sh[wid] = x;
    __syncthreads();
    if (wid == 0) {
        uint32_t t = lane < (uint32_t)NW ? sh[lane] : 0;
        uint32_t s = wave_incl_scan(t, lane);
        if (lane < (uint32_t)NW) sh[lane] = s - t;
        if (lane == NW - 1) sh[NW] = s;
    }
    __syncthreads();
    uint32_t res = x - v + sh[wid];
    *total = sh[NW];
    __syncthreads();
    return res;
}

// first index in [lo,hi) with a[i] >= v
DEV uint64_t lb_u32(const uint32_t *a, uint64_t lo, uint64_t hi, uint32_t v) {
    while (lo < hi) {
        uint64_t mid = lo + ((hi - lo) >> 1);
        if (a[mid] < v) lo = mid + 1; else hi = mid;
    }
    return lo;
}
// first index in [lo,hi) with a[i] > v
DEV uint64_t ub_u32(const uint32_t *a, uint64_t lo, uint64_t hi, uint32_t v) {
    while (lo < hi) {
        uint64_t mid = lo + ((hi - lo) >> 1);
        if (a[mid] <= v) lo = mid + 1; else hi = mid;
    }
    return lo;
}

DEV uint32_t next_pow2(uint32_t x) { return x <= 1 ? 1u : 1u << (32 - __clz(x - 1)); }

// ========================================================================
// methmers of one read in one direction (get_mmr_of_read, blockjoin.c:3357-3451)
// ========================================================================

// Methylation characters (m/u/- = 0/1/2) of read r over real-site indices
// [qlo, qhi): the category of the read's first call at the site's position,
// '-' when the read has no call there -- the successor of the site entry in
// get_mmr_of_read's sorted buffer (blockjoin.c:3390-3436).  A read's calls are
// sorted by (pos, cat), so the first call at a position has the smallest
// category, as in the reference's radix-sorted buffer.
DEV void k2_chars(const pf_dev_batch &d, uint64_t c0, uint64_t c1, const uint32_t *sp, uint32_t qlo,
                  uint32_t qhi, uint32_t lane, uint8_t *chars) {
    const uint32_t nq = qhi - qlo;
    for (uint32_t j = lane; j < nq; j += 64) chars[j] = 2;
    wave_sync();
    const uint32_t plo = sp[qlo], phi = sp[qhi - 1];
    for (uint64_t cb = c0 + lane; cb < c1; cb += 256) {
        uint32_t pos[4], prv[4], cat[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint64_t c = cb + 64 * u;
            const bool ok = c < c1;
            pos[u] = ok ? d.call_pos[c] : 0xFFFFFFFFu;
            prv[u] = (ok && c > c0) ? d.call_pos[c - 1] : 0xFFFFFFFFu;
            cat[u] = ok ? d.call_cat[c] : 2u;
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint64_t c = cb + 64 * u;
            const uint32_t p = pos[u];
            if (c < c1 && (c == c0 || prv[u] != p) && p >= plo && p <= phi) {
                uint32_t lo = qlo, hi = qhi;
                while (lo < hi) {
                    const uint32_t mid = (lo + hi) >> 1;
                    if (sp[mid] < p) lo = mid + 1; else hi = mid;
                }
                if (lo < qhi && sp[lo] == p) chars[lo - qlo] = (uint8_t)cat[u];
            }
        }
    }
    wave_sync();
}

// Lower bounds of two keys in a non-decreasing array a[0, n): lanes 0-31
// search kA, lanes 32-63 kB, narrowing 32-fold per round (one LDS round trip
// each instead of a dependent binary-search chain).
DEV void wave_lb2(const uint32_t *a, uint32_t n, uint32_t kA, uint32_t kB, uint32_t lane, uint32_t &lbA,
                  uint32_t &lbB) {
    const uint32_t h = lane >> 5, j = lane & 31;
    const uint32_t key = h ? kB : kA;
    uint32_t lo = 0, hi = n;
    for (;;) {
        const uint32_t len = hi - lo;
        const uint32_t step = (len + 31) >> 5;
        const uint32_t p = lo + j * step;
        const bool lt = len > 0 && p < hi && a[p] < key;
        const uint64_t bal = __ballot(lt);
        const uint32_t c = (uint32_t)__popc((uint32_t)(bal >> (32 * h)));
        if (len > 0) {
            if (c == 0) hi = lo;
            else {
                const uint32_t pn = lo + c * step;
                lo = lo + (c - 1) * step + 1;
                hi = pn < hi ? pn : hi;
            }
        }
        if (__ballot(hi > lo) == 0) break;
    }
    lbA = rdl(lo, 0);
    lbB = rdl(lo, 32);
}

// Position -> site index hash of a window's sites (LDS), entries
// (pos - pmin) << 13 | index; positions of hash-path windows span < 2^19.
struct K2SiteHash {
    const uint32_t *t;
    uint32_t mask, pmin;
};
DEV uint32_t k2_hash_slot(uint32_t rel) { return (rel * 2654435761u) >> 7; }
DEV uint32_t k2_site_of(const K2SiteHash &hs, uint32_t p) {
    const uint32_t rel = p - hs.pmin;
    if (p < hs.pmin || rel >= (1u << 19)) return PF_NONE;
    uint32_t h = k2_hash_slot(rel) & hs.mask;
    for (;;) {
        const uint32_t e = hs.t[h];
        if (e == PF_NONE) return PF_NONE;
        if ((e >> 13) == rel) return e & 8191u;
        h = (h + 1) & hs.mask;
    }
}

// Per-read scalars of the methmer walk.
struct K2Read {
    uint64_t c0, c1;
    uint32_t F, L, cap, maxcall;
};

// Calls of one read held in registers (reads of up to 64*K2_CR calls): the
// position and, for the first call at a position, its category (3 = none).
#define K2_CR 8
struct K2Calls {
    uint32_t pos[K2_CR], cat[K2_CR], site[K2_CR];
};

// site index of each first call (PF_NONE if its position is not a site), once
// per read for both directions: hash lookup, or lower bound over all sites
// (the hash is passed by value: a pointer to a local struct would put it on
// the scratch stack, and every reload's vmcnt wait would drain the next
// read's prefetched calls)
DEV void k2_calls_sites(K2Calls &cl, const uint32_t *sp, uint32_t S, const K2SiteHash hs, bool use_hash) {
#pragma unroll
    for (int u = 0; u < K2_CR; u++) {
        const uint32_t p = cl.pos[u];
        uint32_t si = PF_NONE;
        if (cl.cat[u] < 3u && S > 0 && p >= sp[0] && p <= sp[S - 1]) {
            if (use_hash) si = k2_site_of(hs, p);
            else {
                uint32_t lo = 0, hi = S;
                while (lo < hi) {
                    const uint32_t mid = (lo + hi) >> 1;
                    if (sp[mid] < p) lo = mid + 1; else hi = mid;
                }
                si = sp[lo] == p ? lo : PF_NONE;
            }
        }
        cl.site[u] = si;
    }
}

DEV void k2_load_scalars(const pf_dev_batch &d, uint32_t r, K2Read &rd) {
    rd.c0 = d.read_call_off[r];
    rd.c1 = d.read_call_off[r + 1];
    rd.F = d.read_first[r];
    rd.L = d.read_last[r];
    rd.cap = d.mmr_cap[r];
    rd.maxcall = 0;
}

// issue the loads of a read's calls (only when they fit the registers)
DEV void k2_issue_calls(const pf_dev_batch &d, const K2Read &rd, uint32_t lane, uint32_t *pos, uint32_t *cat) {
    const bool fits = rd.c1 - rd.c0 <= 64ull * K2_CR && rd.cap <= d.k12_capw;
#pragma unroll
    for (int u = 0; u < K2_CR; u++) {
        const uint64_t c = rd.c0 + lane + 64u * u;
        const bool ok = fits && c < rd.c1;
        pos[u] = ok ? d.call_pos[c] : 0xFFFFFFFFu;
        cat[u] = ok ? (uint32_t)d.call_cat[c] : 3u;
    }
}

// first-call flags: the previous call's position comes from the lane below
// (DPP wave_shr:1) or, for lane 0, from lane 63 of the previous round
DEV void k2_finish_calls(uint64_t c0, uint64_t c1, uint32_t lane, const uint32_t *pos, const uint32_t *cat,
                         K2Calls &cl) {
    uint32_t last = 0xFFFFFFFFu;
#pragma unroll
    for (int u = 0; u < K2_CR; u++) {
        const uint64_t c = c0 + lane + 64u * u;
        uint32_t prv = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)pos[u], 0x138, 0xF, 0xF, false);  // wave_shr:1
        if (lane == 0) prv = last;
        last = rdl(pos[u], 63);
        cl.pos[u] = pos[u];
        cl.cat[u] = (c < c1 && (c == c0 || prv != pos[u])) ? cat[u] : 3u;
    }
}

// k2_chars from calls held in registers with their site indices
DEV void k2_chars_reg(const K2Calls &cl, uint32_t qlo, uint32_t qhi, uint32_t lane, uint8_t *chars) {
    const uint32_t nq = qhi - qlo;
    for (uint32_t j = lane; j < nq; j += 64) chars[j] = 2;
    wave_sync();
#pragma unroll
    for (int u = 0; u < K2_CR; u++) {
        const uint32_t si = cl.site[u];
        if (si >= qlo && si < qhi) chars[si - qlo] = (uint8_t)cl.cat[u];
    }
    wave_sync();
}

// One read, one direction, one wavefront.  sp = real site positions, st =
// the direction's sites_starts, lens = its methmer lengths, q1 = dir-1 real
// index of each start; buffers of capw entries (LDS or HBM scratch).
// With kst, keys go to that LDS staging buffer (the caller copies them to the
// arena) and the number staged is returned; otherwise straight to the arena.
template <typename IR>
DEV uint32_t k2_core(const pf_dev_batch &d, uint32_t r, uint32_t dir, uint32_t lane, uint32_t S,
                     const uint32_t *sp, const uint32_t *st, const uint8_t *lens, const uint32_t *q1,
                     uint8_t *chars, uint8_t *crank, IR *irank, uint32_t capw, const K2Read &rd,
                     const K2Calls *cl, uint64_t koff, unsigned long long *k2acc = nullptr,
                     uint32_t *kst = nullptr) {
    uint32_t staged_n = 0;
    const uint32_t g = 2 * r + dir;
    const uint64_t c0 = rd.c0, c1 = rd.c1;
    uint32_t total = 0, start_i = PF_NONE;
    if (S > 0 && c1 > c0) {
        const uint32_t F = rd.F, L = rd.L;
        const uint32_t sfirst = st[0], slast = st[S - 1];
        // search_arr on sites_starts (blockjoin.c:3375-3384); sites_starts is
        // non-decreasing in both directions, so search_arr1 = lower bound.
        if (!(F > slast || L < sfirst)) {
            uint32_t lbF, lbL;
            wave_lb2(st, S, F, L, lane, lbF, lbL);
            uint32_t xl, xr;
            if (F < sfirst) xl = 0;
            else xl = st[lbF] == F ? lbF : (lbF ? lbF - 1 : 0);
            xr = L > slast ? S : lbL;
            if (xl < xr) {
                const uint32_t qlo = dir ? q1[xl] : xl;
                const uint32_t qhi = dir ? q1[xr - 1] + 1 : xr;
                const uint32_t nq = qhi - qlo;
                const uint32_t cap = rd.cap;
                if (nq > capw || xr - xl > capw) {
                    if (lane == 0) atomicOr(d.status, PF_ST_INTERNAL);
                } else {
                    K2_STAMP(0);
                    if (cl) k2_chars_reg(*cl, qlo, qhi, lane, chars);
                    else k2_chars(d, c0, c1, sp, qlo, qhi, lane, chars);
                    K2_STAMP(1);
                    // buffer site entries: indices of [xl,xr) except repeats of the
                    // previous start, with the i>1 quirk (blockjoin.c:3391)
                    uint32_t E = 0;
                    for (uint32_t i0 = xl; i0 < xr; i0 += 64) {
                        const uint32_t i = i0 + lane;
                        bool ent = false;
                        if (i < xr) ent = !(i > 1 && st[i] == st[i - 1]);
                        const uint64_t m = __ballot(ent);
                        if (ent) {
                            const uint32_t rk = E + (uint32_t)__popcll(m & lanemask_lt(lane));
                            const uint32_t q = dir ? q1[i] : i;
                            crank[rk] = chars[q - qlo];
                            irank[rk] = (IR)i;
                        }
                        E += (uint32_t)__popcll(m);
                    }
                    wave_sync();
                    K2_STAMP(2);
                    if (E > 0) {
                        // the buffer's last element is never a walk position (:3420)
                        const uint32_t maxcall = rd.maxcall;
                        const uint32_t usable = E - (st[irank[E - 1]] > maxcall ? 1u : 0u);
                        // duplicated start at indices 0 and 1: entry 0 is followed by
                        // another site entry, so its character is '-'
                        if (lane == 0 && E >= 2 && irank[0] == 0 && irank[1] == 1 && st[1] == st[0])
                            crank[0] = 2;
                        wave_sync();
                        uint32_t *out = d.keys + koff;
                        const uint64_t room = d.keys_cap > koff ? d.keys_cap - koff : 0;
                        for (uint32_t e0 = 0; e0 < E; e0 += 64) {
                            const uint32_t e = e0 + lane;
                            uint32_t ne = 0, fj = PF_NONE, i = 0, P = 0;
                            if (e < E) {
                                i = irank[e];
                                P = st[i];
                                for (uint32_t j = i; j < S && st[j] == P; j++) {
                                    if (e + lens[j] <= usable) {
                                        if (fj == PF_NONE) fj = j;
                                        ne++;
                                    }
                                }
                            }
                            const uint32_t incl = wave_incl_scan_dpp(ne);
                            const uint32_t tot = rdl(incl, 63);
                            if (start_i == PF_NONE && tot > 0) {
                                const uint64_t m = __ballot(ne > 0);
                                const uint32_t src = (uint32_t)__ffsll((unsigned long long)m) - 1;
                                start_i = rdl(fj, src);
                            }
                            if (ne) {
                                uint32_t pos = total + incl - ne;
                                for (uint32_t j = i; j < S && st[j] == P; j++) {
                                    const uint32_t Lj = lens[j];
                                    if (e + Lj <= usable) {
                                        uint32_t key = 0;
                                        for (uint32_t t = 0; t < Lj; t++) key = key << 2 | crank[e + t];
                                        if (pos < cap && pos < room) {
                                            if (kst) kst[pos] = key;
                                            else out[pos] = key;
                                        }
                                        pos++;
                                    }
                                }
                            }
                            total += tot;
                        }
                        if (total > cap && lane == 0) atomicOr(d.status, PF_ST_KEYS_OVF);
                        staged_n = total < cap ? total : cap;
                        staged_n = staged_n < room ? staged_n : (uint32_t)room;
                        K2_STAMP(3);
                    }
                }
            }
        }
    }
    if (lane == 0) {
        d.mmr_n[g] = total;
        d.mmr_start[g] = total ? start_i : 0;   // store_mmr_of_one_read (:3518-3522)
    }
    return staged_n;
}

// copy n staged keys to the arena (lane-strided, coalesced)
DEV void k2_flush(const pf_dev_batch &d, const uint32_t *kst, uint64_t koff, uint32_t n, uint32_t lane) {
    uint32_t *out = d.keys + koff;
    for (uint32_t t = lane; t < n; t += 64) out[t] = kst[t];
}

// Fallback for reads the fused kernel could not take (site-entry bound above
// its wave buffer, or a window whose sites do not fit LDS): one wavefront per
// (read, dir) from K12's list, site arrays read from HBM.
__global__ __launch_bounds__(PF_K2_WAVES * 64) void pf_k2_methmers(pf_dev_batch d) {
    __shared__ uint8_t s_chars[PF_K2_WAVES][PF_K2_ENT_CAP];
    __shared__ uint8_t s_crank[PF_K2_WAVES][PF_K2_ENT_CAP];
    __shared__ uint32_t s_irank[PF_K2_WAVES][PF_K2_ENT_CAP];
    const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint64_t n = 2ull * (*d.fb_ctr);
    for (uint64_t gw = (uint64_t)blockIdx.x * PF_K2_WAVES + wid; gw < n; gw += (uint64_t)gridDim.x * PF_K2_WAVES) {
        const uint32_t r = d.fb_list[gw >> 1], dir = (uint32_t)(gw & 1);
        const uint32_t w = d.read_win[r];
        const uint32_t S = d.win_S[w];
        const uint64_t sb = d.win_site_off[w];
        const uint32_t *sp = d.site_pos + sb;
        const uint32_t *st = dir ? d.st1_pos + sb : sp;
        const uint8_t *lens = (dir ? d.len1 : d.len0) + sb;
        const uint32_t *q1 = d.site_q1 + sb;
        const uint64_t bo = d.big_off[r];
        K2Read rd;
        rd.c0 = d.read_call_off[r];
        rd.c1 = d.read_call_off[r + 1];
        rd.F = d.read_first[r];
        rd.L = d.read_last[r];
        rd.cap = d.mmr_cap[r];
        rd.maxcall = rd.c1 > rd.c0 ? d.call_pos[rd.c1 - 1] : 0u;
        const uint64_t koff = d.mmr_off[2ull * r + dir];
        if (bo == ~0ull) {
            k2_core(d, r, dir, lane, S, sp, st, lens, q1, s_chars[wid], s_crank[wid], s_irank[wid],
                    PF_K2_ENT_CAP, rd, nullptr, koff);
        } else {
            // large read: HBM scratch reserved by K12, 16 bytes per bound entry:
            // per direction [chars cap][crank cap][pad][irank 4*cap] at dir*8*cap
            const uint32_t cap = d.mmr_cap[r];
            if (bo + 16ull * cap > d.big_cap) {
                if (lane == 0) { d.mmr_n[2 * r + dir] = 0; d.mmr_start[2 * r + dir] = 0; atomicOr(d.status, PF_ST_BIG_OVF); }
                continue;
            }
            uint8_t *b = d.big + bo + (dir ? 8ull * cap : 0);
            k2_core(d, r, dir, lane, S, sp, st, lens, q1, b, b + cap, reinterpret_cast<uint32_t *>(b + 4ull * cap),
                    cap, rd, nullptr, koff);
        }
    }
}

// The methmer phase of one window over its reads i0, i0 + NW, ... < i1 (wave
// wid of NW): one wavefront per read, both directions, the window's site
// arrays in LDS (sp, st1, q1s, l0s, l1s; hsd when use_hash), the wave's
// buffers at wb.  Used by K12 for its own reads and by pf_k12_chunks for the
// read chunks of the windows K12 hands over.
DEV void k12_methmers(const pf_dev_batch &d, uint32_t r0, uint32_t i0, uint32_t i1, uint32_t wid, uint32_t NW,
                      uint32_t lane, uint32_t S, const uint32_t *sp, const uint32_t *st1, const uint32_t *q1s,
                      const uint8_t *l0s, const uint8_t *l1s, const K2SiteHash &hsd, bool use_hash, uint8_t *wb,
                      unsigned long long *k2acc, uint32_t *rctr) {
        uint8_t *chars = wb, *crank = wb + PF_K12_CAPW;
        uint16_t *irank = reinterpret_cast<uint16_t *>(wb + 2 * PF_K12_CAPW);
        uint32_t *kst = reinterpret_cast<uint32_t *>(wb + 4 * PF_K12_CAPW);
        // keys are staged in LDS and copied out at points where no prefetched
        // load is younger than the copy: vmcnt counts loads and stores in
        // issue order, so a load issued before a dynamic number of stores can
        // only be waited for with vmcnt(0), which drains the stores too.  The
        // dir-1 keys of read i are copied out after read i+1's prefetched
        // calls have been consumed, just before read i+2's are issued.
        uint32_t pend_n = 0;
        uint64_t pend_off = 0;
        // software pipeline over this wave's reads: the scalars of the read
        // after next and the calls of the next read are in flight while a read
        // is processed.  A wave's first read is i0 + wid; later ones are taken
        // from the workgroup's counter (*rctr, set to i0 + NW by the caller),
        // one read ahead, so that the waves finish together however the
        // reads' lengths fall (round-robin left the window to its slowest wave)
        auto take = [&]() -> uint32_t {
            uint32_t v = 0;
            if (lane == 0) v = atomicAdd(rctr, 1u);
            return (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
        };
        K2Read rdA, rdB;
        uint32_t pA[K2_CR], tA[K2_CR], pB[K2_CR], tB[K2_CR];
        const uint32_t iw = i0 + wid;
        uint32_t iB = iw < i1 ? take() : i1;
        if (iw < i1) k2_load_scalars(d, r0 + iw, rdA);
        if (iB < i1) k2_load_scalars(d, r0 + iB, rdB);
        k2_issue_calls(d, iw < i1 ? rdA : K2Read{0, 0, 0, 0, 0, 0}, lane, pA, tA);
        for (uint32_t i = iw; i < i1;) {
            const uint32_t r = r0 + i;
            K2_STAMP(6);
            K2Read rd = rdA;
            const uint64_t nc = rd.c1 - rd.c0;
            const bool regs = rd.cap <= d.k12_capw && nc <= 64ull * K2_CR;
            K2Calls cl;
            if (regs) {
                k2_finish_calls(rd.c0, rd.c1, lane, pA, tA, cl);
                // last call position (sorted order) from the registers
                uint32_t mc = 0;
                if (nc) {
                    const uint32_t ul = (uint32_t)((nc - 1) >> 6), ll = (uint32_t)((nc - 1) & 63);
#pragma unroll
                    for (int u = 0; u < K2_CR; u++)
                        if ((uint32_t)u == ul) mc = rdl(cl.pos[u], ll);
                }
                rd.maxcall = mc;
                k2_calls_sites(cl, sp, S, hsd, use_hash);
            }
            K2_STAMP(4);
            k2_flush(d, kst, pend_off, pend_n, lane);
            pend_n = 0;
            K2Read rdC = {0, 0, 0, 0, 0, 0};
            const uint32_t iC = iB < i1 ? take() : i1;
            if (iC < i1) k2_load_scalars(d, r0 + iC, rdC);
            k2_issue_calls(d, iB < i1 ? rdB : K2Read{0, 0, 0, 0, 0, 0}, lane, pB, tB);
            K2_STAMP(8);
            if (rd.cap > d.k12_capw) {
                if (lane == 0) d.fb_list[atomicAdd(d.fb_ctr, 1u)] = r;
            } else {
                const uint64_t k0 = d.mmr_off[2ull * r], k1 = d.mmr_off[2ull * r + 1];
                if (regs) {
                    const uint32_t n0 = k2_core(d, r, 0, lane, S, sp, sp, l0s, q1s, chars, crank, irank, PF_K12_CAPW,
                                                rd, &cl, k0, k2acc, kst);
                    k2_flush(d, kst, k0, n0, lane);
                    K2_STAMP(5);
                    pend_n = k2_core(d, r, 1, lane, S, sp, st1, l1s, q1s, chars, crank, irank, PF_K12_CAPW, rd,
                                     &cl, k1, k2acc, kst);
                    pend_off = k1;
                    K2_STAMP(5);
                } else {
                    rd.maxcall = nc ? d.call_pos[rd.c1 - 1] : 0u;
                    k2_core(d, r, 0, lane, S, sp, sp, l0s, q1s, chars, crank, irank, PF_K12_CAPW, rd, nullptr, k0);
                    k2_core(d, r, 1, lane, S, sp, st1, l1s, q1s, chars, crank, irank, PF_K12_CAPW, rd, nullptr, k1);
                }
            }
            rdA = rdB;
            rdB = rdC;
            i = iB;
            iB = iC;
#pragma unroll
            for (int u = 0; u < K2_CR; u++) { pA[u] = pB[u]; tA[u] = tB[u]; }
            K2_STAMP(7);
        }
        k2_flush(d, kst, pend_off, pend_n, lane);
}

// ========================================================================
// K12: sites + directional methmer ranges + end-order + arena reservation,
// then every read's methmers (both directions) from LDS-resident site arrays
// ========================================================================
__global__ __launch_bounds__(PF_K1_THREADS) void pf_k12_sites_methmers(pf_dev_batch d) {
    __shared__ uint32_t tile[PF_K1_TILE];
    __shared__ uint32_t sh_scan[PF_K1_THREADS / 64 + 1];
    __shared__ uint32_t sh_misc[8];
    __shared__ unsigned long long sh_base[2];
    constexpr uint32_t NT = PF_K1_THREADS, NW = NT / 64;
    // windows heaviest first (k12_order): the big windows of a gap mix start
    // in the first wave of workgroups instead of forming the kernel's tail
    const uint32_t w = d.k12_order[blockIdx.x], tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
#ifdef PF_K3_PROFILE
    unsigned long long k12_t0 = __builtin_amdgcn_s_memtime();
#endif
    const uint32_t r0 = d.win_read_off[w], R = d.win_read_off[w + 1] - r0;
    const int cov = d.win_par[w * 4 + 0];
    const uint32_t s = d.win_start[w];
    const uint64_t sb = d.win_site_off[w];
    const uint32_t scap = d.win_site_cap[w];

    if (tid < 8) sh_misc[tid] = 0;
    __syncthreads();
    if (tid == 0) { sh_misc[2] = 0xFFFFFFFFu; sh_misc[3] = 0; }
    __syncthreads();
    // left-side per-haplotype coverage (blockjoin.c:1127-1133, 1161) and position range
    for (uint32_t i = tid; i < R; i += NT) {
        const uint32_t r = r0 + i;
        if (d.read_start[r] <= s) {
            const uint32_t hp = d.read_hp[r];
            if (hp < 2) atomicAdd(&sh_misc[hp], 1u);
        }
        const uint64_t c0 = d.read_call_off[r], c1 = d.read_call_off[r + 1];
        if (c1 > c0) {
            atomicMin(&sh_misc[2], d.call_pos[c0]);
            atomicMax(&sh_misc[3], d.call_pos[c1 - 1]);
        }
    }
    __syncthreads();
    const bool fail = R == 0 || (int)sh_misc[0] < d.hard_cov || (int)sh_misc[1] < d.hard_cov ||
                      sh_misc[2] > sh_misc[3];
    if (fail) {
        if (tid == 0) { d.win_S[w] = 0; d.win_nreads[w] = 0; }
        for (uint32_t i = tid; i < R; i += NT) {
            const uint32_t r = r0 + i;
            d.mmr_n[2 * r] = 0; d.mmr_n[2 * r + 1] = 0;
            d.mmr_start[2 * r] = 0; d.mmr_start[2 * r + 1] = 0;
            d.mmr_off[2 * r] = 0; d.mmr_off[2 * r + 1] = 0;
            d.mmr_cap[r] = 0;
            d.big_off[r] = ~0ull;
        }
        return;
    }
    K12_STAMP(1);
    const uint32_t pmin = sh_misc[2], pmax = sh_misc[3];
    if (tid == 0) { sh_misc[4] = 0; d.win_nreads[w] = R; }
    __syncthreads();

    // ---- fast path: a bitmap of the positions with >= 2 meth/unmeth calls over
    // a segment [base, base + 64*BW) of the window's positions, one counter per
    // such position indexed by its rank among them (a prefix popcount: no
    // hash, no probing), then the bitmap of qualifying positions, whose prefix
    // popcount is a site's index, so no sort is needed.  A span of up to two
    // segments (1 Mb; the mix's widest windows span 512-760 kb) takes them one
    // after the other, each over all of the window's calls, the site ranks
    // carried in position order.
    constexpr uint32_t BW = 8192, RMAX = 12288, SEGB = BW * 64, MAXSEG = 2;
    static_assert(BW / 2 + RMAX <= PF_K1_TILE / 2, "word ranks + counters fit the first half of the tile");
    uint64_t *bmap = reinterpret_cast<uint64_t *>(tile + PF_K1_TILE / 2);
    const uint32_t nseg = d.k12_dense ? 0u : (uint32_t)min<uint64_t>(((uint64_t)(pmax - pmin) + SEGB) / SEGB, MAXSEG + 1);
    const bool range_ok = nseg >= 1 && nseg <= MAXSEG;
    bool fast = range_ok;
    [[maybe_unused]] uint32_t rep_seen = 0;             // the profile's dense-path reason
    // the window's calls are one contiguous run: flat passes, four
    // independent (cat, pos) loads in flight per thread
    const uint64_t C0 = d.read_call_off[r0], C1 = d.read_call_off[r0 + R];
    // Pass A marks in bmap the positions with >= 2 meth/unmeth calls: a site
    // needs >= cov_sel calls of each kind, so no other position can qualify.
    // Pass B counts only those.  Sequencing errors put CpG calls at positions
    // that one read alone covers; with real reads they outnumber the sites, and
    // filtering them keeps the counters few.
    for (uint32_t seg = 0; fast && seg < nseg; seg++) {
        const uint32_t base = pmin + seg * SEGB;
        {
            uint64_t *once = reinterpret_cast<uint64_t *>(tile);   // the first half of the tile
            for (uint32_t j = tid; j < BW; j += NT) { once[j] = 0; bmap[j] = 0; }
            __syncthreads();
            for (uint64_t cb = C0 + tid; cb < C1; cb += 4ull * NT) {
                uint32_t cat4[4], pos4[4];
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const uint64_t c = cb + (uint64_t)u * NT;
                    const bool ok = c < C1;
                    cat4[u] = ok ? d.call_cat[c] : 2u;
                    pos4[u] = ok ? d.call_pos[c] : 0u;
                }
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const uint32_t o = pos4[u] - base;
                    if (cat4[u] >= 2 || o >= SEGB) continue;
                    const unsigned long long bit = 1ull << (o & 63);
                    if (atomicOr((unsigned long long *)&once[o >> 6], bit) & bit)
                        atomicOr((unsigned long long *)&bmap[o >> 6], bit);
                }
            }
            __syncthreads();
        }
        // more repeated positions than counters: the dense path
        constexpr uint32_t PW = BW / NT;                 // bitmap words per thread
        uint32_t rep = 0, rep_tot = 0;
#pragma unroll
        for (uint32_t j = 0; j < PW; j++) rep += (uint32_t)__popcll(bmap[tid * PW + j]);
        const uint32_t rep_ex = block_excl_scan<NT>(rep, sh_scan, &rep_tot);
        rep_seen = rep_tot > rep_seen ? rep_tot : rep_seen;
        if (rep_tot > RMAX) {
            fast = false;                                // uniform: a block-wide total
            break;
        }
        // over the freed once-bitmap: each word's rank base (u16), then the
        // counters (meth in the low half, unmeth in the high half)
        uint16_t *wrank = reinterpret_cast<uint16_t *>(tile);
        uint32_t *rcnt = tile + BW / 2;
        {
            uint32_t rk = rep_ex;
#pragma unroll
            for (uint32_t j = 0; j < PW; j++) {
                const uint32_t wi = tid * PW + j;
                wrank[wi] = (uint16_t)rk;
                rk += (uint32_t)__popcll(bmap[wi]);
            }
        }
        for (uint32_t j = tid; j < rep_tot; j += NT) rcnt[j] = 0;
        __syncthreads();
        for (uint64_t cb = C0 + tid; cb < C1; cb += 4ull * NT) {
            uint32_t cat4[4], pos4[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const uint64_t c = cb + (uint64_t)u * NT;
                const bool ok = c < C1;
                cat4[u] = ok ? d.call_cat[c] : 2u;
                pos4[u] = ok ? d.call_pos[c] : 0u;
            }
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const uint32_t o = pos4[u] - base;
                if (cat4[u] >= 2 || o >= SEGB) continue;
                const uint64_t bits = bmap[o >> 6];
                const uint64_t below = (1ull << (o & 63)) - 1ull;
                if (!((bits >> (o & 63)) & 1ull)) continue;
                const uint32_t ix = (uint32_t)wrank[o >> 6] + (uint32_t)__popcll(bits & below);
                atomicAdd(&rcnt[ix], cat4[u] == 0 ? 1u : 0x10000u);
            }
        }
        __syncthreads();
        // bmap becomes the qualifying bitmap, each thread over its own words
        // counts are uint16 holding count<<4 in the reference: count mod 4096 (blockjoin.c:3236)
        uint32_t mycount = 0;
        {
            uint32_t rk = rep_ex;
#pragma unroll
            for (uint32_t j = 0; j < PW; j++) {
                const uint32_t wi = tid * PW + j;
                uint64_t bits = bmap[wi], q = 0;
                while (bits) {
                    const uint32_t b = (uint32_t)__ffsll((unsigned long long)bits) - 1;
                    bits &= bits - 1;
                    const uint32_t v = rcnt[rk++];
                    if ((int)(v & 4095u) >= cov && (int)((v >> 16) & 4095u) >= cov) q |= 1ull << b;
                }
                bmap[wi] = q;
                mycount += (uint32_t)__popcll(q);
            }
        }
        // the segment's sites, ranked after the earlier segments'
        uint32_t total;
        const uint32_t excl = block_excl_scan<NT>(mycount, sh_scan, &total);
        const uint32_t carry = sh_misc[4];
        {
            uint32_t rank = carry + excl;
            for (uint32_t j = 0; j < PW; j++) {
                const uint32_t wi = tid * PW + j;
                uint64_t bits = bmap[wi];
                while (bits) {
                    const uint32_t b = __ffsll((unsigned long long)bits) - 1;
                    bits &= bits - 1;
                    if (rank < scap) d.site_pos[sb + rank] = base + wi * 64 + b;
                    else atomicOr(d.status, PF_ST_SITE_OVF);
                    rank++;
                }
            }
        }
        __syncthreads();
        if (tid == 0) sh_misc[4] = carry + total;
        __syncthreads();
    }
    if (range_ok && !fast) {
        // a segment had too many repeated positions: the dense path restarts
        // the window's sites from rank 0
        if (tid == 0) sh_misc[4] = 0;
        __syncthreads();
    }
    // ---- general path (a position range beyond the bitmaps, or more repeated
    // positions than the hash holds: the big windows of a gap mix).  The
    // window's calls are bucketed by 16 K-position chunk into an HBM scratch
    // list of u16 (offset in chunk | meth/unmeth bit), then each chunk is
    // counted with LDS atomics in the tile and scanned in position order.
    // Two flat passes over the calls (histogram, scatter; the chunk counters
    // are wave-aggregated) and one per chunk over its own calls.  Round 2
    // counted 32 K-position LDS tiles each over every read of the window (two
    // binary searches per read and tile); device-scope atomics on an HBM
    // counter array were tried this round: ~15 cycles per call at L2, 6-9 M
    // cycles on a 500 kb gap -- both ~10x this.
    if (!fast) {
        constexpr uint32_t CHB = 14, CH = 1u << CHB, MAXCH = 8191;
        static_assert(CH + 2 * (MAXCH + 1) <= PF_K1_TILE, "chunk counters + chunk offsets fit the tile");
        uint32_t *ccnt = tile, *coff = tile + CH, *cfill = coff + MAXCH + 1;
        const uint64_t ncall = C1 - C0;
        const uint64_t need = (2ull * ncall + 15) & ~15ull;
        if (tid == 0) {
            const unsigned long long o = atomicAdd(d.scr_ctr, (unsigned long long)need);
            sh_base[0] = o;
            if (o + need > d.scr_cap) atomicOr(d.status, PF_ST_SCR_OVF);
        }
        __syncthreads();
        const uint64_t so = sh_base[0];
#ifdef PF_K3_PROFILE
        const unsigned long long dz0 = k3_stamp_now();
#endif
        if (so + need > d.scr_cap) {
            // the scratch arena is full (status set; the host grows it and
            // re-runs): no sites, and K3 skips the window
            if (tid == 0) sh_misc[4] = 0;
            __syncthreads();
        } else {
            uint16_t *sc = reinterpret_cast<uint16_t *>(d.scr + so);
            const uint32_t span = pmax - pmin + 1;
            // one wave-aggregated LDS add per distinct chunk among the lanes
            // (a wave's 64 consecutive calls are mostly one read's, 1-2 chunks)
            auto chunk_add = [&](bool act, uint32_t ch, uint32_t *ctr, bool ret) -> uint32_t {
                uint32_t mine = 0;
                uint64_t todo = __ballot(act);
                while (todo) {
                    const uint32_t l0 = (uint32_t)__ffsll((long long)todo) - 1;
                    const uint32_t lc = rdl(ch, l0);
                    const uint64_t m = __ballot(act && ch == lc);
                    uint32_t base = 0;
                    if (lane == l0) {
                        if (ret) base = atomicAdd(&ctr[lc], (uint32_t)__popcll(m));
                        else atomicAdd(&ctr[lc], (uint32_t)__popcll(m));
                    }
                    base = rdl(base, l0);
                    if (act && ch == lc) mine = base + (uint32_t)__popcll(m & lanemask_lt(lane));
                    todo &= ~m;
                }
                return mine;
            };
            const uint64_t cend4 = C0 + (ncall + 4 * NT - 1) / (4 * NT) * (4 * NT);   // whole waves in every pass
            for (uint64_t sup = 0; sup < span; sup += (uint64_t)MAXCH << CHB) {
                const uint32_t nch = (uint32_t)min<uint64_t>((span - sup + CH - 1) >> CHB, MAXCH);
                const uint64_t slim = min<uint64_t>((uint64_t)nch << CHB, span - sup);
                for (uint32_t j = tid; j <= nch; j += NT) { coff[j] = 0; cfill[j] = 0; }
                __syncthreads();
                // A: calls per chunk (four calls per thread per step, loads first)
                for (uint64_t c0 = C0 + tid; c0 < cend4; c0 += 4ull * NT) {
                    uint32_t cat4[4], pos4[4];
#pragma unroll
                    for (int u = 0; u < 4; u++) {
                        const uint64_t c = c0 + (uint64_t)u * NT;
                        cat4[u] = c < C1 ? d.call_cat[c] : 2u;
                        pos4[u] = c < C1 ? d.call_pos[c] : pmin;
                    }
#pragma unroll
                    for (int u = 0; u < 4; u++) {
                        const uint64_t rel = (uint64_t)(pos4[u] - pmin) - sup;
                        const bool act = cat4[u] < 2 && rel < slim;
                        chunk_add(act, act ? (uint32_t)(rel >> CHB) : 0u, coff, false);
                    }
                }
                __syncthreads();
                // chunk offsets (exclusive scan, 8 chunks per thread)
                {
                    uint32_t v[8], t = 0;
#pragma unroll
                    for (uint32_t u = 0; u < 8; u++) { const uint32_t j = tid * 8 + u; v[u] = j < nch ? coff[j] : 0u; t += v[u]; }
                    uint32_t tot;
                    uint32_t ex = block_excl_scan<NT>(t, sh_scan, &tot);
#pragma unroll
                    for (uint32_t u = 0; u < 8; u++) { const uint32_t j = tid * 8 + u; if (j < nch) coff[j] = ex; ex += v[u]; }
                    if (tid == 0) coff[nch] = tot;
                }
                __syncthreads();
                // C: scatter the calls into their chunks' lists
                for (uint64_t c0 = C0 + tid; c0 < cend4; c0 += 4ull * NT) {
                    uint32_t cat4[4], pos4[4];
#pragma unroll
                    for (int u = 0; u < 4; u++) {
                        const uint64_t c = c0 + (uint64_t)u * NT;
                        cat4[u] = c < C1 ? d.call_cat[c] : 2u;
                        pos4[u] = c < C1 ? d.call_pos[c] : pmin;
                    }
#pragma unroll
                    for (int u = 0; u < 4; u++) {
                        const uint64_t rel = (uint64_t)(pos4[u] - pmin) - sup;
                        const bool act = cat4[u] < 2 && rel < slim;
                        const uint32_t ch = act ? (uint32_t)(rel >> CHB) : 0u;
                        const uint32_t slot = chunk_add(act, ch, cfill, true);
                        if (act) sc[coff[ch] + slot] = (uint16_t)(((uint32_t)rel & (CH - 1)) | (cat4[u] << 15));
                    }
                }
                __threadfence();                         // the lists are read back through L2 (L1 invalidated)
                __syncthreads();
                // D: each chunk counted in LDS, scanned in position order
                for (uint32_t ch = 0; ch < nch; ch++) {
                    const uint32_t l0 = coff[ch], l1 = coff[ch + 1];
                    if (l1 == l0) continue;                  // uniform: no calls, no site
                    for (uint32_t j = tid; j < CH / 4; j += NT) reinterpret_cast<uint4 *>(ccnt)[j] = make_uint4(0, 0, 0, 0);
                    __syncthreads();
                    for (uint32_t t0 = l0 + tid; t0 < l1; t0 += 4 * NT) {   // four list loads in flight
                        uint32_t v4[4];
#pragma unroll
                        for (int u = 0; u < 4; u++) v4[u] = t0 + u * NT < l1 ? sc[t0 + u * NT] : 0xFFFFFFFFu;
#pragma unroll
                        for (int u = 0; u < 4; u++)
                            if (v4[u] != 0xFFFFFFFFu) atomicAdd(&ccnt[v4[u] & (CH - 1)], (v4[u] >> 15) ? 0x10000u : 1u);
                    }
                    __syncthreads();
                    uint32_t qmask = 0;
                    constexpr uint32_t PER = CH / NT;        // 16 positions per thread
#pragma unroll
                    for (uint32_t jj = 0; jj < PER; jj++) {
                        const uint32_t j = (jj + tid) & (PER - 1);   // rotated: conflict-free banks
                        const uint32_t v = ccnt[tid * PER + j];
                        // counts are uint16 holding count<<4 in the reference: count mod 4096 (blockjoin.c:3236)
                        if ((int)(v & 4095u) >= cov && (int)((v >> 16) & 4095u) >= cov) qmask |= 1u << j;
                    }
                    uint32_t total;
                    const uint32_t excl = block_excl_scan<NT>((uint32_t)__popc(qmask), sh_scan, &total);
                    const uint32_t srun = sh_misc[4];
                    uint32_t m = qmask, rank = srun + excl;
                    const uint32_t pb = pmin + (uint32_t)sup + (ch << CHB) + tid * PER;
                    while (m) {
                        const uint32_t j = __ffs(m) - 1;
                        m &= m - 1;
                        if (rank < scap) d.site_pos[sb + rank] = pb + j;
                        else atomicOr(d.status, PF_ST_SITE_OVF);
                        rank++;
                    }
                    __syncthreads();
                    if (tid == 0) sh_misc[4] = srun + total;
                    __syncthreads();
                }
                __syncthreads();
            }
        }
#ifdef PF_K3_PROFILE
        // the dense path: cycles | repeated positions << 32 (0: the span was beyond
        // the bitmap) | span in KiB << 52 | the bitmap's range held << 63
        if (tid == 0)
            d.prof[64ull * d.W + (uint64_t)w * 16] = ((k3_stamp_now() - dz0) & 0xFFFFFFFFull) |
                                                     ((uint64_t)min(rep_seen, 0xFFFFFu) << 32) |
                                                     ((uint64_t)min((pmax - pmin) >> 10, 0x7FFu) << 52) |
                                                     ((uint64_t)range_ok << 63);
#endif
    }
    K12_STAMP(2);
    uint32_t S = sh_misc[4];
    if (S > scap) S = scap;
    if (tid == 0) {
        d.win_S[w] = S;
        d.k12_path[w] = fast ? (uint8_t)nseg : (uint8_t)3;
    }

    // ---- revbuf order: reads ascending by (end<<32 | idx) (blockjoin.c:1126, 1140)
    {
        uint64_t *keyv = reinterpret_cast<uint64_t *>(tile);
        const uint32_t n2 = next_pow2(R);
        if (n2 <= PF_K1_TILE / 2) {
            __syncthreads();
            for (uint32_t i = tid; i < n2; i += NT)
                keyv[i] = i < R ? (((uint64_t)d.read_end[r0 + i]) << 32 | i) : ~0ull;
            __syncthreads();
            for (uint32_t kk = 2; kk <= n2; kk <<= 1) {
                for (uint32_t jj = kk >> 1; jj > 0; jj >>= 1) {
                    for (uint32_t i = tid; i < n2; i += NT) {
                        const uint32_t ixj = i ^ jj;
                        if (ixj > i) {
                            const uint64_t x = keyv[i], y = keyv[ixj];
                            const bool up = (i & kk) == 0;
                            if ((x > y) == up) { keyv[i] = y; keyv[ixj] = x; }
                        }
                    }
                    __syncthreads();
                }
            }
            for (uint32_t i = tid; i < R; i += NT) d.rev_ord[r0 + i] = (uint32_t)keyv[i];
        } else {
            for (uint32_t i = tid; i < R; i += NT) {
                const uint64_t ki = ((uint64_t)d.read_end[r0 + i]) << 32 | i;
                uint32_t rank = 0;
                for (uint32_t j = 0; j < R; j++) rank += (((uint64_t)d.read_end[r0 + j]) << 32 | j) < ki;
                d.rev_ord[r0 + rank] = i;
            }
        }
    }

    K12_STAMP(3);
    // ---- directional methmer lengths/starts (blockjoin.c:3307-3329), into
    // LDS (when the window's sites fit next to the methmer phase's wave
    // buffers) and HBM (K3 and the debug/parity hooks read them there)
    __syncthreads();
    const bool staged = S <= d.k12_smax;
    uint32_t *sp = tile, *st1 = tile + S, *q1s = tile + 2 * S;
    uint8_t *l0s = reinterpret_cast<uint8_t *>(tile + 3 * S), *l1s = l0s + S;
    const uint32_t *a = staged ? sp : d.site_pos + sb;
    if (staged) {
        for (uint32_t p = tid; p < S; p += NT) sp[p] = d.site_pos[sb + p];
        __syncthreads();
    }
    const uint32_t k = (uint32_t)d.k, span = (uint32_t)d.k_span;
    for (uint32_t p = tid; p < S; p += NT) {
        const uint32_t ap = a[p];
        uint32_t j = p + k > S - 1 ? S - 1 : p + k;
        while (a[j] - ap > span) j--;
        const uint8_t v0 = (uint8_t)(j == p ? 1 : j - p);
        uint32_t q = p > k ? p - k : 0;
        while (ap - a[q] > span) q++;
        const uint8_t v1 = (uint8_t)(q == p ? 1 : p - q);
        const uint32_t s1 = a[q];
        d.len0[sb + p] = v0;
        d.len1[sb + p] = v1;
        d.st1_pos[sb + p] = s1;
        d.site_q1[sb + p] = q;
        if (staged) { l0s[p] = v0; l1s[p] = v1; st1[p] = s1; q1s[p] = q; }
    }
    K12_STAMP(4);
    // ---- per-read methmer capacity and arena reservation
    // bound_r = #sites in [first call, last call] + 3k + 4 >= methmers of the read
    // in either direction (entry walk: <= xr-xl + 2k+1, xr-xl <= #sites + k + 1).
    uint32_t tot_keys = 0, tot_big = 0;
    for (uint32_t i0 = 0; i0 < R; i0 += NT) {
        const uint32_t i = i0 + tid;
        uint32_t bound = 0, bigb = 0;
        if (i < R) {
            const uint32_t r = r0 + i;
            const uint64_t c0 = d.read_call_off[r], c1 = d.read_call_off[r + 1];
            if (c1 > c0 && S > 0) {
                const uint32_t F = d.read_first[r], L = d.read_last[r];
                const uint64_t lbF = lb_u32(a, 0, S, F), ubL = ub_u32(a, 0, S, L);
                const uint32_t cnt = ubL > lbF ? (uint32_t)(ubL - lbF) : 0;
                bound = cnt + 3 * k + 4;
                if (bound > d.k2_entcap) bigb = 16 * bound;
            }
            d.mmr_cap[r] = bound;
        }
        uint32_t t1, t2;
        block_excl_scan<NT>(bound, sh_scan, &t1);
        block_excl_scan<NT>(bigb, sh_scan, &t2);
        tot_keys += t1;
        tot_big += t2;
    }
    if (tid == 0) {
        const unsigned long long kb = atomicAdd(d.keys_ctr, 2ull * tot_keys);
        if (kb + 2ull * tot_keys > d.keys_cap) atomicOr(d.status, PF_ST_KEYS_OVF);
        sh_base[0] = kb;
        unsigned long long bb = 0;
        if (tot_big) {
            bb = atomicAdd(d.big_ctr, (unsigned long long)tot_big);
            if (bb + tot_big > d.big_cap) atomicOr(d.status, PF_ST_BIG_OVF);
        }
        sh_base[1] = bb;
    }
    __syncthreads();
    if (sh_base[0] + 2ull * tot_keys > d.keys_cap) {
        // the key arena is full (status set above; the host grows it and
        // re-runs): this window writes no keys and K3 skips it (S = 0)
        for (uint32_t i = tid; i < R; i += NT) {
            const uint32_t r = r0 + i;
            d.mmr_n[2 * r] = 0; d.mmr_n[2 * r + 1] = 0;
            d.mmr_start[2 * r] = 0; d.mmr_start[2 * r + 1] = 0;
            d.mmr_off[2 * r] = 0; d.mmr_off[2 * r + 1] = 0;
            d.big_off[r] = ~0ull;
        }
        if (tid == 0) d.win_S[w] = 0;
        return;
    }
    uint64_t kcarry = sh_base[0], bcarry = sh_base[1];
    for (uint32_t i0 = 0; i0 < R; i0 += NT) {
        const uint32_t i = i0 + tid;
        uint32_t bound = 0, bigb = 0;
        if (i < R) {
            bound = d.mmr_cap[r0 + i];
            if (bound > d.k2_entcap) bigb = 16 * bound;
        }
        uint32_t t1, t2;
        const uint32_t e1 = block_excl_scan<NT>(bound, sh_scan, &t1);
        const uint32_t e2 = block_excl_scan<NT>(bigb, sh_scan, &t2);
        if (i < R) {
            const uint32_t r = r0 + i;
            d.mmr_off[2 * r] = kcarry + 2ull * e1;
            d.mmr_off[2 * r + 1] = kcarry + 2ull * e1 + bound;
            d.big_off[r] = bigb ? bcarry + e2 : ~0ull;
        }
        kcarry += 2ull * t1;
        bcarry += t2;
    }

    K12_STAMP(5);
    // ---- methmers of every read (get_mmr_of_read, blockjoin.c:3357-3451),
    // one wavefront per read, both directions, site arrays in LDS.  Reads
    // whose site-entry bound exceeds the wave buffer (and every read of a
    // window whose sites do not fit LDS) go to the K2 fallback kernel.
    // position -> site index hash (hash-path windows whose hash fits beside
    // the arrays and the wave buffers)
    const uint32_t arr_b = (uint32_t)((14ull * S + 15) & ~15ull);
    // load factor <= 1/4: most lookups are misses (calls at CpGs that are not
    // sites), which linear probing makes long at high load
    uint32_t HS = 1;
    while (HS < S * 4) HS <<= 1;
    const bool use_hash = staged && fast && nseg == 1 && arr_b + 4u * HS + 16u * PF_K12_WB * PF_K12_CAPW <= 4u * PF_K1_TILE;
    uint32_t *hst = reinterpret_cast<uint32_t *>(reinterpret_cast<uint8_t *>(tile) + arr_b);
    if (tid == 0) sh_misc[5] = NW;                       // the methmer phase's read counter
    if (use_hash) {
        for (uint32_t j = tid; j < HS; j += NT) hst[j] = PF_NONE;
        __syncthreads();
        for (uint32_t p = tid; p < S; p += NT) {
            const uint32_t rel = sp[p] - pmin;
            uint32_t h = k2_hash_slot(rel) & (HS - 1);
            while (atomicCAS(&hst[h], PF_NONE, (rel << 13) | p) != PF_NONE) h = (h + 1) & (HS - 1);
        }
    }
    __syncthreads();
    K2SiteHash hsd;
    hsd.t = hst;
    hsd.mask = HS - 1;
    hsd.pmin = pmin;

    if (staged && R >= d.k12c_minr && S <= d.k12c_smax) {
        // a heavy window: its reads go to pf_k12_chunks in chunks of
        // PF_K12C_READS, spread over the device, instead of this workgroup's
        // 16 waves (round 5: the 500 kb window's methmer phase was 1.3 ms of
        // its 1.9 ms here)
        for (uint32_t c = tid; c * PF_K12C_READS < R; c += NT) {
            const uint32_t k = atomicAdd(d.k12c_ctr, 1u);
            d.k12c_list[2ull * k] = w;
            d.k12c_list[2ull * k + 1] = c * PF_K12C_READS;
        }
    } else if (staged) {
        // per-wave buffers: chars, crank (u8), irank (u16), key staging (u32)
        uint8_t *wb = reinterpret_cast<uint8_t *>(tile) + arr_b + (use_hash ? 4u * HS : 0u) +
                      wid * (uint64_t)PF_K12_WB * PF_K12_CAPW;
#ifdef PF_K3_PROFILE
        unsigned long long k2a[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, __builtin_amdgcn_s_memtime()};
        unsigned long long *k2acc = wid == 0 ? k2a : nullptr;
#else
        unsigned long long *k2acc = nullptr;
#endif
        k12_methmers(d, r0, 0, R, wid, NW, lane, S, sp, st1, q1s, l0s, l1s, hsd, use_hash, wb, k2acc, &sh_misc[5]);
#ifdef PF_K3_PROFILE
        if (tid == 0) {
            for (int j = 0; j < 7; j++) d.prof[64ull * d.W + (uint64_t)w * 16 + 8 + j] = k2a[j];
            d.prof[64ull * d.W + (uint64_t)w * 16 + 7] = k2a[7];
            d.prof[64ull * d.W + (uint64_t)w * 16 + 15] = k2a[8];
        }
#endif
    } else {
        for (uint32_t i = tid; i < R; i += NT) d.fb_list[atomicAdd(d.fb_ctr, 1u)] = r0 + i;
    }
    __syncthreads();
    K12_STAMP(6);
}

// The methmer phase of the heavy windows K12 handed over: each item is
// PF_K12C_READS reads of one window; a workgroup stages the window's site
// arrays (14 B per site, written by K12) in LDS and runs k12_methmers over
// the chunk with its PF_K12C_WAVES waves.  Persistent over the item counter.
// No position hash (the heavy windows' calls span beyond K12's bitmap): the
// calls' site indices come from binary searches in LDS, as K12's dense-path
// windows do.
__global__ __launch_bounds__(PF_K12C_WAVES * 64) void pf_k12_chunks(pf_dev_batch d) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    __shared__ uint32_t s_item, s_rctr;
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wid = tid >> 6;
    const uint32_t n = *d.k12c_ctr;
    for (;;) {
        if (tid == 0) s_item = atomicAdd(d.k12c_next, 1u);
        __syncthreads();
        const uint32_t it = s_item;
        if (it >= n) break;
        const uint32_t w = d.k12c_list[2ull * it], c0 = d.k12c_list[2ull * it + 1];
        if (tid == 0) s_rctr = c0 + PF_K12C_WAVES;
        const uint32_t r0 = d.win_read_off[w], R = d.win_read_off[w + 1] - r0;
        const uint32_t S = d.win_S[w];
        const uint64_t sb = d.win_site_off[w];
        uint32_t *sp = reinterpret_cast<uint32_t *>(smem), *st1 = sp + S, *q1s = sp + 2 * S;
        uint8_t *l0s = reinterpret_cast<uint8_t *>(sp + 3 * S), *l1s = l0s + S;
        for (uint32_t p = tid; p < S; p += PF_K12C_WAVES * 64) {
            sp[p] = d.site_pos[sb + p];
            st1[p] = d.st1_pos[sb + p];
            q1s[p] = d.site_q1[sb + p];
            l0s[p] = d.len0[sb + p];
            l1s[p] = d.len1[sb + p];
        }
        __syncthreads();
        const uint32_t arr_b = (uint32_t)((14ull * S + 15) & ~15ull);
        uint8_t *wb = smem + arr_b + wid * (uint64_t)PF_K12_WB * PF_K12_CAPW;
        K2SiteHash hsd;
        hsd.t = nullptr; hsd.mask = 0; hsd.pmin = 0;
        const uint32_t c1 = min(R, c0 + PF_K12C_READS);
        k12_methmers(d, r0, c0, c1, wid, PF_K12C_WAVES, lane, S, sp, st1, q1s, l0s, l1s, hsd, false, wb, nullptr,
                     &s_rctr);
        __syncthreads();                                 // the site arrays are reused by the next item
    }
}

// ========================================================================
// K3: greedy haplotag extension of one (window, direction)
// ========================================================================
struct K3Ctl {
    uint32_t S, R, ntot, nc, L, done, failed, inserted, winner, tag;
    int32_t i_last;
    uint32_t min_i, max_i, fail, summ, nstrict, mxlen, cmax;
    uint32_t path, need, cacheb;              // the P2 variant taken (K3_PATH_*); (profile build) its LDS bytes, cache part
    unsigned long long t_run;                 // (profile build) s_memrealtime at k3_run's start
    uint32_t ins_n, ins_st, ins_mo, ins_tg;   // register variant: winner whose insert is pending
    unsigned long long scr;
    int32_t tab[4];
};

struct K3Cand {
    uint32_t read[PF_MAX_NCAND];
    uint32_t pos[PF_MAX_NCAND];
    uint32_t site0[PF_MAX_NCAND];
    uint32_t len[PF_MAX_NCAND];
    uint32_t kofs[PF_MAX_NCAND];
    unsigned long long key[PF_MAX_NCAND];
    uint8_t tag[PF_MAX_NCAND];
};

// the slim loop's static LDS (k3_greedy_slim): the per-wave queue scratch
// (64 entries per wave), the push/positive count pairs [2][64] and the exact
// hap sums [2][2][64] -- 3.5 KB instead of K3Cand's 7.2 KB, so more problems
// fit a CU beside their dynamic budget
template <int NTH>
struct K3CandSlimT {
    uint32_t read[NTH];
    uint32_t pos[128];
    unsigned long long key[256];
};
using K3CandSlim = K3CandSlimT<PF_K3S_THREADS>;

DEV uint64_t align16(uint64_t x) { return (x + 15) & ~15ull; }

// Every methmer key of the problem's reads (direction dir) that `keep(i)`
// selects: f(read i, index t, site st + t, arena offset, key).  A wave takes
// eight reads at a time with all their scalar fields and key loads issued
// before the first use, so a workgroup keeps 32 reads' loads in flight
// instead of walking one read per wave through two dependent round trips
// (the prologue of a 1,400-read problem was a quarter of its greedy loop).
template <int NT, typename K, typename F>
DEV void k3_each_key(const pf_dev_batch &d, uint32_t r0, uint32_t R, uint32_t dir, K &&keep, F &&f) {
    constexpr uint32_t B = 8, NW = NT / 64;
    const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (uint32_t i0 = wid * B; i0 < R; i0 += NW * B) {
        uint32_t n[B], st[B], key[B];
        uint64_t off[B];
#pragma unroll
        for (uint32_t u = 0; u < B; u++) {
            const uint32_t i = i0 + u;
            const bool ok = i < R && keep(i);
            const uint64_t g = 2ull * (r0 + (ok ? i : 0u)) + dir;
            n[u] = ok ? d.mmr_n[g] : 0u;
            st[u] = d.mmr_start[g];
            off[u] = d.mmr_off[g];
        }
#pragma unroll
        for (uint32_t u = 0; u < B; u++) key[u] = lane < n[u] ? d.keys[off[u] + lane] : 0u;
#pragma unroll
        for (uint32_t u = 0; u < B; u++)
            if (lane < n[u]) f(i0 + u, lane, st[u] + lane, off[u] + lane, key[u]);
#pragma unroll
        for (uint32_t u = 0; u < B; u++)
            for (uint32_t t = 64 + lane; t < n[u]; t += 64) f(i0 + u, t, st[u] + t, off[u] + t, d.keys[off[u] + t]);
    }
}

// dictionary of methmer keys per site -> dense slot ids (replaces the per-site
// key lists + linear search of insert_mmrs_to_counts / query_counts_of_mmrs)
template <int NT = PF_K3_THREADS>
DEV void k3_dict(const pf_dev_batch &d, uint32_t r0, uint32_t R, uint32_t S, uint32_t dir,
                 uint64_t *masks, uint32_t *base, uint32_t *sh_scan, K3Ctl &ctl) {
    const uint32_t tid = threadIdx.x;
    const uint32_t MW = (uint32_t)d.mw;
    for (uint32_t j = tid; j < S * MW; j += NT) masks[j] = 0;
    __syncthreads();
    k3_each_key<NT>(d, r0, R, dir, [](uint32_t) { return true; },
                    [&](uint32_t, uint32_t, uint32_t site, uint64_t, uint32_t key) {
                        if (site < S && key < 64u * MW)
                            atomicOr((unsigned long long *)&masks[(uint64_t)site * MW + (key >> 6)], 1ull << (key & 63));
                    });
    __syncthreads();
    uint32_t carry = 0;
    for (uint32_t p0 = 0; p0 < S; p0 += NT) {
        const uint32_t p = p0 + tid;
        uint32_t c = 0;
        if (p < S)
            for (uint32_t m = 0; m < MW; m++) c += (uint32_t)__popcll(masks[(uint64_t)p * MW + m]);
        uint32_t tot;
        const uint32_t ex = block_excl_scan<NT>(c, sh_scan, &tot);
        if (p < S) base[p] = carry + ex;
        carry += tot;
    }
    if (tid == 0) ctl.ntot = carry;
    __syncthreads();
}

// second half: rewrite every key in place into its slot id (destructive: a
// problem is committed to a kernel before this)
template <int NT = PF_K3_THREADS>
DEV void k3_dict_rewrite(const pf_dev_batch &d, uint32_t r0, uint32_t R, uint32_t S, uint32_t dir,
                         const uint64_t *masks, const uint32_t *base) {
    const uint32_t MW = (uint32_t)d.mw;
    k3_each_key<NT>(d, r0, R, dir, [](uint32_t) { return true; },
                    [&](uint32_t, uint32_t, uint32_t site, uint64_t koff, uint32_t key) {
                        uint32_t slot = PF_NONE;
                        if (site < S && key < 64u * MW) {
                            const uint64_t *row = masks + (uint64_t)site * MW;
                            const uint32_t wi = key >> 6, b = key & 63;
                            slot = base[site];
                            for (uint32_t m = 0; m < wi; m++) slot += (uint32_t)__popcll(row[m]);
                            slot += (uint32_t)__popcll(row[wi] & ((1ull << b) - 1ull));
                        }
                        d.keys[koff] = slot;
                    });
    __syncthreads();
}

// ---- k > 5: the slot dictionary from per-site hash tables (pf_k3_kdict).
// insert_mmrs_to_counts (blockjoin.c:3453-3486) keeps, per site, a linear list
// of the distinct methmer keys it has seen, and query_counts_of_mmrs
// (3669-3691) searches it; the greedy kernels index the counts by a dense
// slot id per (site, key) instead.  For k <= 5 k3_dict numbers the slots from
// a 4^k-bit mask per site.  Past that the masks outgrow any memory (4^15 bits
// a site at the reference's documented maximum, cli.c:243), so this kernel --
// one workgroup per problem, launched before the greedy kernels -- gives each
// site an open-addressing table of 2^ceil(log2(2 cov)) keys in HBM scratch
// (cov: the methmers at the site, <= half full), ranks each site's distinct
// keys, and rewrites every key into base[site] + its rank: the numbering the
// masks give, so both dictionaries yield the same slots (PF_K3_KDICT=1 forces
// this one at any k; tests compare the two).  The greedy kernels then skip
// their dictionary phase and read the problem's slot count from k3_ntot.
DEV uint32_t kd_hash(uint32_t key) {
    const uint32_t h = key * 0x9E3779B1u;
    return h ^ (h >> 15);
}
DEV void kd_sync() {                    // HBM tables written by other waves of the workgroup
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
}

__global__ __launch_bounds__(PF_K3_THREADS) void pf_k3_kdict(pf_dev_batch d) {
    constexpr uint32_t NT = PF_K3_THREADS, NW = NT / 64;
    __shared__ uint32_t sh_scan[NW + 1];
    __shared__ unsigned long long s_o;
    __shared__ uint32_t s_fail;
    const uint32_t prob = blockIdx.x, w = prob >> 1, dir = prob & 1;
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wid = tid >> 6;
    const uint32_t S = d.win_S[w];
    if (S == 0) {
        if (tid == 0) d.k3_ntot[prob] = 0;
        return;
    }
    const uint32_t R = d.win_nreads[w], r0 = d.win_read_off[w];
    auto alloc = [&](uint64_t bytes) -> bool {     // workgroup-uniform scratch allocation
        if (tid == 0) {
            const unsigned long long o = atomicAdd(d.scr_ctr, (unsigned long long)bytes);
            s_fail = o + bytes > d.scr_cap;
            if (s_fail) atomicOr(d.status, PF_ST_SCR_OVF);   // the host grows the scratch and re-runs
            s_o = o;
        }
        __syncthreads();
        return s_fail == 0;
    };
    // per site: the methmer coverage (a difference array first), then the
    // table's capacity; its table offset; its distinct keys, then its base
    if (!alloc(align16(12ull * (S + 1)))) { if (tid == 0) d.k3_ntot[prob] = PF_NONE; return; }
    uint32_t *cap = reinterpret_cast<uint32_t *>(d.scr + s_o), *toff = cap + (S + 1), *base = toff + (S + 1);
    for (uint32_t j = tid; j <= S; j += NT) cap[j] = 0;
    kd_sync();
    for (uint32_t i = tid; i < R; i += NT) {
        const uint64_t g = 2ull * (r0 + i) + dir;
        const uint32_t n = d.mmr_n[g], st = d.mmr_start[g];
        if (n && st < S) {
            atomicAdd(&cap[st], 1u);
            atomicAdd(&cap[st + n < S ? st + n : S], 0xFFFFFFFFu);
        }
    }
    kd_sync();
    // contiguous runs of sites per thread: coverage, capacity, table offsets
    const uint32_t per = (S + NT - 1) / NT, j0 = min(tid * per, S), j1 = min(j0 + per, S);
    uint32_t part = 0, tot = 0;
    for (uint32_t j = j0; j < j1; j++) part += cap[j];
    uint32_t run = block_excl_scan<NT>(part, sh_scan, &tot), csum = 0;
    for (uint32_t j = j0; j < j1; j++) {
        run += cap[j];
        const uint32_t c = run ? 1u << (32 - __builtin_clz(2u * run - 1u)) : 0u;   // >= 2 cov, a power of 2
        cap[j] = c;
        csum += c;
    }
    uint32_t T = 0;
    uint32_t o = block_excl_scan<NT>(csum, sh_scan, &T);
    for (uint32_t j = j0; j < j1; j++) { toff[j] = o; o += cap[j]; }
    if (!alloc(align16(8ull * T))) { if (tid == 0) d.k3_ntot[prob] = PF_NONE; return; }   // keys not rewritten
    uint32_t *tbl = reinterpret_cast<uint32_t *>(d.scr + s_o), *rk = tbl + T;   // key + 1 (0: empty), rank
    for (uint32_t j = tid; j < T; j += NT) tbl[j] = 0;
    kd_sync();
    k3_each_key<NT>(d, r0, R, dir, [](uint32_t) { return true; },
                    [&](uint32_t, uint32_t, uint32_t site, uint64_t, uint32_t key) {
                        if (site >= S) return;
                        const uint32_t m = cap[site] - 1u, ob = toff[site];
                        for (uint32_t h = kd_hash(key) & m;; h = (h + 1u) & m) {
                            const uint32_t prev = atomicCAS(&tbl[ob + h], 0u, key + 1u);
                            if (prev == 0u || prev == key + 1u) break;
                        }
                    });
    kd_sync();
    // one wave per site: each distinct key's rank among the site's keys
    for (uint32_t s = wid; s < S; s += NW) {
        const uint32_t c = cap[s], ob = toff[s];
        uint32_t nd = 0;
        for (uint32_t a0 = 0; a0 < c; a0 += 64) {
            const uint32_t v = a0 + lane < c ? tbl[ob + a0 + lane] : 0u;
            uint32_t r = 0;
            for (uint32_t b0 = 0; b0 < c; b0 += 64) {
                const uint32_t u = b0 + lane < c ? tbl[ob + b0 + lane] : 0u;
                for (uint64_t m = __ballot(u != 0u); m; m &= m - 1) {
                    const uint32_t x = (uint32_t)__builtin_amdgcn_readlane((int)u, __builtin_ctzll(m));
                    r += x < v ? 1u : 0u;
                }
            }
            if (v) rk[ob + a0 + lane] = r;
            nd += (uint32_t)__popcll(__ballot(v != 0u));
        }
        if (lane == 0) base[s] = nd;
    }
    kd_sync();
    part = 0;
    for (uint32_t j = j0; j < j1; j++) part += base[j];
    uint32_t ntot = 0;
    run = block_excl_scan<NT>(part, sh_scan, &ntot);
    for (uint32_t j = j0; j < j1; j++) { const uint32_t x = base[j]; base[j] = run; run += x; }
    if (tid == 0) d.k3_ntot[prob] = ntot;
    kd_sync();
    k3_each_key<NT>(d, r0, R, dir, [](uint32_t) { return true; },
                    [&](uint32_t, uint32_t, uint32_t site, uint64_t koff, uint32_t key) {
                        uint32_t slot = PF_NONE;
                        if (site < S) {
                            const uint32_t m = cap[site] - 1u, ob = toff[site];
                            uint32_t h = kd_hash(key) & m;
                            while (tbl[ob + h] != key + 1u) h = (h + 1u) & m;   // inserted above: found
                            slot = base[site] + rk[ob + h];
                        }
                        d.keys[koff] = slot;
                    });
}

struct K3Mem {
    uint32_t *sum, *cnt, *aux, *mo;
    void *mn, *mst;          // methmers per read, first site index: u16 when m16 (the slim loop: S < 8192), else u32
    bool m16;
    uint16_t *ord;           // dir-1 scan order (window-local read indices, R < 2^16)
    const uint64_t *gmo;     // mo == nullptr: the reads' key offsets in HBM (d.mmr_off, stride 2), minus kbase
    const uint32_t *gmn, *gmst;   // mn == nullptr: the reads' methmer counts / first sites in HBM (stride 2)
    uint64_t kbase;
    uint8_t *hp, *flg;
    uint64_t *untag;
    uint16_t *sl16;          // slot lists in LDS (u16), when they fit
    const uint32_t *kb;      // slot lists in the HBM key arena (window base)
    float2 *recv;            // per-wave record rings
    uint32_t *recc;
    uint32_t rcw;            // records per wave
};

#define K3_NOFF 13
// P2 byte layout.  Returns the bytes needed with `rcw` records per wave;
// slots (u16) are included only when with_slots, the per-read slot-list
// offsets only when with_mo (the candidate cache reads them from HBM), and
// aux_b bytes of T5 scratch (4R, or 0 when it lives in the cache region).
// No per-site divisor cache: a term's divisor is its site's hap total, and
// its reciprocal is taken beside the dependent count load.
DEV uint64_t k3_layout(uint32_t S, uint32_t ntot, uint32_t R, uint32_t dir, uint32_t summ,
                       bool with_slots, uint32_t rcw, uint64_t off[K3_NOFF], bool c8 = false, bool with_mo = true,
                       uint64_t aux_b = ~0ull, bool with_mnst = true, bool with_side = true, bool with_cnt = true) {
    const uint32_t nwords = (R + 63) >> 6;
    const uint64_t sd = with_side ? 1ull : 0ull;       // hp, flg, ord in LDS (else k3_side_mem)
    off[0] = 0;                                        // sum   S*4
    off[1] = align16(off[0] + 4ull * S);               // cnt   ntot*4 (in HBM when !with_cnt: path 6)
    off[2] = align16(off[1] + (with_cnt ? (c8 ? 2ull : 4ull) * ntot : 0ull));   // hp    R (cnt: u8 pairs when c8)
    off[3] = align16(off[2] + sd * R);                 // flg   R
    off[4] = align16(off[3] + sd * R);                 // ord   R*2 (dir 1)
    off[5] = align16(off[4] + (dir ? 2ull * sd * R : 0));   // untag nwords*8
    const uint64_t mw = !with_mnst ? 0ull : S < 8192u ? 2ull : 4ull;   // (u16 when every index fits: see k3_mem)
    off[6] = align16(off[5] + 8ull * nwords);          // mn    R*2|4  methmers per read
    off[7] = align16(off[6] + mw * R);                 // mst   R*2|4  first site index
    off[8] = align16(off[7] + mw * R);                 // mo    R*4  slot-list offset (optional)
    off[9] = align16(off[8] + (with_mo ? 4ull * R : 0));   // sl16  summ*2 (optional)
    off[10] = align16(off[9] + (with_slots ? 2ull * summ : 0));
    off[11] = off[10];                                 // records / aux
    const uint64_t rec = 12ull * PF_K3_WAVES * rcw;
    const uint64_t aux = aux_b == ~0ull ? 4ull * R : aux_b;
    off[12] = off[11] + (rec > aux ? rec : aux);
    return off[12];
}

DEV void k3_mem(uint8_t *base, const uint64_t off[K3_NOFF], uint32_t rcw, bool with_slots,
                const uint32_t *kb, K3Mem &m, bool with_mo = true, uint32_t S = 0xFFFFFFFFu, bool with_mnst = true) {
    m.sum = reinterpret_cast<uint32_t *>(base + off[0]);
    m.cnt = reinterpret_cast<uint32_t *>(base + off[1]);
    m.hp = base + off[2];
    m.flg = base + off[3];
    m.ord = reinterpret_cast<uint16_t *>(base + off[4]);
    m.untag = reinterpret_cast<uint64_t *>(base + off[5]);
    m.mn = with_mnst ? base + off[6] : nullptr;
    m.mst = with_mnst ? base + off[7] : nullptr;
    m.gmn = m.gmst = nullptr;
    m.m16 = S < 8192u;
    m.mo = with_mo ? reinterpret_cast<uint32_t *>(base + off[8]) : nullptr;
    m.gmo = nullptr;
    m.kbase = 0;
    m.sl16 = with_slots ? reinterpret_cast<uint16_t *>(base + off[9]) : nullptr;
    m.kb = kb;
    m.recv = reinterpret_cast<float2 *>(base + off[11]);
    m.recc = reinterpret_cast<uint32_t *>(base + off[11] + 8ull * PF_K3_WAVES * rcw);
    m.aux = reinterpret_cast<uint32_t *>(base + off[11]);
    m.rcw = rcw;
}

// the per-read side arrays (hp, flg, ord, aux) of problem (r0, dir) in the
// batch's HBM buffer d.k3_side: touched by the problem set-up, one store per
// iteration (the winner's hp), a load per 64 queued reads (ord) and the
// finish -- LDS left to the tables the greedy loop reads in every iteration
DEV void k3_side_mem(const pf_dev_batch &d, uint32_t r0, uint32_t dir, K3Mem &m) {
    const uint64_t RB = d.R;
    m.hp = d.k3_side + dir * RB + r0;
    m.flg = d.k3_side + 2 * RB + dir * RB + r0;
    m.ord = reinterpret_cast<uint16_t *>(d.k3_side + 4 * RB) + r0;
    m.aux = reinterpret_cast<uint32_t *>(d.k3_side + ((6 * RB + 3) & ~3ull)) + dir * RB + r0;
}

DEV uint32_t k3_mn(const K3Mem &m, uint32_t i) {
    if (!m.mn) return m.gmn[2ull * i];
    return m.m16 ? (uint32_t)static_cast<const uint16_t *>(m.mn)[i] : static_cast<const uint32_t *>(m.mn)[i];
}
DEV uint32_t k3_mst(const K3Mem &m, uint32_t i) {
    if (!m.mst) return m.gmst[2ull * i];
    return m.m16 ? (uint32_t)static_cast<const uint16_t *>(m.mst)[i] : static_cast<const uint32_t *>(m.mst)[i];
}
// a read's slot-list offset in the HBM key arena (window base)
DEV uint32_t k3_mo(const K3Mem &m, uint32_t rd) {
    return m.mo ? m.mo[rd] : (uint32_t)(m.gmo[2ull * rd] - m.kbase);
}

#define FLG_LEFT 1u
#define FLG_LEFT_STRICT 2u
#define FLG_RIGHT 4u
#define FLG_RIGHT_STRICT 8u

// update_available_methmer_range (blockjoin.c:3669-3691), one wavefront
DEV void k3_range_update(const uint32_t *sum, uint32_t S, int cov_rt, K3Ctl &ctl, uint32_t lane) {
    const int m0 = (int)ctl.min_i;
    if (m0 >= 0) {
        int count = 0;
        for (;;) {
            const int i = m0 - count - (int)lane;
            bool cv = false;
            if (i >= 0) {
                const uint32_t v = sum[i];
                cv = (int)((v & 0xffffu) + (v >> 16)) >= cov_rt;
            }
            const uint64_t bal = __ballot(cv);
            if (bal == ~0ull) { count += 64; continue; }
            count += __ffsll((unsigned long long)~bal) - 1;
            break;
        }
        if (count > 0 && lane == 0) ctl.min_i = (uint32_t)(m0 - count + 1);
    }
    const int M0 = (int)ctl.max_i;
    if (M0 >= 0) {
        int count = 0;
        for (;;) {
            const int i = M0 + count + (int)lane;
            bool cv = false;
            if (i < (int)S) {
                const uint32_t v = sum[i];
                cv = (int)((v & 0xffffu) + (v >> 16)) >= cov_rt;
            }
            const uint64_t bal = __ballot(cv);
            if (bal == ~0ull) { count += 64; continue; }
            count += __ffsll((unsigned long long)~bal) - 1;
            break;
        }
        if (count > 0 && lane == 0) ctl.max_i = (uint32_t)(M0 + count - 1);
    }
    wave_sync();
}

struct K3Stats {
    unsigned long long lookups, inserts, iters, scanned;
};
#define PF_NSTAT 8

// next untagged scan position after p (dir 0: > p) / before p (dir 1: < p);
// -1 if none.  One wavefront; no cross-lane shuffles (ballot + readlane).
DEV int k3_next_untag(const uint64_t *untag, uint32_t nwords, int p, uint32_t dir, uint32_t lane) {
    if (dir == 0) {
        const int q = p + 1;
        if (q >= (int)(nwords * 64)) return -1;
        const uint32_t w0 = (uint32_t)q >> 6;
        for (uint32_t wb = w0; wb < nwords; wb += 64) {
            const uint32_t wi = wb + lane;
            uint64_t bits = wi < nwords ? untag[wi] : 0ull;
            if (wi == w0) bits &= ~0ull << ((uint32_t)q & 63);
            const uint64_t bal = __ballot(bits != 0);
            if (bal) {
                const int src = __ffsll((unsigned long long)bal) - 1;
                const int v = (int)(wi * 64 + (uint32_t)(__ffsll((unsigned long long)bits) - 1));
                return __builtin_amdgcn_readlane(v, src);
            }
        }
        return -1;
    } else {
        const int q = p - 1;
        if (q < 0) return -1;
        const int w0 = q >> 6;
        for (int wb = w0; wb >= 0; wb -= 64) {
            const int wi = wb - (int)lane;
            uint64_t bits = wi >= 0 ? untag[wi] : 0ull;
            if (wi == w0) {
                const uint32_t b = (uint32_t)q & 63;
                bits &= b == 63 ? ~0ull : ((1ull << (b + 1)) - 1ull);
            }
            const uint64_t bal = __ballot(bits != 0);
            if (bal) {
                const int src = __ffsll((unsigned long long)bal) - 1;
                const int v = bits ? wi * 64 + (63 - __clzll((long long)bits)) : 0;
                return __builtin_amdgcn_readlane(v, src);
            }
        }
        return -1;
    }
}

// Candidate queue of the register variant: the untagged reads that follow
// position p in scan order (dir 0: > p, dir 1: < p), up to 64, lane k holding
// entry k with its read and methmer fields.  Reads after the last candidate
// are untouched until they join the list, so one build serves up to 64
// appends.  `cont` is where a further build continues; `more` whether
// anything may lie beyond.
DEV uint32_t k3_qbuild(const K3Mem &m, uint32_t nwords, int p, uint32_t dir, uint32_t lane, uint32_t *qbuf,
                       uint32_t &q_pos, uint32_t &q_rd, uint32_t &q_n, uint32_t &q_st, uint32_t &q_mo,
                       bool &more, int &cont) {
    uint64_t bits = 0;
    int wi, w0;
    bool more_words;
    if (dir == 0) {
        const int q = p + 1;
        if (q >= (int)(nwords * 64)) { more = false; return 0; }
        w0 = q >> 6;
        wi = w0 + (int)lane;
        if (wi < (int)nwords) {
            bits = m.untag[wi];
            if (wi == w0) bits &= ~0ull << (q & 63);
        }
        more_words = w0 + 64 < (int)nwords;
    } else {
        const int q = p - 1;
        if (q < 0) { more = false; return 0; }
        w0 = q >> 6;
        wi = w0 - (int)lane;
        if (wi >= 0) {
            bits = m.untag[wi];
            if (wi == w0) {
                const uint32_t b = (uint32_t)q & 63;
                bits &= b == 63 ? ~0ull : ((1ull << (b + 1)) - 1ull);
            }
        }
        more_words = w0 - 64 >= 0;
    }
    const uint32_t pc = (uint32_t)__popcll(bits);
    const uint32_t incl = wave_incl_scan_dpp(pc);
    const uint32_t tot = rdl(incl, 63);
    uint32_t k = incl - pc;
    while (bits != 0 && k < 64) {
        const int b = dir == 0 ? __ffsll((unsigned long long)bits) - 1 : 63 - __clzll((long long)bits);
        qbuf[k++] = (uint32_t)(wi * 64 + b);
        bits &= ~(1ull << b);
    }
    wave_sync();
    const uint32_t cnt = tot < 64 ? tot : 64;
    if (lane < cnt) {
        q_pos = qbuf[lane];
        q_rd = dir ? m.ord[q_pos] : q_pos;
        q_n = k3_mn(m, q_rd);
        q_st = k3_mst(m, q_rd);
        q_mo = k3_mo(m, q_rd);
    }
    if (tot > 64) cont = (int)qbuf[63];
    else cont = dir == 0 ? (w0 + 64) * 64 - 1 : (w0 - 63) * 64;
    more = tot > 64 || more_words;
    wave_sync();
    return cnt;
}

// per-candidate derived fields for the current range (query_counts_of_mmrs
// only uses sites in [min_i, max_i), blockjoin.c:3500-3501); one wavefront.
DEV void k3_cand_fields(const K3Mem &m, uint32_t nc, uint32_t dir, uint32_t lane, const K3Ctl &ctl,
                        K3Cand &cd, K3Stats &stx) {
    const uint32_t mn_ = ctl.min_i, mx_ = ctl.max_i;
    uint32_t lsum = 0;
    for (uint32_t c = lane; c < nc; c += 64) {
        const uint32_t rd = cd.read[c];
        const uint32_t n = k3_mn(m, rd), st = k3_mst(m, rd);
        const uint64_t lo = st > mn_ ? st : mn_;
        const uint64_t hi0 = (uint64_t)st + n;
        const uint64_t hi = hi0 < mx_ ? hi0 : mx_;
        const uint32_t len = hi > lo ? (uint32_t)(hi - lo) : 0;
        cd.site0[c] = (uint32_t)lo;
        cd.len[c] = len;
        cd.kofs[c] = k3_mo(m, rd) + (len ? (uint32_t)(lo - st) : 0);
        lsum += len;
    }
    // lookups statistic: a wave sum without shuffles (ballot bit-slices)
    uint32_t tot = 0;
#pragma unroll
    for (int b = 0; b < 16; b++) tot += (uint32_t)__popcll(__ballot((lsum >> b) & 1)) << b;
    stx.lookups += tot;
    wave_sync();
}

// full candidate collection from i_last (:4037-4051), one wavefront: used at
// start and after a failed iteration (i_last moves).  Returns with
// ctl.done or a non-empty list.
DEV void k3_collect(const K3Mem &m, uint32_t R, uint32_t dir, uint32_t NC, uint32_t lane,
                    K3Ctl &ctl, K3Cand &cd, K3Stats &stx) {
    const uint32_t nwords = (R + 63) >> 6;
    int il = ctl.i_last;
    uint32_t failed = ctl.failed;
    for (;;) {
        const bool stop = dir == 0 ? il >= (int)R : il <= 0;
        if (stop) {
            if (lane == 0) { ctl.done = 1; ctl.i_last = il; ctl.failed = failed; }
            wave_sync();
            return;
        }
        // first NC set bits from il (scan order), sequential over words
        uint32_t found = 0;
        int p = dir == 0 ? il - 1 : il + 1;
        while (found < NC) {
            const int q = k3_next_untag(m.untag, nwords, p, dir, lane);
            if (q < 0) break;
            if (lane == 0) cd.pos[found] = (uint32_t)q;
            found++;
            p = q;
        }
        wave_sync();
        const uint32_t nc = found;
        if (nc == 0) {
            stx.scanned += dir == 0 ? (uint32_t)((int)R - il) : (uint32_t)(il + 1);
            failed++;
            if (failed > 10) {
                if (lane == 0) { ctl.done = 1; ctl.i_last = il; ctl.failed = failed; }
                wave_sync();
                return;
            }
            il += dir == 0 ? (int)NC : -(int)NC;
            continue;
        }
        for (uint32_t c = lane; c < nc; c += 64) {
            const uint32_t pp = cd.pos[c];
            cd.read[c] = dir ? m.ord[pp] : pp;
        }
        if (lane == 0) { ctl.done = 0; ctl.nc = nc; ctl.i_last = il; ctl.failed = failed; }
        wave_sync();
        return;
    }
}

// reads visited by the reference's scan this iteration (statistic only)
DEV void k3_scanned(const K3Ctl &ctl, const K3Cand &cd, uint32_t R, uint32_t dir, uint32_t NC,
                    K3Stats &stx) {
    const int il = ctl.i_last;
    const uint32_t nc = ctl.nc;
    if (nc >= NC) {
        const uint32_t pl = cd.pos[NC - 1];
        stx.scanned += dir == 0 ? pl - (uint32_t)il + 1 : (uint32_t)il - pl + 1;
    } else stx.scanned += dir == 0 ? (uint32_t)((int)R - il) : (uint32_t)(il + 1);
    stx.iters++;
}

// raw slot-list entry: u16 (0xFFFF = none) in LDS, u32 (PF_NONE) in HBM
template <bool SLDS>
DEV uint32_t k3_slot_raw(const K3Mem &m, uint32_t off) {
    if (SLDS) return m.sl16[off];
    return m.kb[off];
}

template <bool SLDS>
DEV uint32_t k3_slot(const K3Mem &m, uint32_t off) {
    if (SLDS) {
        const uint32_t v = m.sl16[off];
        return v == 0xFFFFu ? PF_NONE : v;
    }
    return m.kb[off];
}

// Fill of one lane's record-row entries t = tstart, tstart+step, ... < tpad
// (entries t >= tend are written as zero); returns the lane's push/positive
// count pair.  Four rounds of loads in flight.
// a slot's (hap0, hap1) counts as hap0 | hap1 << 16: u16 pairs (C8 = false)
// or, when no site is covered by more than 255 reads' methmers (so no count
// can exceed 255), u8 pairs -- half the table, more problems per CU
template <bool C8>
DEV uint32_t k3_cnt_get(const K3Mem &m, uint32_t sl) {
    if (!C8) return m.cnt[sl];
    const uint32_t c = reinterpret_cast<const uint16_t *>(m.cnt)[sl];
    return (c & 0xffu) | ((c >> 8) << 16);
}

template <bool SLDS>
DEV uint32_t k3_fill_rows(const K3Mem &m, uint32_t f_lo, uint32_t f_kofs, uint32_t tstart, uint32_t tend,
                          uint32_t tpad, uint32_t step, float2 *row, double &e0, double &e1) {
    uint32_t lcode = 0;
    for (uint32_t tb = tstart; tb < tpad; tb += 4 * step) {
        // unconditional loads (out-of-span lanes read entry 0 and are masked
        // afterwards)
        uint32_t sl[4], cv[4], sv[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint32_t t = tb + u * step;
            const bool ok = t < tend;
            sl[u] = k3_slot_raw<SLDS>(m, ok ? f_kofs + t : 0u);
            sv[u] = m.sum[ok ? f_lo + t : 0u];
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint32_t t = tb + u * step;
            const bool ok = t < tend && sl[u] != (SLDS ? 0xFFFFu : PF_NONE);
            const uint32_t c = m.cnt[ok ? sl[u] : 0u];
            cv[u] = ok ? c : 0u;
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint32_t t = tb + u * step;
            const uint32_t a0 = cv[u] & 0xffffu, a1 = cv[u] >> 16;
            const uint32_t h0 = sv[u] & 0xffffu, h1 = sv[u] >> 16;
            // key present at this site (inserted at least once) and sum != 0:
            // pushed; cnt > 0: positive (blockjoin.c:3505-3509, :3619-3624)
            const bool p0 = cv[u] != 0 && h0 != 0, p1 = cv[u] != 0 && h1 != 0;
            const float q0 = div_u16_y((float)a0, (float)h0, h0 ? __builtin_amdgcn_rcpf((float)h0) : 0.f);
            const float q1 = div_u16_y((float)a1, (float)h1, h1 ? __builtin_amdgcn_rcpf((float)h1) : 0.f);
            lcode += (p0 ? 1u + (a0 ? 1u : 0u) : 0u) + ((p1 ? 1u + (a1 ? 1u : 0u) : 0u) << 16);
            if (t < tpad) row[t] = make_float2(q0, q1);
            e0 += (double)q0;                        // exact: see k3_pick_exact
            e1 += (double)q1;
        }
    }
    return lcode;
}

#define K3_FADD(acc, x) asm("v_add_f32 %0, %0, %1" : "+v"(acc) : "v"(x))

// insert_mmr_counts of one tagged read (hap tg) by the whole workgroup: its
// sites are distinct, so a plain read-modify-write per site
template <bool SLDS, int NT = PF_K3_THREADS, bool C8 = false>
DEV void k3_insert_all(const K3Mem &m, uint32_t S, uint32_t n, uint32_t st, uint32_t mo, uint32_t tg) {
    const uint32_t inc = tg ? 0x10000u : 1u;
    for (uint32_t tb = 0; tb < n; tb += 2 * NT) {
        uint32_t sl[2], cc[2], sv[2];
        bool ok[2];
#pragma unroll
        for (int u = 0; u < 2; u++) {
            const uint32_t t = tb + u * NT + threadIdx.x;
            ok[u] = t < n && st + t < S;
            sl[u] = k3_slot_raw<SLDS>(m, ok[u] ? mo + t : 0u);
        }
#pragma unroll
        for (int u = 0; u < 2; u++) {
            const uint32_t t = tb + u * NT + threadIdx.x;
            ok[u] = ok[u] && sl[u] != (SLDS ? 0xFFFFu : PF_NONE);
            cc[u] = C8 ? (uint32_t)reinterpret_cast<const uint16_t *>(m.cnt)[ok[u] ? sl[u] : 0u] : m.cnt[ok[u] ? sl[u] : 0u];
            sv[u] = m.sum[ok[u] ? st + t : 0u];
        }
        asm volatile("" ::: "memory");              // every load issued before the first store
#pragma unroll
        for (int u = 0; u < 2; u++) {
            if (ok[u]) {
                const uint32_t site = st + tb + u * NT + threadIdx.x;
                if (C8) reinterpret_cast<uint16_t *>(m.cnt)[sl[u]] = (uint16_t)(cc[u] + (tg ? 0x100u : 1u));
                else m.cnt[sl[u]] = cc[u] + inc;
                m.sum[site] = sv[u] + inc;
            }
        }
    }
}

// Exact-sum fill of the register variant: the lane's terms t = tstart,
// tstart+step, ... < tend, accumulated into the exact fp64 sums (no record
// rows: the sequential fold, needed for 0.05-0.5 % of picks, recomputes its
// terms with k3_fold_direct).  Returns the push/positive count pair.
template <bool SLDS, bool C8 = false>
DEV uint32_t k3_fill_sums(const K3Mem &m, uint32_t f_lo, uint32_t f_kofs, uint32_t tstart, uint32_t tend,
                          uint32_t step, double &e0, double &e1) {
    uint32_t lcode = 0;
    for (uint32_t tb = tstart; tb < tend; tb += 4 * step) {
        uint32_t sl[4], cv[4], sv[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint32_t t = tb + u * step;
            const bool ok = t < tend;
            sl[u] = k3_slot_raw<SLDS>(m, ok ? f_kofs + t : 0u);
            sv[u] = m.sum[ok ? f_lo + t : 0u];
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint32_t t = tb + u * step;
            const bool ok = t < tend && sl[u] != (SLDS ? 0xFFFFu : PF_NONE);
            const uint32_t c = k3_cnt_get<C8>(m, ok ? sl[u] : 0u);
            cv[u] = ok ? c : 0u;
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint32_t a0 = cv[u] & 0xffffu, a1 = cv[u] >> 16;
            // the divisors: the site's hap totals (0 -> a zero reciprocal, so 0/h = 0)
            const uint32_t h0 = sv[u] & 0xffffu, h1 = sv[u] >> 16;
            const float q0 = div_u16_y((float)a0, (float)h0, h0 ? __builtin_amdgcn_rcpf((float)h0) : 0.f);
            const float q1 = div_u16_y((float)a1, (float)h1, h1 ? __builtin_amdgcn_rcpf((float)h1) : 0.f);
            // push/positive counts (:3505-3509, :3619-3624): pushed = key present
            // (cv != 0) and hap total != 0; positive = cnt > 0, which implies
            // pushed.  Both haps packed per u32 half: min(cnt, 1) and
            // min(total, 1) in one v_pk_min_u16 each.
            uint32_t posc, hm;
            asm("v_pk_min_u16 %0, %1, %2" : "=v"(posc) : "v"(cv[u]), "s"(0x00010001u));
            asm("v_pk_min_u16 %0, %1, %2" : "=v"(hm) : "v"(sv[u]), "s"(0x00010001u));
            lcode += posc + (cv[u] ? hm : 0u);
            e0 += (double)q0;
            e1 += (double)q1;
        }
    }
    return lcode;
}

// The reference's sequential float sums (blockjoin.c:3619-3636) of one
// candidate, terms recomputed from the tables in methmer order (the rare
// picks the exact intervals cannot decide).
template <bool SLDS, bool C8 = false>
DEV void k3_fold_direct(const K3Mem &m, uint32_t lo, uint32_t kofs, uint32_t len, float &s0, float &s1) {
    for (uint32_t t0 = 0; t0 < len; t0 += 8) {
        uint32_t sl[8], sv[8];
        float q0[8], q1[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const uint32_t t = t0 + u;
            const bool ok = t < len;
            sl[u] = k3_slot_raw<SLDS>(m, ok ? kofs + t : 0u);
            sv[u] = m.sum[ok ? lo + t : 0u];
        }
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const bool ok = t0 + u < len && sl[u] != (SLDS ? 0xFFFFu : PF_NONE);
            const uint32_t c = ok ? k3_cnt_get<C8>(m, sl[u]) : 0u;
            const uint32_t h0 = sv[u] & 0xffffu, h1 = sv[u] >> 16;
            q0[u] = div_u16_y((float)(c & 0xffffu), (float)h0, h0 ? __builtin_amdgcn_rcpf((float)h0) : 0.f);
            q1[u] = div_u16_y((float)(c >> 16), (float)h1, h1 ? __builtin_amdgcn_rcpf((float)h1) : 0.f);
        }
#pragma unroll
        for (int u = 0; u < 8; u++) {
            K3_FADD(s0, q0[u]);
            K3_FADD(s1, q1[u]);
        }
    }
}

// Pick without the sequential fold.  S_h = exact sum of a candidate's fp32
// terms: every nonzero term is >= 1/65535 (a multiple of 2^-39) and a row
// holds < 2^13 terms <= 1, so the fp64 sums of the fill and of the ds_add_f64
// reduction are exact in any order.  The reference's sequential fp32 sum s_h
// of L non-negative terms satisfies |s_h - S_h| <= gamma_{L-1} S_h (Higham,
// gamma_n = n u / (1 - n u), u = 2^-24), and diff = fl(|s0 - s1|) adds one
// rounding.  With those intervals the eligibility (diff >= 3 unless l0, l1 >=
// 3), the winner (largest diff, ties to the later candidate) and its tag (s0 >
// s1) are decided when no interval overlaps a competitor's or the threshold;
// otherwise pick stays 0 and the caller folds.
DEV void k3_pick_exact(const double *accd, uint32_t lane, uint32_t nc, uint32_t c_len, int l0, int l1,
                       uint32_t &pick, uint32_t &cw, uint32_t &tg) {
    const bool act = lane < nc;
    const double S0 = act ? accd[lane] : 0.0, S1 = act ? accd[64 + lane] : 0.0;
    // gamma_{L-1} <= (L-1) u (1 + 2^-10) for L < 2^13; margin 2^-9
    const double g = (double)(c_len > 1 ? c_len - 1 : 0) * (0x1p-24 * (1.0 + 0x1p-9));
    const double E = g * (S0 + S1);
    const double D = S0 > S1 ? S0 - S1 : S1 - S0;
    const bool sgn = D > E;                            // sign of s0 - s1 known
    const double dlo = sgn ? (D - E) * (1.0 - 0x1p-20) : 0.0;
    const double dhi = (D + E) * (1.0 + 0x1p-20) + 0x1p-60;
    const bool rel = l0 < 3 || l1 < 3;
    const bool el = act && (!rel || dlo >= 3.0);     // certainly eligible
    const bool un = !act || (rel && dhi < 3.0);      // certainly untagged (or no candidate)
    // all lane masks at once, off the dependent chain
    const uint64_t b_und = __ballot(!el && !un), b_el = __ballot(el);
    const uint64_t b_sgn = __ballot(sgn), b_gt = __ballot(S0 > S1);
    if (b_und) return;                                 // eligibility undecided
    if (b_el == 0) { pick = 2; return; }
    // conservative fp32 images of the interval ends (non-negative: bit order = value order)
    const float flo = el ? (float)(dlo * (1.0 - 0x1p-20)) : 0.f;
    const float fhi = (float)(dhi * (1.0 + 0x1p-20));
    const uint32_t key = el ? __float_as_uint(flo) + 1u : 0u;
    // candidates sit in lanes < nc: one DPP row holds them all when nc <= 16
    const uint32_t M = nc <= 16 ? (uint32_t)__builtin_amdgcn_readlane(
                                      (int)dpp_max_step(dpp_max_step(dpp_max_step(dpp_max_step(key, 0), 1), 2), 3), 0)
                                : wave_max_dpp(key);
    const float mf = __uint_as_float(M - 1u);
    // the lane holding the max has fhi >= flo = mf; decided iff it is the
    // only eligible lane whose interval reaches mf (a tie is never decided)
    const uint64_t b_hi = __ballot(el && fhi >= mf);
    if (__popcll(b_hi) != 1) return;
    const uint32_t cs = (uint32_t)__ffsll((unsigned long long)b_hi) - 1u;
    if (!((b_sgn >> cs) & 1ull)) return;
    pick = 1;
    cw = cs;
    tg = ((b_gt >> cs) & 1ull) ? 0u : 1u;
}

// Problem set-up shared by both greedy bodies: tables zeroed, per-read
// state, slot-list offsets (and the u16 LDS copy), reference reads seeding the
// counts (insert_ref_reads_methmer_counts, :3776-3810), the initial range,
// the T5 round trip and the untagged bitmask.
template <bool SLDS, int NT = PF_K3_THREADS, bool C8 = false>
DEV void k3_init(const pf_dev_batch &d, uint32_t w, uint32_t dir, uint32_t r0, uint32_t S, uint32_t R,
                 const K3Mem &m, K3Ctl &ctl, uint32_t *sh_scan, K3Stats &stx) {
    const uint32_t tid = threadIdx.x, lane = tid & 63, wid = uni(tid >> 6);
    const uint32_t ntot = uni(ctl.ntot);
    const int cov_rt = d.win_par[w * 4 + 1];
    const uint32_t s = d.win_start[w], e = d.win_end[w];
    const uint32_t nwords = (R + 63) >> 6;
    const uint64_t sb = d.win_site_off[w];
    const uint64_t kbase = d.mmr_off[2ull * r0];
    const uint32_t *kb = d.keys + kbase;
    uint32_t sum_mmr = 0, mx_mmr = 0;
    // ---- init tables and per-read state
    for (uint32_t j = tid; j < (C8 ? (ntot + 1) / 2 : ntot); j += NT) m.cnt[j] = 0;
    for (uint32_t j = tid; j < S; j += NT) m.sum[j] = 0;
    for (uint32_t i = tid; i < R; i += NT) {
        const uint32_t r = r0 + i;
        const uint32_t st = d.read_start[r], en = d.read_end[r];
        uint32_t f = 0;
        if (st <= s) {                                           // blockjoin.c:1127-1128
            f |= FLG_LEFT;
            if (en > s) f |= FLG_LEFT_STRICT;
        } else if (en >= e) {                                    // blockjoin.c:1134-1135
            f |= FLG_RIGHT;
            if (st < e) f |= FLG_RIGHT_STRICT;
        }
        m.flg[i] = (uint8_t)f;
        m.hp[i] = d.read_hp[r];
        m.aux[i] = 0;
        if (dir) m.ord[i] = (uint16_t)d.rev_ord[r];
        const uint64_t g = 2ull * r + dir;
        const uint32_t n_ = d.mmr_n[g], st_ = d.mmr_start[g];
        if (!m.mn) {
        } else if (m.m16) {
            static_cast<uint16_t *>(m.mn)[i] = (uint16_t)n_;
            static_cast<uint16_t *>(m.mst)[i] = (uint16_t)st_;
        } else {
            static_cast<uint32_t *>(m.mn)[i] = n_;
            static_cast<uint32_t *>(m.mst)[i] = st_;
        }
        sum_mmr += n_;
        mx_mmr = n_ > mx_mmr ? n_ : mx_mmr;
    }
    if (tid == 0) {
        const uint32_t *a = d.site_pos + sb;
        if (dir == 0) {
            ctl.min_i = 0;
            ctl.max_i = (uint32_t)ub_u32(a, 0, S, s);            // #sites <= ref_start (:3994-3998)
        } else {
            ctl.max_i = S - 1;
            ctl.min_i = (uint32_t)((int)ub_u32(a, 0, S, e) - 1); // may wrap to UINT32_MAX (:3999-4003)
        }
        ctl.i_last = dir == 0 ? 0 : (int)R - 1;
        ctl.failed = 0;
        ctl.done = 0;
        ctl.tab[0] = 0;
    }
    __syncthreads();
    // slot-list offsets: LDS copy (prefix sum of mn) or the HBM arena
    if (SLDS) {
        uint32_t carry = 0;
        for (uint32_t i0 = 0; i0 < R; i0 += NT) {
            const uint32_t i = i0 + tid;
            const uint32_t v = i < R ? k3_mn(m, i) : 0;
            uint32_t tot;
            const uint32_t ex = block_excl_scan<NT>(v, sh_scan, &tot);
            if (i < R) m.mo[i] = carry + ex;
            carry += tot;
        }
        __syncthreads();
        for (uint32_t i = wid; i < R; i += (NT / 64)) {
            const uint32_t g = 2 * (r0 + i) + dir;
            const uint32_t *src = kb + (d.mmr_off[g] - kbase);
            uint16_t *dst = m.sl16 + m.mo[i];
            const uint32_t n = k3_mn(m, i);
            for (uint32_t t = lane; t < n; t += 64) {
                const uint32_t v = src[t];
                dst[t] = v == PF_NONE ? (uint16_t)0xFFFFu : (uint16_t)v;
            }
        }
    } else if (m.mo) {
        for (uint32_t i = tid; i < R; i += NT)
            m.mo[i] = (uint32_t)(d.mmr_off[2ull * (r0 + i) + dir] - kbase);
    }
    __syncthreads();
    // ---- reference reads seed the counts (insert_ref_reads_methmer_counts, :3776-3810)
    const uint32_t refbit = dir == 0 ? FLG_LEFT : FLG_RIGHT;
    uint32_t ref_ins = 0;
    auto seed = [&](uint32_t i, uint32_t site, uint32_t slot) {
        const uint32_t hp = m.hp[i];
        if (site < S && slot != PF_NONE) {
            if (C8) atomicAdd(&m.cnt[slot >> 1], (hp ? 0x100u : 1u) << ((slot & 1u) * 16u));
            else atomicAdd(&m.cnt[slot], hp ? 0x10000u : 1u);
            atomicAdd(&m.sum[site], hp ? 0x10000u : 1u);
        }
    };
    auto is_ref = [&](uint32_t i) { return (m.flg[i] & refbit) && m.hp[i] <= 1; };
    if (SLDS) {
        for (uint32_t i = wid; i < R; i += (NT / 64)) {
            if (!is_ref(i)) continue;
            const uint32_t n = k3_mn(m, i), st = k3_mst(m, i), mo = m.mo[i];
            ref_ins += n;
            for (uint32_t t = lane; t < n; t += 64) seed(i, st + t, k3_slot<SLDS>(m, mo + t));
        }
    } else {
        // the slot ids from the rewritten key arena, eight reads' loads in flight
        k3_each_key<NT>(d, r0, R, dir, is_ref, [&](uint32_t i, uint32_t t, uint32_t site, uint64_t, uint32_t slot) {
            if (t == 0) ref_ins += d.mmr_n[2ull * (r0 + i) + dir];
            seed(i, site, slot);
        });
        ref_ins = (uint32_t)__builtin_amdgcn_readfirstlane((int)ref_ins);   // (lane 0 counted every read)
    }
    if (lane == 0 && ref_ins) atomicAdd((uint32_t *)&ctl.tab[0], ref_ins);
    if (sum_mmr) atomicAdd(&ctl.summ, sum_mmr);
    if (mx_mmr) atomicMax(&ctl.mxlen, mx_mmr);
    __syncthreads();
    if (wid == 0) k3_range_update(m.sum, S, cov_rt, ctl, lane);
    // ---- step 1.5 (:4010-4025): all reads unphased, ref reads restored through
    // the (readID<<2)|hp round trip (hp >= 4 lands on readID|(hp>>2)); the last
    // writer in reference order wins.
    for (uint32_t i = tid; i < R; i += NT) {
        if (m.flg[i] & refbit) {
            const uint32_t t = i | ((uint32_t)m.hp[i] >> 2);
            if (t < R) atomicMax(&m.aux[t], i + 1);
        }
    }
    __syncthreads();
    for (uint32_t i = tid; i < R; i += NT) {
        const uint32_t lw = m.aux[i];
        m.hp[i] = lw ? (uint8_t)(d.read_hp[r0 + lw - 1] & 3) : (uint8_t)2;
    }
    __syncthreads();
    // untagged bitmask in scan order (dir 0: read order, dir 1: revbuf order)
    for (uint32_t j = wid; j < nwords; j += (NT / 64)) {
        const uint32_t p = j * 64 + lane;
        bool u = false;
        if (p < R) {
            const uint32_t rd = dir ? m.ord[p] : p;
            const uint32_t h = m.hp[rd];
            u = h != 0 && h != 1;
        }
        const uint64_t b = __ballot(u);
        if (lane == 0) m.untag[j] = b;
    }
    stx.inserts = ctl.tab[0];
    __syncthreads();
}

// 2x2 table, per-read tags of direction 0 and the statistics (wave 0)
DEV void k3_finish(const pf_dev_batch &d, uint32_t w, uint32_t dir, uint32_t r0, uint32_t S, uint32_t R,
                   const K3Mem &m, const K3Ctl &ctl, const K3Stats &stx) {
    const uint32_t lane = threadIdx.x & 63;
    // ---- 2x2 table on the opposite side's strict reads (evaluate_separation, :3940-3956)
    int tab0 = 0, tab1 = 0, tab2 = 0, tab3 = 0;
    uint32_t nstrict = 0;
    const uint32_t strict = dir == 0 ? FLG_RIGHT_STRICT : FLG_LEFT_STRICT;
    for (uint32_t i = lane; i < R; i += 64) {
        if (m.flg[i] & strict) {
            nstrict++;
            const uint32_t ref = d.read_hp[r0 + i], q = m.hp[i];
            if (ref <= 1 && q <= 1) {
                const uint32_t k = ref * 2 + q;
                tab0 += k == 0; tab1 += k == 1; tab2 += k == 2; tab3 += k == 3;
            }
        }
        if (dir == 0) d.hp_fwd[r0 + i] = m.hp[i];
    }
    uint32_t tsum[5] = {(uint32_t)tab0, (uint32_t)tab1, (uint32_t)tab2, (uint32_t)tab3, nstrict};
#pragma unroll
    for (int k = 0; k < 5; k++) {
        uint32_t tot = 0;
        for (int bb = 0; bb < 16; bb++) tot += (uint32_t)__popcll(__ballot((tsum[k] >> bb) & 1)) << bb;
        tsum[k] = tot;
    }
    if (lane < 4) d.table[((uint64_t)w * 2 + dir) * 4 + lane] = (int32_t)tsum[lane];
    if (lane == 0) {
        unsigned long long *sp = d.stats + ((uint64_t)w * 2 + dir) * PF_NSTAT;
        sp[0] = stx.lookups; sp[1] = stx.inserts; sp[3] = stx.scanned;
        sp[2] = stx.iters | ((unsigned long long)ctl.path << 56);      // the slot-list source in the top byte
        sp[4] = ctl.summ; sp[5] = tsum[4]; sp[6] = R; sp[7] = S;
    }
}


// update_range (:3669-3704) on register copies of [min_i, max_i): both ends
// in one ballot, lanes 0-31 walk left from min_i, lanes 32-63 right from max_i
DEV void k3_range_regs(const K3Mem &m, uint32_t S, int cov_rt, uint32_t lane, uint32_t &umin, uint32_t &umax) {
    auto cov_ok = [&](int ii) -> bool {
        const uint32_t v = m.sum[ii];
        return (int)((v & 0xffffu) + (v >> 16)) >= cov_rt;
    };
    const int m0 = (int)umin, M0 = (int)umax;
    const bool left = lane < 32;
    const int i = left ? m0 - (int)lane : M0 + (int)(lane - 32);
    bool cvg = false;
    if (left ? (m0 >= 0 && i >= 0) : (M0 >= 0 && i < (int)S)) cvg = cov_ok(i);
    const uint64_t b = __ballot(cvg);
    const uint32_t bl = (uint32_t)b, br = (uint32_t)(b >> 32);
    int cl = bl == ~0u ? 32 : __ffs(~bl) - 1;
    int cr = br == ~0u ? 32 : __ffs(~br) - 1;
    if (cl == 32) {
        for (;;) {
            const int ii = m0 - cl - (int)lane;
            const uint64_t b2 = __ballot(ii >= 0 && cov_ok(ii));
            if (b2 == ~0ull) { cl += 64; continue; }
            cl += __ffsll((unsigned long long)~b2) - 1;
            break;
        }
    }
    if (cr == 32) {
        for (;;) {
            const int ii = M0 + cr + (int)lane;
            const uint64_t b2 = __ballot(ii < (int)S && cov_ok(ii));
            if (b2 == ~0ull) { cr += 64; continue; }
            cr += __ffsll((unsigned long long)~b2) - 1;
            break;
        }
    }
    if (m0 >= 0 && cl > 0) umin = (uint32_t)(m0 - cl + 1);
    if (M0 >= 0 && cr > 0) umax = (uint32_t)(M0 + cr - 1);
}

// Greedy loop of the main kernel (register candidate list, exact pick).  All
// four waves run the control flow of haplotag_region1 (:4032-4071)
// redundantly -- identical register copies of the candidate list, the queue
// and the range -- so nothing is published between waves; two barriers per
// iteration: after the term fill (B) and after the winner's insert (X).
//
// CACHE: the window's slot lists do not fit LDS, so instead of reading them
// from the HBM key arena in every fill and insert, the candidates' own lists
// live in an LDS cache of n_cand + 1 slots of CL entries (u16, CL = the
// longest list of the problem): a candidate's slot index rides in its lane
// (c_cs), free slots in a wave-uniform mask.  The read the list appends in
// this iteration is known at its top, so its list is loaded from HBM there
// and stored into the free slot before the closing barrier -- the load's
// latency hides behind the fill, the pick and the insert.  (The slots of a
// fresh candidate list are filled in one cooperative copy.)
template <bool SLDS, int NT = PF_K3_THREADS, bool C8 = false, bool CACHE = false, typename CD = K3Cand>
DEV void k3_greedy_slim(const pf_dev_batch &d, uint32_t w, uint32_t dir, uint32_t r0, uint32_t S, uint32_t R,
                        const K3Mem &m, K3Ctl &ctl, CD &cd, uint32_t *sh_scan, uint32_t *qb, uint32_t CL = 0) {
    const uint32_t tid = threadIdx.x, lane = tid & 63, wid = uni(tid >> 6);
    const int cov_rt = d.win_par[w * 4 + 1];
    const uint32_t NC = (uint32_t)d.win_par[w * 4 + 2];
    const uint32_t nwords = (R + 63) >> 6;
    K3Stats stx = {0, 0, 0, 0};
#ifdef PF_K3_PROFILE
    unsigned long long prof_acc[32] = {0};
    unsigned long long prof_last = k3_stamp_now();
    prof_acc[24] = k3_realtime();
#endif
    k3_init<SLDS && !CACHE, NT, C8>(d, w, dir, r0, S, R, m, ctl, sh_scan, stx);
    K3_STAMP(0);
    int il = uni_i(ctl.i_last);
    uint32_t failed = 0;
    uint32_t umin = uni(ctl.min_i), umax = uni(ctl.max_i);
    uint32_t nc = 0;
    uint32_t c_pos = 0, c_rd = 0, c_n = 0, c_st = 0, c_mo = 0;
    uint32_t c_cs = 0;                                   // CACHE: the candidate's cache slot
    uint64_t fmask = 0;                                  // CACHE: free cache slots (wave-uniform)
    const uint32_t NCS = NC + 1;
    uint32_t q_pos = 0, q_rd = 0, q_nn = 0, q_st = 0, q_mo = 0;
    uint32_t q_cnt = 0, q_head = 0;
    bool q_more = false;
    int q_cont = 0;
    uint32_t *qbuf = qb + 64 * wid;                      // per-wave queue scratch
    uint32_t lsum = 0;
    bool need_collect = true, have_win = false;
    // the range walk runs after the first insert (the initial range is not a
    // walk's result) and then only when the insert touched a site that ended
    // the last walk: umin - 1 or umin on the left (it stopped at an uncovered
    // site; coverage only grows, and only by inserts), umax or umax + 1 on the
    // right -- the walk's result is otherwise what it was
    bool rng_walk = true;
    // per-candidate totals, double-buffered by iteration parity: exact fp64
    // hap sums [2][128] and push/positive count pairs [2][64]
    double *accd = reinterpret_cast<double *>(cd.key);
    uint32_t *lcp = cd.pos;
    if (tid < 256) accd[tid] = 0.0;
    if (tid < 128) lcp[tid] = 0u;
    uint32_t par = 0;
    __syncthreads();
    for (;;) {
        // ---- range after the last insert (update_available_methmer_range)
        if (have_win && rng_walk) k3_range_regs(m, S, cov_rt, lane, umin, umax);
        K3_STAMP(4);
        // ---- candidate list: full collection from i_last (:4037-4051)
        if (need_collect) {
            bool done = false;
            for (;;) {
                if (dir == 0 ? il >= (int)R : il <= 0) { done = true; break; }
                q_cnt = k3_qbuild(m, nwords, dir == 0 ? il - 1 : il + 1, dir, lane, qbuf,
                                  q_pos, q_rd, q_nn, q_st, q_mo, q_more, q_cont);
                const uint32_t take = q_cnt < NC ? q_cnt : NC;
                c_pos = q_pos; c_rd = q_rd; c_n = q_nn; c_st = q_st; c_mo = q_mo;
                q_head = take;
                uint32_t found = take;
                while (found < NC && q_more) {
                    q_cnt = k3_qbuild(m, nwords, q_cont, dir, lane, qbuf, q_pos, q_rd, q_nn, q_st, q_mo,
                                      q_more, q_cont);
                    q_head = 0;
                    while (found < NC && q_head < q_cnt) {
                        const uint32_t a0 = rdl(q_pos, q_head), a1 = rdl(q_rd, q_head), a2 = rdl(q_nn, q_head);
                        const uint32_t a3 = rdl(q_st, q_head), a4 = rdl(q_mo, q_head);
                        if (lane == found) { c_pos = a0; c_rd = a1; c_n = a2; c_st = a3; c_mo = a4; }
                        found++;
                        q_head++;
                    }
                }
                if (found == 0) {
                    stx.scanned += dir == 0 ? (uint32_t)((int)R - il) : (uint32_t)(il + 1);
                    if (++failed > 10) { done = true; break; }
                    il += dir == 0 ? (int)NC : -(int)NC;
                    continue;
                }
                nc = found;
                break;
            }
            if (done) break;
            need_collect = false;
            if (CACHE) {
                // a fresh list: candidate c in cache slot c; every list copied
                // by the workgroup (wave v takes candidates v, v + NT/64, ...)
                c_cs = lane;
                fmask = (NCS >= 64 ? ~0ull : ((1ull << NCS) - 1ull)) & (nc >= 64 ? 0ull : ~((1ull << nc) - 1ull));
                for (uint32_t c = wid; c < nc; c += NT / 64) {
                    const uint32_t n_ = rdl(c_n, c), ko = rdl(c_mo, c);
                    uint16_t *dst = m.sl16 + c * CL;
                    for (uint32_t t = lane; t < n_; t += 64) {
                        const uint32_t v = m.kb[ko + t];
                        dst[t] = v == PF_NONE ? (uint16_t)0xFFFFu : (uint16_t)v;
                    }
                }
                __syncthreads();
            }
        }
        K3_STAMP(5);
        // ---- the next untagged read after the list, for this iteration's append
        int qn = -1;
        uint32_t q_rd1 = 0, q_n1 = 0, q_st1 = 0, q_mo1 = 0;
        if (nc == NC) {
            if (q_head == q_cnt && q_more) {
                q_cnt = k3_qbuild(m, nwords, q_cont, dir, lane, qbuf, q_pos, q_rd, q_nn, q_st, q_mo,
                                  q_more, q_cont);
                q_head = 0;
            }
            if (q_head < q_cnt) {
                qn = (int)rdl(q_pos, q_head);
                q_rd1 = rdl(q_rd, q_head); q_n1 = rdl(q_nn, q_head);
                q_st1 = rdl(q_st, q_head); q_mo1 = rdl(q_mo, q_head);
                q_head++;
            }
        }
        K3_STAMP(6);
        // CACHE: the appended read's list, loaded now, stored before (X)
        uint32_t pf0 = PF_NONE, pf1 = PF_NONE, s_sp = 0;
        if (CACHE && qn >= 0) {
            s_sp = (uint32_t)__ffsll((unsigned long long)fmask) - 1u;
            if (tid < q_n1) pf0 = m.kb[q_mo1 + tid];
            if (tid + NT < q_n1) pf1 = m.kb[q_mo1 + tid + NT];
        }
        // ---- lookup spans: sites in [min_i, max_i) (query_counts_of_mmrs, :3500-3501)
        uint32_t c_len, c_lo, c_kofs;
        {
            const uint32_t lo = c_st > umin ? c_st : umin;
            const uint32_t hi0 = c_st + c_n;
            const uint32_t hi = hi0 < umax ? hi0 : umax;
            c_len = lane < nc && hi > lo && umin != 0xFFFFFFFFu ? hi - lo : 0;
            c_lo = lo;
            c_kofs = (CACHE ? c_cs * CL : c_mo) + (c_len ? lo - c_st : 0);
        }
        lsum += c_len;
        if (nc >= NC) {
            const uint32_t pl = rdl(c_pos, NC - 1);
            stx.scanned += dir == 0 ? pl - (uint32_t)il + 1 : (uint32_t)il - pl + 1;
        } else stx.scanned += dir == 0 ? (uint32_t)((int)R - il) : (uint32_t)(il + 1);
        stx.iters++;
        K3_STAMP(2);
        // ---- term fill: G = 64/ncp lanes of each wave per candidate, the waves
        // interleaved along the methmers; exact fp64 sums and the integer
        // push/positive counts per lane, reduced with LDS atomics
        {
            const uint32_t ncp = next_pow2(nc);
            const uint32_t lgn = 31 - __clz(ncp);
            const uint32_t G = 64u >> lgn;
            const uint32_t fc = lane & (ncp - 1), fj = lane >> lgn;
            const uint32_t J = wid * G + fj, GS = (NT / 64) * G;
            const uint32_t f_lo = (uint32_t)__shfl((int)c_lo, (int)fc, 64);
            const uint32_t f_len = (uint32_t)__shfl((int)c_len, (int)fc, 64);
            const uint32_t f_kofs = (uint32_t)__shfl((int)c_kofs, (int)fc, 64);
            double x0 = 0.0, x1 = 0.0;
            const uint32_t lcode = k3_fill_sums<SLDS, C8>(m, f_lo, f_kofs, J, f_len, GS, x0, x1);
            if (fc < nc) {
                atomicAdd(&lcp[par * 64 + fc], lcode);
                atomicAdd(&accd[par * 128 + fc], x0);
                atomicAdd(&accd[par * 128 + 64 + fc], x1);
            }
            // the other parity's totals start from zero next iteration (its last
            // readers finished before barrier X)
            if (wid == 0) {
                accd[(par ^ 1) * 128 + lane] = 0.0;
                accd[(par ^ 1) * 128 + 64 + lane] = 0.0;
                lcp[(par ^ 1) * 64 + lane] = 0u;
            }
        }
        K3_STAMP(10);
        __syncthreads();                                           // (B)
        K3_STAMP(3);
        // ---- pick (every wave alike): use_mmr_count_predict_tag_for_one_read
        // (:3637-3655) and predict_tags_of_reads (:3729-3766), from the exact
        // sums with rounding-error intervals, else the sequential fp32 fold
        uint32_t pick = 0, cw = 0, tg = 0;
        bool folded = false;
        {
            const uint32_t lcode = lcp[par * 64 + lane];
            const int l0 = (int)(lcode & 0xffffu), l1 = (int)(lcode >> 16);
            k3_pick_exact(accd + par * 128, lane, nc, c_len, l0, l1, pick, cw, tg);
            K3_COUNT(14, pick == 0 ? 1u : 0u);
            if (pick == 0) {
                folded = true;
                float s0 = 0.f, s1 = 0.f;
                if (lane < nc) k3_fold_direct<SLDS, C8>(m, c_lo, c_kofs, c_len, s0, s1);
                const float diff = s0 > s1 ? s0 - s1 : s1 - s0;
                const bool elig = lane < nc && !(diff < 3.f && (l0 < 3 || l1 < 3));
                const uint32_t hkey = elig ? __float_as_uint(diff) + 1u : 0u;
                const uint32_t hmax = wave_max_dpp(hkey);
                if (hmax == 0) pick = 2;
                else {
                    pick = 1;
                    cw = 63u - (uint32_t)__clzll((long long)__ballot(hkey == hmax));
                    tg = rdl(s0 > s1 ? 0u : 1u, cw);
                }
            }
        }
        par ^= 1;
        K3_STAMP(19);
        if (pick == 2) {
            // nothing could be tagged (:4064-4069): move i_last, rescan
            if (++failed > 10) break;
            il += dir == 0 ? (int)NC : -(int)NC;
            need_collect = true;
            have_win = false;
            __syncthreads();                                       // (X): totals reused
            continue;
        }
        // ---- the winner: tag, list minus the winner plus the queued read
        const uint32_t rd = rdl(c_rd, cw), n = rdl(c_n, cw), st = rdl(c_st, cw);
        const uint32_t mo = CACHE ? rdl(c_cs, cw) * CL : rdl(c_mo, cw);
        const uint32_t pw = rdl(c_pos, cw);
        stx.inserts += n;
        if (wid == 0 && lane == 0) {
            m.hp[rd] = (uint8_t)tg;
            m.untag[pw >> 6] &= ~(1ull << (pw & 63));
        }
        failed = 0;
        if (CACHE) fmask |= 1ull << (mo / CL);           // the winner's slot: free after this insert
        {
            // the list closes over the winner: lanes >= cw take their upper
            // neighbour's entry (DPP, no LDS round trip)
            const uint32_t a0 = wave_shl1(c_pos), a1 = wave_shl1(c_rd), a2 = wave_shl1(c_n), a3 = wave_shl1(c_st);
            const uint32_t a4 = CACHE ? 0u : wave_shl1(c_mo);
            const uint32_t a5 = CACHE ? wave_shl1(c_cs) : 0u;
            if (lane >= cw) { c_pos = a0; c_rd = a1; c_n = a2; c_st = a3; c_mo = a4; c_cs = a5; }
        }
        // touched sites [st, st + n) against the last walk's end sites
        {
            const uint32_t te = st + n;
            auto hit = [&](uint32_t a) { return a != 0xFFFFFFFFu && a >= st && a < te; };
            rng_walk = !have_win || hit(umin) || hit(umin - 1u) || hit(umax) || hit(umax + 1u);
        }
        uint32_t ncn = nc - 1;
        if (qn >= 0) {
            if (lane == ncn) { c_pos = (uint32_t)qn; c_rd = q_rd1; c_n = q_n1; c_st = q_st1; c_mo = q_mo1; c_cs = s_sp; }
            if (CACHE) fmask &= ~(1ull << s_sp);
            ncn++;
        }
        nc = ncn;
        if (nc == 0) need_collect = true;     // an empty batch: the failure path of the reference (:4046-4051)
        K3_STAMP(20);
        // ---- insert_mmr_counts of the winner, the whole workgroup (after every
        // wave's fold, if the pick needed one, has read the tables)
        if (folded) __syncthreads();
        k3_insert_all<SLDS, NT, C8>(m, S, n, st, mo, tg);
        if (CACHE && qn >= 0) {
            // the appended read's list into its (free until now) cache slot
            uint16_t *dst = m.sl16 + s_sp * CL;
            if (tid < q_n1) dst[tid] = pf0 == PF_NONE ? (uint16_t)0xFFFFu : (uint16_t)pf0;
            if (tid + NT < q_n1) dst[tid + NT] = pf1 == PF_NONE ? (uint16_t)0xFFFFu : (uint16_t)pf1;
        }
        have_win = true;
        K3_STAMP(21);
        __syncthreads();                                           // (X)
        K3_STAMP(8);
    }
    {
        uint32_t tot = 0;
#pragma unroll
        for (int bb = 0; bb < 32; bb++) tot += (uint32_t)__popcll(__ballot((lsum >> bb) & 1)) << bb;
        stx.lookups += tot;
    }
    if (wid != 0) return;
    k3_finish(d, w, dir, r0, S, R, m, ctl, stx);
#ifdef PF_K3_PROFILE
    if (lane == 0) {
        unsigned long long *pp = d.prof + ((uint64_t)w * 2 + dir) * 32;
        prof_acc[29] = ctl.path;
        prof_acc[25] = k3_realtime();
        prof_acc[26] = ctl.t_run;
        prof_acc[30] = ctl.ntot;
        prof_acc[31] = ctl.need;
        prof_acc[27] = ctl.cacheb;
        for (int i = 0; i < 32; i++) pp[i] = prof_acc[i];
    }
#endif
}

template <bool SLDS, bool FULL>
DEV void k3_greedy_body(const pf_dev_batch &d, uint32_t w, uint32_t dir, uint32_t r0, uint32_t S,
                        uint32_t R, const K3Mem &m, K3Ctl &ctl, K3Cand &cd, uint32_t *sh_scan) {
    const uint32_t tid = threadIdx.x, lane = tid & 63, wid = uni(tid >> 6);
    const int cov_rt = d.win_par[w * 4 + 1];
    const uint32_t NC = (uint32_t)d.win_par[w * 4 + 2];
    const uint32_t nwords = (R + 63) >> 6;
    K3Stats stx = {0, 0, 0, 0};
#ifdef PF_K3_PROFILE
    unsigned long long prof_acc[32] = {0};
    unsigned long long prof_last = k3_stamp_now();
#endif

    k3_init<SLDS>(d, w, dir, r0, S, R, m, ctl, sh_scan, stx);

    // ---- step 2: greedy extension, one read per iteration (:4032-4071), run by
    // wavefront 0 alone (no workgroup barriers on the serial chain).  The
    // candidate list is kept incrementally: after a tag it loses the winner and
    // gains the next untagged read after its last entry -- exactly the
    // reference's rescan from i_last, since tags never revert.
    K3_STAMP(0);
    const uint32_t rec_cap = PF_K3_WAVES * m.rcw;
    if (!FULL || NC <= 64) {
    // ---- register-resident variant (n_cand <= 64): lane c holds candidate c
    // (scan position, read, methmer count/start/slot offset and the range-
    // clipped lookup span); control state lives in scalars.
    int il = uni_i(ctl.i_last);
    uint32_t failed = 0;
    uint32_t umin = uni(ctl.min_i), umax = uni(ctl.max_i);
    uint32_t nc = 0;
    uint32_t c_pos = 0, c_rd = 0, c_n = 0, c_st = 0, c_mo = 0;
    uint32_t c_lo = 0, c_len = 0, c_kofs = 0;
    uint32_t q_pos = 0, q_rd = 0, q_nn = 0, q_st = 0, q_mo = 0;
    uint32_t q_cnt = 0, q_head = 0;
    bool q_more = false;
    int q_cont = 0;
    uint32_t *qbuf = cd.read;
    uint32_t lsum = 0;
    // one chunk per iteration when a row can hold the longest methmer list
    // of the window, zero-padded to 32 terms (pitch = 4 mod 32 for the banks)
    // (the register variant keeps no push codes, so the whole 12-byte record
    // region holds float2 terms)
    // exact sums need rows of < 2^13 terms (k3_pick_exact); longer lists
    // take the chunked record-row path with the sequential fold
    // (the main kernel only takes windows of < 8192 sites: mxlen <= S)
    const bool exact_path = !FULL || (uni(ctl.mxlen) < 8192u && d.k3_mode != 2u);
    K3_COUNT(15, exact_path ? 1 : 0);
    bool need_collect = true, stop = false;
    int qn = -1;
    uint32_t q_rd1 = 0, q_n1 = 0, q_st1 = 0, q_mo1 = 0;
    uint32_t p_n = 0, p_st = 0, p_mo = 0, p_tg = 0;           // pending insert (wavefront 0)
    uint32_t *lcp = reinterpret_cast<uint32_t *>(cd.key);    // per-wave push/positive partials
    double *accd = reinterpret_cast<double *>(cd.key + 128);  // exact hap sums per candidate
    K3_STAMP(1);
    for (;;) {
    // wavefront 0: candidate list upkeep, then publish the lookup spans
    if (wid == 0) {
        K3_STAMP(28);
        if (!stop && need_collect) {
            bool done = false;
            for (;;) {
                if (dir == 0 ? il >= (int)R : il <= 0) { done = true; break; }
                K3_COUNT(25, 1);
                q_cnt = k3_qbuild(m, nwords, dir == 0 ? il - 1 : il + 1, dir, lane, qbuf,
                                  q_pos, q_rd, q_nn, q_st, q_mo, q_more, q_cont);
                const uint32_t take = q_cnt < NC ? q_cnt : NC;
                c_pos = q_pos; c_rd = q_rd; c_n = q_nn; c_st = q_st; c_mo = q_mo;
                q_head = take;
                uint32_t found = take;
                while (found < NC && q_more) {
                    // fewer than n_cand untagged reads in the first 4096 scan
                    // positions: continue the scan entry by entry
                    K3_COUNT(26, 1);
                    q_cnt = k3_qbuild(m, nwords, q_cont, dir, lane, qbuf, q_pos, q_rd, q_nn, q_st, q_mo,
                                      q_more, q_cont);
                    q_head = 0;
                    while (found < NC && q_head < q_cnt) {
                        const uint32_t a0 = rdl(q_pos, q_head), a1 = rdl(q_rd, q_head), a2 = rdl(q_nn, q_head);
                        const uint32_t a3 = rdl(q_st, q_head), a4 = rdl(q_mo, q_head);
                        if (lane == found) { c_pos = a0; c_rd = a1; c_n = a2; c_st = a3; c_mo = a4; }
                        found++;
                        q_head++;
                    }
                }
                if (found == 0) {
                    stx.scanned += dir == 0 ? (uint32_t)((int)R - il) : (uint32_t)(il + 1);
                    if (++failed > 10) { done = true; break; }
                    il += dir == 0 ? (int)NC : -(int)NC;
                    continue;
                }
                nc = found;
                break;
            }
            if (done) stop = true;
        }
        K3_STAMP(16);
        if (!stop && need_collect) {
            need_collect = false;
            // span of query_counts_of_mmrs: sites in [min_i, max_i) (:3500-3501)
            {
                const uint64_t lo = c_st > umin ? c_st : umin;
                const uint64_t hi0 = (uint64_t)c_st + c_n;
                const uint64_t hi = hi0 < umax ? hi0 : umax;
                c_len = lane < nc && hi > lo ? (uint32_t)(hi - lo) : 0;
                c_lo = (uint32_t)lo;
                c_kofs = c_mo + (c_len ? (uint32_t)(lo - c_st) : 0);
                lsum += c_len;
            }
            if (nc >= NC) {
                const uint32_t pl = rdl(c_pos, NC - 1);
                stx.scanned += dir == 0 ? pl - (uint32_t)il + 1 : (uint32_t)il - pl + 1;
            } else stx.scanned += dir == 0 ? (uint32_t)((int)R - il) : (uint32_t)(il + 1);
            stx.iters++;
        }
        // the next untagged read after the last candidate, from the queue
        qn = -1;
        if (!stop && nc == NC) {
            if (q_head == q_cnt && q_more) {
                K3_COUNT(27, 1);
                q_cnt = k3_qbuild(m, nwords, q_cont, dir, lane, qbuf, q_pos, q_rd, q_nn, q_st, q_mo,
                                  q_more, q_cont);
                q_head = 0;
            }
            if (q_head < q_cnt) {
                qn = (int)rdl(q_pos, q_head);
                q_rd1 = rdl(q_rd, q_head); q_n1 = rdl(q_nn, q_head);
                q_st1 = rdl(q_st, q_head); q_mo1 = rdl(q_mo, q_head);
                q_head++;
            }
        }
        K3_STAMP(17);
        const uint32_t lmax0 = stop || exact_path ? 0u : wave_max_dpp(c_len);
        cd.site0[lane] = c_lo;
        cd.len[lane] = c_len;
        cd.kofs[lane] = c_kofs;
        accd[lane] = 0.0;
        accd[64 + lane] = 0.0;
        lcp[lane] = 0u;
        if (lane == 0) {
            ctl.done = stop ? 1u : 0u; ctl.nc = nc; ctl.L = lmax0;
            ctl.ins_n = p_n; ctl.ins_st = p_st; ctl.ins_mo = p_mo; ctl.ins_tg = p_tg;
        }
        p_n = 0;
        K3_STAMP(2);
    }
    __syncthreads();                                           // (A)
    if (uni(ctl.done)) break;
    K3_STAMP(8);
    // the previous winner's insert, deferred to here so that the whole
    // workgroup shares it; wavefront 0 has already applied it virtually to
    // its range update
    if (const uint32_t ins_n = uni(ctl.ins_n)) {
        k3_insert_all<SLDS>(m, S, ins_n, uni(ctl.ins_st), uni(ctl.ins_mo), uni(ctl.ins_tg));
        __syncthreads();                                       // (A2)
    }
    {
        // ---- fill, all four waves: the value pair of every (candidate,
        // methmer) lookup into per-candidate record rows; G = 64/ncp lanes of
        // each wave per candidate, the waves interleaved along the methmers.
        // The push/positive counts (integer, order-free) are summed in
        // registers, reduced across lanes and waves.
        const uint32_t ncs = uni(ctl.nc);
        const uint32_t ncp = next_pow2(ncs);
        const uint32_t lgn = 31 - __clz(ncp);
        const uint32_t G = 64u >> lgn;
        const uint32_t fc = lane & (ncp - 1), fj = lane >> lgn;
        const uint32_t J = wid * G + fj, GS = PF_K3_WAVES * G;
        const uint32_t f_lo = cd.site0[fc], f_len = cd.len[fc], f_kofs = cd.kofs[fc];
        float s0 = 0.f, s1 = 0.f;
        uint32_t lcode = 0;
        bool exact_ok = false;
        if (!FULL || exact_path) {
            K3_COUNT(13, ncs);
            K3_STAMP(9);
            double x0 = 0.0, x1 = 0.0;
            lcode = k3_fill_sums<SLDS>(m, f_lo, f_kofs, J, f_len, GS, x0, x1);
            K3_STAMP(10);
            // every lane adds into its candidate's totals: integer counts and
            // exact fp64 sums are order-free, and the G same-address lanes of
            // one ds_add cost G LDS cycles, far below a DPP reduction chain
            if (fc < ncs) {
                atomicAdd(&lcp[fc], lcode);
                atomicAdd(&accd[fc], x0);
                atomicAdd(&accd[64 + fc], x1);
            }
            K3_STAMP(11);
            __syncthreads();                                   // (B)
            K3_STAMP(3);
            exact_ok = true;
            K3_STAMP(4);
        } else {
        if constexpr (FULL) {
        const uint32_t lmax = uni(ctl.L);
        // row pitch P (float2) = 4 mod 32: the fold's 16-byte row reads of up
        // to 8 candidates and the fill's 8-lane row segments spread over the
        // LDS banks; chunks of CHK (8 | CHK) terms
        const uint32_t cap = rec_cap >> lgn;
        const uint32_t P = cap >= 36 ? ((cap - 4) & ~31u) + 4 : (cap & ~7u);
        const uint32_t CHK = P & ~7u;
        // rows are zero-padded to a multiple of 8 terms so that the fold reads
        // whole 8-term blocks (+0.0f leaves a non-negative sum unchanged)
        const uint32_t lmaxp = (lmax + 7) & ~7u;
        K3_COUNT(12, lmax);
        K3_COUNT(13, ncs);
        const uint32_t f_lenp = (f_len + 7) & ~7u;
        for (uint32_t t0 = 0; t0 < lmaxp; t0 += CHK) {
            const uint32_t tlim = lmaxp - t0 < CHK ? lmaxp - t0 : CHK;  // wave-uniform, 8 | tlim
            const uint32_t tend = f_len < t0 + tlim ? f_len : t0 + tlim;
            const uint32_t tpad = f_lenp < t0 + tlim ? f_lenp : t0 + tlim;
            double x0 = 0.0, x1 = 0.0;
            lcode += k3_fill_rows<SLDS>(m, f_lo, f_kofs, t0 + J, tend, tpad, GS, m.recv + fc * P - t0, x0, x1);
            const bool last_chunk = t0 + CHK >= lmaxp;
            if (last_chunk) {
                const uint32_t lc = wave_group_sum(lcode, ncp);
                if (lane < ncp) lcp[wid * 64 + lane] = lc;
            }
            __syncthreads();                                   // (B)
            K3_STAMP(3);
            // the reference's sequential float sums (:3619-3636), one candidate
            // per lane of wavefront 0, 8-term blocks double-buffered
            if (wid == 0 && lane < ncs) {
                const uint32_t lp = (c_len + 7) & ~7u;
                const uint32_t nt = lp > t0 ? (lp - t0 < tlim ? lp - t0 : tlim) : 0;
                const float4 *rv4 = reinterpret_cast<const float4 *>(m.recv + lane * P);
                const uint32_t nb = nt >> 3;
                float4 A[4], B[4];
                if (nb) {
#pragma unroll
                    for (int u = 0; u < 4; u++) A[u] = rv4[u];
                }
                for (uint32_t bk = 0; bk < nb; bk += 2) {
                    if (bk + 1 < nb) {
#pragma unroll
                        for (int u = 0; u < 4; u++) B[u] = rv4[((bk + 1) << 2) + u];
                    }
#pragma unroll
                    for (int u = 0; u < 4; u++) { s0 += A[u].x; s1 += A[u].y; s0 += A[u].z; s1 += A[u].w; }
                    if (bk + 2 < nb) {
#pragma unroll
                        for (int u = 0; u < 4; u++) A[u] = rv4[((bk + 2) << 2) + u];
                    }
                    if (bk + 1 < nb) {
#pragma unroll
                        for (int u = 0; u < 4; u++) { s0 += B[u].x; s1 += B[u].y; s0 += B[u].z; s1 += B[u].w; }
                    }
                }
            }
            if (!last_chunk) __syncthreads();                  // rows reused by the next chunk
            K3_STAMP(4);
        }
        }
        }
        if (wid != 0) continue;
        lcode = exact_ok ? lcp[lane] : lcp[lane] + lcp[64 + lane] + lcp[128 + lane] + lcp[192 + lane];
        const int l0 = (int)(lcode & 0xffffu), l1 = (int)(lcode >> 16);
        K3_STAMP(18);
        // use_mmr_count_predict_tag_for_one_read (:3637-3655) and the pick of
        // predict_tags_of_reads (:3729-3766): max score, ties to the later
        // candidate (stable merge sort walked from the end).  First from the
        // exact sums with rounding-error intervals; the sequential fp32 fold
        // only when the intervals cannot decide.
        uint32_t pick = 0;                         // 0 undecided, 1 winner, 2 none
        uint32_t cw = 0, tg = 0;
        if (exact_ok && d.k3_mode == 0u) k3_pick_exact(accd, lane, nc, c_len, l0, l1, pick, cw, tg);
        K3_STAMP(19);
        K3_COUNT(14, pick == 0 ? 1u : 0u);
        if (pick == 0) {
            if (exact_ok && lane < nc) k3_fold_direct<SLDS>(m, c_lo, c_kofs, c_len, s0, s1);
            const float diff = s0 > s1 ? s0 - s1 : s1 - s0;
            const bool elig = lane < nc && !(diff < 3.f && (l0 < 3 || l1 < 3));
            const uint32_t hkey = elig ? __float_as_uint(diff) + 1u : 0u;
            const uint32_t hmax = wave_max_dpp(hkey);
            if (hmax == 0) pick = 2;
            else {
                pick = 1;
                cw = 63u - (uint32_t)__clzll((long long)__ballot(hkey == hmax));
                tg = rdl(s0 > s1 ? 0u : 1u, cw);
            }
        }
        K3_STAMP(5);
        if (pick == 2) {
            // nothing could be tagged (:4064-4069): move i_last, rescan
            K3_COUNT(24, 1);
            K3_STAMP(6);
            if (++failed > 10) stop = true;
            else {
                il += dir == 0 ? (int)NC : -(int)NC;
                need_collect = true;
            }
            K3_STAMP(7);
            continue;
        }
        K3_MARK("tail_begin");
        const uint32_t rd = rdl(c_rd, cw), n = rdl(c_n, cw), st = rdl(c_st, cw), mo = rdl(c_mo, cw);
        const uint32_t pw = rdl(c_pos, cw);
        K3_STAMP(6);
        stx.inserts += n;
        // the insert itself runs on the whole workgroup after the next barrier (A)
        p_n = n; p_st = st; p_mo = mo; p_tg = tg;
        K3_STAMP(20);
        if (lane == 0) {
            m.hp[rd] = (uint8_t)tg;
            m.untag[pw >> 6] &= ~(1ull << (pw & 63));
        }
        failed = 0;
        K3_STAMP(21);
        // candidate list minus the winner, plus the prefetched next read
        {
            const int src = (int)lane + 1;
            const uint32_t a0 = (uint32_t)__shfl((int)c_pos, src, 64), a1 = (uint32_t)__shfl((int)c_rd, src, 64);
            const uint32_t a2 = (uint32_t)__shfl((int)c_n, src, 64), a3 = (uint32_t)__shfl((int)c_st, src, 64);
            const uint32_t a4 = (uint32_t)__shfl((int)c_mo, src, 64);
            if (lane >= cw) { c_pos = a0; c_rd = a1; c_n = a2; c_st = a3; c_mo = a4; }
        }
        uint32_t ncn = nc - 1;
        if (qn >= 0) {
            if (lane == ncn) { c_pos = (uint32_t)qn; c_rd = q_rd1; c_n = q_n1; c_st = q_st1; c_mo = q_mo1; }
            ncn++;
        }
        nc = ncn;
        wave_sync();
        K3_STAMP(22);
        // update_range (:3669-3704): both ends in one ballot, lanes 0-31 walk
        // left from min_i, lanes 32-63 right from max_i
        {
            const int m0 = (int)umin, M0 = (int)umax;
            const bool left = lane < 32;
            const int i = left ? m0 - (int)lane : M0 + (int)(lane - 32);
            // coverage after the pending insert of the winner (+1 at its sites)
            auto cov_at = [&](int ii) -> int {
                const uint32_t v = m.sum[ii];
                const uint32_t t = (uint32_t)ii - st;
                int c = (int)((v & 0xffffu) + (v >> 16));
                if (t < n && k3_slot_raw<SLDS>(m, mo + t) != (SLDS ? 0xFFFFu : PF_NONE)) c++;
                return c;
            };
            bool cvg = false;
            if (left ? (m0 >= 0 && i >= 0) : (M0 >= 0 && i < (int)S)) cvg = cov_at(i) >= cov_rt;
            const uint64_t b = __ballot(cvg);
            const uint32_t bl = (uint32_t)b, br = (uint32_t)(b >> 32);
            int cl = bl == ~0u ? 32 : __ffs(~bl) - 1;
            int cr = br == ~0u ? 32 : __ffs(~br) - 1;
            if (cl == 32) {
                for (;;) {
                    const int ii = m0 - cl - (int)lane;
                    bool c2 = false;
                    if (ii >= 0) c2 = cov_at(ii) >= cov_rt;
                    const uint64_t b2 = __ballot(c2);
                    if (b2 == ~0ull) { cl += 64; continue; }
                    cl += __ffsll((unsigned long long)~b2) - 1;
                    break;
                }
            }
            if (cr == 32) {
                for (;;) {
                    const int ii = M0 + cr + (int)lane;
                    bool c2 = false;
                    if (ii < (int)S) c2 = cov_at(ii) >= cov_rt;
                    const uint64_t b2 = __ballot(c2);
                    if (b2 == ~0ull) { cr += 64; continue; }
                    cr += __ffsll((unsigned long long)~b2) - 1;
                    break;
                }
            }
            if (m0 >= 0 && cl > 0) umin = (uint32_t)(m0 - cl + 1);
            if (M0 >= 0 && cr > 0) umax = (uint32_t)(M0 + cr - 1);
        }
        K3_STAMP(23);
        if (nc == 0) {
            // an empty batch: the failure path of the reference (:4046-4051)
            need_collect = true;
        } else {
            const uint64_t lo = c_st > umin ? c_st : umin;
            const uint64_t hi0 = (uint64_t)c_st + c_n;
            const uint64_t hi = hi0 < umax ? hi0 : umax;
            c_len = lane < nc && hi > lo ? (uint32_t)(hi - lo) : 0;
            c_lo = (uint32_t)lo;
            c_kofs = c_mo + (c_len ? (uint32_t)(lo - c_st) : 0);
            lsum += c_len;
            if (nc >= NC) {
                const uint32_t pl = rdl(c_pos, NC - 1);
                stx.scanned += dir == 0 ? pl - (uint32_t)il + 1 : (uint32_t)il - pl + 1;
            } else stx.scanned += dir == 0 ? (uint32_t)((int)R - il) : (uint32_t)(il + 1);
            stx.iters++;
        }
        K3_MARK("tail_end");
        K3_STAMP(7);
    }
    }
    if (wid != 0) return;
    {
        uint32_t tot = 0;
#pragma unroll
        for (int bb = 0; bb < 32; bb++) tot += (uint32_t)__popcll(__ballot((lsum >> bb) & 1)) << bb;
        stx.lookups += tot;
    }
    } else if constexpr (FULL) {
    // ---- general variant (n_cand > 64): candidate list in LDS, wavefront 0
    if (wid != 0) return;
    k3_collect(m, R, dir, NC, lane, ctl, cd, stx);
    if (!ctl.done) {
        k3_cand_fields(m, ctl.nc, dir, lane, ctl, cd, stx);
        k3_scanned(ctl, cd, R, dir, NC, stx);
    }
    K3_STAMP(1);
    while (!ctl.done) {
        const uint32_t nc = ctl.nc;
        const uint32_t ng = (nc + 63) >> 6;     // candidate groups of 64 lanes
        uint32_t lmax = 0;
        for (uint32_t g = 0; g < ng; g++) {
            const uint32_t c = (g << 6) + lane;
            const uint32_t l = c < nc ? cd.len[c] : 0u;
            lmax = l > lmax ? l : lmax;
        }
        lmax = wave_max_u32(lmax);
        // rows of `ch` records per candidate (power of two), chunked along t
        uint32_t ch = next_pow2(lmax ? lmax : 1);
        while (ch > 1 && ch * nc > rec_cap) ch >>= 1;
        const uint32_t lgc = 31 - __clz(ch);
        float s0[4] = {0.f, 0.f, 0.f, 0.f}, s1[4] = {0.f, 0.f, 0.f, 0.f};
        uint32_t lcode[4] = {0u, 0u, 0u, 0u};
        for (uint32_t t0 = 0; t0 < lmax; t0 += ch) {
            const uint32_t nrec = nc << lgc;
            // records: value pair + push/positive code of (candidate c, methmer t0+tt)
#pragma unroll 2
            for (uint32_t idx = lane; idx < nrec; idx += 64) {
                const uint32_t c = idx >> lgc, tt = idx & (ch - 1), t = t0 + tt;
                float v0 = 0.f, v1 = 0.f;
                uint32_t code = 0;
                const uint32_t len = cd.len[c];
                if (t < len) {
                    const uint32_t site = cd.site0[c] + t;
                    const uint32_t sv = m.sum[site];
                    const uint32_t slot = k3_slot<SLDS>(m, cd.kofs[c] + t);
                    const uint32_t cv = slot != PF_NONE ? m.cnt[slot] : 0u;
                    if (cv != 0) {                               // key present at this site
                        const uint32_t h0 = sv & 0xffffu, h1 = sv >> 16;
                        if (h0) {
                            v0 = (float)(cv & 0xffffu) / (float)h0;
                            code += 1u + (v0 > 0.f ? 1u : 0u);   // pushed + positive (:3619-3624)
                        }
                        if (h1) {
                            v1 = (float)(cv >> 16) / (float)h1;
                            code += (1u + (v1 > 0.f ? 1u : 0u)) << 16;
                        }
                    }
                }
                m.recv[idx] = make_float2(v0, v1);
                m.recc[idx] = code;
            }
            wave_sync_mem();
            K3_STAMP(3);
            // the reference's sequential float sums (:3619-3636), one candidate
            // per lane; absent terms are +0.0f and leave the sum unchanged
            const uint32_t n_t = lmax - t0 < ch ? lmax - t0 : ch;
#pragma unroll
            for (uint32_t g = 0; g < 4; g++) {
                const uint32_t c = (g << 6) + lane;
                if (g < ng && c < nc) {
                    const float2 *rv = m.recv + (c << lgc);
                    const uint32_t *rc = m.recc + (c << lgc);
                    float a0 = s0[g], a1 = s1[g];
                    uint32_t lc = lcode[g];
                    uint32_t t = 0;
                    for (; t + 8 <= n_t; t += 8) {
                        float2 v[8];
                        uint32_t cc[8];
#pragma unroll
                        for (int u = 0; u < 8; u++) { v[u] = rv[t + u]; cc[u] = rc[t + u]; }
#pragma unroll
                        for (int u = 0; u < 8; u++) { a0 += v[u].x; a1 += v[u].y; lc += cc[u]; }
                    }
                    for (; t < n_t; t++) {
                        const float2 v = rv[t];
                        a0 += v.x;
                        a1 += v.y;
                        lc += rc[t];
                    }
                    s0[g] = a0; s1[g] = a1; lcode[g] = lc;
                }
            }
            wave_sync_mem();
            K3_STAMP(4);
        }
        // use_mmr_count_predict_tag_for_one_read (:3637-3655); selection key
        // (score, index): max wins, ties go to the later candidate = the stable
        // merge sort + walk from the end of predict_tags_of_reads (:3729-3766)
#pragma unroll
        for (uint32_t g = 0; g < 4; g++) {
            const uint32_t c = (g << 6) + lane;
            if (g < ng && c < nc) {
                const float diff = s0[g] > s1[g] ? s0[g] - s1[g] : s1[g] - s0[g];
                const int l0 = (int)(lcode[g] & 0xffffu), l1 = (int)(lcode[g] >> 16);
                const bool untagged = diff < 3.f && (l0 < 3 || l1 < 3);
                cd.tag[c] = s0[g] > s1[g] ? 0 : 1;
                cd.key[c] = untagged ? 0ull : (((unsigned long long)__float_as_uint(diff) << 32) | (c + 1));
            }
        }
        wave_sync();
        K3_STAMP(5);
        unsigned long long b = 0;
        {
            uint32_t c = 0;
            for (; c + 4 <= nc; c += 4) {
                const unsigned long long k0 = cd.key[c], k1 = cd.key[c + 1], k2 = cd.key[c + 2], k3 = cd.key[c + 3];
                const unsigned long long m01 = k0 > k1 ? k0 : k1, m23 = k2 > k3 ? k2 : k3;
                const unsigned long long mm = m01 > m23 ? m01 : m23;
                b = mm > b ? mm : b;
            }
            for (; c < nc; c++) { const unsigned long long k = cd.key[c]; b = k > b ? k : b; }
        }
        K3_STAMP(6);
        if (b == 0) {
            // nothing could be tagged (:4064-4069): move i_last, rescan
            if (lane == 0) {
                ctl.failed = ctl.failed + 1;
                if (ctl.failed > 10) ctl.done = 1;
                else ctl.i_last += dir == 0 ? (int)NC : -(int)NC;
            }
            wave_sync();
            if (!ctl.done) {
                k3_collect(m, R, dir, NC, lane, ctl, cd, stx);
                if (!ctl.done) {
                    k3_cand_fields(m, ctl.nc, dir, lane, ctl, cd, stx);
                    k3_scanned(ctl, cd, R, dir, NC, stx);
                }
            }
        } else {
            const uint32_t cw = (uint32_t)(b & 0xffffffffu) - 1;
            const uint32_t rd = cd.read[cw];
            const uint32_t tg = cd.tag[cw];
            const uint32_t pw = cd.pos[cw];
            const uint32_t n = k3_mn(m, rd), st = k3_mst(m, rd), mo = k3_mo(m, rd);
            const uint32_t inc = tg ? 0x10000u : 1u;
            stx.inserts += n;
            // the sites of one read are distinct: plain read-modify-write
            for (uint32_t t = lane; t < n; t += 64) {
                const uint32_t site = st + t;
                const uint32_t slot = k3_slot<SLDS>(m, mo + t);
                if (site < S && slot != PF_NONE) {
                    m.cnt[slot] += inc;
                    m.sum[site] += inc;
                }
            }
            // candidate list minus the winner, plus the next untagged read after
            // the last one when the list was full
            const uint32_t last = cd.pos[nc - 1];
            uint32_t pos_c = 0, read_c = 0;
            for (uint32_t c0 = 0; c0 < nc; c0 += 64) {
                const uint32_t c = c0 + lane;
                if (c >= cw && c + 1 < nc) { pos_c = cd.pos[c + 1]; read_c = cd.read[c + 1]; }
                wave_sync();
                if (c >= cw && c + 1 < nc) { cd.pos[c] = pos_c; cd.read[c] = read_c; }
                wave_sync();
            }
            if (lane == 0) {
                ctl.failed = 0;
                m.hp[rd] = (uint8_t)tg;
                m.untag[pw >> 6] &= ~(1ull << (pw & 63));
            }
            wave_sync();
            k3_range_update(m.sum, S, cov_rt, ctl, lane);
            uint32_t ncn = nc - 1;
            if (nc == NC) {
                const int q = k3_next_untag(m.untag, nwords, (int)last, dir, lane);
                if (q >= 0) {
                    if (lane == 0) {
                        cd.pos[ncn] = (uint32_t)q;
                        cd.read[ncn] = dir ? m.ord[q] : (uint32_t)q;
                    }
                    ncn++;
                }
            }
            if (lane == 0) ctl.nc = ncn;
            wave_sync();
            if (ncn == 0) {
                // an empty batch: the failure path of the reference (:4046-4051)
                k3_collect(m, R, dir, NC, lane, ctl, cd, stx);
                if (!ctl.done) {
                    k3_cand_fields(m, ctl.nc, dir, lane, ctl, cd, stx);
                    k3_scanned(ctl, cd, R, dir, NC, stx);
                }
            } else {
                k3_cand_fields(m, ncn, dir, lane, ctl, cd, stx);
                k3_scanned(ctl, cd, R, dir, NC, stx);
            }
        }
        K3_STAMP(7);
    }
    }

    k3_finish(d, w, dir, r0, S, R, m, ctl, stx);
    if (lane == 0) {
#ifdef PF_K3_PROFILE
        unsigned long long *pp = d.prof + ((uint64_t)w * 2 + dir) * 32;
        for (int i = 0; i < 32; i++) pp[i] = prof_acc[i];
#endif
    }
}

// hand a problem the main kernel does not take to pf_k3_fallback
DEV void k3_defer(const pf_dev_batch &d, uint32_t prob) {
    if (threadIdx.x == 0) d.k3_fb_list[atomicAdd(d.k3_fb_ctr, 1u)] = prob;
}

// One greedy problem (window w, direction dir) on one workgroup.  FULL =
// false is the main kernel's slim build: slot dictionary and lists in LDS,
// n_cand <= 64 (register candidate list), < 8192 sites (exact-interval pick
// only); anything else is deferred to the FULL build.
template <bool FULL, int NT = PF_K3_THREADS, typename CD = K3Cand>
DEV void k3_run(const pf_dev_batch &d, uint32_t prob, uint8_t *smem, K3Ctl &ctl, CD &cd, uint32_t *sh_scan,
                const uint32_t lds, uint32_t *qb = nullptr) {
    // qb: per-wave queue scratch of the slim loop, 64 entries per wave; the
    // kernels that pass none (fallback, heavy: 256 threads) use cd.read
    static_assert(sizeof(cd.read) / sizeof(cd.read[0]) >= (size_t)NT, "cd.read holds 64 entries per wave");
    const uint32_t tid = threadIdx.x;
    const uint32_t w = prob >> 1, dir = prob & 1;
    const uint32_t S = d.win_S[w];
    if (S == 0) {
        if (tid < 4) d.table[((uint64_t)w * 2 + dir) * 4 + tid] = 0;
        if (tid < PF_NSTAT) d.stats[((uint64_t)w * 2 + dir) * PF_NSTAT + tid] = 0;
        return;
    }
    const uint32_t R = d.win_nreads[w];
    const uint32_t r0 = d.win_read_off[w];
    const uint32_t MW = (uint32_t)d.mw;
    const uint64_t kbase = d.mmr_off[2ull * r0];
#ifdef PF_K3_PROFILE
    if (tid == 0) ctl.t_run = k3_realtime();
#endif

    // ---- P1: slot dictionary (built by pf_k3_kdict when d.kdict)
    const bool kd = d.kdict != 0u;
    const uint64_t need1 = kd ? 0ull : align16(8ull * S * MW) + 4ull * S;
    const bool p1_lds = need1 <= lds;
    // the slim loop: register candidate list (n_cand <= 64), exact-interval
    // pick (< 8192 sites), dictionary in LDS
    const bool slim_ok = p1_lds && d.win_par[w * 4 + 2] <= 64 && S < 8192u && d.k3_mode == 0u;
    if (!FULL && !slim_ok) {
        k3_defer(d, prob);
        return;
    }
    if (tid == 0) {
        ctl.fail = 0;
        ctl.summ = 0;
        ctl.nstrict = 0;
        ctl.mxlen = 0;
        if (!p1_lds) {
            const unsigned long long o = atomicAdd(d.scr_ctr, (unsigned long long)align16(need1));
            if (o + need1 > d.scr_cap) { ctl.fail = 1; atomicOr(d.status, PF_ST_SCR_OVF); }
            ctl.scr = o;
        }
    }
    __syncthreads();
    if (uni(ctl.fail)) return;
    uint64_t *masks;
    uint32_t *mbase;
    if (!FULL || p1_lds) {
        masks = reinterpret_cast<uint64_t *>(smem);
        mbase = reinterpret_cast<uint32_t *>(smem + align16(8ull * S * MW));
    } else {
        uint8_t *g = d.scr + ctl.scr;
        masks = reinterpret_cast<uint64_t *>(g);
        mbase = reinterpret_cast<uint32_t *>(g + align16(8ull * S * MW));
    }
    if (!kd) k3_dict<NT>(d, r0, R, S, dir, masks, mbase, sh_scan, ctl);
    const uint32_t ntot = kd ? uni(d.k3_ntot[prob]) : uni(ctl.ntot);
    if (kd && ntot == PF_NONE) return;               // pf_k3_kdict ran out of scratch: the host re-runs
    if (kd && tid == 0) ctl.ntot = ntot;             // the greedy loop's init reads it (k3_init; a barrier follows)
    // sum of methmers over the window's reads (slot-list size) and the longest list
    uint32_t summ = 0, lmx = 0;
    for (uint32_t i = tid; i < R; i += NT) {
        const uint32_t n_ = d.mmr_n[2ull * (r0 + i) + dir];
        summ += n_;
        lmx = n_ > lmx ? n_ : lmx;
    }
    if (lmx) atomicMax(&ctl.mxlen, lmx);
    uint32_t summ_tot;
    block_excl_scan<NT>(summ, sh_scan, &summ_tot);

    // ---- P2: greedy.  Prefer everything in LDS (u16 slot lists), then LDS
    // tables with slot lists read from the HBM arena, then all in HBM.  The
    // slim loop keeps no record rows (rcw = 0): either kernel runs it when the
    // problem fits this launch's LDS; the fallback kernel's general loop
    // takes the rest.
    uint64_t off[K3_NOFF];
    const bool slots_ok = ntot < 0xFFFFu;
    // u8 count pairs when no site is covered by more than 255 reads' methmer
    // spans [st, st+n) (every count is bounded by that coverage): the deepest
    // coverage from a difference array in the LDS left after the dictionary
    bool c8 = false;
    if (slim_ok && (!FULL || p1_lds) && need1 + align16(4ull * (S + 1)) <= lds) {
        uint32_t *cov = reinterpret_cast<uint32_t *>(smem + need1);
        for (uint32_t j = tid; j <= S; j += NT) cov[j] = 0;
        if (tid == 0) ctl.cmax = 0;
        __syncthreads();
        for (uint32_t i = tid; i < R; i += NT) {
            const uint64_t g = 2ull * (r0 + i) + dir;
            const uint32_t n = d.mmr_n[g], st = d.mmr_start[g];
            if (n && st < S) {
                atomicAdd(&cov[st], 1u);
                atomicAdd(&cov[st + n < S ? st + n : S], 0xFFFFFFFFu);
            }
        }
        __syncthreads();
        const uint32_t per = (S + NT) / NT;                 // S + 1 entries, contiguous per thread
        const uint32_t j0 = tid * per, j1 = min(j0 + per, S + 1);
        uint32_t part = 0;
        for (uint32_t j = j0; j < j1; j++) part += cov[j];
        uint32_t tot;
        uint32_t run = block_excl_scan<NT>(part, sh_scan, &tot), mx = 0;
        for (uint32_t j = j0; j < j1; j++) { run += cov[j]; mx = run > mx ? run : mx; }
        if (mx) atomicMax(&ctl.cmax, mx);
        __syncthreads();
        c8 = uni(ctl.cmax) < 256u;
    }
    const uint64_t slim_s = k3_layout(S, ntot, R, dir, summ_tot, true, 0, off, c8);
    const uint64_t slim_n = k3_layout(S, ntot, R, dir, summ_tot, false, 0, off, c8);
    // the candidate slot-list cache (k3_greedy_slim CACHE) when the window's
    // lists do not fit: n_cand + 1 slots of the longest list, u16 entries
    const uint32_t CL = (uni(ctl.mxlen) + 1u) & ~1u;
    const uint32_t NCc = (uint32_t)d.win_par[w * 4 + 2];
    const bool cache_ok = slim_ok && slots_ok && NCc <= 63u && CL > 0 && CL <= 2u * NT && (d.k3_cache & 1u) != 0u;
    const bool lists_ok = slots_ok && d.k3_cache < 2u;         // (tests force the cache / the HBM lists)
    // no per-read slot-list offsets (the cache copies from HBM), and the
    // per-read side arrays and the T5 scratch of k3_init in HBM (k3_side_mem)
    const uint64_t cache_b = 2ull * (NCc + 1) * CL;
    const uint64_t slim_cn = k3_layout(S, ntot, R, dir, summ_tot, false, 0, off, c8, false, 0, false, false);
    const uint64_t slim_c = align16(slim_cn) + cache_b;
    const bool slim_fit0 = slim_ok && ((lists_ok && slim_s <= lds) || (cache_ok && slim_c <= lds) || slim_n <= lds);
    // path 6 (round 5): a candidate-cache problem past the budget (the main
    // kernel's four-per-CU budget leaves the largest windows of a batch a few
    // KB short) keeps its count table -- the bulk of its need -- in HBM
    // scratch: it runs at once, heaviest first, instead of in the fallback
    // kernel after the main one.  u8 count pairs only (c8); PF_K3_GCNT=force
    // takes it for every such problem (tests)
    const uint64_t cnt_b = align16(2ull * ntot);
    const uint64_t slim_g =
        align16(k3_layout(S, ntot, R, dir, summ_tot, false, 0, off, c8, false, 0, false, false, false)) + cache_b;
    const bool gcnt = !FULL && cache_ok && c8 && slim_g <= lds && (!slim_fit0 || d.k3_gcnt != 0u);
    const bool slim_fit = slim_fit0 || gcnt;
    if (!FULL && !slim_fit) {
        k3_defer(d, prob);           // keys still intact: the fallback rebuilds the dictionary
        return;
    }
    if (gcnt) {
        __syncthreads();
        if (tid == 0) {
            const unsigned long long o = atomicAdd(d.scr_ctr, (unsigned long long)cnt_b);
            ctl.fail = 0;
            if (o + cnt_b > d.scr_cap) { ctl.fail = 1; atomicOr(d.status, PF_ST_SCR_OVF); }   // the host grows it, re-runs
            ctl.scr = o;
        }
        __syncthreads();
        if (uni(ctl.fail)) return;
    }
    if (!kd) k3_dict_rewrite<NT>(d, r0, R, S, dir, masks, mbase);
    const uint32_t *kb = d.keys + kbase;
    if (tid == 0) {
        // 1 slot lists in LDS, 2 the candidate cache, 3 slot lists in HBM (slim loop); 4 the general body;
        // reported with the problem's stats (pf_batch_k3_paths)
        ctl.path = !slim_fit ? 4u : gcnt ? 6u : (lists_ok && slim_s <= lds) ? 1u : (cache_ok && slim_c <= lds) ? 2u : 3u;
#ifdef PF_K3_PROFILE
        ctl.need = (uint32_t)(cache_ok ? slim_c : ctl.path == 1 ? slim_s : slim_n);   // the cache layout's need (path 6: with its counts)
        ctl.cacheb = (uint32_t)cache_b;
#endif
    }
    if (slim_fit) {
        K3Mem m;
        uint32_t *qq = qb ? qb : cd.read;
        if constexpr (!FULL) {
            if (gcnt) {
                (void)k3_layout(S, ntot, R, dir, summ_tot, false, 0, off, c8, false, 0, false, false, false);
                k3_mem(smem, off, 0, false, kb, m, false, S, false);
                k3_side_mem(d, r0, dir, m);
                m.cnt = reinterpret_cast<uint32_t *>(d.scr + ctl.scr);
                m.gmo = d.mmr_off + 2ull * r0 + dir;
                m.gmn = d.mmr_n + 2ull * r0 + dir;
                m.gmst = d.mmr_start + 2ull * r0 + dir;
                m.kbase = kbase;
                m.sl16 = reinterpret_cast<uint16_t *>(smem + (slim_g - cache_b));
                k3_greedy_slim<true, NT, true, true, CD>(d, w, dir, r0, S, R, m, ctl, cd, sh_scan, qq, CL);
                return;
            }
        }
        if (lists_ok && slim_s <= lds) {
            (void)k3_layout(S, ntot, R, dir, summ_tot, true, 0, off, c8);
            k3_mem(smem, off, 0, true, kb, m, true, S);
            if (c8) k3_greedy_slim<true, NT, true, false, CD>(d, w, dir, r0, S, R, m, ctl, cd, sh_scan, qq);
            else k3_greedy_slim<true, NT, false, false, CD>(d, w, dir, r0, S, R, m, ctl, cd, sh_scan, qq);
        } else if (cache_ok && slim_c <= lds) {
            (void)k3_layout(S, ntot, R, dir, summ_tot, false, 0, off, c8, false, 0, false, false);
            k3_mem(smem, off, 0, false, kb, m, false, S, false);
            k3_side_mem(d, r0, dir, m);
            m.gmo = d.mmr_off + 2ull * r0 + dir;
            m.gmn = d.mmr_n + 2ull * r0 + dir;
            m.gmst = d.mmr_start + 2ull * r0 + dir;
            m.kbase = kbase;
            m.sl16 = reinterpret_cast<uint16_t *>(smem + align16(slim_cn));
            if (c8) k3_greedy_slim<true, NT, true, true, CD>(d, w, dir, r0, S, R, m, ctl, cd, sh_scan, qq, CL);
            else k3_greedy_slim<true, NT, false, true, CD>(d, w, dir, r0, S, R, m, ctl, cd, sh_scan, qq, CL);
        } else {
            (void)k3_layout(S, ntot, R, dir, summ_tot, false, 0, off, c8);
            k3_mem(smem, off, 0, false, kb, m, true, S);
            if (c8) k3_greedy_slim<false, NT, true, false, CD>(d, w, dir, r0, S, R, m, ctl, cd, sh_scan, qq);
            else k3_greedy_slim<false, NT, false, false, CD>(d, w, dir, r0, S, R, m, ctl, cd, sh_scan, qq);
        }
        return;
    }
    if constexpr (FULL) {
        const uint32_t rcw_min = 256, rcw_max = 1024;
        const uint64_t need_s = k3_layout(S, ntot, R, dir, summ_tot, true, rcw_min, off);
        const uint64_t need_n = k3_layout(S, ntot, R, dir, summ_tot, false, rcw_min, off);
        if (slots_ok && need_s <= lds) {
            (void)k3_layout(S, ntot, R, dir, summ_tot, true, rcw_min, off);
            uint32_t rcw = (uint32_t)((lds - off[11]) / (12ull * PF_K3_WAVES));
            rcw = rcw > rcw_max ? rcw_max : rcw;
            (void)k3_layout(S, ntot, R, dir, summ_tot, true, rcw, off);
            K3Mem m;
            k3_mem(smem, off, rcw, true, kb, m, true, S);
            k3_greedy_body<true, true>(d, w, dir, r0, S, R, m, ctl, cd, sh_scan);
        } else if (need_n <= lds) {
            (void)k3_layout(S, ntot, R, dir, summ_tot, false, rcw_min, off);
            uint32_t rcw = (uint32_t)((lds - off[11]) / (12ull * PF_K3_WAVES));
            rcw = rcw > rcw_max ? rcw_max : rcw;
            (void)k3_layout(S, ntot, R, dir, summ_tot, false, rcw, off);
            K3Mem m;
            k3_mem(smem, off, rcw, false, kb, m, true, S);
            k3_greedy_body<false, true>(d, w, dir, r0, S, R, m, ctl, cd, sh_scan);
        } else {
            const uint32_t rcw = rcw_min;
            const uint64_t need2 = align16(k3_layout(S, ntot, R, dir, summ_tot, false, rcw, off));
            __syncthreads();
            if (tid == 0) {
                const unsigned long long o = atomicAdd(d.scr_ctr, (unsigned long long)need2);
                ctl.fail = 0;
                if (o + need2 > d.scr_cap) { ctl.fail = 1; atomicOr(d.status, PF_ST_SCR_OVF); }
                ctl.scr = o;
            }
            __syncthreads();
            if (uni(ctl.fail)) return;
            K3Mem m;
            k3_mem(d.scr + ctl.scr, off, rcw, false, kb, m, true, S);
            k3_greedy_body<false, true>(d, w, dir, r0, S, R, m, ctl, cd, sh_scan);
        }
    }
}

// Main greedy kernel: every problem, heaviest first (k3_order); the slim build.
// PF_K3S_THREADS threads per problem.  The greedy loop's control runs
// redundantly in every wave, so more waves shorten only the parallel parts of
// an iteration (the term fill, the winner's insert); 512 threads were measured
// in round 3 (50 kb batch 5.25 -> 4.96 ms, gap mix 7.3 -> 10.3 ms: register-
// limited to two problems per CU; with 6 waves per SIMD forced, spills, 5.48 /
// 11.2 ms) and 256 kept.
// Persistent: the grid is what the device holds at once (pf_api.hip
// k3_resident); each workgroup takes the next problem of k3_order (heaviest
// first) from the counter d.k3_next until k3_n are taken -- list scheduling,
// so a slot freed on any CU takes the next problem at once.  Every workgroup
// leaves when the counter passes k3_n.
// At most 128 VGPRs (four waves per SIMD): four problems per CU when the LDS
// budget allows it (pf_api.hip k3_lds_four; round 4's 132 VGPRs held three).
__global__ __launch_bounds__(PF_K3S_THREADS) __attribute__((amdgpu_waves_per_eu(4))) void pf_k3_greedy(pf_dev_batch d) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    __shared__ K3Ctl ctl;
    __shared__ K3CandSlim cd;
    __shared__ uint32_t sh_scan[PF_K3S_THREADS / 64 + 1];
    __shared__ uint32_t s_rank;
    static_assert(PF_K3S_THREADS <= PF_MAX_NCAND, "cd.read holds the per-wave queue scratch");
    for (;;) {
        if (threadIdx.x == 0) s_rank = atomicAdd(d.k3_next, 1u);
        __syncthreads();
        const uint32_t rank = uni(s_rank);
        if (rank >= d.k3_n) break;
        k3_run<false, PF_K3S_THREADS>(d, d.k3_order[rank], smem, ctl, cd, sh_scan, d.lds_bytes);
        __syncthreads();                                 // every thread has read s_rank and left the problem
    }
}

// The heavy problems (k3_order's first n, pf_api.hip): the slim build with
// the larger budget d.lds_heavy, launched on a second stream beside the main
// kernel; a problem that does not fit is deferred to pf_k3_fallback like the
// main kernel's.
// Round 6: PF_K3H_THREADS (512) threads per problem -- a heavy problem's
// chain is its window's critical path, and the term fill, the winner's insert
// and the range walk split over twice the waves (the pick runs in every wave).
__global__ __launch_bounds__(PF_K3H_THREADS) __attribute__((amdgpu_waves_per_eu(4))) void pf_k3_heavy(pf_dev_batch d) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    __shared__ K3Ctl ctl;
    __shared__ K3CandSlimT<PF_K3H_THREADS> cd;
    __shared__ uint32_t sh_scan[PF_K3H_THREADS / 64 + 1];
    k3_run<false, PF_K3H_THREADS>(d, d.k3_order[blockIdx.x], smem, ctl, cd, sh_scan, d.lds_heavy);
}

// Problems the main kernel deferred (dictionary or tables beyond the LDS
// budget, n_cand > 64, >= 8192 sites, test overrides): all variants.
__global__ __launch_bounds__(PF_K3_THREADS) void pf_k3_fallback(pf_dev_batch d) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    __shared__ K3Ctl ctl;
    __shared__ K3Cand cd;
    __shared__ uint32_t sh_scan[PF_K3_WAVES + 1];
    const uint32_t n = *d.k3_fb_ctr;
    for (uint32_t i = blockIdx.x; i < n; i += gridDim.x) {
        k3_run<true>(d, d.k3_fb_list[i], smem, ctl, cd, sh_scan, d.lds_fb);
        __syncthreads();
    }
}

// ========================================================================
// K3W: one wavefront per (window, direction) -- the main greedy kernel
// ========================================================================
// The greedy loop of haplotag_region1 (:4032-4071) is a serial chain of one
// tagged read per iteration; its per-iteration work (n_cand candidates x
// their in-range methmers, ~10^3 lookups at 60x) fits one wavefront.  One
// wave per problem needs no workgroup barriers, no LDS reductions and no
// redundant control across waves, and a compact LDS image lets 6-8 problems
// share a CU, so the whole batch is resident at once.  LDS per problem:
//   srec  16 B per site: (h0, h1, 1/h0, 1/h1) as floats, exact hap totals
//         (they replace the u32 sum array: the range update reads h0 + h1)
//   cnt   per slot, hap0 | hap1 packed: u8 pairs when no site is covered by
//         more than 255 reads' methmers (no count can exceed that; checked
//         per problem), else u16 pairs
//   hp, flg 1 B per read, untag 1 bit per read
// Slot lists stay in the HBM key arena (rewritten in place into slot ids by
// the dictionary build); per-read methmer fields and the dir-1 scan order
// are read from HBM when a read joins the candidate queue.
#define K3W_NOFF 7
#define K3W_LSMAX 512u            // longest methmer list the candidate cache holds (8 regs per lane)

template <bool C8>
DEV uint64_t k3w_layout(uint32_t S, uint32_t ntot, uint32_t R, uint32_t nc, uint32_t ls, uint64_t off[K3W_NOFF]) {
    const uint32_t nwords = (R + 63) >> 6;
    off[0] = 0;                                                   // srec  16*S
    off[1] = align16(16ull * S);                                  // cnt   ntot * (2 | 4)
    off[2] = align16(off[1] + (C8 ? 2ull : 4ull) * ntot);         // cache nc * ls u16 slot ids
    off[3] = align16(off[2] + 2ull * nc * ls);                    // hp    R
    off[4] = align16(off[3] + R);                                 // flg   R
    off[5] = align16(off[4] + R);                                 // untag nwords*8
    off[6] = off[5] + 8ull * nwords;
    return off[6];
}

struct K3WMem {
    float4 *srec;
    uint8_t *cnt;
    uint16_t *cc;                // candidate slot-list cache: nc lists of ls u16 slot ids (0xFFFF: none)
    uint32_t ls;
    uint8_t *hp, *flg;
    uint64_t *untag;
    const uint32_t *kb;          // slot lists (HBM key arena, window base)
    uint64_t kbase;
};

DEV uint32_t k3w_slot(const K3WMem &m, uint32_t i) {
    const uint32_t v = m.cc[i];
    return v == 0xFFFFu ? PF_NONE : v;
}

// one read's slot list (n entries at arena offset mo) into cache list cs
DEV void k3w_cache_load(const K3WMem &m, uint32_t cs, uint32_t mo, uint32_t n, uint32_t lane) {
    uint16_t *dst = m.cc + cs * m.ls;
    for (uint32_t t = lane; t < n; t += 64) {
        const uint32_t v = m.kb[mo + t];
        dst[t] = v == PF_NONE ? (uint16_t)0xFFFFu : (uint16_t)v;
    }
}

// count pair of slot s: (hap0, hap1)
template <bool C8>
DEV uint32_t k3w_cnt(const K3WMem &m, uint32_t s) {
    if (C8) return reinterpret_cast<const uint16_t *>(m.cnt)[s];
    return reinterpret_cast<const uint32_t *>(m.cnt)[s];
}
template <bool C8> DEV uint32_t k3w_c0(uint32_t c) { return C8 ? (c & 0xffu) : (c & 0xffffu); }
template <bool C8> DEV uint32_t k3w_c1(uint32_t c) { return C8 ? (c >> 8) : (c >> 16); }

// per-read methmer fields of window-local read rd, direction dir, from HBM
DEV void k3w_read_fields(const pf_dev_batch &d, uint32_t r0, uint32_t rd, uint32_t dir, uint64_t kbase,
                         uint32_t &n, uint32_t &st, uint32_t &mo) {
    const uint64_t g = 2ull * (r0 + rd) + dir;
    n = d.mmr_n[g];
    st = d.mmr_start[g];
    mo = (uint32_t)(d.mmr_off[g] - kbase);
}

// k3_qbuild with the per-read fields from HBM
DEV uint32_t k3w_qbuild(const pf_dev_batch &d, const K3WMem &m, uint32_t r0, uint32_t nwords, int p, uint32_t dir,
                        uint32_t lane, uint32_t *qbuf, uint32_t &q_pos, uint32_t &q_rd, uint32_t &q_n,
                        uint32_t &q_st, uint32_t &q_mo, bool &more, int &cont) {
    uint64_t bits = 0;
    int wi, w0;
    bool more_words;
    if (dir == 0) {
        const int q = p + 1;
        if (q >= (int)(nwords * 64)) { more = false; return 0; }
        w0 = q >> 6;
        wi = w0 + (int)lane;
        if (wi < (int)nwords) {
            bits = m.untag[wi];
            if (wi == w0) bits &= ~0ull << (q & 63);
        }
        more_words = w0 + 64 < (int)nwords;
    } else {
        const int q = p - 1;
        if (q < 0) { more = false; return 0; }
        w0 = q >> 6;
        wi = w0 - (int)lane;
        if (wi >= 0) {
            bits = m.untag[wi];
            if (wi == w0) {
                const uint32_t b = (uint32_t)q & 63;
                bits &= b == 63 ? ~0ull : ((1ull << (b + 1)) - 1ull);
            }
        }
        more_words = w0 - 64 >= 0;
    }
    const uint32_t pc = (uint32_t)__popcll(bits);
    const uint32_t incl = wave_incl_scan_dpp(pc);
    const uint32_t tot = rdl(incl, 63);
    uint32_t k = incl - pc;
    while (bits != 0 && k < 64) {
        const int b = dir == 0 ? __ffsll((unsigned long long)bits) - 1 : 63 - __clzll((long long)bits);
        qbuf[k++] = (uint32_t)(wi * 64 + b);
        bits &= ~(1ull << b);
    }
    wave_sync();
    const uint32_t cnt = tot < 64 ? tot : 64;
    if (lane < cnt) {
        q_pos = qbuf[lane];
        q_rd = dir ? d.rev_ord[r0 + q_pos] : q_pos;
        k3w_read_fields(d, r0, q_rd, dir, m.kbase, q_n, q_st, q_mo);
    }
    if (tot > 64) cont = (int)qbuf[63];
    else cont = dir == 0 ? (w0 + 64) * 64 - 1 : (w0 - 63) * 64;
    more = tot > 64 || more_words;
    wave_sync();
    return cnt;
}

// update_available_methmer_range (:3669-3691) from the exact float totals
DEV void k3w_range(const K3WMem &m, uint32_t S, int cov_rt, uint32_t lane, uint32_t &umin, uint32_t &umax) {
    auto cov_ok = [&](int ii) -> bool {
        const float4 r = m.srec[ii];
        return (int)((uint32_t)r.x + (uint32_t)r.y) >= cov_rt;
    };
    const int m0 = (int)umin, M0 = (int)umax;
    const bool left = lane < 32;
    const int i = left ? m0 - (int)lane : M0 + (int)(lane - 32);
    bool cvg = false;
    if (left ? (m0 >= 0 && i >= 0) : (M0 >= 0 && i < (int)S)) cvg = cov_ok(i);
    const uint64_t b = __ballot(cvg);
    const uint32_t bl = (uint32_t)b, br = (uint32_t)(b >> 32);
    int cl = bl == ~0u ? 32 : __ffs(~bl) - 1;
    int cr = br == ~0u ? 32 : __ffs(~br) - 1;
    if (cl == 32) {
        for (;;) {
            const int ii = m0 - cl - (int)lane;
            const uint64_t b2 = __ballot(ii >= 0 && cov_ok(ii));
            if (b2 == ~0ull) { cl += 64; continue; }
            cl += __ffsll((unsigned long long)~b2) - 1;
            break;
        }
    }
    if (cr == 32) {
        for (;;) {
            const int ii = M0 + cr + (int)lane;
            const uint64_t b2 = __ballot(ii < (int)S && cov_ok(ii));
            if (b2 == ~0ull) { cr += 64; continue; }
            cr += __ffsll((unsigned long long)~b2) - 1;
            break;
        }
    }
    if (m0 >= 0 && cl > 0) umin = (uint32_t)(m0 - cl + 1);
    if (M0 >= 0 && cr > 0) umax = (uint32_t)(M0 + cr - 1);
}

// fp32 partial sums and push/positive counts of the lane's terms t =
// tstart, tstart + step, ... < tend, eight terms' loads in flight.  Each
// partial is a sequential fp32 sum of at most L terms (L = the candidate's
// length), so it lies within gamma_{L-1} of its exact value; the partials
// meet in fp64 exactly (fp32 values >= 2^-16 are multiples of 2^-39), and
// k3w_pick_exact widens its intervals by that second gamma.
template <bool C8>
DEV uint32_t k3w_fill(const K3WMem &m, uint32_t f_lo, uint32_t f_kofs, uint32_t tstart, uint32_t tend,
                      uint32_t step, float &e0, float &e1) {
    uint32_t lcode = 0;
    for (uint32_t tb = tstart; tb < tend; tb += 8 * step) {
        uint32_t sl[8], cv[8];
        float4 sr[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const uint32_t t = tb + u * step;
            const bool ok = t < tend;
            sl[u] = k3w_slot(m, ok ? f_kofs + t : 0u);
            sr[u] = m.srec[ok ? f_lo + t : 0u];
            sl[u] = ok ? sl[u] : PF_NONE;
        }
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const bool ok = sl[u] != PF_NONE;
            const uint32_t c = k3w_cnt<C8>(m, ok ? sl[u] : 0u);
            cv[u] = ok ? c : 0u;
        }
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const uint32_t a0 = k3w_c0<C8>(cv[u]), a1 = k3w_c1<C8>(cv[u]);
            const float q0 = div_u16_y((float)a0, sr[u].x, sr[u].z);
            const float q1 = div_u16_y((float)a1, sr[u].y, sr[u].w);
            // pushed: key present (cv != 0) and hap total != 0 (:3505-3509);
            // positive: cnt > 0 (:3619-3624); branch-free
            const uint32_t hm = (sr[u].z != 0.f ? 1u : 0u) | (sr[u].w != 0.f ? 0x10000u : 0u);
            const uint32_t pc = (a0 != 0u ? 1u : 0u) | (a1 != 0u ? 0x10000u : 0u);
            lcode += pc + (cv[u] != 0u ? hm : 0u);
            e0 += q0;
            e1 += q1;
        }
    }
    return lcode;
}

// the reference's sequential fp32 fold of one candidate (:3619-3636)
template <bool C8>
DEV void k3w_fold(const K3WMem &m, uint32_t lo, uint32_t kofs, uint32_t len, float &s0, float &s1) {
    for (uint32_t t0 = 0; t0 < len; t0 += 8) {
        uint32_t sl[8];
        float4 sr[8];
        float q0[8], q1[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const uint32_t t = t0 + u;
            const bool ok = t < len;
            sl[u] = ok ? k3w_slot(m, kofs + t) : PF_NONE;
            sr[u] = m.srec[ok ? lo + t : 0u];
        }
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const bool ok = sl[u] != PF_NONE;
            const uint32_t c = ok ? k3w_cnt<C8>(m, sl[u]) : 0u;
            q0[u] = div_u16_y((float)k3w_c0<C8>(c), sr[u].x, sr[u].z);
            q1[u] = div_u16_y((float)k3w_c1<C8>(c), sr[u].y, sr[u].w);
        }
#pragma unroll
        for (int u = 0; u < 8; u++) {
            K3_FADD(s0, q0[u]);
            K3_FADD(s1, q1[u]);
        }
    }
}

// insert_mmr_counts of one tagged read into hap tg (its sites are distinct)
template <bool C8>
DEV void k3w_insert(const K3WMem &m, uint32_t S, uint32_t n, uint32_t st, uint32_t mo, uint32_t tg, uint32_t lane) {
    for (uint32_t tb = 0; tb < n; tb += 128) {
        uint32_t sl[2], cc[2];
        float4 sr[2];
        bool ok[2];
#pragma unroll
        for (int u = 0; u < 2; u++) {
            const uint32_t t = tb + u * 64 + lane;
            ok[u] = t < n && st + t < S;
            sl[u] = k3w_slot(m, ok[u] ? mo + t : 0u);
        }
#pragma unroll
        for (int u = 0; u < 2; u++) {
            ok[u] = ok[u] && sl[u] != PF_NONE;
            cc[u] = k3w_cnt<C8>(m, ok[u] ? sl[u] : 0u);
            sr[u] = m.srec[ok[u] ? st + tb + u * 64 + lane : 0u];
        }
#pragma unroll
        for (int u = 0; u < 2; u++) {
            if (ok[u]) {
                const uint32_t site = st + tb + u * 64 + lane;
                if (C8) reinterpret_cast<uint16_t *>(m.cnt)[sl[u]] = (uint16_t)(cc[u] + (tg ? 0x100u : 1u));
                else reinterpret_cast<uint32_t *>(m.cnt)[sl[u]] = cc[u] + (tg ? 0x10000u : 1u);
                const float h = (tg ? sr[u].y : sr[u].x) + 1.f;
                float *f = reinterpret_cast<float *>(&m.srec[site]);
                f[tg] = h;
                f[2 + tg] = __builtin_amdgcn_rcpf(h);
            }
        }
    }
    wave_sync();
}

// per-problem set-up (k3_init for one wave): flags and tags, reference
// reads seeding the counts (:3776-3810), the initial range, the T5 round
// trip, the site records and the untagged bitmask
template <bool C8>
DEV void k3w_init(const pf_dev_batch &d, uint32_t w, uint32_t dir, uint32_t r0, uint32_t S, uint32_t R,
                  uint32_t ntot, const K3WMem &m, uint32_t &umin, uint32_t &umax, K3Stats &stx, uint32_t &summ) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t s = d.win_start[w], e = d.win_end[w];
    const uint32_t refbit = dir == 0 ? FLG_LEFT : FLG_RIGHT;
    uint32_t *cw = reinterpret_cast<uint32_t *>(m.cnt);
    const uint32_t cwords = C8 ? (ntot + 1) / 2 : ntot;
    for (uint32_t j = lane; j < cwords; j += 64) cw[j] = 0;
    for (uint32_t j = lane; j < S; j += 64) m.srec[j] = make_float4(0.f, 0.f, 0.f, 0.f);
    uint32_t sum_mmr = 0;
    for (uint32_t i = lane; i < R; i += 64) {
        const uint32_t r = r0 + i;
        const uint32_t st = d.read_start[r], en = d.read_end[r];
        uint32_t f = 0;
        if (st <= s) {                                           // blockjoin.c:1127-1128
            f |= FLG_LEFT;
            if (en > s) f |= FLG_LEFT_STRICT;
        } else if (en >= e) {                                    // blockjoin.c:1134-1135
            f |= FLG_RIGHT;
            if (st < e) f |= FLG_RIGHT_STRICT;
        }
        m.flg[i] = (uint8_t)f;
        m.hp[i] = d.read_hp[r];
        sum_mmr += d.mmr_n[2ull * r + dir];
    }
    {
        const uint32_t *a = d.site_pos + d.win_site_off[w];
        if (dir == 0) {
            umin = 0;
            umax = (uint32_t)ub_u32(a, 0, S, s);                 // #sites <= ref_start (:3994-3998)
        } else {
            umax = S - 1;
            umin = (uint32_t)((int)ub_u32(a, 0, S, e) - 1);      // may wrap to UINT32_MAX (:3999-4003)
        }
        umin = uni(umin);
        umax = uni(umax);
    }
    wave_sync();
    // ---- reference reads seed the counts: eight reads' slot loads in flight
    uint32_t ref_ins = 0;
    for (uint32_t i0 = 0; i0 < R; i0 += 64) {
        const uint32_t i = i0 + lane;
        const bool isref = i < R && (m.flg[i] & refbit) && m.hp[i] <= 1;
        uint64_t bal = __ballot(isref);
        while (bal) {
            uint32_t rd[8] = {0}, n[8] = {0}, st[8] = {0}, mo[8] = {0}, inc[8] = {0};
            int k = 0;
            for (; k < 8 && bal; k++) {
                const uint32_t b = (uint32_t)__ffsll((unsigned long long)bal) - 1u;
                bal &= bal - 1;
                rd[k] = i0 + b;
                k3w_read_fields(d, r0, rd[k], dir, m.kbase, n[k], st[k], mo[k]);
                inc[k] = m.hp[rd[k]] ? 1u : 0u;
                ref_ins += n[k];
            }
            uint32_t mx = 0;
            for (int u = 0; u < k; u++) mx = n[u] > mx ? n[u] : mx;
            for (uint32_t t0 = 0; t0 < mx; t0 += 64) {
                uint32_t sl[8];
#pragma unroll
                for (int u = 0; u < 8; u++) {
                    const uint32_t t = t0 + lane;
                    const bool ok = t < n[u] && st[u] + t < S;
                    sl[u] = ok ? m.kb[mo[u] + t] : PF_NONE;
                }
#pragma unroll
                for (int u = 0; u < 8; u++) {
                    if (sl[u] != PF_NONE) {
                        const uint32_t site = st[u] + t0 + lane;
                        if (C8) atomicAdd(&cw[sl[u] >> 1], (inc[u] ? 0x100u : 1u) << ((sl[u] & 1u) * 16u));
                        else atomicAdd(&cw[sl[u]], inc[u] ? 0x10000u : 1u);
                        // exact hap totals as floats (ds_add_f32 of 1.0: integers < 2^24)
                        atomicAdd(reinterpret_cast<float *>(&m.srec[site]) + inc[u], 1.f);
                    }
                }
            }
        }
    }
    wave_sync();
    // reciprocals of the totals (0 for a zero total: its terms are never pushed)
    for (uint32_t j = lane; j < S; j += 64) {
        const float4 r = m.srec[j];
        m.srec[j] = make_float4(r.x, r.y, r.x != 0.f ? __builtin_amdgcn_rcpf(r.x) : 0.f,
                                r.y != 0.f ? __builtin_amdgcn_rcpf(r.y) : 0.f);
    }
    wave_sync();
    summ = 0;
#pragma unroll
    for (int bb = 0; bb < 32; bb++) summ += (uint32_t)__popcll(__ballot((sum_mmr >> bb) & 1)) << bb;
    stx.inserts = uni(ref_ins);                      // wave-uniform: the reads came from a ballot
}

// the T5 round trip and the untagged bitmask (aux: 4 B per read after the
// layout)
DEV void k3w_tags(const pf_dev_batch &d, uint32_t dir, uint32_t r0, uint32_t R, const K3WMem &m, uint32_t *aux) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t nwords = (R + 63) >> 6;
    const uint32_t refbit = dir == 0 ? FLG_LEFT : FLG_RIGHT;
    for (uint32_t i = lane; i < R; i += 64) aux[i] = 0;
    wave_sync();
    // step 1.5 (:4010-4025): all reads unphased, ref reads restored through
    // the (readID<<2)|hp round trip (hp >= 4 lands on readID|(hp>>2)); the
    // last writer in reference order wins
    for (uint32_t i = lane; i < R; i += 64)
        if (m.flg[i] & refbit) {
            const uint32_t t = i | ((uint32_t)m.hp[i] >> 2);
            if (t < R) atomicMax(&aux[t], i + 1);
        }
    wave_sync();
    for (uint32_t i = lane; i < R; i += 64) {
        const uint32_t lw = aux[i];
        m.hp[i] = lw ? (uint8_t)(d.read_hp[r0 + lw - 1] & 3) : (uint8_t)2;
    }
    wave_sync();
    for (uint32_t j = 0; j < nwords; j++) {
        const uint32_t p = j * 64 + lane;
        bool u = false;
        if (p < R) {
            const uint32_t rd = dir ? d.rev_ord[r0 + p] : p;
            const uint32_t h = m.hp[rd];
            u = h != 0 && h != 1;
        }
        const uint64_t b = __ballot(u);
        if (lane == 0) m.untag[j] = b;
    }
    wave_sync();
}

// 2x2 table on the opposite side's strict reads (:3940-3956), dir-0 tags, stats
DEV void k3w_finish(const pf_dev_batch &d, uint32_t w, uint32_t dir, uint32_t r0, uint32_t S, uint32_t R,
                    const K3WMem &m, uint32_t summ, const K3Stats &stx) {
    const uint32_t lane = threadIdx.x & 63;
    int tab0 = 0, tab1 = 0, tab2 = 0, tab3 = 0;
    uint32_t nstrict = 0;
    const uint32_t strict = dir == 0 ? FLG_RIGHT_STRICT : FLG_LEFT_STRICT;
    for (uint32_t i = lane; i < R; i += 64) {
        if (m.flg[i] & strict) {
            nstrict++;
            const uint32_t ref = d.read_hp[r0 + i], q = m.hp[i];
            if (ref <= 1 && q <= 1) {
                const uint32_t k = ref * 2 + q;
                tab0 += k == 0; tab1 += k == 1; tab2 += k == 2; tab3 += k == 3;
            }
        }
        if (dir == 0) d.hp_fwd[r0 + i] = m.hp[i];
    }
    uint32_t tsum[5] = {(uint32_t)tab0, (uint32_t)tab1, (uint32_t)tab2, (uint32_t)tab3, nstrict};
#pragma unroll
    for (int k = 0; k < 5; k++) {
        uint32_t tot = 0;
        for (int bb = 0; bb < 16; bb++) tot += (uint32_t)__popcll(__ballot((tsum[k] >> bb) & 1)) << bb;
        tsum[k] = tot;
    }
    if (lane < 4) d.table[((uint64_t)w * 2 + dir) * 4 + lane] = (int32_t)tsum[lane];
    if (lane == 0) {
        unsigned long long *sp = d.stats + ((uint64_t)w * 2 + dir) * PF_NSTAT;
        sp[0] = stx.lookups; sp[1] = stx.inserts; sp[3] = stx.scanned;
        sp[2] = stx.iters | (5ull << 56);                              // the slot-list source: the one-wave kernel
        sp[4] = summ; sp[5] = tsum[4]; sp[6] = R; sp[7] = S;
    }
}

// pick from registers (k3_pick_exact with the per-candidate sums in lanes)
DEV void k3w_pick_exact(double S0, double S1, uint32_t lane, uint32_t nc, uint32_t c_len, int l0, int l1,
                        uint32_t &pick, uint32_t &cw, uint32_t &tg) {
    const bool act = lane < nc;
    if (!act) { S0 = 0.0; S1 = 0.0; }
    // the reference's sequential sum within gamma_{L-1} of the exact sum, the
    // per-lane fp32 partials within another gamma_{L-1} (k3w_fill): twice
    // the single-sum margin, and 2^-8 of slack for the second-order terms
    const double g = (double)(c_len > 1 ? c_len - 1 : 0) * (0x1p-23 * (1.0 + 0x1p-8));
    const double E = g * (S0 + S1);
    const double D = S0 > S1 ? S0 - S1 : S1 - S0;
    const bool sgn = D > E;
    const double dlo = sgn ? (D - E) * (1.0 - 0x1p-20) : 0.0;
    const double dhi = (D + E) * (1.0 + 0x1p-20) + 0x1p-60;
    const bool rel = l0 < 3 || l1 < 3;
    const bool el = act && (!rel || dlo >= 3.0);
    const bool un = !act || (rel && dhi < 3.0);
    const uint64_t b_und = __ballot(!el && !un), b_el = __ballot(el);
    const uint64_t b_sgn = __ballot(sgn), b_gt = __ballot(S0 > S1);
    if (b_und) return;
    if (b_el == 0) { pick = 2; return; }
    const float flo = el ? (float)(dlo * (1.0 - 0x1p-20)) : 0.f;
    const float fhi = (float)(dhi * (1.0 + 0x1p-20));
    const uint32_t key = el ? __float_as_uint(flo) + 1u : 0u;
    const uint32_t M = nc <= 16 ? (uint32_t)__builtin_amdgcn_readlane(
                                      (int)dpp_max_step(dpp_max_step(dpp_max_step(dpp_max_step(key, 0), 1), 2), 3), 0)
                                : wave_max_dpp(key);
    const float mf = __uint_as_float(M - 1u);
    const uint64_t b_hi = __ballot(el && fhi >= mf);
    if (__popcll(b_hi) != 1) return;
    const uint32_t cs = (uint32_t)__ffsll((unsigned long long)b_hi) - 1u;
    if (!((b_sgn >> cs) & 1ull)) return;
    pick = 1;
    cw = cs;
    tg = ((b_gt >> cs) & 1ull) ? 0u : 1u;
}

// per-wave fill scratch (static LDS): candidate fields and exact partial sums
struct K3WFill {
    uint4 cf[64];                // lo, kofs, first lane, length << 8 | lanes
    double acc[128];             // hap 0 | hap 1 sums per candidate
    uint32_t lcs[64];            // push/positive count pairs per candidate
};

template <bool C8>
DEV void k3w_greedy(const pf_dev_batch &d, uint32_t w, uint32_t dir, uint32_t r0, uint32_t S, uint32_t R,
                    uint32_t ntot, const K3WMem &m, uint32_t *qbuf, uint32_t *aux, K3WFill *fsc) {
    const uint32_t lane = threadIdx.x & 63;
    fsc->acc[lane] = 0.0;
    fsc->acc[64 + lane] = 0.0;
    fsc->lcs[lane] = 0u;
    const int cov_rt = d.win_par[w * 4 + 1];
    const uint32_t NC = (uint32_t)d.win_par[w * 4 + 2];
    const uint32_t nwords = (R + 63) >> 6;
    K3Stats stx = {0, 0, 0, 0};
#ifdef PF_K3_PROFILE
    unsigned long long prof_acc[32] = {0};
    unsigned long long prof_last = k3_stamp_now();
#endif
    uint32_t umin, umax, summ;
    k3w_init<C8>(d, w, dir, r0, S, R, ntot, m, umin, umax, stx, summ);
    k3w_tags(d, dir, r0, R, m, aux);
    k3w_range(m, S, cov_rt, lane, umin, umax);
    K3_STAMP(0);
    int il = dir == 0 ? 0 : (int)R - 1;
    uint32_t failed = 0;
    uint32_t nc = 0;
    uint32_t c_pos = 0, c_rd = 0, c_n = 0, c_st = 0, c_mo = 0, c_cs = 0;
    uint32_t q_pos = 0, q_rd = 0, q_nn = 0, q_st = 0, q_mo = 0;
    uint32_t q_cnt = 0, q_head = 0;
    bool q_more = false;
    int q_cont = 0;
    uint32_t lsum = 0;
    bool need_collect = true, have_win = false;
    const bool force_fold = d.k3_mode == 1u;
    uint32_t pfv[K3W_LSMAX / 64];                 // the queued read's slot list, loaded ahead
    for (;;) {
        if (have_win) k3w_range(m, S, cov_rt, lane, umin, umax);
        // ---- candidate list: full collection from i_last (:4037-4051)
        if (need_collect) {
            bool done = false;
            for (;;) {
                if (dir == 0 ? il >= (int)R : il <= 0) { done = true; break; }
                q_cnt = k3w_qbuild(d, m, r0, nwords, dir == 0 ? il - 1 : il + 1, dir, lane, qbuf,
                                   q_pos, q_rd, q_nn, q_st, q_mo, q_more, q_cont);
                const uint32_t take = q_cnt < NC ? q_cnt : NC;
                c_pos = q_pos; c_rd = q_rd; c_n = q_nn; c_st = q_st; c_mo = q_mo;
                q_head = take;
                uint32_t found = take;
                while (found < NC && q_more) {
                    q_cnt = k3w_qbuild(d, m, r0, nwords, q_cont, dir, lane, qbuf, q_pos, q_rd, q_nn, q_st, q_mo,
                                       q_more, q_cont);
                    q_head = 0;
                    while (found < NC && q_head < q_cnt) {
                        const uint32_t a0 = rdl(q_pos, q_head), a1 = rdl(q_rd, q_head), a2 = rdl(q_nn, q_head);
                        const uint32_t a3 = rdl(q_st, q_head), a4 = rdl(q_mo, q_head);
                        if (lane == found) { c_pos = a0; c_rd = a1; c_n = a2; c_st = a3; c_mo = a4; }
                        found++;
                        q_head++;
                    }
                }
                if (found == 0) {
                    stx.scanned += dir == 0 ? (uint32_t)((int)R - il) : (uint32_t)(il + 1);
                    if (++failed > 10) { done = true; break; }
                    il += dir == 0 ? (int)NC : -(int)NC;
                    continue;
                }
                nc = found;
                break;
            }
            if (done) break;
            need_collect = false;
            // every candidate's slot list into cache list c
            c_cs = lane;
            for (uint32_t c = 0; c < nc; c++) k3w_cache_load(m, c, rdl(c_mo, c), rdl(c_n, c), lane);
            wave_sync();
        }
        // ---- the next untagged read after the list, for this iteration's
        // append; its slot list is loaded now and lands in the cache at the end
        int qn = -1;
        uint32_t q_rd1 = 0, q_n1 = 0, q_st1 = 0, q_mo1 = 0;
        if (nc == NC) {
            if (q_head == q_cnt && q_more) {
                q_cnt = k3w_qbuild(d, m, r0, nwords, q_cont, dir, lane, qbuf, q_pos, q_rd, q_nn, q_st, q_mo,
                                   q_more, q_cont);
                q_head = 0;
            }
            if (q_head < q_cnt) {
                qn = (int)rdl(q_pos, q_head);
                q_rd1 = rdl(q_rd, q_head); q_n1 = rdl(q_nn, q_head);
                q_st1 = rdl(q_st, q_head); q_mo1 = rdl(q_mo, q_head);
                q_head++;
#pragma unroll
                for (uint32_t u = 0; u < K3W_LSMAX / 64; u++) {
                    const uint32_t t = u * 64 + lane;
                    pfv[u] = t < q_n1 ? m.kb[q_mo1 + t] : PF_NONE;
                }
            }
        }
        // ---- lookup spans: sites in [min_i, max_i) (query_counts_of_mmrs, :3500-3501)
        uint32_t c_len, c_lo, c_kofs;
        {
            const uint32_t lo = c_st > umin ? c_st : umin;
            const uint32_t hi0 = c_st + c_n;
            const uint32_t hi = hi0 < umax ? hi0 : umax;
            c_len = lane < nc && hi > lo && umin != 0xFFFFFFFFu ? hi - lo : 0;
            c_lo = lo;
            c_kofs = c_cs * m.ls + (c_len ? lo - c_st : 0);
        }
        lsum += c_len;
        if (nc >= NC) {
            const uint32_t pl = rdl(c_pos, NC - 1);
            stx.scanned += dir == 0 ? pl - (uint32_t)il + 1 : (uint32_t)il - pl + 1;
        } else stx.scanned += dir == 0 ? (uint32_t)((int)R - il) : (uint32_t)(il + 1);
        stx.iters++;
        K3_STAMP(2);
        // ---- term fill, balanced: candidate c gets g_c >= 1 lanes in
        // proportion to its in-range methmers (sum <= 64), its lanes stride
        // its terms; exact per-lane partial sums meet in LDS (fp64 sums are
        // exact in any order)
        uint32_t lcode;
        double S0, S1;
        {
            const uint32_t incl = wave_incl_scan_dpp(c_len);
            const uint32_t T = rdl(incl, 63);
            const uint32_t g = lane < nc ? (T ? (uint32_t)(((uint64_t)c_len * (64u - nc)) / T) + 1u : 1u) : 0u;
            const uint32_t gincl = wave_incl_scan_dpp(g);
            if (lane < nc) fsc->cf[lane] = make_uint4(c_lo, c_kofs, gincl - g, (c_len << 8) | g);
            wave_sync();
            uint32_t c = 0;
            for (uint32_t k = 0; k < nc; k++) c += rdl(gincl, k) <= lane ? 1u : 0u;
            if (c < nc) {
                const uint4 f = fsc->cf[c];
                float x0 = 0.f, x1 = 0.f;
                const uint32_t lc = k3w_fill<C8>(m, f.x, f.y, lane - f.z, f.w >> 8, f.w & 0xffu, x0, x1);
                atomicAdd(&fsc->acc[c], (double)x0);
                atomicAdd(&fsc->acc[64 + c], (double)x1);
                atomicAdd(&fsc->lcs[c], lc);
            }
            wave_sync();
            S0 = fsc->acc[lane];
            S1 = fsc->acc[64 + lane];
            lcode = fsc->lcs[lane];
            fsc->acc[lane] = 0.0;
            fsc->acc[64 + lane] = 0.0;
            fsc->lcs[lane] = 0u;
            wave_sync();
        }
        K3_STAMP(10);
        // ---- pick: exact intervals, else the sequential fp32 fold
        uint32_t pick = 0, cw = 0, tg = 0;
        {
            const int l0 = (int)(lcode & 0xffffu), l1 = (int)(lcode >> 16);
            if (!force_fold) k3w_pick_exact(S0, S1, lane, nc, c_len, l0, l1, pick, cw, tg);
            if (pick == 0) {
                float s0 = 0.f, s1 = 0.f;
                if (lane < nc) k3w_fold<C8>(m, c_lo, c_kofs, c_len, s0, s1);
                const float diff = s0 > s1 ? s0 - s1 : s1 - s0;
                const bool elig = lane < nc && !(diff < 3.f && (l0 < 3 || l1 < 3));
                const uint32_t hkey = elig ? __float_as_uint(diff) + 1u : 0u;
                const uint32_t hmax = wave_max_dpp(hkey);
                if (hmax == 0) pick = 2;
                else {
                    pick = 1;
                    cw = 63u - (uint32_t)__clzll((long long)__ballot(hkey == hmax));
                    tg = rdl(s0 > s1 ? 0u : 1u, cw);
                }
            }
        }
        K3_STAMP(19);
        if (pick == 2) {
            // nothing could be tagged (:4064-4069): move i_last, rescan
            if (++failed > 10) break;
            il += dir == 0 ? (int)NC : -(int)NC;
            need_collect = true;
            have_win = false;
            continue;
        }
        // ---- the winner: tag, list minus the winner plus the queued read
        const uint32_t rd = rdl(c_rd, cw), n = rdl(c_n, cw), st = rdl(c_st, cw), fs = rdl(c_cs, cw);
        const uint32_t pw = rdl(c_pos, cw);
        stx.inserts += n;
        if (lane == 0) {
            m.hp[rd] = (uint8_t)tg;
            m.untag[pw >> 6] &= ~(1ull << (pw & 63));
        }
        failed = 0;
        {
            const int src = (int)lane + 1;
            const uint32_t a0 = (uint32_t)__shfl((int)c_pos, src, 64), a1 = (uint32_t)__shfl((int)c_rd, src, 64);
            const uint32_t a2 = (uint32_t)__shfl((int)c_n, src, 64), a3 = (uint32_t)__shfl((int)c_st, src, 64);
            const uint32_t a4 = (uint32_t)__shfl((int)c_cs, src, 64);
            if (lane >= cw) { c_pos = a0; c_rd = a1; c_n = a2; c_st = a3; c_cs = a4; }
        }
        uint32_t ncn = nc - 1;
        if (qn >= 0) {
            if (lane == ncn) { c_pos = (uint32_t)qn; c_rd = q_rd1; c_n = q_n1; c_st = q_st1; c_cs = fs; }
            ncn++;
        }
        nc = ncn;
        if (nc == 0) need_collect = true;     // an empty batch: the reference's failure path (:4046-4051)
        K3_STAMP(20);
        k3w_insert<C8>(m, S, n, st, fs * m.ls, tg, lane);
        K3_STAMP(21);
        if (qn >= 0) {                        // the appended read takes the winner's cache list
            uint16_t *dst = m.cc + fs * m.ls;
#pragma unroll
            for (uint32_t u = 0; u < K3W_LSMAX / 64; u++) {
                const uint32_t t = u * 64 + lane;
                if (t < q_n1) dst[t] = pfv[u] == PF_NONE ? (uint16_t)0xFFFFu : (uint16_t)pfv[u];
            }
            wave_sync();
        }
        have_win = true;
        K3_STAMP(22);
    }
    {
        uint32_t tot = 0;
#pragma unroll
        for (int bb = 0; bb < 32; bb++) tot += (uint32_t)__popcll(__ballot((lsum >> bb) & 1)) << bb;
        stx.lookups += tot;
    }
    k3w_finish(d, w, dir, r0, S, R, m, summ, stx);
#ifdef PF_K3_PROFILE
    if (lane == 0) {
        unsigned long long *pp = d.prof + ((uint64_t)w * 2 + dir) * 32;
        for (int i = 0; i < 32; i++) pp[i] = prof_acc[i];
    }
#endif
}

// slot dictionary of one problem by one wave (k3_dict / k3_dict_rewrite with
// eight reads' key loads in flight)
DEV void k3w_dict(const pf_dev_batch &d, uint32_t r0, uint32_t R, uint32_t S, uint32_t dir, uint64_t *masks,
                  uint32_t *base, uint32_t *sh_scan, K3Ctl &ctl, bool rewrite) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t MW = (uint32_t)d.mw;
    if (!rewrite) {
        for (uint32_t j = lane; j < S * MW; j += 64) masks[j] = 0;
        wave_sync();
    }
    for (uint32_t i0 = 0; i0 < R; i0 += 8) {
        uint32_t n[8], st[8];
        uint32_t *kp[8];
        uint32_t mx = 0;
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const uint32_t i = i0 + u < R ? i0 + u : i0;
            const uint64_t g = 2ull * (r0 + i) + dir;
            n[u] = i0 + u < R ? d.mmr_n[g] : 0u;
            st[u] = d.mmr_start[g];
            kp[u] = d.keys + d.mmr_off[g];
            mx = n[u] > mx ? n[u] : mx;
        }
        for (uint32_t t0 = 0; t0 < mx; t0 += 64) {
            const uint32_t t = t0 + lane;
            uint32_t key[8];
#pragma unroll
            for (int u = 0; u < 8; u++) key[u] = t < n[u] ? kp[u][t] : 0xFFFFFFFFu;
#pragma unroll
            for (int u = 0; u < 8; u++) {
                if (t >= n[u]) continue;
                const uint32_t site = st[u] + t;
                const bool ok = site < S && key[u] < 64u * MW;
                if (!rewrite) {
                    if (ok) atomicOr((unsigned long long *)&masks[(uint64_t)site * MW + (key[u] >> 6)],
                                     1ull << (key[u] & 63));
                } else {
                    uint32_t slot = PF_NONE;
                    if (ok) {
                        const uint64_t *row = masks + (uint64_t)site * MW;
                        const uint32_t wi = key[u] >> 6, b = key[u] & 63;
                        slot = base[site];
                        for (uint32_t mm = 0; mm < wi; mm++) slot += (uint32_t)__popcll(row[mm]);
                        slot += (uint32_t)__popcll(row[wi] & ((1ull << b) - 1ull));
                    }
                    kp[u][t] = slot;
                }
            }
        }
    }
    wave_sync();
    if (rewrite) return;
    uint32_t carry = 0;
    for (uint32_t p0 = 0; p0 < S; p0 += 64) {
        const uint32_t p = p0 + lane;
        uint32_t c = 0;
        if (p < S)
            for (uint32_t mm = 0; mm < MW; mm++) c += (uint32_t)__popcll(masks[(uint64_t)p * MW + mm]);
        const uint32_t incl = wave_incl_scan_dpp(c);
        if (p < S) base[p] = carry + incl - c;
        carry += rdl(incl, 63);
    }
    if (lane == 0) ctl.ntot = carry;
    wave_sync();
}

// LDS of the dictionary phase: masks, slot bases, and the per-site coverage
// by methmer spans (S + 1 counters)
DEV uint64_t k3w_p1_bytes(uint32_t S, uint32_t MW) {
    return align16(8ull * S * MW) + align16(4ull * S) + 4ull * (S + 1);
}

DEV void k3w_run(const pf_dev_batch &d, uint32_t prob, uint8_t *smem, K3Ctl &ctl, uint32_t *qbuf,
                 uint32_t *sh_scan, K3WFill *fsc, const uint32_t lds) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t w = prob >> 1, dir = prob & 1;
    const uint32_t S = d.win_S[w];
    if (S == 0) {
        if (lane < 4) d.table[((uint64_t)w * 2 + dir) * 4 + lane] = 0;
        if (lane < PF_NSTAT) d.stats[((uint64_t)w * 2 + dir) * PF_NSTAT + lane] = 0;
        return;
    }
    const uint32_t R = d.win_nreads[w];
    const uint32_t r0 = d.win_read_off[w];
    const uint32_t MW = (uint32_t)d.mw;
    const uint64_t kbase = d.mmr_off[2ull * r0];
    // the wave build: n_cand <= 64 (register candidate list), < 8192 sites
    // (exact-interval pick), the dictionary in LDS, the exact or fold pick
    if (d.win_par[w * 4 + 2] > 64 || S >= 8192u || d.k3_mode > 1u || d.kdict || k3w_p1_bytes(S, MW) > lds) {
        k3_defer(d, prob);
        return;
    }
    uint64_t *masks = reinterpret_cast<uint64_t *>(smem);
    uint32_t *mbase = reinterpret_cast<uint32_t *>(smem + align16(8ull * S * MW));
    uint32_t *cov = reinterpret_cast<uint32_t *>(smem + align16(8ull * S * MW) + align16(4ull * S));
    k3w_dict(d, r0, R, S, dir, masks, mbase, sh_scan, ctl, false);
    const uint32_t ntot = uni(ctl.ntot);
    // deepest site coverage by methmer spans [st, st+n): it bounds every count
    for (uint32_t j = lane; j <= S; j += 64) cov[j] = 0;
    wave_sync();
    for (uint32_t i = lane; i < R; i += 64) {
        const uint64_t g = 2ull * (r0 + i) + dir;
        const uint32_t n = d.mmr_n[g], st = d.mmr_start[g];
        if (n && st < S) {
            atomicAdd(&cov[st], 1u);
            atomicAdd(&cov[st + n < S ? st + n : S], 0xFFFFFFFFu);
        }
    }
    wave_sync();
    uint32_t carry = 0, mx = 0;
    for (uint32_t j0 = 0; j0 < S; j0 += 64) {
        const uint32_t j = j0 + lane;
        const uint32_t v = j < S ? cov[j] : 0u;
        const uint32_t incl = wave_incl_scan_dpp(v) + carry;
        carry = rdl(incl, 63);
        const uint32_t c = j < S ? incl : 0u;
        mx = c > mx ? c : mx;
    }
    mx = wave_max_dpp(mx);
    const bool c8 = mx < 256u;
    // longest methmer list of the direction: the candidate cache's stride
    uint32_t mxl = 0;
    for (uint32_t i = lane; i < R; i += 64) {
        const uint32_t n = d.mmr_n[2ull * (r0 + i) + dir];
        mxl = n > mxl ? n : mxl;
    }
    mxl = wave_max_dpp(mxl);
    const uint32_t ls = (mxl + 7u) & ~7u;
    const uint32_t NCw = (uint32_t)d.win_par[w * 4 + 2];
    uint64_t off[K3W_NOFF];
    const uint64_t need = c8 ? k3w_layout<true>(S, ntot, R, NCw, ls, off) : k3w_layout<false>(S, ntot, R, NCw, ls, off);
    // the T5 scratch (4 B per read) goes after the layout when it fits there
    const uint64_t need_aux = align16(need) + 4ull * R;
    if (need_aux > lds || mxl > K3W_LSMAX || ntot >= 0xFFFFu) {
        k3_defer(d, prob);           // keys still intact: the fallback rebuilds the dictionary
        return;
    }
    k3w_dict(d, r0, R, S, dir, masks, mbase, sh_scan, ctl, true);
    K3WMem m;
    m.srec = reinterpret_cast<float4 *>(smem + off[0]);
    m.cnt = smem + off[1];
    m.cc = reinterpret_cast<uint16_t *>(smem + off[2]);
    m.ls = ls;
    m.hp = smem + off[3];
    m.flg = smem + off[4];
    m.untag = reinterpret_cast<uint64_t *>(smem + off[5]);
    m.kb = d.keys + kbase;
    m.kbase = kbase;
    uint32_t *aux2 = reinterpret_cast<uint32_t *>(smem + align16(need));
    if (c8) k3w_greedy<true>(d, w, dir, r0, S, R, ntot, m, qbuf, aux2, fsc);
    else k3w_greedy<false>(d, w, dir, r0, S, R, ntot, m, qbuf, aux2, fsc);
}

// Main greedy kernel: one wavefront per problem, heaviest first (k3_order);
// problems it cannot take go to pf_k3_fallback.
__global__ __launch_bounds__(64) void pf_k3_wave(pf_dev_batch d) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    __shared__ K3Ctl ctl;
    __shared__ uint32_t qbuf[64];
    __shared__ uint32_t sh_scan[2];
    __shared__ K3WFill fsc;
    k3w_run(d, d.k3_order[blockIdx.x], smem, ctl, qbuf, sh_scan, &fsc, d.lds_w);
}

// ------------------------------------------------------------------------
// self-test: div_u16 against the correctly rounded fp32 division over every
// (a, b) with 0 <= a <= 65535, 1 <= b <= 65535 (block = one b)
__global__ __launch_bounds__(256) void pf_selftest_div(unsigned long long *bad) {
    const uint32_t b = blockIdx.x + 1;
    uint32_t nb = 0;
    for (uint32_t a = threadIdx.x; a < 65536u; a += 256) {
        const float ref = (float)a / (float)b;
        nb += __float_as_uint(div_u16(a, b)) != __float_as_uint(ref);
    }
    if (nb) atomicAdd(bad, (unsigned long long)nb);
}

// self-test of the DPP / permlane wave primitives against LDS references
__global__ __launch_bounds__(64) void pf_selftest_wave(unsigned long long *bad) {
    __shared__ uint32_t v[64];
    const uint32_t lane = threadIdx.x;
    uint32_t h = (blockIdx.x * 64 + lane) * 2654435761u;
    h ^= h >> 15;
    h *= 2246822519u;
    h ^= h >> 13;
    const uint32_t x = blockIdx.x & 1 ? (h & 0xffffu) : (h & 7u);
    v[lane] = x;
    __syncthreads();
    uint32_t nb = 0;
    uint32_t ref = 0, mx = 0;
    for (uint32_t i = 0; i <= lane; i++) ref += v[i];
    for (uint32_t i = 0; i < 64; i++) mx = v[i] > mx ? v[i] : mx;
    nb += wave_incl_scan_dpp(x) != ref;
    {
        const uint32_t sh = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x138, 0xF, 0xF, false);
        if (lane > 0) nb += sh != v[lane - 1];
        const uint32_t sl = wave_shl1(x);
        nb += sl != (lane < 63 ? v[lane + 1] : 0u);
    }
    nb += wave_max_dpp(x) != mx;
    for (uint32_t ncp = 1; ncp <= 64; ncp <<= 1) {
        uint32_t gs = 0;
        for (uint32_t i = lane & (ncp - 1); i < 64; i += ncp) gs += v[i];
        nb += wave_group_sum(x, ncp) != gs;
    }
    if (nb) atomicAdd(bad, (unsigned long long)nb);
}
