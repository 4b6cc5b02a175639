// pf_kernels.hip -- gfx950 kernels of the methphase hot path.
//
// Three launches per batch (reference call stack in SURVEY.md section 3.1):
//
//   pf_k1_sites    one 1024-thread workgroup per window.
//                  get_methmer_sites_and_ranges (blockjoin.c:3202-3354) for both
//                  directions + the left-coverage check of load_reads_given_interval
//                  (blockjoin.c:1161-1163) + the revbuf end-order (blockjoin.c:1126,1140).
//                  Per-position meth/unmeth counts are accumulated in a dense
//                  32768-position LDS tile (no hashing), tiles swept in position
//                  order so sites come out sorted; every call is labelled with its
//                  site index for the next kernel.
//   pf_k2_methmers one wavefront per (read, direction).
//                  get_mmr_of_read (blockjoin.c:3357-3451), restated as an
//                  "entry walk": the merged site/call buffer the reference radix
//                  sorts per read is never materialised; each site entry gets its
//                  methylation character from the call labels, and each methmer is
//                  assembled from the characters of the following entries.
//   pf_k3_greedy   one 256-thread workgroup per (window, direction).
//                  haplotag_region1 (blockjoin.c:3958-4080) and the 2x2 table of
//                  evaluate_separation (blockjoin.c:3940-3956).  The per-site methmer
//                  key lists of the reference (linear search, blockjoin.c:3453-3515)
//                  are replaced by a dense per-site slot dictionary built once per
//                  problem, so a lookup is one LDS load; candidate scoring runs over
//                  (methmer, candidate) pairs in parallel and only the order-sensitive
//                  float sums (blockjoin.c:3619-3636) run sequentially, one lane per
//                  candidate, in methmer order.
//
// Bit-exactness notes: fp32 division is IEEE (no fast-math), the score sums are
// strictly sequential in methmer order, and candidate selection reproduces the
// stable merge sort + walk-from-end of predict_tags_of_reads (blockjoin.c:3729-3766)
// as "max score, ties to the later candidate".
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "pf_device.h"

#define DEV static __device__ __forceinline__

// Diagnostic build only (-DPF_K3_PROFILE): per-phase s_memtime cycle shares of
// the greedy loop, written to d.prof.  The real kernel executes no stamp.
#ifdef PF_K3_PROFILE
#define K3_STAMP(i) do { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
    prof_acc[i] += t_ - prof_last; prof_last = t_; } while (0)
#else
#define K3_STAMP(i) do { } while (0)
#endif

// ------------------------------------------------------------------------
// small helpers
DEV uint64_t lanemask_lt(uint32_t lane) { return lane ? (~0ull >> (64 - lane)) : 0ull; }

DEV void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
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

DEV uint32_t next_pow2(uint32_t x) {
    uint32_t p = 1;
    while (p < x) p <<= 1;
    return p;
}

// ========================================================================
// K1: sites + directional methmer ranges + end-order + arena reservation
// ========================================================================
__global__ __launch_bounds__(PF_K1_THREADS) void pf_k1_sites(pf_dev_batch d) {
    __shared__ uint32_t tile[PF_K1_TILE];
    __shared__ uint32_t sh_scan[PF_K1_THREADS / 64 + 1];
    __shared__ uint32_t sh_misc[8];
    __shared__ uint32_t sh_tbase[PF_K1_THREADS];
    __shared__ unsigned long long sh_base[2];
    constexpr uint32_t NT = PF_K1_THREADS, NW = NT / 64;
    const uint32_t w = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
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
        return;
    }
    const uint32_t pmin = sh_misc[2], pmax = sh_misc[3];
    if (tid == 0) { sh_misc[4] = 0; d.win_nreads[w] = R; }
    __syncthreads();

    // ---- fast path: LDS hash of call positions (meth/unmeth only) + a bitmap of
    // qualifying positions over [pmin, pmin + 64*BW): a site's index (its rank in
    // position order) is a prefix popcount, so no sort is needed.
    constexpr uint32_t HN = 8192, HMAX = 6144, BW = 8192;
    uint32_t *hkeys = tile, *hcnt = tile + HN;
    uint64_t *bmap = reinterpret_cast<uint64_t *>(tile + 2 * HN);
    bool hash_ok = (uint64_t)(pmax - pmin) < (uint64_t)BW * 64;
    if (hash_ok) {
        for (uint32_t j = tid; j < HN; j += NT) { hkeys[j] = PF_NONE; hcnt[j] = 0; }
        for (uint32_t j = tid; j < BW; j += NT) bmap[j] = 0;
        if (tid == 0) { sh_misc[5] = 0; sh_misc[6] = 0; }
        __syncthreads();
        for (uint32_t i = wid; i < R; i += NW) {
            const uint32_t r = r0 + i;
            const uint64_t c0 = d.read_call_off[r], c1 = d.read_call_off[r + 1];
            for (uint64_t c = c0 + lane; c < c1; c += 64) {
                const uint32_t cat = d.call_cat[c];
                if (cat >= 2) continue;
                const uint32_t pos = d.call_pos[c];
                const uint32_t inc = cat == 0 ? 1u : 0x10000u;
                uint32_t h = (pos * 2654435761u) >> 19;
                for (;;) {
                    const uint32_t k = __hip_atomic_load(&hkeys[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    if (k == pos) { atomicAdd(&hcnt[h], inc); break; }
                    if (k == PF_NONE) {
                        // reserve before inserting: at most HMAX keys ever enter the
                        // table, so probing always terminates
                        if (atomicAdd(&sh_misc[5], 1u) >= HMAX) { sh_misc[6] = 1; break; }
                        const uint32_t old = atomicCAS(&hkeys[h], PF_NONE, pos);
                        if (old == PF_NONE || old == pos) { atomicAdd(&hcnt[h], inc); break; }
                    }
                    h = (h + 1) & (HN - 1);
                }
            }
        }
        __syncthreads();
        hash_ok = sh_misc[6] == 0;
    }
    if (hash_ok) {
        for (uint32_t j = tid; j < HN; j += NT) {
            const uint32_t k = hkeys[j];
            if (k == PF_NONE) continue;
            const uint32_t v = hcnt[j];
            if ((int)(v & 4095u) >= cov && (int)((v >> 16) & 4095u) >= cov) {
                const uint32_t o = k - pmin;
                atomicOr((unsigned long long *)&bmap[o >> 6], 1ull << (o & 63));
            } else hcnt[j] = PF_NONE;
        }
        __syncthreads();
        uint32_t mycount = 0;
#pragma unroll
        for (uint32_t j = 0; j < BW / NT; j++) mycount += (uint32_t)__popcll(bmap[tid * (BW / NT) + j]);
        uint32_t total;
        const uint32_t excl = block_excl_scan<NT>(mycount, sh_scan, &total);
        sh_tbase[tid] = excl;
        {
            uint32_t rank = excl;
            for (uint32_t j = 0; j < BW / NT; j++) {
                const uint32_t wi = tid * (BW / NT) + j;
                uint64_t bits = bmap[wi];
                while (bits) {
                    const uint32_t b = __ffsll((unsigned long long)bits) - 1;
                    bits &= bits - 1;
                    if (rank < scap) d.site_pos[sb + rank] = pmin + wi * 64 + b;
                    else atomicOr(d.status, PF_ST_SITE_OVF);
                    rank++;
                }
            }
        }
        __syncthreads();
        for (uint32_t j = tid; j < HN; j += NT) {
            const uint32_t k = hkeys[j];
            if (k == PF_NONE || hcnt[j] == PF_NONE) continue;
            const uint32_t o = k - pmin, wi = o >> 6, t = wi / (BW / NT);
            uint32_t rk = sh_tbase[t];
            for (uint32_t q = t * (BW / NT); q < wi; q++) rk += (uint32_t)__popcll(bmap[q]);
            rk += (uint32_t)__popcll(bmap[wi] & ((1ull << (o & 63)) - 1ull));
            hcnt[j] = rk;
        }
        __syncthreads();
        for (uint32_t i = wid; i < R; i += NW) {
            const uint32_t r = r0 + i;
            const uint64_t c0 = d.read_call_off[r], c1 = d.read_call_off[r + 1];
            for (uint64_t c = c0 + lane; c < c1; c += 64) {
                const uint32_t pos = d.call_pos[c];
                const bool first = (c == c0) || d.call_pos[c - 1] != pos;
                uint32_t v = PF_NONE;
                if (first) {
                    uint32_t h = (pos * 2654435761u) >> 19;
                    for (;;) {
                        const uint32_t k = hkeys[h];
                        if (k == pos) { v = hcnt[h]; break; }
                        if (k == PF_NONE) break;
                        h = (h + 1) & (HN - 1);
                    }
                }
                d.call_site[c] = v;
            }
        }
        if (tid == 0) sh_misc[4] = total;
        __syncthreads();
    }
    // ---- general path: dense per-position counts, tile by tile, in position order
    for (uint64_t base = pmin; !hash_ok && base <= pmax; base += PF_K1_TILE) {
        const uint64_t top = base + PF_K1_TILE;
        for (uint32_t j = tid; j < PF_K1_TILE; j += NT) tile[j] = 0;
        __syncthreads();
        for (uint32_t i = wid; i < R; i += NW) {
            const uint32_t r = r0 + i;
            const uint64_t c0 = d.read_call_off[r], c1 = d.read_call_off[r + 1];
            if (c1 == c0) continue;
            if ((uint64_t)d.call_pos[c1 - 1] < base || (uint64_t)d.call_pos[c0] >= top) continue;
            const uint64_t lo = lb_u32(d.call_pos, c0, c1, (uint32_t)base);
            const uint64_t hi = top > 0xFFFFFFFFull ? c1 : lb_u32(d.call_pos, lo, c1, (uint32_t)top);
            for (uint64_t c = lo + lane; c < hi; c += 64) {
                const uint32_t cat = d.call_cat[c];
                if (cat < 2) atomicAdd(&tile[d.call_pos[c] - (uint32_t)base], cat == 0 ? 1u : 0x10000u);
            }
        }
        __syncthreads();
        // each thread owns 32 consecutive positions, visited in a rotated order
        // (bank = (j + tid) mod 32: conflict-free)
        uint32_t qmask = 0;
#pragma unroll 8
        for (uint32_t jj = 0; jj < 32; jj++) {
            const uint32_t j = (jj + tid) & 31;
            const uint32_t v = tile[tid * 32 + j];
            // counts are uint16 holding count<<4 in the reference: count mod 4096 (blockjoin.c:3236)
            if ((int)(v & 4095u) >= cov && (int)((v >> 16) & 4095u) >= cov) qmask |= 1u << j;
        }
        uint32_t total;
        const uint32_t excl = block_excl_scan<NT>((uint32_t)__popc(qmask), sh_scan, &total);
        const uint32_t srun = sh_misc[4];
        {
            uint32_t m = qmask, rank = srun + excl;
            while (m) {
                const uint32_t j = __ffs(m) - 1;
                m &= m - 1;
                if (rank < scap) d.site_pos[sb + rank] = (uint32_t)base + tid * 32 + j;
                else atomicOr(d.status, PF_ST_SITE_OVF);
                rank++;
            }
        }
#pragma unroll 8
        for (uint32_t jj = 0; jj < 32; jj++) {
            const uint32_t j = (jj + tid) & 31;
            const uint32_t below = (uint32_t)__popc(qmask & ((1u << j) - 1u));
            tile[tid * 32 + j] = ((qmask >> j) & 1u) ? srun + excl + below : PF_NONE;
        }
        __syncthreads();
        if (tid == 0) sh_misc[4] = srun + total;
        // label calls with their site index (first call at a position only)
        for (uint32_t i = wid; i < R; i += NW) {
            const uint32_t r = r0 + i;
            const uint64_t c0 = d.read_call_off[r], c1 = d.read_call_off[r + 1];
            if (c1 == c0) continue;
            if ((uint64_t)d.call_pos[c1 - 1] < base || (uint64_t)d.call_pos[c0] >= top) continue;
            const uint64_t lo = lb_u32(d.call_pos, c0, c1, (uint32_t)base);
            const uint64_t hi = top > 0xFFFFFFFFull ? c1 : lb_u32(d.call_pos, lo, c1, (uint32_t)top);
            for (uint64_t c = lo + lane; c < hi; c += 64) {
                const uint32_t pos = d.call_pos[c];
                const bool first = (c == c0) || d.call_pos[c - 1] != pos;
                d.call_site[c] = first ? tile[pos - (uint32_t)base] : PF_NONE;
            }
        }
        __syncthreads();
    }
    uint32_t S = sh_misc[4];
    if (S > scap) S = scap;
    if (tid == 0) d.win_S[w] = S;

    // ---- directional methmer lengths/starts (blockjoin.c:3307-3329)
    const uint32_t *a = d.site_pos + sb;
    const uint32_t k = (uint32_t)d.k, span = (uint32_t)d.k_span;
    for (uint32_t p = tid; p < S; p += NT) {
        const uint32_t ap = a[p];
        uint32_t j = p + k > S - 1 ? S - 1 : p + k;
        while (a[j] - ap > span) j--;
        d.len0[sb + p] = (uint8_t)(j == p ? 1 : j - p);
        uint32_t q = p > k ? p - k : 0;
        while (ap - a[q] > span) q++;
        d.len1[sb + p] = (uint8_t)(q == p ? 1 : p - q);
        d.st1_pos[sb + p] = a[q];
        d.site_q1[sb + p] = q;
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
                if (bound > PF_K2_ENT_CAP) bigb = 16 * bound;
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
    uint64_t kcarry = sh_base[0], bcarry = sh_base[1];
    for (uint32_t i0 = 0; i0 < R; i0 += NT) {
        const uint32_t i = i0 + tid;
        uint32_t bound = 0, bigb = 0;
        if (i < R) {
            bound = d.mmr_cap[r0 + i];
            if (bound > PF_K2_ENT_CAP) bigb = 16 * bound;
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
}

// ========================================================================
// K2: methmers of one read in one direction (one wavefront)
// ========================================================================
template <bool LDSBUF>
DEV void k2_one(const pf_dev_batch &d, uint32_t r, uint32_t dir, uint32_t lane, uint8_t *chars,
                uint8_t *crank, uint32_t *irank) {
    const uint32_t g = 2 * r + dir;
    const uint32_t w = d.read_win[r];
    const uint32_t S = d.win_S[w];
    const uint64_t c0 = d.read_call_off[r], c1 = d.read_call_off[r + 1];
    uint32_t total = 0, start_i = PF_NONE;
    if (S > 0 && c1 > c0) {
        const uint64_t sb = d.win_site_off[w];
        const uint32_t *st = (dir ? d.st1_pos : d.site_pos) + sb;
        const uint8_t *lens = (dir ? d.len1 : d.len0) + sb;
        const uint32_t *q1 = d.site_q1 + sb;
        const uint32_t F = d.read_first[r], L = d.read_last[r];
        const uint32_t sfirst = st[0], slast = st[S - 1];
        // search_arr on sites_starts (blockjoin.c:3375-3384); sites_starts is
        // non-decreasing in both directions, so search_arr1 = lower bound.
        if (!(F > slast || L < sfirst)) {
            uint32_t xl, xr;
            if (F < sfirst) xl = 0;
            else {
                const uint32_t lb = (uint32_t)lb_u32(st, 0, S, F);
                xl = st[lb] == F ? lb : (lb ? lb - 1 : 0);
            }
            xr = L > slast ? S : (uint32_t)lb_u32(st, 0, S, L);
            if (xl < xr) {
                const uint32_t qlo = dir ? q1[xl] : xl;
                const uint32_t qhi = dir ? q1[xr - 1] + 1 : xr;
                const uint32_t nq = qhi - qlo;
                const uint32_t cap = d.mmr_cap[r];
                if (LDSBUF && (nq > PF_K2_ENT_CAP || xr - xl > PF_K2_ENT_CAP)) {
                    if (lane == 0) atomicOr(d.status, PF_ST_INTERNAL);
                } else {
                    // methylation character of each site for this read:
                    // m/u/- = category of the first call at the site, or '-' (2)
                    for (uint32_t j = lane; j < nq; j += 64) chars[j] = 2;
                    wave_sync();
                    for (uint64_t c = c0 + lane; c < c1; c += 64) {
                        const uint32_t si = d.call_site[c];
                        if (si != PF_NONE && si >= qlo && si < qhi) chars[si - qlo] = d.call_cat[c];
                    }
                    wave_sync();
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
                            irank[rk] = i;
                        }
                        E += (uint32_t)__popcll(m);
                    }
                    wave_sync();
                    if (E > 0) {
                        // the buffer's last element is never a walk position (:3420)
                        const uint32_t maxcall = d.call_pos[c1 - 1];
                        const uint32_t usable = E - (st[irank[E - 1]] > maxcall ? 1u : 0u);
                        // duplicated start at indices 0 and 1: entry 0 is followed by
                        // another site entry, so its character is '-'
                        if (lane == 0 && E >= 2 && irank[0] == 0 && irank[1] == 1 && st[1] == st[0])
                            crank[0] = 2;
                        wave_sync();
                        uint32_t *out = d.keys + d.mmr_off[g];
                        const uint64_t room = d.keys_cap > d.mmr_off[g] ? d.keys_cap - d.mmr_off[g] : 0;
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
                            const uint32_t incl = wave_incl_scan(ne, lane);
                            const uint32_t tot = __shfl(incl, 63, 64);
                            if (start_i == PF_NONE && tot > 0) {
                                const uint64_t m = __ballot(ne > 0);
                                const int src = __ffsll((unsigned long long)m) - 1;
                                start_i = __shfl(fj, src, 64);
                            }
                            if (ne) {
                                uint32_t pos = total + incl - ne;
                                for (uint32_t j = i; j < S && st[j] == P; j++) {
                                    const uint32_t Lj = lens[j];
                                    if (e + Lj <= usable) {
                                        uint32_t key = 0;
                                        for (uint32_t t = 0; t < Lj; t++) key = key << 2 | crank[e + t];
                                        if (pos < cap && pos < room) out[pos] = key;
                                        pos++;
                                    }
                                }
                            }
                            total += tot;
                        }
                        if (total > cap && lane == 0) atomicOr(d.status, PF_ST_KEYS_OVF);
                    }
                }
            }
        }
    }
    if (lane == 0) {
        d.mmr_n[g] = total;
        d.mmr_start[g] = total ? start_i : 0;   // store_mmr_of_one_read (:3518-3522)
    }
}

__global__ __launch_bounds__(PF_K2_WAVES * 64) void pf_k2_methmers(pf_dev_batch d) {
    __shared__ uint8_t s_chars[PF_K2_WAVES][PF_K2_ENT_CAP];
    __shared__ uint8_t s_crank[PF_K2_WAVES][PF_K2_ENT_CAP];
    __shared__ uint32_t s_irank[PF_K2_WAVES][PF_K2_ENT_CAP];
    const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint64_t gw = (uint64_t)blockIdx.x * PF_K2_WAVES + wid;
    if (gw >= 2ull * d.R) return;
    const uint32_t r = (uint32_t)(gw >> 1), dir = (uint32_t)(gw & 1);
    const uint64_t bo = d.big_off[r];
    if (bo == ~0ull) {
        k2_one<true>(d, r, dir, lane, s_chars[wid], s_crank[wid], s_irank[wid]);
    } else {
        // large read: HBM scratch reserved by K1, 16 bytes per bound entry:
        // per direction [chars cap][crank cap][pad][irank 4*cap] at dir*8*cap
        const uint32_t cap = d.mmr_cap[r];
        if (bo + 16ull * cap > d.big_cap) {
            if (lane == 0) { d.mmr_n[2 * r + dir] = 0; d.mmr_start[2 * r + dir] = 0; atomicOr(d.status, PF_ST_BIG_OVF); }
            return;
        }
        uint8_t *b = d.big + bo + (dir ? 8ull * cap : 0);
        k2_one<false>(d, r, dir, lane, b, b + cap, reinterpret_cast<uint32_t *>(b + 4ull * cap));
    }
}

// ========================================================================
// K3: greedy haplotag extension of one (window, direction)
// ========================================================================
struct K3Ctl {
    uint32_t S, R, ntot, nc, L, done, failed, inserted, winner, tag;
    int32_t i_last;
    uint32_t min_i, max_i, fail, summ, nstrict;
    unsigned long long scr;
    unsigned long long wbest[PF_K3_WAVES];
    int32_t tab[4];
};

struct K3Cand {
    uint32_t read[PF_MAX_NCAND];
    uint32_t pos[PF_MAX_NCAND];
    uint32_t site0[PF_MAX_NCAND];
    uint32_t len[PF_MAX_NCAND];
    uint64_t kofs[PF_MAX_NCAND];
    uint8_t tag[PF_MAX_NCAND];
};

DEV uint64_t align16(uint64_t x) { return (x + 15) & ~15ull; }

// dictionary of methmer keys per site -> dense slot ids (replaces the per-site
// key lists + linear search of insert_mmrs_to_counts / query_counts_of_mmrs)
template <bool LDS1>
DEV void k3_dict(const pf_dev_batch &d, uint32_t r0, uint32_t R, uint32_t S, uint32_t dir,
                 uint64_t *masks, uint32_t *base, uint32_t *sh_scan, K3Ctl &ctl) {
    const uint32_t tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const uint32_t MW = (uint32_t)d.mw;
    for (uint32_t j = tid; j < S * MW; j += PF_K3_THREADS) masks[j] = 0;
    __syncthreads();
    for (uint32_t i = wid; i < R; i += PF_K3_WAVES) {
        const uint32_t g = 2 * (r0 + i) + dir;
        const uint32_t n = d.mmr_n[g], st = d.mmr_start[g];
        const uint32_t *kp = d.keys + d.mmr_off[g];
        for (uint32_t t = lane; t < n; t += 64) {
            const uint32_t site = st + t;
            const uint32_t key = kp[t];
            if (site < S && key < 64u * MW)
                atomicOr((unsigned long long *)&masks[(uint64_t)site * MW + (key >> 6)], 1ull << (key & 63));
        }
    }
    __syncthreads();
    uint32_t carry = 0;
    for (uint32_t p0 = 0; p0 < S; p0 += PF_K3_THREADS) {
        const uint32_t p = p0 + tid;
        uint32_t c = 0;
        if (p < S)
            for (uint32_t m = 0; m < MW; m++) c += (uint32_t)__popcll(masks[(uint64_t)p * MW + m]);
        uint32_t tot;
        const uint32_t ex = block_excl_scan<PF_K3_THREADS>(c, sh_scan, &tot);
        if (p < S) base[p] = carry + ex;
        carry += tot;
    }
    if (tid == 0) ctl.ntot = carry;
    __syncthreads();
    for (uint32_t i = wid; i < R; i += PF_K3_WAVES) {
        const uint32_t g = 2 * (r0 + i) + dir;
        const uint32_t n = d.mmr_n[g], st = d.mmr_start[g];
        uint32_t *kp = d.keys + d.mmr_off[g];
        for (uint32_t t = lane; t < n; t += 64) {
            const uint32_t site = st + t;
            uint32_t slot = PF_NONE;
            const uint32_t key = kp[t];
            if (site < S && key < 64u * MW) {
                const uint64_t *row = masks + (uint64_t)site * MW;
                const uint32_t wi = key >> 6, b = key & 63;
                slot = base[site];
                for (uint32_t m = 0; m < wi; m++) slot += (uint32_t)__popcll(row[m]);
                slot += (uint32_t)__popcll(row[wi] & ((1ull << b) - 1ull));
            }
            kp[t] = slot;
        }
    }
    __syncthreads();
}

struct K3Mem {
    uint32_t *sum, *cnt, *aux, *ord, *mn, *mst, *mo;
    uint8_t *hp, *flg;
    uint64_t *untag;
    float2 *recv;
    uint32_t *recc;
    uint32_t rc;        // record capacity (multiple of ncp)
};

#define K3_NOFF 11
// P2 byte layout for given sizes; returns the bytes needed before the records
DEV uint64_t k3_layout(uint32_t S, uint32_t ntot, uint32_t R, uint32_t dir, uint64_t off[K3_NOFF]) {
    const uint32_t nwords = (R + 63) >> 6;
    off[0] = 0;                                        // sum   S*4
    off[1] = align16(off[0] + 4ull * S);               // cnt   ntot*4
    off[2] = align16(off[1] + 4ull * ntot);            // hp    R
    off[3] = align16(off[2] + R);                      // flg   R
    off[4] = align16(off[3] + R);                      // aux   R*4
    off[5] = align16(off[4] + 4ull * R);               // ord   R*4 (dir 1)
    off[6] = align16(off[5] + (dir ? 4ull * R : 0));   // untag nwords*8
    off[7] = align16(off[6] + 8ull * nwords);          // mn    R*4  methmers per read
    off[8] = align16(off[7] + 4ull * R);               // mst   R*4  first site index
    off[9] = align16(off[8] + 4ull * R);               // mo    R*4  key offset (window-relative)
    off[10] = align16(off[9] + 4ull * R);              // records
    return off[10];
}

DEV void k3_mem(uint8_t *base, const uint64_t off[K3_NOFF], uint32_t rc, K3Mem &m) {
    m.sum = reinterpret_cast<uint32_t *>(base + off[0]);
    m.cnt = reinterpret_cast<uint32_t *>(base + off[1]);
    m.hp = base + off[2];
    m.flg = base + off[3];
    m.aux = reinterpret_cast<uint32_t *>(base + off[4]);
    m.ord = reinterpret_cast<uint32_t *>(base + off[5]);
    m.untag = reinterpret_cast<uint64_t *>(base + off[6]);
    m.mn = reinterpret_cast<uint32_t *>(base + off[7]);
    m.mst = reinterpret_cast<uint32_t *>(base + off[8]);
    m.mo = reinterpret_cast<uint32_t *>(base + off[9]);
    m.recv = reinterpret_cast<float2 *>(base + off[10]);
    m.recc = reinterpret_cast<uint32_t *>(base + off[10] + 8ull * rc);
    m.rc = rc;
}

#define FLG_LEFT 1u
#define FLG_LEFT_STRICT 2u
#define FLG_RIGHT 4u
#define FLG_RIGHT_STRICT 8u

// update_available_methmer_range (blockjoin.c:3669-3691), one wavefront
DEV void k3_range_update(const uint32_t *sum, uint32_t S, int cov_rt, K3Ctl &ctl, uint32_t lane) {
    // left: extend down from (int)min_i while covered
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
    // right: extend up from (int)max_i while covered; max_i = last covered index
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

// per-problem counters for the algorithmic-byte model (B_tag)
struct K3Stats {
    unsigned long long lookups, inserts, iters, scanned;
};
#define PF_NSTAT 8

// step 1 of an iteration (wave 0 only): collect up to NC untagged reads in scan
// order from i_last (:4037-4045); empty batches advance i_last (:4046-4051).
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
        uint32_t found = 0;
        if (dir == 0) {
            const uint32_t w0 = (uint32_t)il >> 6;
            for (uint32_t wb = w0; wb < nwords && found < NC; wb += 64) {
                const uint32_t wi = wb + lane;
                uint64_t bits = wi < nwords ? m.untag[wi] : 0ull;
                if (wi == w0) bits &= ~0ull << ((uint32_t)il & 63);
                const uint32_t c = (uint32_t)__popcll(bits);
                const uint32_t incl = wave_incl_scan(c, lane);
                uint32_t rk = found + incl - c;
                while (bits && rk < NC) {
                    const uint32_t b = __ffsll((unsigned long long)bits) - 1;
                    cd.pos[rk++] = wi * 64 + b;
                    bits &= bits - 1;
                }
                found += __shfl(incl, 63, 64);
            }
        } else {
            const int w0 = il >> 6;
            for (int wb = w0; wb >= 0 && found < NC; wb -= 64) {
                const int wi = wb - (int)lane;
                uint64_t bits = wi >= 0 ? m.untag[wi] : 0ull;
                if (wi == w0) {
                    const uint32_t b = (uint32_t)il & 63;
                    bits &= b == 63 ? ~0ull : ((1ull << (b + 1)) - 1ull);
                }
                const uint32_t c = (uint32_t)__popcll(bits);
                const uint32_t incl = wave_incl_scan(c, lane);
                uint32_t rk = found + incl - c;
                while (bits && rk < NC) {
                    const uint32_t b = 63 - __clzll((long long)bits);
                    cd.pos[rk++] = (uint32_t)wi * 64 + b;
                    bits &= ~(1ull << b);
                }
                found += __shfl(incl, 63, 64);
            }
        }
        const uint32_t nc = found < NC ? found : NC;
        wave_sync();
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
        if (found >= NC) {
            const uint32_t pl = cd.pos[NC - 1];
            stx.scanned += dir == 0 ? pl - (uint32_t)il + 1 : (uint32_t)il - pl + 1;
        } else stx.scanned += dir == 0 ? (uint32_t)((int)R - il) : (uint32_t)(il + 1);
        uint32_t lmax = 0, lsum = 0;
        const uint32_t mn_ = ctl.min_i, mx_ = ctl.max_i;
        for (uint32_t c = lane; c < nc; c += 64) {
            const uint32_t p = cd.pos[c];
            const uint32_t rd = dir ? m.ord[p] : p;
            const uint32_t n = m.mn[rd], st = m.mst[rd];
            // in-range methmers: site index in [min_i, max_i) (query_counts_of_mmrs, :3500-3501)
            const uint64_t lo = st > mn_ ? st : mn_;
            const uint64_t hi0 = (uint64_t)st + n;
            const uint64_t hi = hi0 < mx_ ? hi0 : mx_;
            const uint32_t len = hi > lo ? (uint32_t)(hi - lo) : 0;
            cd.read[c] = rd;
            cd.site0[c] = (uint32_t)lo;
            cd.len[c] = len;
            cd.kofs[c] = (uint64_t)m.mo[rd] + (len ? (lo - st) : 0);
            lmax = len > lmax ? len : lmax;
            lsum += len;
        }
        lmax = wave_max_u32(lmax);
        lsum = wave_incl_scan(lsum, lane);
        stx.lookups += __shfl(lsum, 63, 64);
        stx.iters++;
        if (lane == 0) { ctl.done = 0; ctl.nc = nc; ctl.L = lmax; ctl.i_last = il; ctl.failed = failed; }
        wave_sync();
        return;
    }
}

template <bool LDS2>
DEV void k3_greedy_body(const pf_dev_batch &d, uint32_t w, uint32_t dir, uint32_t r0, uint32_t S,
                        uint32_t R, const K3Mem &m, K3Ctl &ctl, K3Cand &cd) {
    const uint32_t tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const uint32_t ntot = ctl.ntot;
    const int cov_rt = d.win_par[w * 4 + 1];
    const uint32_t NC = (uint32_t)d.win_par[w * 4 + 2];
    const uint32_t s = d.win_start[w], e = d.win_end[w];
    const uint32_t nwords = (R + 63) >> 6;
    const uint64_t sb = d.win_site_off[w];
    const uint32_t ncp = next_pow2(NC);
    const uint32_t lg = 31 - __clz(ncp);
    const uint64_t kbase = d.mmr_off[2ull * r0];
    const uint32_t *kb = d.keys + kbase;
    K3Stats stx = {0, 0, 0, 0};
    uint32_t sum_mmr = 0;
#ifdef PF_K3_PROFILE
    unsigned long long prof_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long prof_last = __builtin_amdgcn_s_memtime();
#endif

    // ---- init tables and per-read state
    for (uint32_t j = tid; j < ntot; j += PF_K3_THREADS) m.cnt[j] = 0;
    for (uint32_t j = tid; j < S; j += PF_K3_THREADS) m.sum[j] = 0;
    for (uint32_t i = tid; i < R; i += PF_K3_THREADS) {
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
        if (dir) m.ord[i] = d.rev_ord[r];
        const uint64_t g = 2ull * r + dir;
        m.mn[i] = d.mmr_n[g];
        sum_mmr += m.mn[i];
        m.mst[i] = d.mmr_start[g];
        m.mo[i] = (uint32_t)(d.mmr_off[g] - kbase);
    }
    if (tid == 0) {
        // haplotag_region1 step 1 (blockjoin.c:3976-4004)
        const uint32_t *a = d.site_pos + sb;
        if (dir == 0) {
            ctl.min_i = 0;
            ctl.max_i = (uint32_t)ub_u32(a, 0, S, s);            // #sites <= ref_start
        } else {
            ctl.max_i = S - 1;
            ctl.min_i = (uint32_t)((int)ub_u32(a, 0, S, e) - 1); // may wrap to UINT32_MAX
        }
        ctl.i_last = dir == 0 ? 0 : (int)R - 1;
        ctl.failed = 0;
        ctl.done = 0;
        ctl.tab[0] = 0;
    }
    __syncthreads();
    // ---- reference reads seed the counts (insert_ref_reads_methmer_counts, :3776-3810)
    const uint32_t refbit = dir == 0 ? FLG_LEFT : FLG_RIGHT;
    uint32_t ref_ins = 0;
    for (uint32_t i = wid; i < R; i += PF_K3_WAVES) {
        const uint32_t hp = m.hp[i];
        if (!(m.flg[i] & refbit) || hp > 1) continue;
        const uint32_t n = m.mn[i], st = m.mst[i];
        const uint32_t *kp = kb + m.mo[i];
        const uint32_t inc = hp ? 0x10000u : 1u;
        ref_ins += n;
        for (uint32_t t = lane; t < n; t += 64) {
            const uint32_t site = st + t;
            const uint32_t slot = kp[t];
            if (site < S && slot != PF_NONE) {
                atomicAdd(&m.cnt[slot], inc);
                atomicAdd(&m.sum[site], inc);
            }
        }
    }
    if (lane == 0 && ref_ins) atomicAdd((uint32_t *)&ctl.tab[0], ref_ins);
    if (sum_mmr) atomicAdd(&ctl.summ, sum_mmr);
    __syncthreads();
    if (wid == 0) k3_range_update(m.sum, S, cov_rt, ctl, lane);
    // ---- step 1.5 (:4010-4025): all reads unphased, ref reads restored through
    // the (readID<<2)|hp round trip (hp >= 4 lands on readID|(hp>>2)); the last
    // writer in reference order wins.
    for (uint32_t i = tid; i < R; i += PF_K3_THREADS) {
        if (m.flg[i] & refbit) {
            const uint32_t t = i | ((uint32_t)m.hp[i] >> 2);
            if (t < R) atomicMax(&m.aux[t], i + 1);
        }
    }
    __syncthreads();
    for (uint32_t i = tid; i < R; i += PF_K3_THREADS) {
        const uint32_t lw = m.aux[i];
        m.hp[i] = lw ? (uint8_t)(d.read_hp[r0 + lw - 1] & 3) : (uint8_t)2;
    }
    __syncthreads();
    // untagged bitmask in scan order (dir 0: read order, dir 1: revbuf order)
    for (uint32_t j = wid; j < nwords; j += PF_K3_WAVES) {
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

    // ---- step 2: greedy extension, one read per iteration (:4032-4071)
    // Barriers per iteration: (a) candidates ready, (b) records ready, (c) keys
    // ready.  Winner pick, insertion, range update and the next candidate scan
    // run in wavefront 0 between (c) and the next (a).
    K3_STAMP(0);
    if (wid == 0) k3_collect(m, R, dir, NC, lane, ctl, cd, stx);
    K3_STAMP(1);
    for (;;) {
        __syncthreads();                                         // (a)
        K3_STAMP(2);
        if (ctl.done) break;
        const uint32_t nc = ctl.nc;
        const uint32_t L = ctl.L;
        const uint32_t lc = m.rc >> lg;                           // t-steps per record chunk
        float s0 = 0.f, s1 = 0.f;
        uint32_t lcode = 0;
        for (uint32_t t0 = 0; t0 < L; t0 += lc) {
            const uint32_t t1 = t0 + lc < L ? t0 + lc : L;
            const uint32_t nrec = (t1 - t0) << lg;
            for (uint32_t idx = tid; idx < nrec; idx += PF_K3_THREADS) {
                const uint32_t t = t0 + (idx >> lg), c = idx & (ncp - 1);
                float v0 = 0.f, v1 = 0.f;
                uint32_t code = 0;
                if (c < nc && t < cd.len[c]) {
                    const uint32_t site = cd.site0[c] + t;
                    const uint32_t slot = kb[cd.kofs[c] + t];
                    const uint32_t cv = slot != PF_NONE ? m.cnt[slot] : 0u;
                    if (cv != 0) {                               // key present at this site
                        const uint32_t sv = m.sum[site];
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
            K3_STAMP(3);
            __syncthreads();                                     // (b)
            K3_STAMP(4);
            if (tid < nc) {
                // sequential in methmer order; absent terms are +0.0f and leave the
                // float sum unchanged
                const uint32_t n = t1 - t0;
                const float2 *rv = m.recv + tid;
                const uint32_t *rcc = m.recc + tid;
                uint32_t t = 0;
                for (; t + 8 <= n; t += 8) {
                    float2 v[8];
                    uint32_t cc[8];
#pragma unroll
                    for (int u = 0; u < 8; u++) { v[u] = rv[(t + u) << lg]; cc[u] = rcc[(t + u) << lg]; }
#pragma unroll
                    for (int u = 0; u < 8; u++) { s0 += v[u].x; s1 += v[u].y; lcode += cc[u]; }
                }
                for (; t < n; t++) {
                    const float2 v = rv[t << lg];
                    s0 += v.x;
                    s1 += v.y;
                    lcode += rcc[t << lg];
                }
            }
            if (t1 < L) __syncthreads();
        }
        // use_mmr_count_predict_tag_for_one_read (:3637-3655) + best pick (:3729-3766)
        unsigned long long key = 0;
        if (tid < nc) {
            const float diff = s0 > s1 ? s0 - s1 : s1 - s0;
            const int l0 = (int)(lcode & 0xffffu), l1 = (int)(lcode >> 16);
            const bool untagged = diff < 3.f && (l0 < 3 || l1 < 3);
            cd.tag[tid] = s0 > s1 ? 0 : 1;
            if (!untagged) key = ((unsigned long long)__float_as_uint(diff) << 32) | (tid + 1);
        }
        key = wave_max_u64(key);
        if (lane == 0) ctl.wbest[wid] = key;
        K3_STAMP(5);
        __syncthreads();                                         // (c)
        K3_STAMP(6);
        if (wid == 0) {
            unsigned long long b = 0;
            for (int i = 0; i < PF_K3_WAVES; i++) b = ctl.wbest[i] > b ? ctl.wbest[i] : b;
            if (b == 0) {
                // nothing could be tagged (:4064-4069)
                const uint32_t f = ctl.failed + 1;
                wave_sync();
                if (lane == 0) {
                    ctl.failed = f;
                    if (f > 10) ctl.done = 1;
                    else ctl.i_last += dir == 0 ? (int)NC : -(int)NC;
                }
                wave_sync();
            } else {
                const uint32_t c = (uint32_t)(b & 0xffffffffu) - 1;
                const uint32_t rd = cd.read[c];
                const uint32_t tg = cd.tag[c];
                const uint32_t p = cd.pos[c];
                const uint32_t n = m.mn[rd], st = m.mst[rd];
                const uint32_t *kp = kb + m.mo[rd];
                const uint32_t inc = tg ? 0x10000u : 1u;
                stx.inserts += n;
                // the sites of one read are distinct: plain read-modify-write
                for (uint32_t t = lane; t < n; t += 64) {
                    const uint32_t site = st + t;
                    const uint32_t slot = kp[t];
                    if (site < S && slot != PF_NONE) {
                        m.cnt[slot] += inc;
                        m.sum[site] += inc;
                    }
                }
                if (lane == 0) {
                    ctl.failed = 0;
                    m.hp[rd] = (uint8_t)tg;
                    m.untag[p >> 6] &= ~(1ull << (p & 63));
                }
                wave_sync();
                k3_range_update(m.sum, S, cov_rt, ctl, lane);
            }
            K3_STAMP(7);
            if (!ctl.done) k3_collect(m, R, dir, NC, lane, ctl, cd, stx);
            K3_STAMP(1);
        }
    }

    // ---- 2x2 table on the opposite side's strict reads (evaluate_separation, :3940-3956)
    if (tid < 4) ctl.tab[tid] = 0;
    __syncthreads();
    const uint32_t strict = dir == 0 ? FLG_RIGHT_STRICT : FLG_LEFT_STRICT;
    for (uint32_t i = tid; i < R; i += PF_K3_THREADS) {
        if (m.flg[i] & strict) {
            atomicAdd(&ctl.nstrict, 1u);
            const uint32_t ref = d.read_hp[r0 + i], q = m.hp[i];
            if (ref <= 1 && q <= 1) atomicAdd(&ctl.tab[ref * 2 + q], 1);
        }
        if (dir == 0) d.hp_fwd[r0 + i] = m.hp[i];
    }
    __syncthreads();
    if (tid < 4) d.table[((uint64_t)w * 2 + dir) * 4 + tid] = ctl.tab[tid];
    if (tid == 0) {
        unsigned long long *sp = d.stats + ((uint64_t)w * 2 + dir) * PF_NSTAT;
        sp[0] = stx.lookups; sp[1] = stx.inserts; sp[2] = stx.iters; sp[3] = stx.scanned;
        sp[4] = ctl.summ; sp[5] = ctl.nstrict; sp[6] = R; sp[7] = S;
#ifdef PF_K3_PROFILE
        unsigned long long *pp = d.prof + ((uint64_t)w * 2 + dir) * 8;
        for (int i = 0; i < 8; i++) pp[i] = prof_acc[i];
#endif
    }
}

__global__ __launch_bounds__(PF_K3_THREADS) void pf_k3_greedy(pf_dev_batch d) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    __shared__ K3Ctl ctl;
    __shared__ K3Cand cd;
    __shared__ uint32_t sh_scan[PF_K3_WAVES + 1];
    const uint32_t tid = threadIdx.x;
    const uint32_t w = blockIdx.x >> 1, dir = blockIdx.x & 1;
    const uint32_t S = d.win_S[w];
    if (S == 0) {
        if (tid < 4) d.table[((uint64_t)w * 2 + dir) * 4 + tid] = 0;
        if (tid < PF_NSTAT) d.stats[((uint64_t)w * 2 + dir) * PF_NSTAT + tid] = 0;
        return;
    }
    const uint32_t R = d.win_nreads[w];
    const uint32_t r0 = d.win_read_off[w];
    const uint32_t MW = (uint32_t)d.mw;
    const uint32_t NC = (uint32_t)d.win_par[w * 4 + 2];
    const uint32_t ncp = next_pow2(NC);

    // ---- P1: slot dictionary
    const uint64_t need1 = align16(8ull * S * MW) + 4ull * S;
    const bool p1_lds = need1 <= d.lds_bytes;
    if (tid == 0) {
        ctl.fail = 0;
        ctl.summ = 0;
        ctl.nstrict = 0;
        if (!p1_lds) {
            const unsigned long long o = atomicAdd(d.scr_ctr, (unsigned long long)align16(need1));
            if (o + need1 > d.scr_cap) { ctl.fail = 1; atomicOr(d.status, PF_ST_SCR_OVF); }
            ctl.scr = o;
        }
    }
    __syncthreads();
    if (ctl.fail) return;
    if (p1_lds) {
        k3_dict<true>(d, r0, R, S, dir, reinterpret_cast<uint64_t *>(smem),
                      reinterpret_cast<uint32_t *>(smem + align16(8ull * S * MW)), sh_scan, ctl);
    } else {
        uint8_t *g = d.scr + ctl.scr;
        k3_dict<false>(d, r0, R, S, dir, reinterpret_cast<uint64_t *>(g),
                       reinterpret_cast<uint32_t *>(g + align16(8ull * S * MW)), sh_scan, ctl);
    }
    const uint32_t ntot = ctl.ntot;

    // ---- P2: greedy
    uint64_t off[K3_NOFF];
    const uint64_t fixed = k3_layout(S, ntot, R, dir, off);
    const uint64_t min_rec = 12ull * ncp * 8;
    const bool p2_lds = fixed + min_rec <= d.lds_bytes;
    const uint32_t lgc = 31 - __clz(ncp);
    if (p2_lds) {
        uint32_t rc = (uint32_t)((d.lds_bytes - fixed) / 12);
        rc = (rc >> lgc) << lgc;
        if (rc > (ncp << 9)) rc = ncp << 9;
        K3Mem m;
        k3_mem(smem, off, rc, m);
        k3_greedy_body<true>(d, w, dir, r0, S, R, m, ctl, cd);
    } else {
        const uint32_t rc = ncp << 8;
        const uint64_t need2 = align16(fixed + 12ull * rc);
        __syncthreads();
        if (tid == 0) {
            const unsigned long long o = atomicAdd(d.scr_ctr, (unsigned long long)need2);
            ctl.fail = 0;
            if (o + need2 > d.scr_cap) { ctl.fail = 1; atomicOr(d.status, PF_ST_SCR_OVF); }
            ctl.scr = o;
        }
        __syncthreads();
        if (ctl.fail) return;
        K3Mem m;
        k3_mem(d.scr + ctl.scr, off, rc, m);
        k3_greedy_body<false>(d, w, dir, r0, S, R, m, ctl, cd);
    }
}
