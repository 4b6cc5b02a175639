/*
 * pf_device.h -- device-side layout shared by the methphase kernels.
 *
 * HBM layout of one resident batch (all SoA, one allocation per array):
 *   windows : win_start/win_end/win_read_off/win_par          [W]
 *   reads   : read_start/end/first/last/win, read_hp           [R]
 *             read_call_off                                     [R+1]
 *   calls   : call_pos (u32), call_cat (u8)                     [N]
 *             calls of a read sorted by (pos, cat)
 *   sites   : per window a slice [site_off[w], +site_cap[w]) of
 *             site_pos, st1_pos, site_q1 (u32) and len0, len1 (u8)
 *   methmers: per (read, dir) a slice of the key arena (u32): methmer keys,
 *             rewritten in place to per-site slot ids before the greedy loop
 */
#ifndef PF_DEVICE_H
#define PF_DEVICE_H
#include <stdint.h>

#define PF_WAVE 64
#define PF_K1_THREADS 1024
#define PF_K1_TILE 32768          /* positions per dense LDS tile (128 KB of u32 counters) */
#define PF_K2_WAVES 4
#define PF_K2_ENT_CAP 1024        /* per-wave LDS entry buffer; larger reads use HBM scratch */
#define PF_K3_THREADS 256
#define PF_K3_WAVES (PF_K3_THREADS / PF_WAVE)
#define PF_K3S_THREADS 256         /* the main (slim) greedy kernel (512 measured: DESIGN.md 8) */
#ifndef PF_K3H_THREADS
#define PF_K3H_THREADS 256         /* pf_k3_heavy (512 measured in round 6: critical window 3.37 -> 3.65 ms, profiles/r06/ab_k3_heavy512.txt) */
#endif
#define PF_MAX_NCAND 256
#define PF_K12_CAPW 512           /* per-wave site-entry buffer of the fused methmer phase */
#define PF_K12_WB 8               /* bytes per wave-buffer entry: chars, crank, u16 irank, u32 staged key */
#define PF_K12_SMAX 4600          /* sites whose arrays (14 B/site) fit LDS beside 16 such buffers */
#define PF_K12C_READS 64          /* reads per item of pf_k12_chunks (the heavy windows' methmer phase) */
#define PF_K12C_WAVES 8           /* its waves per workgroup */
#define PF_K12C_LDS 61440         /* its dynamic LDS: 14 B per site + PF_K12C_WAVES wave buffers (2 per CU) */
#define PF_NONE 0xFFFFFFFFu

/* status bits */
#define PF_ST_KEYS_OVF   1u
#define PF_ST_BIG_OVF    2u
#define PF_ST_SCR_OVF    4u
#define PF_ST_SITE_OVF   8u
#define PF_ST_INTERNAL  16u

struct pf_dev_batch {
    uint32_t W, R;
    uint64_t N;
    int32_t k, k_span, hard_cov, mw;   /* mw: 64-bit mask words per site = max(1, 4^k/64) */
    /* windows */
    const uint32_t *win_start, *win_end, *win_read_off;
    const int32_t *win_par;            /* [W*4]: cov_sel, cov_rt, n_cand, 0 */
    const uint64_t *win_site_off;
    const uint32_t *win_site_cap;
    /* reads */
    const uint32_t *read_start, *read_end, *read_first, *read_last, *read_win;
    const uint8_t *read_hp;
    const uint64_t *read_call_off;
    /* calls */
    const uint32_t *call_pos;
    const uint8_t *call_cat;
    uint32_t *fb_list, *fb_ctr;        /* reads left to the K2 fallback kernel */
    uint32_t *k12c_list, *k12c_ctr;    /* (window, first read) chunks of the heavy windows for pf_k12_chunks */
    uint32_t *k12c_next;               /* pf_k12_chunks' next item */
    uint32_t k12c_minr, k12c_smax;     /* windows with >= k12c_minr reads and <= k12c_smax sites go there */
    /* per-window results of K1 */
    uint32_t *win_S, *win_nreads;
    const uint32_t *k3_order;          /* [2W] greedy problems (w<<1|dir), heaviest first */
    const uint32_t *k12_order;         /* [W] windows for K12's workgroups, heaviest first */
    uint32_t *k3_fb_list, *k3_fb_ctr;  /* problems the main greedy kernel defers to pf_k3_fallback */
    uint32_t *k3_next;                 /* the persistent main greedy kernel's next problem (rank in k3_order) */
    uint32_t k3_n;                     /* its problems: k3_order[0, k3_n) */
    uint32_t *site_pos, *st1_pos, *site_q1;
    uint8_t *len0, *len1;
    uint32_t *rev_ord;                 /* [R] window-local read index, ascending (end, idx) */
    /* methmers */
    uint32_t *mmr_n, *mmr_start;       /* [2R] */
    uint64_t *mmr_off;                 /* [2R] */
    uint32_t *mmr_cap;                 /* [R]  */
    uint64_t *big_off;                 /* [R]  */
    uint32_t *keys; uint64_t keys_cap; unsigned long long *keys_ctr;
    uint8_t *big; uint64_t big_cap; unsigned long long *big_ctr;
    uint8_t *scr; uint64_t scr_cap; unsigned long long *scr_ctr;
    /* the slim greedy loop's per-read side arrays in HBM, when its slot lists
     * miss LDS (k3_side_mem): hp, flg [2R] bytes, ord [R] u16, aux [2R] u32 */
    uint8_t *k3_side;
    /* outputs */
    int32_t *table;                    /* [W*2*4] */
    uint8_t *hp_fwd;                   /* [R] */
    unsigned long long *stats;         /* [W*2*4] per problem: lookups, inserts, iterations, scanned */
    uint32_t *status;
    unsigned long long *prof;          /* [W*2*8] diagnostic build only */
    uint32_t lds_bytes;                /* dynamic LDS of the main greedy kernel */
    uint32_t lds_fb;                   /* dynamic LDS of the fallback greedy kernel (>= lds_bytes) */
    uint32_t lds_heavy;                /* dynamic LDS of pf_k3_heavy (the heavy problems' slim loop) */
    uint32_t lds_w;                    /* dynamic LDS of the one-wave greedy kernel */
    uint32_t k12_capw, k12_smax;       /* fused methmer phase limits (test overrides) */
    uint32_t k12_dense;                /* 1: every window takes K12's dense (HBM) site path (tests) */
    uint32_t k2_entcap;                /* fallback reads above this bound use HBM scratch */
    uint32_t k3_mode;                  /* test override: 0 exact pick, 1 always fold, 2 chunked record rows */
    uint32_t k3_cache;                 /* 1: candidate slot-list cache when a window's lists miss LDS (PF_K3_CACHE=0: off) */
    uint32_t k3_gcnt;                  /* 1: path 6 (cache + count table in HBM) for every cache problem (PF_K3_GCNT=force) */
    /* k > 5 (or PF_K3_KDICT=1): the slot dictionary is built by pf_k3_kdict
     * before the greedy kernels (per-site hash tables in HBM scratch instead
     * of 4^k-bit masks), which rewrite no keys and read ntot from k3_ntot */
    uint32_t kdict;
    uint8_t *k12_path;                 /* [W] K12's sites path of the last run: 1 / 2 the fast path over 1 / 2
                                          segments, 3 the dense path, 0 none (no calls, left coverage) */
    uint32_t *k3_ntot;                 /* [2W] slots of each problem (kdict) */
};

#endif
