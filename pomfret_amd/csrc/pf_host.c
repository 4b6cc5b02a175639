/*
 * pf_host.c -- host-side epilogue of the methphase hot path (product code).
 *
 * After the device has run both greedy directions of every window it returns
 * one 2x2 table per (window, direction).  This file turns those tables into
 * join decisions exactly as the reference does on its CPU:
 *   evaluate_separation1   /root/reference/blockjoin.c:3881-3939
 *   haplotag_region2 summary at n_permutations=1   blockjoin.c:4147-4206
 *   final decision          blockjoin.c:4313-4320
 * and provides the two-sided Fisher exact test the reference takes from
 * htslib (kt_fisher_exact, called at blockjoin.c:3926; htslib kfunc.c,
 * third-party and not vendored in the reference -- restated here from its
 * published algorithm: hypergeometric tail sums via lgamma).
 */
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include "pf_host.h"

/* log k! = lgamma(k + 1) for k < PF_LFACT_N, tabulated once: the same libm
 * values the direct calls return, so the p-values are unchanged bit for bit,
 * at a fraction of the cost (a 2x2 table of a window has n <= 65535 reads). */
#define PF_LFACT_N 65537
static double *pf_lfact;
static pthread_once_t pf_lfact_once = PTHREAD_ONCE_INIT;
static void pf_lfact_init(void) {
    double *t = (double *)malloc(PF_LFACT_N * sizeof(double));
    if (t)
        for (int k = 0; k < PF_LFACT_N; k++) t[k] = lgamma(k + 1);
    pf_lfact = t;
}
static inline double pf_lfac(int k) {
    return (pf_lfact && k >= 0 && k < PF_LFACT_N) ? pf_lfact[k] : lgamma(k + 1);
}

static double pf_lbinom(int n, int k) {
    if (k == 0 || n == k) return 0;
    return pf_lfac(n) - pf_lfac(k) - pf_lfac(n - k);
}

static double pf_hypergeo(int n11, int n1_, int n_1, int n) {
    return exp(pf_lbinom(n1_, n11) + pf_lbinom(n - n1_, n_1 - n11) - pf_lbinom(n, n_1));
}

typedef struct { int n11, n1_, n_1, n; double p; } pf_hgacc_t;

/* incremental hypergeometric probability: moving n11 by +-1 reuses the last
 * value (same recurrence and the same n11%11 re-anchoring as htslib) */
static double pf_hypergeo_acc(int n11, int n1_, int n_1, int n, pf_hgacc_t *h) {
    if (n1_ || n_1 || n) {
        h->n11 = n11; h->n1_ = n1_; h->n_1 = n_1; h->n = n;
    } else {
        if (n11 % 11 && n11 + h->n - h->n1_ - h->n_1) {
            if (n11 == h->n11 + 1) {
                h->p *= (double)(h->n1_ - h->n11) / n11 * (h->n_1 - h->n11) /
                        (n11 + h->n - h->n1_ - h->n_1);
                h->n11 = n11;
                return h->p;
            }
            if (n11 == h->n11 - 1) {
                h->p *= (double)h->n11 / (h->n1_ - n11) * (h->n11 + h->n - h->n1_ - h->n_1) /
                        (h->n_1 - n11);
                h->n11 = n11;
                return h->p;
            }
        }
        h->n11 = n11;
    }
    h->p = pf_hypergeo(h->n11, h->n1_, h->n_1, h->n);
    return h->p;
}

double pf_fisher_exact(int n11, int n12, int n21, int n22, double *left_out, double *right_out,
                       double *two_out) {
    pthread_once(&pf_lfact_once, pf_lfact_init);
    double l_dummy, r_dummy, t_dummy;
    double *pl = left_out ? left_out : &l_dummy;
    double *pr = right_out ? right_out : &r_dummy;
    double *pt = two_out ? two_out : &t_dummy;
    int n1_ = n11 + n12, n_1 = n11 + n21, n = n11 + n12 + n21 + n22;
    int hi = n_1 < n1_ ? n_1 : n1_;      /* largest feasible n11  */
    int lo = n1_ + n_1 - n;              /* smallest feasible n11 */
    if (lo < 0) lo = 0;
    *pt = *pl = *pr = 1.0;
    if (lo == hi) return 1.0;
    pf_hgacc_t h;
    double q = pf_hypergeo_acc(n11, n1_, n_1, n, &h);
    if (q == 0.0) {  /* underflow: both tails ~0; report the closer side as 0 */
        if ((double)n11 * (n + 2) < (double)(n_1 + 1) * (n1_ + 1)) { *pl = 0.0; *pr = 1.0; }
        else { *pl = 1.0; *pr = 0.0; }
        *pt = 0.0;
        return 0.0;
    }
    double p, left, right;
    int i, j;
    p = pf_hypergeo_acc(lo, 0, 0, 0, &h);
    for (left = 0.0, i = lo + 1; p < 0.99999999 * q && i <= hi; ++i)
        left += p, p = pf_hypergeo_acc(i, 0, 0, 0, &h);
    --i;
    if (p < 1.00000001 * q) left += p; else --i;
    p = pf_hypergeo_acc(hi, 0, 0, 0, &h);
    for (right = 0.0, j = hi - 1; p < 0.99999999 * q && j >= 0; --j)
        right += p, p = pf_hypergeo_acc(j, 0, 0, 0, &h);
    ++j;
    if (p < 1.00000001 * q) right += p; else ++j;
    *pt = left + right;
    if (*pt > 1.0) *pt = 1.0;
    if (abs(i - n11) < abs(j - n11)) right = 1.0 - left + q;
    else left = 1.0 - right + q;
    *pl = left; *pr = right;
    return q;
}

/* evaluate_separation1 on a device-reduced table t = {n00, n01, n10, n11}
 * (buf[raw][new]).  Returns the score; *which_way = join direction or -9. */
float pf_evaluate_table(const int32_t t[4], int *which_way, double *p_two) {
    const int HARD_COV = 15, HARD_CONTAM = 5;
    int b00 = t[0], b01 = t[1], b10 = t[2], b11 = t[3];
    int m0 = b00 < b01 ? b00 : b01, m1 = b10 < b11 ? b10 : b11;
    int hard_cov_fail = (m0 > HARD_COV || m1 > HARD_COV);
    float scores[2];
    int way = 0;
    *p_two = 1.0;
    for (int i = 0; i < 2; i++) {
        int x0 = i == 0 ? b00 : b10, x1 = i == 0 ? b01 : b11;
        float mn, mx;
        if (x0 > x1) { mn = (float)x1; mx = (float)x0; way += i == 0 ? 1 : -1; }
        else { mn = (float)x0; mx = (float)x1; way += i == 0 ? -1 : 1; }
        if (m0 > HARD_CONTAM || m1 > HARD_CONTAM) { *which_way = -9; return 1.0f; }
        if (mx == 0) { *which_way = -9; return 1.0f; }
        if (mn == 0) mn = 1;
        if (mx / mn < 3) { *which_way = -9; return 1.0f; }
        scores[i] = mx / mn;
    }
    double l, r, two;
    pf_fisher_exact(b00, b01, b10, b11, &l, &r, &two);
    *p_two = two;
    if (two < 0.001 && !hard_cov_fail) {
        *which_way = way;
        return scores[0] <= scores[1] ? scores[0] : scores[1];
    }
    *which_way = -9;
    return 1.0f;
}

/* haplotag_region2's n_permutations=1 summary: join 0 (cis) / 1 (trans) / -1 */
int pf_join_from_eval(float score, int which_way) {
    if (score >= 2 && which_way != 0) return which_way > 0 ? 0 : 1;
    return -1;
}

void pf_decide_windows(uint32_t n_windows, const uint32_t *win_read_off, const uint32_t *n_sites,
                       const int32_t *tables, const uint8_t *hp_raw, const uint8_t *hp_fwd,
                       pf_window_out_t *out) {
    for (uint32_t w = 0; w < n_windows; w++) {
        int join[2] = {-1, -1}, way[2] = {-9, -9};
        double p[2] = {1.0, 1.0};
        float sc[2] = {1.0f, 1.0f};
        int decision = -1;
        uint32_t r0 = win_read_off[w], r1 = win_read_off[w + 1];
        int skipped = n_sites[w] == 0;
        if (!skipped) {
            for (int d = 0; d < 2; d++) {
                sc[d] = pf_evaluate_table(tables + ((size_t)w * 2 + d) * 4, &way[d], &p[d]);
                join[d] = pf_join_from_eval(sc[d], way[d]);
            }
            if (join[0] != join[1] || (join[0] == -1 && join[1] == -1)) decision = -1;
            else decision = join[0];
        }
        if (out->decision) out->decision[w] = (int8_t)decision;
        if (out->read_hp) {
            for (uint32_t r = r0; r < r1; r++)
                out->read_hp[r] = skipped ? hp_raw[r] : (decision < 0 ? 2 : hp_fwd[r]);
        }
        for (int d = 0; d < 2; d++) {
            size_t i = (size_t)w * 2 + d;
            if (out->dir_table) memcpy(out->dir_table + i * 4, tables + i * 4, 4 * sizeof(int32_t));
            if (out->dir_join) out->dir_join[i] = join[d];
            if (out->dir_which_way) out->dir_which_way[i] = way[d];
            if (out->dir_fisher_p) out->dir_fisher_p[i] = p[d];
            if (out->dir_score) out->dir_score[i] = sc[d];
        }
        if (out->win_n_sites) out->win_n_sites[w] = n_sites[w];
    }
}
