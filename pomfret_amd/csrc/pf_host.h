/* pf_host.h -- host-side epilogue helpers shared by the HIP driver (product). */
#ifndef PF_HOST_H
#define PF_HOST_H
#include "../../include/pomfret_amd.h"
#ifdef __cplusplus
extern "C" {
#endif
float pf_evaluate_table(const int32_t t[4], int *which_way, double *p_two);
int pf_join_from_eval(float score, int which_way);
void pf_decide_windows(uint32_t n_windows, const uint32_t *win_read_off, const uint32_t *n_sites,
                       const int32_t *tables, const uint8_t *hp_raw, const uint8_t *hp_fwd,
                       pf_window_out_t *out);
#ifdef __cplusplus
}
#endif
#endif
