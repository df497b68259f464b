// gs_fold.h — the reference's binary64 window folds, shared by the sweep and the
// greedy kernels.
#pragma once
#include <hip/hip_runtime.h>

#include "gs_common.h"

namespace gs {

// S_k and G_k of window k: the reference's left folds (.fs:291-292, .fs:124).
// tab: symbol-major [E][tab_stride(WM)] (PWM, PCV) pairs, columns j >= W hold
// (1.0, 1.0); the column offset j*16 is a ds_read immediate and the odd row
// stride spreads the symbols' rows over distinct banks.
template <int WM>
__device__ __forceinline__ void window_products(const uint8_t *sseq, const unsigned char *tab,
                                                int k, double &S, double &G) {
    constexpr int ND = WM / 4 + 1, RS = tab_stride(WM) * 16;
    const int kb = k & ~3, off = k & 3;
    uint32_t d[ND];
#pragma unroll
    for (int i = 0; i < ND; ++i) d[i] = *(const uint32_t *)(sseq + kb + 4 * i);
    S = 1.0;
    G = 1.0;
#pragma unroll
    for (int i = 0; i < WM / 4; ++i) {
        const uint32_t x = __builtin_amdgcn_alignbyte(d[i + 1], d[i], off);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int j = 4 * i + t;
            const uint32_t e = (x >> (8 * t)) & 0xffu;
            const double2 v = *(const double2 *)(tab + e * RS + j * 16);
            S = S * v.x;
            G = G * v.y;
        }
        // four table rows in flight at a time: hoisting all W loads would hold 4W
        // VGPRs at the peak
        __builtin_amdgcn_sched_barrier(0);
    }
    // materialise both folds here: otherwise the G fold is sunk below the caller's
    // log2 branch and every table operand stays live across it (VGPRs, occupancy)
    asm volatile("" ::"v"(S), "v"(G));
}

// Exact view: the reference's binary64 G_k and, when it passes the cut-off,
// log2 S_k (.fs:735-738, .fs:759-777); M = -inf when window k is no motif
// category.  thr_lo: S below it certainly fails the cut-off (the log can wait).
template <int WM>
__device__ __forceinline__ void exact_eval(const uint8_t *sseq, const unsigned char *tab,
                                           double thr_lo, double cutoff, int k, double &G,
                                           double &M) {
    double S;
    window_products<WM>(sseq, tab, k, S, G);
    M = -INFINITY;
    if (S >= thr_lo) {
        const double l2 = log(S * 1.0) / kLn2;
        if (l2 > cutoff) M = l2;
    }
}

}  // namespace gs
