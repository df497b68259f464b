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

// The same folds for a latency-bound caller with registers to spare (one wavefront
// per SIMD or two): every table row of a chunk of CH columns is requested before
// the first product, so a window costs ~W/CH LDS round trips instead of W.
template <int WM, int CH = 16>
__device__ __forceinline__ void window_products_wide(const uint8_t *sseq, const unsigned char *tab,
                                                     int k, double &S, double &G) {
    constexpr int ND = WM / 4 + 1, RS = tab_stride(WM) * 16;
    const int kb = k & ~3, off = k & 3;
    uint32_t d[ND];
#pragma unroll
    for (int i = 0; i < ND; ++i) d[i] = *(const uint32_t *)(sseq + kb + 4 * i);
    uint32_t x[WM / 4];
#pragma unroll
    for (int i = 0; i < WM / 4; ++i) x[i] = __builtin_amdgcn_alignbyte(d[i + 1], d[i], off);
    S = 1.0;
    G = 1.0;
#pragma unroll
    for (int c0 = 0; c0 < WM; c0 += CH) {
        double2 v[CH];
#pragma unroll
        for (int t = 0; t < CH; ++t) {
            const int j = c0 + t;
            if (j < WM) {
                const uint32_t e = (x[j / 4] >> (8 * (j % 4))) & 0xffu;
                v[t] = *(const double2 *)(tab + e * RS + j * 16);
            }
        }
#pragma unroll
        for (int t = 0; t < CH; ++t) {
            if (c0 + t < WM) {
                S = S * v[t].x;
                G = G * v[t].y;
            }
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    asm volatile("" ::"v"(S), "v"(G));
}

// Two windows k0, k1 of the same lane at once (independent folds interleaved: one
// LDS round trip per chunk serves both).
template <int WM, int CH = 16>
__device__ __forceinline__ void window_products_wide2(const uint8_t *sseq,
                                                      const unsigned char *tab, int k0, int k1,
                                                      double &S0, double &G0, double &S1,
                                                      double &G1) {
    constexpr int ND = WM / 4 + 1, RS = tab_stride(WM) * 16;
    uint32_t x0[WM / 4], x1[WM / 4];
    {
        const int kb0 = k0 & ~3, off0 = k0 & 3, kb1 = k1 & ~3, off1 = k1 & 3;
        uint32_t d0[ND], d1[ND];
#pragma unroll
        for (int i = 0; i < ND; ++i) {
            d0[i] = *(const uint32_t *)(sseq + kb0 + 4 * i);
            d1[i] = *(const uint32_t *)(sseq + kb1 + 4 * i);
        }
#pragma unroll
        for (int i = 0; i < WM / 4; ++i) {
            x0[i] = __builtin_amdgcn_alignbyte(d0[i + 1], d0[i], off0);
            x1[i] = __builtin_amdgcn_alignbyte(d1[i + 1], d1[i], off1);
        }
    }
    S0 = G0 = S1 = G1 = 1.0;
#pragma unroll
    for (int c0 = 0; c0 < WM; c0 += CH) {
        double2 v0[CH], v1[CH];
#pragma unroll
        for (int t = 0; t < CH; ++t) {
            const int j = c0 + t;
            if (j < WM) {
                const uint32_t e0 = (x0[j / 4] >> (8 * (j % 4))) & 0xffu;
                const uint32_t e1 = (x1[j / 4] >> (8 * (j % 4))) & 0xffu;
                v0[t] = *(const double2 *)(tab + e0 * RS + j * 16);
                v1[t] = *(const double2 *)(tab + e1 * RS + j * 16);
            }
        }
#pragma unroll
        for (int t = 0; t < CH; ++t) {
            if (c0 + t < WM) {
                S0 = S0 * v0[t].x;
                G0 = G0 * v0[t].y;
                S1 = S1 * v1[t].x;
                G1 = G1 * v1[t].y;
            }
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    asm volatile("" ::"v"(S0), "v"(G0), "v"(S1), "v"(G1));
}

// Motif category of a window with product S (.fs:735-738): log2 S when it passes
// the cut-off, else -inf.  thr_lo: S below it certainly fails (the log can wait).
__device__ __forceinline__ double motif_weight(double S, double thr_lo, double cutoff) {
    double M = -INFINITY;
    if (S >= thr_lo) {
        const double l2 = log(S * 1.0) / kLn2;
        if (l2 > cutoff) M = l2;
    }
    return M;
}

// exact_eval on window_products_wide.
template <int WM>
__device__ __forceinline__ void exact_eval_wide(const uint8_t *sseq, const unsigned char *tab,
                                                double thr_lo, double cutoff, int k, double &G,
                                                double &M) {
    double S;
    window_products_wide<WM>(sseq, tab, k, S, G);
    M = -INFINITY;
    if (S >= thr_lo) {
        const double l2 = log(S * 1.0) / kLn2;
        if (l2 > cutoff) M = l2;
    }
}

// binary64 log out of line: a kernel that takes it only on rare paths keeps the
// polynomial's constants out of its loops' registers
__device__ __noinline__ inline double log_ool(double x) { return log(x); }

// Exact view: the reference's binary64 G_k and, when it passes the cut-off,
// log2 S_k (.fs:735-738, .fs:759-777); M = -inf when window k is no motif
// category.  thr_lo: S below it certainly fails the cut-off (the log can wait).
// OOL: the log out of line (log_ool).
template <int WM, bool OOL = false>
__device__ __forceinline__ void exact_eval(const uint8_t *sseq, const unsigned char *tab,
                                           double thr_lo, double cutoff, int k, double &G,
                                           double &M) {
    double S;
    window_products<WM>(sseq, tab, k, S, G);
    M = -INFINITY;
    if (S >= thr_lo) {
        const double l2 = (OOL ? log_ool(S * 1.0) : log(S * 1.0)) / kLn2;
        if (l2 > cutoff) M = l2;
    }
}

}  // namespace gs
