// gs_bgregime.h — the all-background state of the sweep chain.
//
// A snapshot is in the all-background state when no window of any sequence can
// pass the cut-off (.fs:735): every target's categories are then its K background
// products only, and the sweep is the background pick of every target
// (gs_sweep_bg.hip).  Bound, for every target n and window k:
//   log2 S_k = sum_j log2 PPM'[s][j] - sum_j log2 PCV_n[s]
//           <= sum_j log2 max_e PPM[e][j] - W log2 min_e PCV_lo[e]
// with PPM' <= PPM cellwise (the own segment's cells count C - 1) and
// PCV_n[e] = (T[e] + x + pc) / (sum T + (W or L_n) + A pc) >= PCV_lo[e] =
// (T[e] + xlo + pc) / (sum T + max(W, Lmax) + A pc), x the target's own counts of e:
// its segment's (>= 0) or, without a motif, its whole composition (>= cmin, the
// fewest occurrences of a symbol in any sequence): xlo = cmin when no target keeps
// a motif (every C cell 0), else 0.
// The margin 1e-6 covers the binary64 roundings of the reference's folds and logs
// and of these ones.  Every kernel that reads a snapshot evaluates it with this one
// function on the same aggregates, so they agree on which kernel sweeps it.
#pragma once
#include <hip/hip_runtime.h>

#include "gs_common.h"

namespace gs {

// C[e * W + j] (int32) and T[e] (int64) in LDS; scratch: 2 W + 3 doubles of LDS.
// Called by every thread of the workgroup (two barriers).  Threads 0..W-1 take a
// column each (its largest count, the log of its PPM bound), thread W both
// candidate PCV bounds (xlo = cmin and xlo = 0); thread 0 combines them in column
// order, so every kernel gets the same value.
__device__ __forceinline__ bool bg_regime(const int32_t *C, const int64_t *T, int A, int W, double pc,
                                          double den, double apc, int32_t Lmax, int32_t cmin,
                                          double cutoff, double *scratch, int tid) {
    if (tid < W) {
        int mx = 0;
        for (int e = 0; e < A; ++e) mx = max(mx, C[e * W + tid]);
        scratch[tid] = log2(((double)mx + pc) / den);  // normalizePPM (.fs:257-260)
        scratch[W + 3 + tid] = (double)mx;
    } else if (tid == W) {
        int64_t s = 0, tmin = T[0];
        for (int e = 0; e < A; ++e) {
            s += T[e];
            tmin = min(tmin, T[e]);
        }
        const double d = (double)s + (double)max(Lmax, W) + apc;
        const double lo0 = ((double)tmin + pc) / d;
        const double lo1 = ((double)(tmin + (int64_t)max(cmin, 0)) + pc) / d;
        scratch[W] = lo0 > 0.0 ? log2(lo0) : -INFINITY;
        scratch[W + 1] = lo1 > 0.0 ? log2(lo1) : -INFINITY;
    }
    __syncthreads();
    if (tid == 0) {
        double ub = 0.0, cmax = 0.0;
        for (int j = 0; j < W; ++j) {
            ub += scratch[j];
            cmax = fmax(cmax, scratch[W + 3 + j]);
        }
        // no target keeps a motif (every C cell 0): each target's own counts are its
        // whole composition, at least cmin
        const double llo = cmax == 0.0 ? scratch[W + 1] : scratch[W];
        const double b = ub - (double)W * llo;
        scratch[W + 2] = (b < cutoff - 1e-6 && fabs(cutoff) < 1000.0) ? 1.0 : 0.0;
    }
    __syncthreads();
    return scratch[W + 2] != 0.0;
}

}  // namespace gs
