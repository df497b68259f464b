// gs_greedy.hip — MotifSampler.findBestMotifIndicesWithStartPositions
// (GibbsSampling.fs:885-929, motifAmount = 1) for gfx950.
//
// The reference refines the sampled positions greedily: target after target it
// rebuilds the background and the count matrix from the LIVE positions (acc,
// .fs:891-893 — Gauss–Seidel: a target sees the moves of the targets before it in
// the same pass), scores every window exactly like the sweep (.fs:894-916), takes
// the head of the stable List.sortByDescending of the categories (.fs:917-920) and
// keeps it when its weight beats the target's current one (.fs:921-925).  Passes
// repeat until a pass moves no position (.fs:926-929).
//
// Only a MOVE changes what later targets see (the aggregates C[A][W], T[A]); a
// target that keeps its position at most rewrites its own PWMS.  One persistent
// workgroup therefore scores the next `waves` targets at once, one wavefront each,
// against the current aggregates (speculation), and commits them in order up to and
// including the first that moves; the targets after it are scored again in the next
// step against the updated aggregates.  Every committed result is the one the
// sequential loop computes — bit-identical picks and PWMS — while runs of
// non-moving targets go `waves` at a time.
//
// Data movement: C/T and the PPM tables live in LDS and change by one segment per
// move; sequences, compositions and positions of the upcoming visits are staged in
// an LDS ring of 2*waves slots, prefetched one step ahead into registers.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <climits>

#include "gs_common.h"
#include "gs_fold.h"
#include "gs_stamps.h"
#include "gs_wave.h"

using namespace gs;

namespace {

// (v, o) comes before (bv, bo) in the stable sortByDescending (.fs:917-920): a
// larger weight, or the same weight earlier in the category list (G_0..G_{K-1},
// then the motif categories in window order).  F# generic comparison ranks NaN
// below every number; "none" is (NaN, INT_MAX).
__device__ __forceinline__ bool sorts_first(double v, int o, double bv, int bo) {
    if (v > bv) return true;
    if (v == bv) return o < bo;
    if (bv != bv) return v == v || o < bo;
    return false;
}

__device__ __forceinline__ int load_relaxed(const int32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double load_relaxed(const double *p) {
    const unsigned long long b = __hip_atomic_load((const unsigned long long *)p, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT);
    return __longlong_as_double((long long)b);
}

struct Shared {
    int32_t *C;       // [A][W] counts of the live segments
    int64_t *T;       // [A] Σ over motif-bearing sequences of (composition − segment)
    int64_t *sumT;    // Σ_a T[a]
    double *ppmG;     // [A][W] normalizePPM of C          (.fs:257-260)
    double *ppmM;     // [A][W] normalizePPM of C − 1 (own-segment cells)
    int32_t *ctl;     // [32] per-wave events
    uint8_t *rseq;    // ring sequences
    int32_t *rt, *rL, *rp, *rcomp;
    double *rpw;
};

// Count of symbol e in sseq[p, p + W) (p >= 0): the segment read as aligned
// words, matching bytes found with the exact zero-byte test (no LDS atomics).
template <int WM>
__device__ __forceinline__ int segment_count(const uint8_t *sseq, int p, int W, int e) {
    constexpr int ND = WM / 4 + 1;
    const int kb = p & ~3, off = p & 3;
    uint32_t d[ND];
#pragma unroll
    for (int i = 0; i < ND; ++i) d[i] = *(const uint32_t *)(sseq + kb + 4 * i);
    const uint32_t pat = (uint32_t)e * 0x01010101u;
    int cnt = 0;
#pragma unroll
    for (int i = 0; i < WM / 4; ++i) {
        uint32_t y = __builtin_amdgcn_alignbyte(d[i + 1], d[i], off) ^ pat;
        const int rem = W - 4 * i;  // bytes of this word inside the segment
        const uint32_t outside = rem >= 4 ? 0u : (rem <= 0 ? ~0u : ~((1u << (8 * rem)) - 1u));
        y |= outside & 0x01010101u;  // never a match
        const uint32_t z = ~(((y & 0x7f7f7f7fu) + 0x7f7f7f7fu) | y | 0x7f7f7f7fu);
        cnt += __popc(z);
    }
    return cnt;
}

// One target scored against the current aggregates: the hold-one-out background
// and PWM (.fs:891-916), every window folded in binary64 (gs_fold.h), and the head
// of the category sort.  Wave-uniform results: pick value bv and the new position
// (-1 = a background category); segc (lane e < E) = the old segment's counts.
template <int WM>
__device__ __forceinline__ void score_target(const GreedyArgs &a, const Shared &sh,
                                             const uint8_t *sseq, int L, int p, int my_comp,
                                             int na, unsigned char *tab, double *pcv,
                                             int lane, double &bv_out, int &newp_out,
                                             int &segc_out, bool &overflow STAMP_PARAMS) {
    constexpr int WS = tab_stride(WM);
    const int A = a.A, W = a.W, E = a.E;
    const int K = L - W + 1;
    const int segc = (p >= 0 && lane < E) ? segment_count<WM>(sseq, p, W, lane) : 0;
    const int seg_alpha = wave_sum_i32(lane < A ? segc : 0);
    const int64_t sumT = *sh.sumT;
    const int64_t bgc = lane < A ? sh.T[lane] + (p >= 0 ? segc : my_comp) : 0;
    const int64_t tot = sumT + (p >= 0 ? seg_alpha : L - na) + na;
    overflow = !a.pcv_fixed && tot > 2147483647LL;  // Checked Array.sum (.fs:117)
    segc_out = segc;
    if (overflow) return;
    // PCV (.fs:119); outside the alphabet the raw count (Q3); the ByPCV twin
    // (.fs:788-823) takes the caller's vector
    const double sbg = (double)tot + a.apc;
    const double pe = a.pcv_fixed ? a.pcv_fixed[lane < E ? lane : 0]
                                  : (lane < A ? ((double)bgc + a.pc) / sbg : (double)my_comp);
    if (lane < E) pcv[lane] = pe;
    wave_sync();
    STAMP(7);
    // PWM of the others (.fs:282-287): own-segment cells count C − 1
    const uint32_t magicW = 0xffffffffu / (uint32_t)W + 1u;
    // two cells per lane per step, all their LDS reads issued before the divisions
    const int pp = p >= 0 ? p : 0;
    for (int c0 = lane; c0 < E * W; c0 += 128) {
        const int c1 = c0 + 64 < E * W ? c0 + 64 : c0;
        const int e0 = magic_div((uint32_t)c0, (uint32_t)W, magicW), j0 = c0 - e0 * W;
        const int e1 = magic_div((uint32_t)c1, (uint32_t)W, magicW), j1 = c1 - e1 * W;
        const int a0 = (e0 < A ? e0 : 0) * W + j0, a1 = (e1 < A ? e1 : 0) * W + j1;
        const double q0 = pcv[e0], q1 = pcv[e1];
        const double g0 = sh.ppmG[a0], m0 = sh.ppmM[a0], g1 = sh.ppmG[a1], m1 = sh.ppmM[a1];
        const int s0 = sseq[pp + j0], s1 = sseq[pp + j1];
        const double v0 = e0 < A ? ((p >= 0 && s0 == e0) ? m0 : g0) / q0 : 0.0;
        const double v1 = e1 < A ? ((p >= 0 && s1 == e1) ? m1 : g1) / q1 : 0.0;
        *(double2 *)(tab + (e0 * WS + j0) * 16) = make_double2(v0, q0);
        *(double2 *)(tab + (e1 * WS + j1) * 16) = make_double2(v1, q1);
    }
    wave_sync();
    STAMP(8);
    // categories (.fs:759-782) and the head of their descending sort
    double bv = __builtin_nan("");
    int bo = INT_MAX;
    auto consider = [&](double g, double m, int k) {
        if (sorts_first(g, k, bv, bo)) {
            bv = g;
            bo = k;
        }
        if (m > -INFINITY && sorts_first(m, K + k, bv, bo)) {
            bv = m;
            bo = K + k;
        }
    };
    for (int k = lane; k < K; k += 64) {
        double S, G;
        window_products_wide<WM>(sseq, tab, k, S, G);
        consider(G, motif_weight(S, a.thr_lo, a.cutoff), k);
    }
    STAMP(9);
    // across lanes (DPP, no LDS round trips): the largest order key, then the
    // earliest category holding it
    const unsigned long long key = order_key(bv);
    const unsigned long long kmax = wave_max_u64(key);
    const int omin = wave_min_i32(key == kmax ? bo : INT_MAX);
    const unsigned long long win = __ballot(key == kmax && bo == omin);
    bv_out = lane_read_f64(bv, __builtin_ctzll(win));
    newp_out = omin < K ? -1 : omin - K;
    STAMP(10);
}

// score_target with every wavefront of the workgroup on ONE visit (the move-heavy
// regime: the speculation width has fallen to one visit per step).  The same
// integers, PCV, (PWM, PCV) table cells and window folds as score_target — the table
// in wavefront 0's slice, one cell per thread; the windows dealt over all threads —
// and the head of the category sort by a workgroup reduction on order keys.  Every
// wavefront must call it (two barriers, plus one for the reduction).
template <int WM>
__device__ __forceinline__ void score_target_coop(const GreedyArgs &a, const Shared &sh,
                                                  const uint8_t *sseq, int L, int p, int my_comp,
                                                  int na, unsigned char *tab, double *pcv,
                                                  unsigned long long *red, int lane, int w,
                                                  int NW, double &bv_out, int &newp_out,
                                                  int &segc_out, bool &overflow) {
    constexpr int WS = tab_stride(WM);
    const int A = a.A, W = a.W, E = a.E;
    const int K = L - W + 1, NT = 64 * NW, tid = 64 * w + lane;
    const int segc = (p >= 0 && lane < E) ? segment_count<WM>(sseq, p, W, lane) : 0;
    const int seg_alpha = wave_sum_i32(lane < A ? segc : 0);
    const int64_t sumT = *sh.sumT;
    const int64_t bgc = lane < A ? sh.T[lane] + (p >= 0 ? segc : my_comp) : 0;
    const int64_t tot = sumT + (p >= 0 ? seg_alpha : L - na) + na;
    overflow = !a.pcv_fixed && tot > 2147483647LL;  // Checked Array.sum (.fs:117)
    segc_out = segc;
    if (overflow) return;  // uniform over the workgroup
    const double sbg = (double)tot + a.apc;
    const double pe = a.pcv_fixed ? a.pcv_fixed[lane < E ? lane : 0]
                                  : (lane < A ? ((double)bgc + a.pc) / sbg : (double)my_comp);
    if (w == 0 && lane < E) pcv[lane] = pe;
    __syncthreads();
    const uint32_t magicW = 0xffffffffu / (uint32_t)W + 1u;
    const int pp = p >= 0 ? p : 0;
    for (int c = tid; c < E * W; c += NT) {
        const int e = magic_div((uint32_t)c, (uint32_t)W, magicW), j = c - e * W;
        const int ai = (e < A ? e : 0) * W + j;
        const double q = pcv[e];
        const double g = sh.ppmG[ai], m = sh.ppmM[ai];
        const double v = e < A ? ((p >= 0 && sseq[pp + j] == e) ? m : g) / q : 0.0;
        *(double2 *)(tab + (e * WS + j) * 16) = make_double2(v, q);
    }
    __syncthreads();
    double bv = __builtin_nan("");
    int bo = INT_MAX;
    for (int k = tid; k < K; k += NT) {
        double S, G;
        window_products_wide<WM>(sseq, tab, k, S, G);
        if (sorts_first(G, k, bv, bo)) {
            bv = G;
            bo = k;
        }
        const double m = motif_weight(S, a.thr_lo, a.cutoff);
        if (m > -INFINITY && sorts_first(m, K + k, bv, bo)) {
            bv = m;
            bo = K + k;
        }
    }
    const unsigned long long key = order_key(bv);
    const unsigned long long kmax = wave_max_u64(key);
    const int omin = wave_min_i32(key == kmax ? bo : INT_MAX);
    const unsigned long long win = __ballot(key == kmax && bo == omin);
    const double bw = lane_read_f64(bv, __builtin_ctzll(win));
    if (lane == 0) {
        red[2 * w] = kmax;
        red[2 * w + 1] = (unsigned long long)(unsigned)omin;
        red[2 * NW + w] = (unsigned long long)__double_as_longlong(bw);
    }
    __syncthreads();
    unsigned long long gk = 0;
    int go = INT_MAX;
    double gb = __builtin_nan("");
    for (int v = 0; v < NW; ++v) {
        const unsigned long long kv = red[2 * v];
        const int ov = (int)red[2 * v + 1];
        if (kv > gk || (kv == gk && ov < go)) {
            gk = kv;
            go = ov;
            gb = __longlong_as_double((long long)red[2 * NW + v]);
        }
    }
    bv_out = gb;
    newp_out = go < K ? -1 : go - K;
}

// Inclusive prefix sum of an int within each 16-lane row (DPP row shifts only).
__device__ __forceinline__ int row_incl_scan_i32(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, true);
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, true);
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, true);
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, true);
    return v;
}

// S_k of window k under the drifting background (.fs:463-479): per column the PCV
// entry ((f + pc) / Σ_k, createNormalizedPCVOfFCV) and the PWM entry (PPM' / PCV),
// then the reference's left fold.  Branch-free over the WM unrolled columns (columns
// past W multiply by exactly 1.0, non-alphabet symbols by 0.0, as the fold would) so
// that the columns' binary64 divisions interleave instead of running one after the
// other.
template <int WM, typename DT>
__device__ __forceinline__ double site_window(const uint8_t *sseq, int k, int p, int W, int A,
                                              const double *ppmG, const double *ppmM,
                                              const int64_t *wbg, const int32_t *wcomp,
                                              const DT *Dt, double pc, double sbg) {
    const int64_t kk = (int64_t)k + 1;
    double v[WM];
#pragma unroll
    for (int j = 0; j < WM; ++j) {
        const int jc = j < W ? j : 0;
        const int e = sseq[k + jc];
        const int ec = e < A ? e : 0;
        const int64_t f = wbg[ec] + kk * (int64_t)wcomp[ec] - (int64_t)Dt[k * A + ec];
        const double q = ((double)f + pc) / sbg;
        const double x = (sseq[p + jc] == e ? ppmM : ppmG)[ec * W + jc] / q;
        v[j] = j < W ? (e < A ? x : 0.0) : 1.0;
    }
    double S = 1.0;
#pragma unroll
    for (int j = 0; j < WM; ++j) S = S * v[j];  // calculateSegmentScoreBy (.fs:290-293)
    return S;
}

// Site-sampler twin (getBestPWMSsWithStartPositions, .fs:554-585): getBestPWMSs of
// the target (.fs:462-479) with the others at their live positions.  The
// background drifts window after window (quirk Q1, closed form as in gs_starts.hip):
//   fcv_k[b] = B[b] + (k+1)·comp[b] − D_k[b],  D_k[b] = Σ_{i<=k} count_b(window i),
// B = the others' background T − (comp − seg).  D is built lane-blocked (each lane
// slides a window count over its own block of windows, one DPP prefix over the
// lanes per symbol) into the wavefront's Dt[K][A].  Wave-uniform results: the log2
// of the first maximal window score and its start (0 when no score beats 0.0).
template <int WM, typename DT>
__device__ __forceinline__ void score_site(const GreedyArgs &a, const Shared &sh,
                                           const uint8_t *sseq, int L, int p, int my_comp,
                                           int na, DT *Dt, int64_t *wbg, int32_t *wcomp,
                                           int lane, double &sc_out, int &newp_out,
                                           int &segc_out, bool &overflow STAMP_PARAMS) {
    const int A = a.A, W = a.W, E = a.E;
    const int K = L - W + 1;
    const int segc = lane < E ? segment_count<WM>(sseq, p, W, lane) : 0;
    segc_out = segc;
    const int seg_alpha = wave_sum_i32(lane < A ? segc : 0);
    // Σ_a B[a]: the others' alphabet symbols outside their segments
    const int64_t bsum = *sh.sumT - (int64_t)((L - na) - seg_alpha);
    const double *pcvf = a.pcv_fixed;  // findBestMotifWithStartPosition (.fs:381-409)
    // Checked Array.sum (.fs:117) of fcv_k: bsum + (k+1)(L − W) grows with k
    overflow = !pcvf && bsum + (int64_t)K * (L - W) > 2147483647LL;
    if (overflow) return;
    if (pcvf) {  // getBestPWMSsWithBPV (.fs:301-313): no background, no drift
        double best = 0.0;
        int bestk = INT_MAX;
        for (int k = lane; k < K; k += 64) {
            double S = 1.0;
#pragma unroll
            for (int j = 0; j < WM; ++j) {
                if (j < W) {
                    const int e = sseq[k + j];
                    const double v =
                        e < A ? (sseq[p + j] == e ? sh.ppmM : sh.ppmG)[e * W + j] / pcvf[e] : 0.0;
                    S = S * v;
                }
            }
            if (S > best) {
                best = S;
                bestk = k;
            }
        }
        const unsigned long long key = order_key(best);
        const unsigned long long kmax = wave_max_u64(key);
        const int kmin = wave_min_i32(key == kmax ? bestk : INT_MAX);
        const unsigned long long win = __ballot(key == kmax && bestk == kmin);
        const double bmax = kmin == INT_MAX ? 0.0 : lane_read_f64(best, __builtin_ctzll(win));
        sc_out = log(bmax) / kLn2;
        newp_out = kmin == INT_MAX ? 0 : kmin;
        return;
    }
    if (lane < A) {
        wbg[lane] = sh.T[lane] - (my_comp - segc);
        wcomp[lane] = my_comp;
    }
    const int R = (K + 63) >> 6, k0 = lane * R, k1 = min(K, k0 + R);
    for (int x = 0; x < A; ++x) {
        const int cw0 = k0 < K ? segment_count<WM>(sseq, k0, W, x) : 0;
        int cw = cw0, bs = 0;
#pragma unroll 4
        for (int k = k0; k < k1; ++k) {
            bs += cw;
            cw += (sseq[k + W] == x) - (sseq[k] == x);
        }
        int d = wave_incl_scan_i32(bs) - bs;  // D_{k0 - 1}
        cw = cw0;
#pragma unroll 4
        for (int k = k0; k < k1; ++k) {
            d += cw;
            Dt[k * A + x] = (DT)d;
            cw += (sseq[k + W] == x) - (sseq[k] == x);
        }
    }
    wave_sync();
    STAMP(7);
    double best = 0.0;
    int bestk = INT_MAX;
    for (int k = lane; k < K; k += 64) {
        const int64_t kk = (int64_t)k + 1;
        const double sbg = (double)(bsum + kk * (int64_t)(L - W)) + a.apc;
        const double S = site_window<WM, DT>(sseq, k, p, W, A, sh.ppmG, sh.ppmM, wbg, wcomp, Dt,
                                             a.pc, sbg);
        if (S > best) {  // strict '>' from (0.0, 0) (.fs:477)
            best = S;
            bestk = k;
        }
    }
    STAMP(9);
    const unsigned long long key = order_key(best);
    const unsigned long long kmax = wave_max_u64(key);
    const int kmin = wave_min_i32(key == kmax ? bestk : INT_MAX);
    const unsigned long long win = __ballot(key == kmax && bestk == kmin);
    const double bmax = kmin == INT_MAX ? 0.0 : lane_read_f64(best, __builtin_ctzll(win));
    sc_out = log(bmax) / kLn2;
    newp_out = kmin == INT_MAX ? 0 : kmin;
    STAMP(10);
}

// score_site with every wavefront of the workgroup on ONE visit (the move-heavy
// regime, where the speculation width has fallen to one visit per step): the D
// table by 16-lane rows (one symbol per row, each lane sliding over a block of
// windows, one row scan), the windows dealt over all threads, the first maximum by a
// workgroup reduction.  Same integers and binary64 operations per window as
// score_site, so the same result.  Every wavefront must call it (two barriers).
template <int WM, typename DT>
__device__ __forceinline__ void score_site_coop(const GreedyArgs &a, const Shared &sh,
                                                const uint8_t *sseq, int L, int p, int my_comp,
                                                int na, DT *Dt, int64_t *wbg, int32_t *wcomp,
                                                unsigned long long *red, int lane, int w, int NW,
                                                double &sc_out, int &newp_out, int &segc_out,
                                                bool &overflow STAMP_PARAMS) {
    const int A = a.A, W = a.W, E = a.E;
    const int K = L - W + 1, NT = 64 * NW, tid = 64 * w + lane;
    const int segc = lane < E ? segment_count<WM>(sseq, p, W, lane) : 0;
    segc_out = segc;
    const int seg_alpha = wave_sum_i32(lane < A ? segc : 0);
    const int64_t bsum = *sh.sumT - (int64_t)((L - na) - seg_alpha);
    const double *pcvf = a.pcv_fixed;
    overflow = !pcvf && bsum + (int64_t)K * (L - W) > 2147483647LL;
    if (overflow) return;  // uniform over the workgroup
    double best = 0.0;
    int bestk = INT_MAX;
    if (pcvf) {
        for (int k = tid; k < K; k += NT) {
            double S = 1.0;
#pragma unroll
            for (int j = 0; j < WM; ++j) {
                if (j < W) {
                    const int e = sseq[k + j];
                    const double v =
                        e < A ? (sseq[p + j] == e ? sh.ppmM : sh.ppmG)[e * W + j] / pcvf[e] : 0.0;
                    S = S * v;
                }
            }
            if (S > best) {
                best = S;
                bestk = k;
            }
        }
    } else {
        if (w == 0 && lane < A) {
            wbg[lane] = sh.T[lane] - (my_comp - segc);
            wcomp[lane] = my_comp;
        }
        // segments of SL lanes (16: DPP row scans, or 64: a wavefront scan) each build
        // D[.][x] for one symbol x at a time, every lane sliding over its block of
        // windows; the segment size with the shorter serial slide is taken (few
        // symbols: whole wavefronts; protein: rows)
        const int R16 = (K + 15) >> 4, R64 = (K + 63) >> 6;
        const int n16 = NT >> 4;
        const bool wide = ((A + NW - 1) / NW) * R64 < ((A + n16 - 1) / n16) * R16;
        const int SL = wide ? 64 : 16, nseg = wide ? NW : n16;
        const int li = wide ? lane : (lane & 15), RB = wide ? R64 : R16;
        const int k0 = li * RB, k1 = min(K, k0 + RB);
        for (int x0 = 0; x0 < A; x0 += nseg) {  // workgroup-uniform trip count
            const int x = x0 + tid / SL;
            const bool ok = x < A;
            const int cw0 = ok && k0 < K ? segment_count<WM>(sseq, k0, W, x) : 0;
            int cw = cw0, bs = 0;
            if (ok)
#pragma unroll 4
                for (int k = k0; k < k1; ++k) {
                    bs += cw;
                    cw += (sseq[k + W] == x) - (sseq[k] == x);
                }
            int d = (wide ? wave_incl_scan_i32(bs) : row_incl_scan_i32(bs)) - bs;  // D_{k0 - 1}
            cw = cw0;
            if (ok)
#pragma unroll 4
                for (int k = k0; k < k1; ++k) {
                    d += cw;
                    Dt[k * A + x] = (DT)d;
                    cw += (sseq[k + W] == x) - (sseq[k] == x);
                }
        }
        __syncthreads();
        STAMP(7);
        for (int k = tid; k < K; k += NT) {
            const int64_t kk = (int64_t)k + 1;
            const double sbg = (double)(bsum + kk * (int64_t)(L - W)) + a.apc;
            const double S = site_window<WM, DT>(sseq, k, p, W, A, sh.ppmG, sh.ppmM, wbg, wcomp,
                                                 Dt, a.pc, sbg);
            if (S > best) {  // strict '>' from (0.0, 0) (.fs:477)
                best = S;
                bestk = k;
            }
        }
    }
    STAMP(9);
    // the first maximum: per wavefront, then over the wavefronts (a thread's windows
    // ascend, so the earliest window among equal keys is the reference's)
    const unsigned long long key = order_key(best);
    const unsigned long long kmax = wave_max_u64(key);
    const int kmin = wave_min_i32(key == kmax ? bestk : INT_MAX);
    const unsigned long long win = __ballot(key == kmax && bestk == kmin);
    const double bw = kmin == INT_MAX ? 0.0 : lane_read_f64(best, __builtin_ctzll(win));
    if (lane == 0) {
        red[2 * w] = kmax;
        red[2 * w + 1] = ((unsigned long long)(unsigned)kmin << 32) |
                         (unsigned long long)(unsigned)(kmin == INT_MAX ? 0 : 1);
        red[2 * NW + w] = (unsigned long long)__double_as_longlong(bw);
    }
    __syncthreads();
    unsigned long long gk = 0;
    int gmin = INT_MAX;
    double gb = 0.0;
    for (int v = 0; v < NW; ++v) {
        const unsigned long long kv = red[2 * v];
        const int mv = (int)(red[2 * v + 1] >> 32);
        if (kv > gk || (kv == gk && mv < gmin)) {
            gk = kv;
            gmin = mv;
            gb = __longlong_as_double((long long)red[2 * NW + v]);
        }
    }
    const double bmax = gmin == INT_MAX ? 0.0 : gb;
    sc_out = log(bmax) / kLn2;
    newp_out = gmin == INT_MAX ? 0 : gmin;
    STAMP(10);
}

// The aggregates after sequence sseq moves from p to newp: the old segment leaves
// C and T, the new one enters (PPM tables and Σ T follow the changed cells).
template <int WM>
__device__ __forceinline__ void move_segment(const GreedyArgs &a, const Shared &sh,
                                             const uint8_t *sseq, int p, int newp, int my_comp,
                                             int segc, int lane) {
    const int A = a.A, W = a.W;
    auto refresh = [&](int c) {
        sh.ppmG[c] = ((double)sh.C[c] + a.pc) / a.den;
        sh.ppmM[c] = ((double)(sh.C[c] - 1) + a.pc) / a.den;
    };
    int64_t t = lane < A ? sh.T[lane] : 0;
    if (p >= 0) {
        for (int j = lane; j < W; j += 64) {
            const int s = sseq[p + j];
            if (s < A) {
                sh.C[s * W + j] -= 1;
                refresh(s * W + j);
            }
        }
        t -= my_comp - segc;
    }
    wave_sync();
    if (newp >= 0) {
        for (int j = lane; j < W; j += 64) {
            const int s = sseq[newp + j];
            if (s < A) {
                sh.C[s * W + j] += 1;
                refresh(s * W + j);
            }
        }
        t += my_comp - (lane < A ? segment_count<WM>(sseq, newp, W, lane) : 0);
    }
    if (lane < A) sh.T[lane] = t;
    const int64_t s = (int64_t)wave_sum_f64(lane < A ? (double)t : 0.0);
    if (lane == 0) *sh.sumT = s;
}

}  // namespace

// SITE = false: the motif sampler's greedy passes (.fs:885-929); SITE = true: the
// site sampler's getBestPWMSsWithStartPositions (.fs:554-585).
// DT: the D table's element type (uint16_t when every D_k[b] <= K*W fits, halving the
// site slice so more wavefronts fit in LDS; int32_t otherwise and for the motif sampler)
template <bool SITE, int WM, typename DT>
__global__ void __launch_bounds__(512) gs_greedy_kernel(GreedyArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    constexpr int WS = tab_stride(WM);
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int NW = blockDim.x >> 6, R = 2 * NW;  // NW a power of two
    // the motif sampler's lone-visit mode is compiled for wide motifs only: for
    // WM <= 12 (DNA configs) its code alone slowed the one-wavefront path by ~5 %
    constexpr bool kMotifCoop = !SITE && WM >= 16;
    STAMP_DECL
    const int A = a.A, W = a.W, E = a.E, AW = A * W, CS = E + 1;
    const int N = a.n;
    Shared sh;
    sh.C = (int32_t *)(lds + a.o_C);
    sh.T = (int64_t *)(lds + a.o_T);
    sh.ppmG = (double *)(lds + a.o_ppmG);
    sh.ppmM = (double *)(lds + a.o_ppmM);
    sh.ctl = (int32_t *)(lds + a.o_ctl);
    sh.sumT = (int64_t *)(sh.ctl + 32);
    sh.rseq = (uint8_t *)(lds + a.o_ring);
    sh.rt = (int32_t *)(lds + a.o_rt);
    sh.rL = (int32_t *)(lds + a.o_rL);
    sh.rp = (int32_t *)(lds + a.o_rp);
    sh.rpw = (double *)(lds + a.o_rpw);
    sh.rcomp = (int32_t *)(lds + a.o_rcomp);
    unsigned char *wv = lds + a.o_wave + w * a.wave_bytes;
    unsigned char *tab = wv + a.w_tab;
    double *pcv = (double *)(wv + a.w_pcv);
    DT *Dt = (DT *)(wv + a.w_dt);
    int64_t *wbg = (int64_t *)(wv + a.w_bg);
    int32_t *wcomp = (int32_t *)(wv + a.w_comp);
    const int RS = a.ring_seq_bytes;

    if (__builtin_amdgcn_readfirstlane(*a.err_code) != 0) return;  // void snapshot

    for (int c = tid; c < a.cells; c += blockDim.x) {
        int64_t s = 0;
#pragma unroll
        for (int r = 0; r < kRepl; ++r) s += a.agg[(int64_t)r * a.stride + c];
        if (c < AW) {
            sh.C[c] = (int32_t)s;
            sh.ppmG[c] = ((double)s + a.pc) / a.den;
            sh.ppmM[c] = ((double)(s - 1) + a.pc) / a.den;
        } else {
            sh.T[c - AW] = s;
        }
    }
    // columns past the motif fold as exact 1.0 factors
    if (!SITE)
        for (int c = lane; c < E * WS; c += 64)
            if (c % WS >= W) *(double2 *)(tab + c * 16) = make_double2(1.0, 1.0);

    // visit v scores target v mod N; tb = b mod N for the current step's base b
    int tb = 0;
    auto target_at = [&](int d) {  // (b + d) mod N for 0 <= d < 2 * NW
        int t = tb + d;
        while (t >= N) t -= N;
        return t;
    };
    // Ring slot of a visit: the sequence with a zero tail, then its metadata.
    auto store_slot = [&](int slot, const uint4 &pf, int cpf, int t, int L, int64_t off, int p,
                          double pw) {
        uint8_t *d = sh.rseq + (int64_t)slot * RS;
        if (L <= 1024) {
            if (lane * 16 < L) *(uint4 *)(d + lane * 16) = keep_bytes(pf, L - lane * 16);
        } else {
            const uint8_t *g = a.seq + off;
            for (int i = lane * 16; i < L; i += 1024)
                *(uint4 *)(d + i) = keep_bytes(*(const uint4 *)(g + i), L - i);
        }
        // zero tail: unrolled window reads past L see symbol 0 (a valid table row)
        for (int i = ((L + 15) & ~15) + lane * 16; i < L + WM + 16; i += 1024)
            *(uint4 *)(d + i) = make_uint4(0, 0, 0, 0);
        if (lane < CS) sh.rcomp[slot * 64 + lane] = cpf;
        if (lane == 0) {
            sh.rt[slot] = t;
            sh.rL[slot] = L;
            sh.rp[slot] = p;
            sh.rpw[slot] = pw;
        }
    };
    auto load_seq = [&](int L, int64_t off) {
        uint4 pf = make_uint4(0, 0, 0, 0);
        if (L <= 1024 && lane * 16 < L) pf = *(const uint4 *)(a.seq + off + lane * 16);
        return pf;
    };
    // the first 2*waves visits
    for (int d = w; d < R; d += NW) {
        const int t = target_at(d);
        const int L = a.len[t];
        const int64_t off = a.doff[t];
        const uint4 pf = load_seq(L, off);
        const int cpf = lane < CS ? a.comp[(int64_t)t * CS + lane] : 0;
        store_slot(d, pf, cpf, t, L, off, load_relaxed(&a.pos[t]), load_relaxed(&a.pwms[t]));
    }
    // the ring holds visits [b, b + 2*waves) at the end of every step: a step that
    // advances by `fresh` leaves the last `fresh` wavefronts to fetch the new ones
    int fresh = 0;  // the prologue staged [0, 2*waves)
    int tpf = 0, Lpf = 0, cpf = 0;
    int64_t opf = 0;
    __syncthreads();
    if (w == 0) {
        const int64_t st = (int64_t)wave_sum_f64(lane < A ? (double)sh.T[lane] : 0.0);
        if (lane == 0) *sh.sumT = st;
    }
    __syncthreads();

    int64_t b = 0, pass_end = N;
    constexpr bool kCoop = SITE || kMotifCoop;
    // recent moves per visit (uniform over the workgroup), from the threshold: a launch
    // starts neither forced into lone visits nor out of them
    float mrate = a.coop_rate;
    int64_t chunk_start = 0;  // mid-pass exit bookkeeping (uniform over the workgroup)
    int chunk_moves = 0;
    bool exit_mid = false;
    // targets scored per step: the last run of non-moving targets, doubled after a
    // step without a move (frequent moves: few wavefronts share the CU, so each
    // scores faster; rare moves: the whole workgroup)
    int width = NW;
    int passes = 0;
    bool moved = false;
    int64_t steps = 0;
    STAMP(0);
    for (;;) {
        ++steps;
        const int nb = (int)min<int64_t>(width, pass_end - b);
        const bool act = w < nb;
        // fetch of visit b + waves + w by the last `fresh` wavefronts.  Positions and
        // PWMS are read now, after every earlier commit reached L2.
        const bool fetch = w >= NW - fresh;
        uint4 pf = make_uint4(0, 0, 0, 0);
        int ppf = 0;
        double pwpf = 0.0;
        if (fetch) {
            pf = load_seq(Lpf, opf);
            ppf = load_relaxed(&a.pos[tpf]);
            pwpf = load_relaxed(&a.pwms[tpf]);
        }
        STAMP(1);

        int ev = 0, t = 0, p = -1, newp = -1, segc = 0, my_comp = 0, s = 0;
        double bv = 0.0, pw_old = 0.0;
        // one visit this step: every wavefront scores it (site sampler)
        // (motif sampler: only for visits with at least motif_coop window cells, K*W —
        // short DNA visits score faster on one wavefront than across barriers)
        const bool coop =
            nb == 1 && NW > 1 &&
            (SITE ? a.site_coop != 0
                  : kMotifCoop && a.motif_coop > 0 &&
                        (sh.rL[b & (R - 1)] - W + 1) * W >= a.motif_coop);
        if (act || coop) {
            s = (int)((b + (coop ? 0 : w)) & (R - 1));
            t = sh.rt[s];
            p = sh.rp[s];
            pw_old = sh.rpw[s];
            const int L = sh.rL[s];
            const int cv = sh.rcomp[s * 64 + (lane < CS ? lane : 0)];
            my_comp = lane < E ? cv : 0;
            const int na = sh.rcomp[s * 64 + E];
            bool overflow;
            if constexpr (SITE) {
                if (coop) {
                    unsigned char *w0 = lds + a.o_wave;  // wavefront 0's slice holds the tables
                    score_site_coop<WM, DT>(a, sh, sh.rseq + (int64_t)s * RS, L, p, my_comp, na,
                                        (DT *)(w0 + a.w_dt), (int64_t *)(w0 + a.w_bg),
                                        (int32_t *)(w0 + a.w_comp),
                                        (unsigned long long *)(lds + a.o_red), lane, w, NW, bv,
                                        newp, segc, overflow STAMP_ARGS);
                } else {
                    score_site<WM, DT>(a, sh, sh.rseq + (int64_t)s * RS, L, p, my_comp, na, Dt, wbg,
                                   wcomp, lane, bv, newp, segc, overflow STAMP_ARGS);
                }
            } else if (kMotifCoop && coop) {
                unsigned char *w0 = lds + a.o_wave;
                score_target_coop<WM>(a, sh, sh.rseq + (int64_t)s * RS, L, p, my_comp, na,
                                      w0 + a.w_tab, (double *)(w0 + a.w_pcv),
                                      (unsigned long long *)(lds + a.o_red), lane, w, NW, bv,
                                      newp, segc, overflow);
            } else {
                score_target<WM>(a, sh, sh.rseq + (int64_t)s * RS, L, p, my_comp, na, tab, pcv,
                                 lane, bv, newp, segc, overflow STAMP_ARGS);
            }
            ev = !act ? 0 : overflow ? 2 : ((bv > pw_old && newp != p) ? 1 : 0);
        }
        STAMP(2);
        // the fetched visit's slot is not read in this step
        if (fetch) store_slot((int)((b + NW + w) & (R - 1)), pf, cpf, tpf, Lpf, opf, ppf, pwpf);
        if (lane == 0) sh.ctl[w] = ev;
        STAMP(3);
        __syncthreads();
        STAMP(4);
        // the first event (a move or an overflow) in visit order
        const unsigned long long evm = __ballot(lane < nb && sh.ctl[lane < nb ? lane : 0] != 0);
        const int f = evm ? __builtin_ctzll(evm) : nb;
        const int fev = f < nb ? sh.ctl[f] : 0;
        if (fev == 2) {  // the sequential loop raises here (.fs:117)
            if (w == f && lane == 0) {
                atomicCAS(a.err_code, 0, 3);
                atomicMin(a.err_index, (unsigned long long)t);
            }
            break;
        }
        if (act && w <= f && bv > pw_old) {  // .fs:921-925
            const bool mv = w == f;
            if (lane == 0) {  // to L2: later prefetches read it there
                __hip_atomic_store((unsigned long long *)&a.pwms[t],
                                   (unsigned long long)__double_as_longlong(bv), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
                if (mv) __hip_atomic_store(&a.pos[t], newp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            // ring slots holding this target carry its new state
            if (lane < R && sh.rt[lane] == t) {
                sh.rpw[lane] = bv;
                if (mv) sh.rp[lane] = newp;
            }
            if (mv) move_segment<WM>(a, sh, sh.rseq + (int64_t)s * RS, p, newp, my_comp, segc, lane);
        }
        moved |= f < nb;
        const int adv = f < nb ? f + 1 : nb;
        width = f < nb ? max(1, f) : min(NW, 2 * nb);
        if (kCoop) {
            // moves per visit, a running average over ~16 visits; while it stays above
            // coop_rate the steps keep one visit (scored by the whole workgroup): a
            // widened step of single-wavefront visits costs ~3 lone visits there
            mrate += ((float)(f < nb) - (float)adv * mrate) * (1.0f / 16.0f);
            mrate = fminf(fmaxf(mrate, 0.0f), 1.0f);
            if (a.coop_rate > 0.0f && mrate > a.coop_rate && NW > 1 &&
                (SITE ? a.site_coop != 0 : a.motif_coop > 0))
                width = 1;
        }
        b += adv;
        if (a.exit_chunk > 0) {
            chunk_moves += f < nb;
            if (b - chunk_start >= a.exit_chunk) {
                exit_mid = b < pass_end &&
                           (int64_t)chunk_moves * a.exit_ratio < b - chunk_start;
                chunk_start = b;
                chunk_moves = 0;
            }
        }
        tb = target_at(adv);
        // descriptors of the next step's fetch, in flight across the barrier
        fresh = adv;
        if (w >= NW - fresh) {
            tpf = target_at(NW + w);
            Lpf = a.len[tpf];
            opf = a.doff[tpf];
            cpf = lane < CS ? a.comp[(int64_t)tpf * CS + lane] : 0;
        }
        STAMP(5);
        __syncthreads();
        STAMP(6);
        if (b == pass_end) {
            ++passes;
            if (!moved || passes >= a.max_passes) break;
            moved = false;
            pass_end += N;
            chunk_start = b;
            chunk_moves = 0;
        }
        if (exit_mid) break;  // the rest of this pass goes to the speculative steps
    }
    __syncthreads();
    // the aggregates of the final positions: replica 0, the others zero
    for (int64_t i = tid; i < (int64_t)kRepl * a.stride; i += blockDim.x) {
        int64_t v = 0;
        if (i < a.cells) v = i < AW ? (int64_t)sh.C[i] : sh.T[i - AW];
        a.agg[i] = v;
    }
    if (tid == 0) {
        *a.passes_out = passes;
        if (a.exit_out) {
            a.exit_out[0] = exit_mid ? (int32_t)(b - (pass_end - N)) : 0;
            a.exit_out[1] = moved ? 1 : 0;
        }
    }
    (void)steps;
    STAMP_FLUSH(steps);
}

#define GS_FOR_EACH_WM(X) X(4) X(8) X(12) X(16) X(20) X(24) X(28) X(32) X(40) X(48) X(56) X(64)

static const void *greedy_kernel_ptr(int wm, bool site, bool d16) {
    switch (wm) {
#define GS_CASE(N) \
    case N:        \
        return !site ? (const void *)&gs_greedy_kernel<false, N, int32_t> \
               : d16 ? (const void *)&gs_greedy_kernel<true, N, uint16_t> \
                     : (const void *)&gs_greedy_kernel<true, N, int32_t>;
        GS_FOR_EACH_WM(GS_CASE)
#undef GS_CASE
    }
    return nullptr;
}

int gs_sweep_wm(int W);

// One workgroup of `waves` wavefronts; lds_bytes from the host carve (gs_api.cpp).
hipError_t gs_greedy_launch(const GreedyArgs &a, int waves, size_t lds_bytes, hipStream_t stream,
                            hipEvent_t start, hipEvent_t stop) {
    const void *k = greedy_kernel_ptr(gs_sweep_wm(a.W), a.site != 0, a.dt16 != 0);
    if (!k || waves < 1 || waves > 8 || (waves & (waves - 1))) return hipErrorInvalidValue;
    GreedyArgs args = a;
    void *params[] = {&args};
    return hipExtLaunchKernel(k, dim3(1), dim3(64 * waves), params, lds_bytes, stream, start, stop,
                              0);
}
