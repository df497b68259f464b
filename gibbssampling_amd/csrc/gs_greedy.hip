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
// The target order is a true data dependence, so one persistent wavefront walks
// the targets: the count aggregates C[A][W] and T[A] live in LDS
// and change by one segment when a target moves (O(W + A) integer updates), the
// next target's sequence is prefetched into registers while the current one is
// scored, and every window is folded in binary64 exactly as the reference does
// (gs_fold.h), so the picks are bit-identical.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <climits>

#include "gs_common.h"
#include "gs_fold.h"
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

}  // namespace

template <int WM>
__global__ void __launch_bounds__(64) gs_greedy_kernel(GreedyArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    constexpr int WS = tab_stride(WM);
    const int lane = threadIdx.x;
    const int A = a.A, W = a.W, E = a.E, AW = A * W, CS = E + 1;
    int32_t *C = (int32_t *)(lds + a.o_C);          // [A][W] counts of the live segments
    int64_t *T = (int64_t *)(lds + a.o_T);          // [A] Σ (composition − segment)
    unsigned char *tab = lds + a.o_tab;              // [E][WS] (PWM, PCV) binary64 pairs
    double *pcv = (double *)(lds + a.o_pcv);         // [64]
    uint8_t *sseq = (uint8_t *)(lds + a.o_seq);      // the target's symbols + zero tail
    int32_t *scnt = (int32_t *)(lds + a.o_misc);     // [64] segment symbol counts

    if (__builtin_amdgcn_readfirstlane(*a.err_code) != 0) return;  // void snapshot

    for (int c = lane; c < a.cells; c += 64) {
        int64_t s = 0;
#pragma unroll
        for (int r = 0; r < kRepl; ++r) s += a.agg[(int64_t)r * a.stride + c];
        if (c < AW)
            C[c] = (int32_t)s;
        else
            T[c - AW] = s;
    }
    // columns past the motif fold as exact 1.0 factors
    for (int c = lane; c < E * WS; c += 64)
        if (c % WS >= W) *(double2 *)(tab + c * 16) = make_double2(1.0, 1.0);
    __syncthreads();

    const int N = a.n;
    // the first target, then one-ahead prefetch of the next
    int nL = a.len[0];
    int64_t nO = a.doff[0];
    uint4 pf = make_uint4(0, 0, 0, 0);
    if (nL <= 1024 && lane * 16 < nL) pf = *(const uint4 *)(a.seq + nO + lane * 16);
    int cpf = lane < CS ? a.comp[lane] : 0;
    int npos = load_relaxed(&a.pos[0]);
    double npw = load_relaxed(&a.pwms[0]);

    int passes = 0;
    bool failed = false;
    for (;;) {
        bool moved = false;
        for (int n = 0; n < N; ++n) {
            const int L = nL, p = npos;
            const int64_t off = nO;
            const double pw_old = npw;
            const int K = L - W + 1;
            if (L <= 1024) {
                if (lane * 16 < L) *(uint4 *)(sseq + lane * 16) = keep_bytes(pf, L - lane * 16);
            } else {
                for (int i = lane * 16; i < L; i += 1024)
                    *(uint4 *)(sseq + i) = keep_bytes(*(const uint4 *)(a.seq + off + i), L - i);
            }
            // createFCVOf (.fs:60-62), precomputed: lane e < E holds the count of e
            const int my_comp = lane < E ? cpf : 0;
            const int na = __builtin_amdgcn_readlane(cpf, E);  // symbols outside the alphabet
            const int nn = n + 1 < N ? n + 1 : 0;
            nL = a.len[nn];
            nO = a.doff[nn];
            if (nL <= 1024 && lane * 16 < nL) pf = *(const uint4 *)(a.seq + nO + lane * 16);
            if (lane < CS) cpf = a.comp[(int64_t)nn * CS + lane];
            npos = load_relaxed(&a.pos[nn]);
            npw = load_relaxed(&a.pwms[nn]);
            // zero tail: unrolled window reads past L see symbol 0 (a valid table row)
            for (int i = ((L + 15) & ~15) + lane * 16; i < L + WM + 16; i += 1024)
                *(uint4 *)(sseq + i) = make_uint4(0, 0, 0, 0);
            scnt[lane] = 0;
            wave_sync();

            // ---- hold-one-out background from the live positions (.fs:891-893) ----
            if (p >= 0)
                for (int j = lane; j < W; j += 64) atomicAdd(&scnt[sseq[p + j]], 1);
            wave_sync();
            const int segc = lane < E ? scnt[lane] : 0;
            const int seg_alpha = wave_sum_i32(lane < A ? segc : 0);
            const int64_t sumT = (int64_t)wave_sum_f64(lane < A ? (double)T[lane] : 0.0);
            const int64_t bgc = lane < A ? T[lane] + (p >= 0 ? segc : my_comp) : 0;
            const int64_t tot = sumT + (p >= 0 ? seg_alpha : L - na) + na;
            if (tot > 2147483647LL) {  // Checked Array.sum (.fs:117)
                if (lane == 0) {
                    atomicCAS(a.err_code, 0, 3);
                    atomicMin(a.err_index, (unsigned long long)n);
                }
                failed = true;
                break;
            }
            // PCV (.fs:119); outside the alphabet the raw count (Q3)
            const double sbg = (double)tot + a.apc;
            const double pe = lane < A ? ((double)bgc + a.pc) / sbg : (double)my_comp;
            if (lane < E) pcv[lane] = pe;
            wave_sync();
            // ---- PWM of the others (.fs:255-261, .fs:282-287): own cells count C - 1 ----
            for (int c = lane; c < E * W; c += 64) {
                const int e = c / W, j = c - e * W;
                const double pe_e = pcv[e];
                double v = 0.0;
                if (e < A) {
                    const bool own = (p >= 0) && (sseq[p + j] == e);
                    const double pm = ((double)(C[e * W + j] - (own ? 1 : 0)) + a.pc) / a.den;
                    v = pm / pe_e;
                }
                *(double2 *)(tab + (e * WS + j) * 16) = make_double2(v, pe_e);
            }
            wave_sync();
            // ---- categories (.fs:759-782) and the head of their descending sort ----
            double bv = __builtin_nan("");
            int bo = INT_MAX;
            for (int k = lane; k < K; k += 64) {
                double g, m;
                exact_eval<WM>(sseq, tab, a.thr_lo, a.cutoff, k, g, m);
                if (sorts_first(g, k, bv, bo)) {
                    bv = g;
                    bo = k;
                }
                if (m > -INFINITY && sorts_first(m, K + k, bv, bo)) {
                    bv = m;
                    bo = K + k;
                }
            }
#pragma unroll
            for (int d = 32; d >= 1; d >>= 1) {
                const double ov = __shfl_xor(bv, d, 64);
                const int oo = __shfl_xor(bo, d, 64);
                if (sorts_first(ov, oo, bv, bo)) {
                    bv = ov;
                    bo = oo;
                }
            }
            const int newp = bo < K ? -1 : bo - K;
            int p_now = p;
            double pw_now = pw_old;
            if (bv > pw_old) {  // .fs:921-925
                pw_now = bv;
                if (lane == 0) a.pwms[n] = bv;
                if (newp != p) {
                    // the old segment leaves the aggregates, the new one enters
                    if (p >= 0) {
                        for (int j = lane; j < W; j += 64) {
                            const int s = sseq[p + j];
                            if (s < A) C[s * W + j] -= 1;
                        }
                        if (lane < A) T[lane] -= my_comp - segc;
                        scnt[lane] = 0;
                    }
                    wave_sync();
                    if (newp >= 0) {
                        for (int j = lane; j < W; j += 64) {
                            const int s = sseq[newp + j];
                            atomicAdd(&scnt[s], 1);
                            if (s < A) C[s * W + j] += 1;
                        }
                        wave_sync();
                        if (lane < A) T[lane] += my_comp - scnt[lane];
                    }
                    if (lane == 0) a.pos[n] = newp;
                    p_now = newp;
                    moved = true;
                }
            }
            if (nn == n) {  // a single target: the prefetch predates its own update
                npos = p_now;
                npw = pw_now;
            }
            wave_sync();
        }
        if (failed) break;
        ++passes;
        if (!moved || passes >= a.max_passes) break;
    }
    // the aggregates of the final positions: replica 0, the others zero
    for (int64_t i = lane; i < (int64_t)kRepl * a.stride; i += 64) {
        int64_t v = 0;
        if (i < a.cells) v = i < AW ? (int64_t)C[i] : T[i - AW];
        a.agg[i] = v;
    }
    if (lane == 0) *a.passes_out = passes;
}

#define GS_FOR_EACH_WM(X) X(4) X(8) X(12) X(16) X(20) X(24) X(28) X(32) X(40) X(48) X(56) X(64)

static const void *greedy_kernel_ptr(int wm) {
    switch (wm) {
#define GS_CASE(N) \
    case N:        \
        return (const void *)&gs_greedy_kernel<N>;
        GS_FOR_EACH_WM(GS_CASE)
#undef GS_CASE
    }
    return nullptr;
}

int gs_sweep_wm(int W);

// One wavefront; lds_bytes from the host carve (gs_api.cpp greedy_carve).
hipError_t gs_greedy_launch(const GreedyArgs &a, size_t lds_bytes, hipStream_t stream,
                            hipEvent_t start, hipEvent_t stop) {
    const void *k = greedy_kernel_ptr(gs_sweep_wm(a.W));
    if (!k) return hipErrorInvalidValue;
    GreedyArgs args = a;
    void *params[] = {&args};
    return hipExtLaunchKernel(k, dim3(1), dim3(64), params, lds_bytes, stream, start, stop, 0);
}
