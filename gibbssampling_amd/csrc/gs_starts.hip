// gs_starts.hip — site-sampler kernels for gfx950: the argmax scan
// SiteSampler.getBestPWMSs (.fs:462-479) and the passes built on it:
// getPWMOfRandomStarts (.fs:589-611) and the Jacobi scans of the ±1 shifted passes
// (.fs:483-550).  The Gauss–Seidel getBestPWMSsWithStartPositions (.fs:554-585)
// shares the greedy kernel's speculative engine (gs_greedy.hip, score_site).
//
// getBestPWMSs mutates its background vector in place window after window
// (increaseInPlaceFCVOf + aliased substractSegmentCountsFrom, .fs:471-472, quirk
// Q1), so the background of window k is
//   fcv_k[b] = bg0[b] + (k+1)·comp(s_n)[b] − D_k[b],   D_k[b] = Σ_{i≤k} count_b(window_i).
// The kernels build D_k with wavefront prefix sums (integer exact), which makes
// all windows independent; the argmax keeps the reference's strict '>' from
// (0.0, 0): the first maximal window wins.
#include <hip/hip_runtime.h>

#include "gs_common.h"

using namespace gs;

namespace {

__device__ __forceinline__ int32_t wave_incl_scan_i32(int32_t x, int lane) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        int32_t y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    return x;
}
__device__ __forceinline__ int64_t wave_sum_i64(int64_t x) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
    return x;
}

// getBestPWMSs (.fs:462-479) of the staged sequence sseq[0, L) for a one-wavefront
// workgroup: ppm [A][W] of the others (normalizePPM, LDS), their background bg0[A]
// (fuseFrequencyVectors over the alphabet) with bsum = Σ_a bg0[a], comp[] the
// sequence's symbol counts by encoded symbol; Dt is [(L+1)][A] int32 scratch.
// Returns the wave-uniform first maximum of S_k (0.0 / window 0 when no S_k > 0)
// and whether a window's background sum overflows int32 (Checked Array.sum, .fs:117).
__device__ __forceinline__ void best_pwms_scan(const uint8_t *sseq, int L, int W, int A, const double *ppm,
                               const int64_t *bg0, int64_t bsum, const int32_t *comp,
                               int32_t *Dt, double pc, double apc, const double *pcvf, int lane,
                               double &best_out, int &bestk_out, bool &overflow_out) {
    const int K = L - W + 1;
    if (pcvf) {  // getBestPWMSsWithBPV (.fs:301-313): the caller's PCV, no drift
        double best = 0.0;
        int bestk = 0x7fffffff;
        for (int k = lane; k < K; k += 64) {
            double S = 1.0;
            for (int j = 0; j < W; ++j) {
                const int e = sseq[k + j];
                S = S * (e < A ? ppm[e * W + j] / pcvf[e] : 0.0);
            }
            if (S > best) {
                best = S;
                bestk = k;
            }
        }
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) {
            double ob = __shfl_xor(best, d, 64);
            int ok = __shfl_xor(bestk, d, 64);
            if (ob > best || (ob == best && ok < bestk)) {
                best = ob;
                bestk = ok;
            }
        }
        best_out = best;
        bestk_out = bestk == 0x7fffffff ? 0 : bestk;
        overflow_out = false;
        __syncthreads();
        return;
    }
    // ---- D_k[a] = Σ_{i≤k} count_a(window_i) by two prefix sums per symbol ----
    for (int x = 0; x < A; ++x) {
        // P_x(i) = #x in s[0, i), kept in Dt row i (rows up to L are carved)
        int32_t carry = 0;
        for (int i0 = 0; i0 < L + 1; i0 += 64) {
            const int i = i0 + lane;
            int32_t ind = (i < L && sseq[i] == x) ? 1 : 0;
            int32_t incl = wave_incl_scan_i32(ind, lane);
            if (i <= L) Dt[i * A + x] = carry + incl - ind;
            carry += __shfl(incl, 63, 64);
        }
    }
    __syncthreads();
    // count_x(window_k) = P_x(k+W) − P_x(k); inclusive scan over k -> D_k
    for (int x = 0; x < A; ++x) {
        int32_t carry = 0;
        for (int k0 = 0; k0 < K; k0 += 64) {
            const int k = k0 + lane;
            int32_t cw = 0;
            if (k < K) cw = Dt[(k + W) * A + x] - Dt[k * A + x];
            int32_t incl = wave_incl_scan_i32(cw, lane);
            // all lanes have read their P values for this chunk before any write
            __syncthreads();
            if (k < K) Dt[k * A + x] = carry + incl;
            carry += __shfl(incl, 63, 64);
            __syncthreads();
        }
    }
    __syncthreads();
    // ---- window scan with the drifting background (.fs:463-479) ----
    double best = 0.0;
    int bestk = 0x7fffffff;
    bool overflow = false;
    for (int k0 = 0; k0 < K; k0 += 64) {
        const int k = k0 + lane;
        if (k >= K) continue;
        const int64_t kk = (int64_t)k + 1;
        // Σ over all 49 slots of fcv_k (Checked Array.sum, .fs:117)
        const int64_t tot = bsum + kk * (int64_t)L - kk * (int64_t)W;
        if (tot > 2147483647LL) overflow = true;
        const double sbg = (double)tot + apc;
        // four columns per step, branch-free (columns past W multiply by exactly 1.0,
        // non-alphabet symbols by 0.0): their binary64 divisions overlap; the fold
        // stays the reference's left fold
        double S = 1.0;
        for (int j0 = 0; j0 < W; j0 += 4) {
            double v[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int j = j0 + i, jc = j < W ? j : W - 1;
                const int e = sseq[k + jc];
                const int ec = e < A ? e : 0;
                const int64_t f = bg0[ec] + kk * (int64_t)comp[ec] - (int64_t)Dt[k * A + ec];
                const double pcv = ((double)f + pc) / sbg;
                const double x = ppm[ec * W + jc] / pcv;
                v[i] = j < W ? (e < A ? x : 0.0) : 1.0;
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) S = S * v[i];
        }
        if (S > best) {  // strict '>' (.fs:477); per lane k increases
            best = S;
            bestk = k;
        }
    }
    overflow_out = __ballot(overflow) != 0ull;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        double ob = __shfl_xor(best, d, 64);
        int ok = __shfl_xor(bestk, d, 64);
        if (ob > best || (ob == best && ok < bestk)) {
            best = ob;
            bestk = ok;
        }
    }
    best_out = best;
    bestk_out = bestk == 0x7fffffff ? 0 : bestk;
    __syncthreads();  // Dt is rewritten by the caller's next sequence
}

// Stage sequence n (16-byte chunks; bytes past L are never read) and its symbol
// counts by encoded symbol (createFCVOf, .fs:60-62).
__device__ void stage_sequence(const uint8_t *g, int L, uint8_t *sseq, int32_t *comp, int lane) {
    for (int i = lane * 16; i < L; i += 64 * 16) *(uint4 *)(sseq + i) = *(const uint4 *)(g + i);
    comp[lane] = 0;
    comp[lane + 64] = 0;
    __syncthreads();
    for (int i = lane; i < L; i += 64) atomicAdd(&comp[sseq[i]], 1);
    __syncthreads();
}

}  // namespace

// Exact mode: for every global target t, the PFM of the other sequences of this
// rank at their own fresh random starts r_{t,m} (createPFMOf/fuse, .fs:603-606).
extern "C" __global__ void __launch_bounds__(64) gs_starts_partial_kernel(PartialArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    int32_t *cnt = (int32_t *)lds;
    const int lane = threadIdx.x;
    const int AW = a.A * a.W;
    for (int64_t t = blockIdx.x; t < a.n_global; t += gridDim.x) {
        for (int c = lane; c < AW; c += 64) cnt[c] = 0;
        __syncthreads();
        const uint64_t st = stream_init((uint64_t)t);
        for (int m = lane; m < a.n_local; m += 64) {
            const int64_t mg = a.global_offset + m;
            if (mg == t) continue;
            const int L = a.len[m];
            const int r = uniform_int(a.seed, st, (uint64_t)mg, L - a.W + 1);
            const uint8_t *s = a.seq + a.doff[m] + r;
            for (int j = 0; j < a.W; ++j) {
                const int e = s[j];
                if (e < a.A) atomicAdd(&cnt[e * a.W + j], 1);
            }
        }
        __syncthreads();
        for (int c = lane; c < AW; c += 64) a.cpart[t * AW + c] = cnt[c];
        __syncthreads();
    }
}

// One Jacobi pass: getBestPWMSs of every local target with the others at their
// start vector (mode 0: per-target draws via cpart; 1: shared draws; 2: `starts`).
// GD: the D table in HBM (a.dt_global, sequences too long for the LDS carve); the
// workgroup is one wavefront, so its own global writes and reads need no fence.
template <bool GD>
__global__ void __launch_bounds__(64) gs_starts_kernel(StartsArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int lane = threadIdx.x;
    const int A = a.A, W = a.W, AW = A * W;
    double *ppm = (double *)(lds + a.o_ppm);        // [A][W]
    int32_t *Dt = GD ? a.dt_global + (int64_t)blockIdx.x * a.dt_stride
                     : (int32_t *)(lds + a.o_Dt);   // [Lmax+1][A]
    int32_t *cg = (int32_t *)(lds + a.o_cg);        // [A*W] + [A*W] scratch
    int64_t *compall = (int64_t *)(lds + a.o_compall);  // [A]
    int64_t *bg0 = (int64_t *)(lds + a.o_bg);       // [A]
    int32_t *comp = (int32_t *)(lds + a.o_comp);    // [128]
    uint8_t *sseq = (uint8_t *)(lds + a.o_seq);

    for (int c = lane; c < a.cells; c += 64) {
        int64_t s = 0;
#pragma unroll
        for (int r = 0; r < kRepl; ++r) s += a.agg[(int64_t)r * a.stride + c];
        if (c < AW)
            cg[c] = (int32_t)s;
        else
            compall[c - AW] = s;  // Σ (composition - segment) over the start vector
    }
    __syncthreads();
    // composition totals: the background cells plus the segments' counts
    if (lane < A) {
        int64_t s = 0;
        for (int j = 0; j < W; ++j) s += cg[lane * W + j];
        compall[lane] += s;
    }
    __syncthreads();

    // speculative Gauss–Seidel step: one visit per workgroup from the control block
    int n_first = blockIdx.x, n_end = a.n_local, n_step = gridDim.x, base = 0;
    if (a.spec_ctl) {
        const SpecCtl ctl = *a.spec_ctl;
        if (ctl.done) return;
        base = ctl.base;
        n_first = base + blockIdx.x;
        n_end = min(n_first + 1, a.n_local);
        n_step = 1;
    }
    if (a.single > 0) {
        if (blockIdx.x > 0) return;
        n_first = a.single - 1;
        n_end = a.single;
        n_step = 1;
    }
    for (int n = n_first; n < n_end; n += n_step) {
        const int L = a.len[n];
        const int K = L - W + 1;
        const int64_t gidx = a.global_offset + n;
        stage_sequence(a.seq + a.doff[n], L, sseq, comp, lane);

        // ---- others' count matrix and background (.fs:599-609) ----
        int r = 0;
        if (a.mode == 1) r = uniform_int(a.seed, stream_init_shared(), (uint64_t)gidx, K);
        if (a.mode == 2) r = a.starts[n];
        for (int c = lane; c < AW; c += 64) {
            const int x = c / W, j = c - x * W;
            int32_t v;
            if (a.mode != 0)
                v = cg[c] - (sseq[r + j] == x ? 1 : 0);
            else
                v = a.cpart[gidx * AW + c];
            // normalizePPM (.fs:257-260), or the caller's PPM (.fs:644-662)
            ppm[c] = a.ppm_fixed ? a.ppm_fixed[c] : ((double)v + a.pc) / a.den;
            cg[AW + c] = v;
        }
        __syncthreads();
        int64_t bsum = 0;
        if (lane < A) {
            int64_t s = 0;
            for (int j = 0; j < W; ++j) s += cg[AW + lane * W + j];
            // Σ_{m≠n} (comp_m − comp(seg_m))[a] = (Σ_all comp − comp_n)[a] − Σ_j C_{−n}[a][j]
            int64_t v = compall[lane] - comp[lane] - s;
            if (a.bg_fixed) v = a.bg_fixed[lane];  // the caller's FrequencyCompositeVector
            bg0[lane] = v;
            bsum = v;
        }
        bsum = wave_sum_i64(bsum);
        if (a.bg_fixed) bsum = a.bg_fixed[A];  // its sum over all 49 slots
        __syncthreads();
        double best;
        int bestk;
        bool overflow;
        best_pwms_scan(sseq, L, W, A, ppm, bg0, bsum, comp, Dt, a.pc, a.apc, a.pcv_fixed, lane,
                       best, bestk, overflow);
        if (overflow) {
            if (lane == 0) {
                atomicCAS(a.err_code, 0, 3);
                atomicMin(a.err_index, (unsigned long long)gidx);
            }
            continue;
        }
        if (lane == 0) {
            const double sc = log(best) / kLn2;
            if (a.spec_ctl) {
                a.spec_res[n - base].score = sc;
                a.spec_res[n - base].pos = bestk;
            } else {
                a.pos_out[n] = bestk;
                a.score_out[n] = sc;
            }
        }
    }
}

// Commit of one speculative step of getBestPWMSsWithStartPositions (.fs:554-585):
// the scored visits [base, base + slots) in order, each taking its scan's result when
// strictly better (fst tmp > fst acc.[n]), up to and including the first whose start
// changes; the live aggregates follow that move, base moves past it.  Pass end as in
// .fs:556-559: stop when a pass changed no start, or at max_passes.
extern "C" __global__ void __launch_bounds__(64) gs_site_spec_commit_kernel(SiteCommitArgs a) {
    const SpecCtl c0 = *a.ctl;
    if (c0.done) return;
    const int lane = threadIdx.x;
    const int base = c0.base, nres = min(a.slots, a.n - base);
    int first = nres;
    for (int w0 = 0; w0 < nres; w0 += 64) {
        const int w = w0 + lane;
        const bool f = w < nres && a.res[w].score > a.score[base + w] &&
                       a.res[w].pos != a.pos[base + w];
        const unsigned long long m = __ballot(f);
        if (m) {
            first = w0 + __ffsll((long long)m) - 1;
            break;
        }
    }
    for (int w = lane; w < first; w += 64)
        if (a.res[w].score > a.score[base + w]) a.score[base + w] = a.res[w].score;  // same start
    int nbase = base + nres, changed = c0.changed;
    if (first < nres) {
        const int n = base + first;
        const int po = a.pos[n], pn = a.res[first].pos;
        const uint8_t *s = a.seq + a.doff[n];
        unsigned long long *C = (unsigned long long *)a.agg, *T = C + a.A * a.W;
        if (lane < a.W) {
            const int eo = s[po + lane], en = s[pn + lane];
            if (eo < a.A) {
                atomicAdd(&C[eo * a.W + lane], ~0ull);
                atomicAdd(&T[eo], 1ull);
            }
            if (en < a.A) {
                atomicAdd(&C[en * a.W + lane], 1ull);
                atomicAdd(&T[en], ~0ull);
            }
        }
        __syncthreads();
        if (lane == 0) {
            a.pos[n] = pn;
            a.score[n] = a.res[first].score;
        }
        changed = 1;
        nbase = n + 1;
    }
    if (lane == 0) {
        SpecCtl c = c0;
        c.base = nbase;
        c.changed = changed;
        if (nbase >= a.n) {
            ++c.pass;
            if (!c.changed || c.pass >= a.max_passes)
                c.done = 1;
            else {
                c.base = 0;
                c.changed = 0;
            }
        }
        *a.ctl = c;
    }
}

// The others' start vector of a shifted pass (.fs:489-492, .fs:525-527): +1 while the
// segment still fits, -1 while the start is positive.
extern "C" __global__ void __launch_bounds__(256)
gs_site_shift_kernel(const int32_t *pos, const int32_t *len, int32_t n, int32_t W, int32_t dir,
                     int32_t *out) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const int p = pos[i];
    out[i] = dir > 0 ? (p <= len[i] - W - 1 ? p + 1 : p) : (p > 0 ? p - 1 : p);
}

// acc.[n] <- tmp when fst tmp > fst acc.[n] (.fs:509, .fs:544); moved counts the
// targets whose position changed (the pass-end comparison with bestMotif).
extern "C" __global__ void __launch_bounds__(256)
gs_site_accept_kernel(const double *tmp_score, const int32_t *tmp_pos, double *score,
                      int32_t *pos, int32_t n, int32_t *moved) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    bool mv = false;
    if (i < n && tmp_score[i] > score[i]) {
        score[i] = tmp_score[i];
        mv = tmp_pos[i] != pos[i];
        pos[i] = tmp_pos[i];
    }
    const unsigned long long b = __ballot(mv);
    if ((threadIdx.x & 63) == 0 && b) atomicAdd(moved, __popcll(b));
}

hipError_t gs_starts_launch(const StartsArgs &a, int grid, size_t lds_bytes, hipStream_t s) {
    if (a.dt_global)
        hipLaunchKernelGGL(gs_starts_kernel<true>, dim3(grid), dim3(64), lds_bytes, s, a);
    else
        hipLaunchKernelGGL(gs_starts_kernel<false>, dim3(grid), dim3(64), lds_bytes, s, a);
    return hipGetLastError();
}
// `steps` speculative Gauss–Seidel steps of the site sampler (score + commit each).
hipError_t gs_site_spec_launch(const StartsArgs &a, const SiteCommitArgs &ca, size_t lds_bytes,
                               int steps, hipStream_t s) {
    for (int i = 0; i < steps; ++i) {
        if (a.dt_global)
            hipLaunchKernelGGL(gs_starts_kernel<true>, dim3(ca.slots), dim3(64), lds_bytes, s, a);
        else
            hipLaunchKernelGGL(gs_starts_kernel<false>, dim3(ca.slots), dim3(64), lds_bytes, s, a);
        hipLaunchKernelGGL(gs_site_spec_commit_kernel, dim3(1), dim3(64), 0, s, ca);
    }
    return hipGetLastError();
}

hipError_t gs_starts_partial_launch(const PartialArgs &a, int grid, hipStream_t s) {
    hipLaunchKernelGGL(gs_starts_partial_kernel, dim3(grid), dim3(64),
                       (size_t)a.A * a.W * sizeof(int32_t), s, a);
    return hipGetLastError();
}
hipError_t gs_site_shift_launch(const int32_t *pos, const int32_t *len, int32_t n, int32_t W,
                                int32_t dir, int32_t *out, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(gs_site_shift_kernel, dim3((n + 255) / 256), dim3(256), 0, s, pos, len, n,
                       W, dir, out);
    return hipGetLastError();
}
hipError_t gs_site_accept_launch(const double *tmp_score, const int32_t *tmp_pos, double *score,
                                 int32_t *pos, int32_t n, int32_t *moved, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(gs_site_accept_kernel, dim3((n + 255) / 256), dim3(256), 0, s, tmp_score,
                       tmp_pos, score, pos, n, moved);
    return hipGetLastError();
}
