// gs_sweep.hip — fused Gibbs sweep kernel for gfx950 (MI355X).
//
// A workgroup is 4 independent 64-lane wavefronts; each wavefront grid-strides
// over this rank's sequences.  Per sequence n (MotifSampler.
// findBestMotifIndicesByWithStartPositions, .fs:935-970, motifAmount = 1):
//   1. stage the encoded sequence into the wavefront's LDS slice (16-byte loads,
//      prefetched one sequence ahead), symbol histogram (createFCVOf, .fs:60-62);
//   2. hold-one-out background counts and PCV from the snapshot aggregates
//      (createFCVWithout/fuseFrequencyVectors/increaseInPlaceFCVOf/
//      createNormalizedPCVOfFCV, .fs:945-954) — integer exact;
//   3. PWM = PPM/PCV (.fs:955-965).  The PPM of the global counts and of the
//      counts minus one are built once per workgroup; per sequence only the
//      division by the PCV remains.  Staged as a [j][symbol] table of
//      (PWM, PCV) pairs so one ds_read_b128 feeds both window products;
//   4. every W-mer window (.fs:759-777): S_k = left fold of PWM factors,
//      G_k = left fold of PCV factors, IEEE binary64 in the reference's order;
//      the W-loop is unrolled (template WM = W rounded up, padded with factors
//      1.0, which multiply exactly); log2 cut-off test (.fs:735-738).  Lane l
//      scores the contiguous windows [l*R, l*R+R) so its category sums stay in
//      registers;
//   5. roulette pick (.fs:746-754): one wavefront prefix sum of the lane sums
//      gives a certified pick; if u lies within the rounding bound of a CDF
//      boundary one lane redoes the reference's sequential sums exactly;
//   6. the picked segment is folded into per-wavefront aggregates of the new
//      snapshot, flushed to XCD-replicated global accumulators once per
//      workgroup: the next sweep's count matrix and background totals.
//
// Compiled with -ffp-contract=off: no FMA contraction.
#include <hip/hip_runtime.h>

#include "gs_common.h"
#include "gs_wave.h"

using namespace gs;

namespace {

constexpr int kWavesPerBlock = 4;

// In-kernel phase stamps, diagnostic build only (make STAMPS=1): never in the
// shipped library; their run time is not quoted, only the phase shares.
#ifdef GS_STAMPS
#define STAMP_DECL                      \
    unsigned long long st_acc[8] = {0}; \
    unsigned long long st_prev = __builtin_amdgcn_s_memtime();
#define STAMP(i)                                              \
    do {                                                      \
        __builtin_amdgcn_sched_barrier(0);                    \
        unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
        st_acc[i] += t_ - st_prev;                            \
        st_prev = t_;                                         \
        __builtin_amdgcn_sched_barrier(0);                    \
    } while (0)
#define STAMP_FLUSH(nseq)                                                        \
    do {                                                                         \
        if (lane == 0 && a.stamps) {                                             \
            for (int i_ = 0; i_ < 7; ++i_) atomicAdd(&a.stamps[i_], st_acc[i_]); \
            atomicAdd(&a.stamps[7], (unsigned long long)(nseq));                 \
        }                                                                        \
    } while (0)
#else
#define STAMP_DECL
#define STAMP(i) \
    do {         \
    } while (0)
#define STAMP_FLUSH(nseq) \
    do {                  \
    } while (0)
#endif

__device__ __forceinline__ void raise_error(const SweepArgs &a, int code, int64_t gidx) {
    atomicCAS(a.err_code, 0, code);
    atomicMin(a.err_index, (unsigned long long)gidx);
}

// S_k and G_k of window k: the reference's left folds (.fs:291-292, .fs:124).
// tab: [WM][E] (PWM, PCV) pairs, columns j >= W hold (1.0, 1.0).
template <int WM>
__device__ __forceinline__ void window_products(const uint8_t *sseq, const unsigned char *tab,
                                                int E16, int k, double &S, double &G) {
    constexpr int ND = WM / 4 + 1;
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
            const double2 v = *(const double2 *)(tab + j * E16 + (e << 4));
            S = S * v.x;
            G = G * v.y;
        }
    }
    // materialise both folds here: otherwise the G fold is sunk below the caller's
    // log2 branch and every table operand stays live across it (VGPRs, occupancy)
    asm volatile("" ::"v"(S), "v"(G));
}

}  // namespace

template <int WM>
__global__ void __launch_bounds__(256) gs_sweep_kernel(SweepArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar loads
    if (__hip_atomic_load(a.err_code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return;

    const int A = a.A, E = a.E, W = a.W, AW = A * W;
    // workgroup-shared
    int32_t *cg = (int32_t *)(lds + a.o_cg);          // [A*W] global counts C
    int64_t *T = (int64_t *)(lds + a.o_T);            // [A+1] others' background totals, sum
    double *ppmG = (double *)(lds + a.o_ppmG);        // [A*W] ((C + pc)/den)
    double *ppmM = (double *)(lds + a.o_ppmM);        // [A*W] ((C - 1 + pc)/den)
    // wavefront slice
    unsigned char *wl = lds + a.o_wave + wid * a.wave_bytes;
    unsigned char *tab = wl + a.w_tab;                // [WM][E] double2
    double *Gs = (double *)(wl + a.w_G);              // [64*R] background products
    double *Ms = (double *)(wl + a.w_M);              // [64*R] log2 scores, -inf = not a category
    int32_t *aggC = (int32_t *)(wl + a.w_aggC);       // [A*W]
    int64_t *aggM = (int64_t *)(wl + a.w_aggM);       // [A]
    int32_t *comp = (int32_t *)(wl + a.w_comp);       // [64] by encoded symbol
    double *pcv = (double *)(wl + a.w_pcv);           // [64]
    int32_t *misc = (int32_t *)(wl + a.w_misc);
    uint8_t *sseq = (uint8_t *)(wl + a.w_seq);
    const int E16 = E * 16;
    STAMP_DECL
    int nseq_done = 0;

    // ---- prologue: aggregates of the snapshot (sum of the replicas) ----
    for (int c = tid; c < a.cells; c += 256) {
        int64_t s = 0;
        if (a.agg_in) {
#pragma unroll
            for (int r = 0; r < kRepl; ++r) s += a.agg_in[(int64_t)r * a.stride + c];
        }
        if (c < AW)
            cg[c] = (int32_t)s;
        else
            T[c - AW] = s;  // composition total of the motif-bearing sequences
    }
    for (int c = lane; c < AW; c += 64) aggC[c] = 0;
    if (lane < A) aggM[lane] = 0;
    if (blockIdx.x == 0 && a.agg_zero)
        for (int i = tid; i < kRepl * a.stride; i += 256) a.agg_zero[i] = 0;
    __syncthreads();
    if (a.mode == 0) {
        for (int c = tid; c < AW; c += 256) {
            ppmG[c] = ((double)cg[c] + a.pc) / a.den;      // normalizePPM (.fs:257-260)
            ppmM[c] = ((double)(cg[c] - 1) + a.pc) / a.den;
        }
        if (tid < A) {
            int64_t s = T[tid];
            for (int j = 0; j < W; ++j) s -= cg[tid * W + j];
            T[tid] = s;
        }
        __syncthreads();
        if (tid == 0) {
            int64_t s = 0;
            for (int x = 0; x < A; ++x) s += T[x];
            T[A] = s;
        }
        // padding columns j >= W of the window table multiply by exactly 1.0
        for (int c = lane; c < (WM - W) * E; c += 64)
            *(double2 *)(tab + W * E16 + c * 16) = make_double2(1.0, 1.0);
    }
    __syncthreads();

    const int wstride = gridDim.x * kWavesPerBlock;
    const int64_t sumT = a.mode == 0 ? T[A] : 0;  // Σ_a T[a], set in the prologue
    // table build mapping: lane -> (column offset jj, symbol e), cols columns per pass
    const int cols = E <= 64 ? 64 / E : 1;
    const int tb_jj = lane / E, tb_e = lane - (lane / E) * E;
    // This wavefront's sequences are n0 + i*wstride, i < cnt.  Their descriptors
    // (length, offset, snapshot position, uniform) are loaded 64 at a time into
    // lane registers and their results stored 64 at a time, so the only vector
    // memory operations inside the loop are the one-ahead sequence prefetches
    // (vmcnt waits are in order: a descriptor load behind a prefetch or a store
    // would otherwise wait for it).
    const int n0 = blockIdx.x * kWavesPerBlock + wid;
    const int cnt = n0 < a.n_local ? (a.n_local - 1 - n0) / wstride + 1 : 0;
    int b_len = 0, b_pos = -1, r_pos = -1;
    int64_t b_off = 0;
    double b_u = 0.0, r_pw = 0.0;
    auto load_batch = [&](int base) {
        const int i = base + lane;
        if (i < cnt) {
            const int nb = n0 + i * wstride;
            b_len = a.len[nb];
            b_off = a.doff[nb];
            b_pos = a.pos_in[nb];
            if (a.mode == 0)
                b_u = a.u_in ? a.u_in[nb]
                             : uniform(a.seed, a.stream, (uint64_t)(a.global_offset + nb));
        }
    };
    load_batch(0);
    // one-sequence-ahead prefetch (sequences up to 1024 symbols)
    uint4 pf = make_uint4(0, 0, 0, 0);
    if (cnt > 0) {
        const int L0 = __builtin_amdgcn_readlane(b_len, 0);
        const int64_t o0 = __builtin_amdgcn_readlane(b_off, 0);
        if (L0 <= 1024 && lane * 16 < L0) pf = *(const uint4 *)(a.seq + o0 + lane * 16);
    }
    STAMP(0);

    for (int it = 0; it < cnt; ++it) {
        const int jb = it & 63;
        const int n = n0 + it * wstride;
        const int L = __builtin_amdgcn_readlane(b_len, jb);
        const int64_t off = __builtin_amdgcn_readlane(b_off, jb);
        const int p = __builtin_amdgcn_readlane(b_pos, jb);
        const double u = lane_read_f64(b_u, jb);
        const int K = L - W + 1;
        const int64_t gidx = a.global_offset + n;
        ++nseq_done;
        if (L <= 1024) {
            if (lane * 16 < L) *(uint4 *)(sseq + lane * 16) = pf;
        } else {
            const uint8_t *g = a.seq + off;
            for (int i = lane * 16; i < L; i += 64 * 16)
                *(uint4 *)(sseq + i) = *(const uint4 *)(g + i);
        }
        if (it + 1 < cnt) {
            int Ln;
            int64_t on;
            if (jb < 63) {
                Ln = __builtin_amdgcn_readlane(b_len, jb + 1);
                on = __builtin_amdgcn_readlane(b_off, jb + 1);
            } else {  // next batch: once per 64 sequences.  readfirstlane moves the values
                      // to SGPRs here, so no load into a VGPR is pending past this branch
                      // (its wait would also wait for the prefetch issued below)
                Ln = __builtin_amdgcn_readfirstlane(a.len[n + wstride]);
                const int64_t x = a.doff[n + wstride];
                on = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(x >> 32)) << 32) |
                               (uint32_t)__builtin_amdgcn_readfirstlane((int)x));
            }
            if (Ln <= 1024 && lane * 16 < Ln) pf = *(const uint4 *)(a.seq + on + lane * 16);
        }
        // zero tail: unrolled window reads past L see symbol 0 (a valid table row)
        for (int i = L + lane; i < L + WM + 72; i += 64) sseq[i] = 0;
        if (E > 8) comp[lane] = 0;
        wave_sync();

        // ---- composition of the sequence (createFCVOf, .fs:60-62) ----
        int my_comp = 0, na = 0;  // lane e < E: count of symbol e; na: symbols outside A
#if defined(GS_ABL) && GS_ABL & 1  // ablation build (timing only, wrong outputs): no composition pass
        my_comp = lane < E ? L / E : 0;
        for (int c0 = L; c0 < L; c0 += 64) {
#else
        for (int c0 = 0; c0 < L; c0 += 64) {
#endif
            const int i = c0 + lane;
            const int sym = i < L ? (int)sseq[i] : 0xff;
            na += popc64(__ballot(sym >= A && sym != 0xff));
            if (E <= 8) {
                for (int e = 0; e < E; ++e) {
                    const int cnt = popc64(__ballot(sym == e));
                    if (lane == e) my_comp += cnt;
                }
            } else if (sym != 0xff) {
                atomicAdd(&comp[sym], 1);
            }
        }
        if (E > 8) {
            wave_sync();
            my_comp = lane < E ? comp[lane] : 0;
        }
        const int alpha_tot = L - na;
        STAMP(1);

        int newp = p;
        if (a.mode == 0) {
            // ---- hold-one-out background (integer exact) ----
            const int sj = (p >= 0 && lane < W) ? (int)sseq[p + lane] : 0xff;
            int my_segc = 0;
            for (int x = 0; x < A; ++x) {
                const int cnt = popc64(__ballot(sj == x));
                if (lane == x) my_segc = cnt;
            }
            const int seg_alpha = popc64(__ballot(sj < A));
            const int64_t bgc = lane < A ? T[lane] + (p >= 0 ? my_segc : my_comp) : 0;
            // Σ over the 49 slots: alphabet part + the sequence's own other symbols
            const int64_t tot = sumT + (p >= 0 ? seg_alpha : alpha_tot) + na;
            if (tot > 2147483647LL) {  // Checked Array.sum (.fs:117)
                if (lane == 0) raise_error(a, 3, gidx);
                goto seq_end;
            }
            const double sbg = (double)tot + a.apc;
            if (lane < A)
                pcv[lane] = ((double)bgc + a.pc) / sbg;  // .fs:119
            else if (lane < E)
                pcv[lane] = (double)my_comp;             // raw count outside the alphabet (Q3)
            wave_sync();
            // ---- (PWM, PCV) window table (.fs:286): cols columns per pass ----
#if defined(GS_ABL) && GS_ABL & 8  // ablation build: table left as it is
            if (false) {
#else
            if (tb_jj < cols) {
#endif
                const double pe = pcv[tb_e];
                for (int j = tb_jj; j < W; j += cols) {
                    double v = 0.0;
                    if (tb_e < A) {
                        const int cell = tb_e * W + j;
                        const bool own = p >= 0 && sseq[p + j] == tb_e;
                        v = (own ? ppmM[cell] : ppmG[cell]) / pe;
                    }
                    *(double2 *)(tab + j * E16 + tb_e * 16) = make_double2(v, pe);
                }
            }
            wave_sync();
            STAMP(2);
            // ---- score every window (.fs:759-782); lane owns windows [k_lo, k_lo+R) ----
            const int R = (K + 63) >> 6;
            const int k_lo = lane * R;
            double sG = 0.0, sM = 0.0, sA = 0.0;
            bool neg = false;
            int npass = 0;
            for (int r = 0; r < R; ++r) {
                const int k = k_lo + r;
                const bool valid = k < K;
                double S, G;
#if defined(GS_ABL) && GS_ABL & 2  // ablation build: no window products
                S = 0.25 * (double)((k * 2654435761u) >> 28);
                G = 1e-7 * (double)(k & 15);
#else
                window_products<WM>(sseq, tab, E16, k, S, G);
#endif
                double M = -INFINITY;
                if (valid && S >= a.thr_lo) {
                    const double l2 = log(S * 1.0) / kLn2;
                    if (l2 > a.cutoff) M = l2;
                }
                // [r][lane] layout: window k = lane*R + r lives at r*64 + lane, so
                // these stores and the walk's loads are bank-conflict-free
                Gs[r * 64 + lane] = G;
                Ms[r * 64 + lane] = M;
                npass += popc64(__ballot(M != -INFINITY));
                if (valid) {
                    sG = sG + G;
                    sA = sA + fabs(G);
                    neg |= !(G >= 0.0);
                    if (M != -INFINITY) {
                        sM = sM + M;
                        sA = sA + fabs(M);
                        neg |= !(M >= 0.0);
                    }
                }
            }
            wave_sync();
            STAMP(3);

            // ---- certified roulette (.fs:746-754) ----
            const double inclG = wave_incl_scan_f64(sG);
            const double inclM = wave_incl_scan_f64(sM);
            const double exclG = dpp_f64<0x138, 0xf>(inclG);  // wave_shr:1
            const double exclM = dpp_f64<0x138, 0xf>(inclM);
            const double totG = lane_read_f64(inclG, 63);
            const double totM = lane_read_f64(inclM, 63);
            const double total = totG + totM;
            const double sumAbs = __ballot(neg) ? wave_sum_f64(sA) : total;
            const double ncat = (double)(K + npass + 2);
            const double delta = 8.0 * ncat * 0x1.0p-53 * (sumAbs / fabs(total));
            const double inv = 1.0 / total;
            const int k_hi = min(K, k_lo + R);

            int kind = -1, pk = -1;  // kind 0 = background category, 1 = motif category
            bool fallback = false;
            // background categories (G_0 .. G_{K-1}) come first in the list (.fs:782)
            if (!(u > totG * inv + 2.0 * delta)) {
                double acc = exclG * inv;
                int st = 0, ik = -1;
                for (int r = 0; k_lo + r < k_hi; ++r) {
                    const double w = Gs[r * 64 + lane] * inv;
                    const double hi = acc + w;
                    if (!((u < acc - delta) || (u > hi + delta))) {
                        st = ((u >= acc + delta) && (u <= hi - delta)) ? 1 : 2;
                        ik = k_lo + r;
                        break;
                    }
                    acc = hi;
                }
                const unsigned long long b = __ballot(st != 0);
                if (b) {
                    const int f = __ffsll((long long)b) - 1;
                    const int sf = __builtin_amdgcn_readlane(st, f);
                    if (sf == 1) {
                        kind = 0;
                        pk = __builtin_amdgcn_readlane(ik, f);
                    } else {
                        fallback = true;
                    }
                }
            }
            if (kind < 0 && !fallback && npass > 0) {
                double acc = (totG + exclM) * inv;
                int st = 0, ik = -1;
                for (int r = 0; k_lo + r < k_hi; ++r) {
                    const double m = Ms[r * 64 + lane];
                    if (m == -INFINITY) continue;
                    const double w = m * inv;
                    const double hi = acc + w;
                    if (!((u < acc - delta) || (u > hi + delta))) {
                        st = ((u >= acc + delta) && (u <= hi - delta)) ? 1 : 2;
                        ik = k_lo + r;
                        break;
                    }
                    acc = hi;
                }
                const unsigned long long b = __ballot(st != 0);
                if (b) {
                    const int f = __ffsll((long long)b) - 1;
                    const int sf = __builtin_amdgcn_readlane(st, f);
                    if (sf == 1) {
                        kind = 1;
                        pk = __builtin_amdgcn_readlane(ik, f);
                    } else {
                        fallback = true;
                    }
                }
            }
            if (fallback) {
                // exact sequential restatement of .fs:747-754, one lane
                if (lane == 0) {
                    atomicAdd(a.fallbacks, 1ull);
#define GS_AT(arr, k) arr[((k) % R) * 64 + (k) / R]
                    double s = 0.0;
                    for (int k = 0; k < K; ++k) s = s + GS_AT(Gs, k);
                    for (int k = 0; k < K; ++k)
                        if (GS_AT(Ms, k) != -INFINITY) s = s + GS_AT(Ms, k);
                    double acc = 0.0;
                    int rk = -1, rp = -1;
                    for (int k = 0; k < K && rk < 0; ++k) {
                        const double w = GS_AT(Gs, k) / s;
                        if (acc <= u && u <= acc + w) {
                            rk = 0;
                            rp = k;
                        }
                        acc = acc + w;
                    }
                    for (int k = 0; k < K && rk < 0; ++k) {
                        if (GS_AT(Ms, k) == -INFINITY) continue;
                        const double w = GS_AT(Ms, k) / s;
                        if (acc <= u && u <= acc + w) {
                            rk = 1;
                            rp = k;
                        }
                        acc = acc + w;
                    }
                    misc[0] = rk;
                    misc[1] = rp;
                }
                wave_sync();
                kind = misc[0];
                pk = misc[1];
            }
            if (kind < 0) {  // every category missed: the reference's list index overruns
                if (lane == 0) raise_error(a, 2, gidx);
                goto seq_end;
            }
            newp = kind == 0 ? -1 : pk;
            if (lane == jb) {  // results wait in lane registers, stored 64 at a time
                r_pos = newp;
                r_pw = kind == 0 ? GS_AT(Gs, pk) : GS_AT(Ms, pk);
            }
        }
        STAMP(4);
        // ---- fold the chosen segment into the next snapshot's aggregates ----
        // lane j < W owns column j: one cell per lane, no conflicts
        if (newp >= 0) {
            if (lane < W) {
                const int s = sseq[newp + lane];
                if (s < A) aggC[s * W + lane] += 1;
            }
            if (lane < A) aggM[lane] += my_comp;
        }
        wave_sync();
        STAMP(5);
    seq_end:
        if (jb == 63 || it + 1 == cnt) {
            if (a.mode == 0 && lane <= jb) {
                const int nb = n0 + (it - jb + lane) * wstride;
                a.pos_out[nb] = r_pos;
                a.pwms_out[nb] = r_pw;
            }
            if (jb == 63 && it + 1 < cnt) load_batch(it + 1);
        }
    }
    // ---- flush: sum the 4 wavefronts' aggregates, one atomic per cell ----
    __syncthreads();
    STAMP(6);
    STAMP_FLUSH(nseq_done);
    int64_t *dst = a.agg_out + (int64_t)(blockIdx.x % kRepl) * a.stride;
    for (int c = tid; c < a.cells; c += 256) {
        int64_t v = 0;
#pragma unroll
        for (int w = 0; w < kWavesPerBlock; ++w) {
            const unsigned char *ow = lds + a.o_wave + w * a.wave_bytes;
            v += c < AW ? (int64_t)((const int32_t *)(ow + a.w_aggC))[c]
                        : ((const int64_t *)(ow + a.w_aggM))[c - AW];
        }
        if (v != 0) atomicAdd((unsigned long long *)&dst[c], (unsigned long long)v);
    }
}

// Host-side launch helpers (the C-ABI translation unit stays free of kernel code).
#define GS_FOR_EACH_WM(X) X(4) X(8) X(12) X(16) X(20) X(24) X(28) X(32) X(40) X(48) X(56) X(64)

static const void *sweep_kernel_ptr(int wm) {
    switch (wm) {
#define GS_CASE(N) \
    case N:        \
        return (const void *)&gs_sweep_kernel<N>;
        GS_FOR_EACH_WM(GS_CASE)
#undef GS_CASE
    }
    return nullptr;
}

int gs_sweep_wm(int W) {
    const int r = (W + 3) / 4 * 4;
    if (r <= 32) return r;
    return (W + 7) / 8 * 8;
}

hipError_t gs_sweep_occupancy(int *blocks_per_cu, int W, size_t lds_bytes) {
    const void *k = sweep_kernel_ptr(gs_sweep_wm(W));
    if (!k) return hipErrorInvalidValue;
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, k, 256, lds_bytes);
}

hipError_t gs_sweep_launch(const SweepArgs &a, int grid, size_t lds_bytes, hipStream_t stream) {
    switch (gs_sweep_wm(a.W)) {
#define GS_CASE(N)                                                                          \
    case N:                                                                                 \
        hipLaunchKernelGGL(gs_sweep_kernel<N>, dim3(grid), dim3(256), lds_bytes, stream, a); \
        break;
        GS_FOR_EACH_WM(GS_CASE)
#undef GS_CASE
        default:
            return hipErrorInvalidValue;
    }
    return hipGetLastError();
}
