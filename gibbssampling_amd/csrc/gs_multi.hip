// gs_multi.hip — the motif sampler with motifAmount >= 1 (Positions lists) on gfx950.
//
// With motifAmount = M >= 2 a sequence may carry up to M motif copies, and the
// categories of calculateNormalizedSegmentScores (.fs:759-784) are
//   [(G_k, []) for every window k]
//   ++ combos(1) ++ combos(2) ++ ... ++ combos(M)
// where combos(m) = calculatePWMsForSegmentCombinations cutOff W m (.fs:727-742): the
// m-tuples of windows k1 < k2 < ... < km, pairwise more than W apart
// (ceckForDistance, .fs:129-140), whose every prefix product passes
// log2(prefix) > cutOff, in the depth-first include-first order of the F# sequence
// expression (lexicographic in (k1, ..., km)), weighted log2(S_km * (... * (S_k1 * 1.0))).
//
// The key identity: the admissible (m-1)-prefixes of combos(m) are exactly the
// categories of combos(m-1) (same products, same tests), so level m is generated
// from level m-1 in order: for each parent tuple, its admissible next windows in
// ascending order.  Levels live in a per-workgroup arena in HBM (product, log2
// weight, last window, parent index); a pick is decoded by walking parents, which
// yields the F# cons order (most recent position first).
//
// One 64-lane wavefront per workgroup scores one target at a time:
//   1. hold-one-out from the snapshot aggregates (C, T) with every position of the
//      target's list removed (.fs:940-965, SURVEY §8(a) identities generalised to
//      lists: a sequence with p positions contributes p segments to C and
//      p·comp(s) − Σ comp(seg) to the background, exactly as Array.map2/concat do);
//   2. PCV, PPM, PWM in binary64 (.fs:115-120, .fs:255-261, .fs:282-287), every
//      window folded in binary64 in the reference's order (.fs:291-292, .fs:124);
//   3. the category levels (above);
//   4. roulette (.fs:746-754): parallel binary64 sums and prefix scans locate the
//      pick; it is accepted only when u is farther than a rounding bound from
//      every CDF boundary, else one lane replays the reference's sequential
//      List.sum and running acc exactly.  The greedy (.fs:917-920) takes the first
//      maximum of the stable descending sort instead (NaN ranks lowest).
// The greedy passes (Gauss–Seidel over the live positions) run in one persistent
// workgroup whose live aggregates sit in LDS.
//
// Compiled with -ffp-contract=off: no FMA contraction.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "gs_common.h"
#include "gs_wave.h"

using namespace gs;

namespace {

__device__ __forceinline__ int64_t wsum_i64(int64_t x) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
    return x;
}

__device__ __forceinline__ void raise_err(const MultiArgs &a, int64_t gidx, int status) {
    atomicMin(a.err, ((unsigned long long)gidx << 4) | (unsigned long long)status);
}

// Category weight in the reference's order: backgrounds first, then the arena.
struct Cats {
    const double *G;     // [K]
    const double *wgt;   // [total]
    int K;
    __device__ __forceinline__ double w(int c) const { return c < K ? G[c] : wgt[c - K]; }
};

struct Slot {
    double *S, *G, *prod, *wgt;
    int32_t *last, *parent;
};

__device__ __forceinline__ Slot slot_of(const MultiArgs &a, int idx) {
    Slot s;
    double *b = a.scratch + (int64_t)idx * a.slot_doubles;
    s.S = b;
    s.G = b + a.kmax;
    s.prod = b + 2 * (int64_t)a.kmax;
    s.wgt = s.prod + a.arena_cap;
    s.last = (int32_t *)(s.wgt + a.arena_cap);
    s.parent = s.last + a.arena_cap;
    return s;
}

// Result of one target: category index in the reference's order and its count.
struct Pick {
    int cat;      // -1 on error
    int status;   // 0 ok, 2 roulette overrun, 3 int32 overflow, kMultiErrArena
    int K, total;
};

// Stage the target's sequence into LDS (16-byte chunks; the upload pads each
// sequence to 16 bytes plus a 64-byte tail, so the last chunk stays in bounds).
__device__ __forceinline__ void stage(const uint8_t *g, int L, uint8_t *sseq, int lane) {
    for (int i = lane * 16; i < L; i += 64 * 16) *(uint4 *)(sseq + i) = *(const uint4 *)(g + i);
}

// Steps 1-4 for target n (all 64 lanes).  C/T: aggregates of the snapshot
// including the target's own list (cnt, pos[0..cnt)); sseq: its staged sequence.
__device__ Pick score_target(const MultiArgs &a, int n, int L, const uint8_t *sseq, int cnt,
                             const int32_t *pos, const int64_t *C, const int64_t *T, double *tab,
                             double *pcv, const Slot &sl, bool greedy, double u, int lane) {
    const int A = a.A, W = a.W, E = a.E;
    const int K = L - W + 1;
    Pick pk{-1, 0, K, 0};
    // ---- 1. hold-one-out background and PCV (.fs:945-954, .fs:115-120) ----
    int64_t bgc = 0;
    if (lane < E) {
        const int64_t ce = a.comp[(int64_t)n * (E + 1) + lane];
        bgc = ce;
        if (lane < A) {
            bgc += T[lane];
            for (int i = 0; i < cnt; ++i) {
                const int p = pos[i];
                int64_t sc = 0;
                for (int j = 0; j < W; ++j) sc += sseq[p + j] == lane;
                bgc -= ce - sc;  // createFCVWithout of the target's own segment
            }
        }
    }
    if (a.pcv_fixed) {
        if (lane < E) pcv[lane] = a.pcv_fixed[lane];
    } else {
        const int64_t tot = wsum_i64(bgc);
        if (tot > 0x7fffffffll) {  // Checked Array.sum (.fs:117)
            pk.status = 3;
            return pk;
        }
        const double sum = (double)tot + a.apc;
        if (lane < E) pcv[lane] = lane < A ? ((double)bgc + a.pc) / sum : (double)bgc;
    }
    __syncthreads();
    // ---- 2. PWM of the others (.fs:955-965, .fs:255-261, .fs:282-287) ----
    for (int c = lane; c < E * W; c += 64) {
        const int e = c / W, j = c - e * W;
        double v = 0.0;
        if (e < A) {
            int64_t x = C[c];
            for (int i = 0; i < cnt; ++i) x -= sseq[pos[i] + j] == e;
            const double ppm = ((double)x + a.pc) / a.den;
            v = ppm / pcv[e];
        }
        tab[c] = v;
    }
    __syncthreads();
    // every window, the reference's left folds (.fs:291-292, .fs:124)
    for (int k = lane; k < K; k += 64) {
        double S = 1.0, G = 1.0;
        for (int j = 0; j < W; ++j) {
            const int e = sseq[k + j];
            S = S * tab[e * W + j];
            G = G * pcv[e];
        }
        sl.S[k] = S;
        sl.G[k] = G;
    }
    __threadfence_block();
    __syncthreads();
    // ---- 3. category levels (.fs:727-742) ----
    const unsigned long long below = (1ull << lane) - 1ull;
    int total = 0;
    bool ovf = false;
    auto append = [&](bool pass, double prod, double lv, int last, int parent) {
        const unsigned long long m = __ballot(pass);
        const int off = total + __popcll(m & below);
        if (pass && off < a.arena_cap) {
            sl.prod[off] = prod;
            sl.wgt[off] = lv;
            sl.last[off] = last;
            sl.parent[off] = parent;
        }
        total += __popcll(m);
        ovf = total > a.arena_cap;
    };
    // level 1: (log2(S_k * 1.0), [k]) for log2(S_k * 1.0) > cutOff (.fs:735-738)
    for (int k0 = 0; k0 < K && !ovf; k0 += 64) {
        const int k = k0 + lane;
        bool pass = false;
        double pr = 0.0, lv = 0.0;
        if (k < K) {
            pr = sl.S[k] * 1.0;
            lv = log(pr) / kLn2;
            pass = lv > a.cutoff;
        }
        append(pass, pr, lv, k, -1);
    }
    // level m from level m-1: children j > last + W with log2(S_j * prod) > cutOff
    int lo = 0, hi = total;
    for (int m = 2; m <= a.M && !ovf && lo < hi; ++m) {
        for (int q = lo; q < hi && !ovf; ++q) {
            __threadfence_block();
            const double pq = sl.prod[q];
            const int lq = sl.last[q];
            for (int j0 = lq + W + 1; j0 < K && !ovf; j0 += 64) {
                const int j = j0 + lane;
                bool pass = false;
                double pr = 0.0, lv = 0.0;
                if (j < K) {
                    pr = sl.S[j] * pq;  // fst x * prob
                    lv = log(pr) / kLn2;
                    pass = lv > a.cutoff;
                }
                append(pass, pr, lv, j, q);
            }
        }
        lo = hi;
        hi = total;
    }
    if (ovf) {
        pk.status = kMultiErrArena;
        return pk;
    }
    __threadfence_block();
    __syncthreads();
    pk.total = total;
    const Cats cats{sl.G, sl.wgt, K};
    const int ncat = K + total;
    if (greedy) {
        // ---- List.sortByDescending PWMS |> List.head (.fs:917-920): first maximum ----
        unsigned long long bk = 0;
        int bi = -1;
        for (int c = lane; c < ncat; c += 64) {
            const unsigned long long key = order_key(cats.w(c));
            if (bi < 0 || key > bk) {
                bk = key;
                bi = c;
            }
        }
        const unsigned long long mk = wave_max_u64(bi >= 0 ? bk : 0ull);
        pk.cat = wave_min_i32(bi >= 0 && bk == mk ? bi : 0x7fffffff);
        return pk;
    }
    // ---- 4. rouletteWheelSelection (.fs:746-754) ----
    double s = 0.0;
    bool bad = false;
    for (int c = lane; c < ncat; c += 64) {
        const double w = cats.w(c);
        bad |= !(w >= 0.0 && w < INFINITY);
        s += w;
    }
    const double tot = wave_sum_f64(s);
    int pick = -1;
    bool serial = __ballot(bad) != 0ull || !(tot > 0.0 && tot < INFINITY);
    if (!serial) {
        // the reference's boundaries acc_c are within (2 ncat + 2) 2^-53 of the exact
        // prefix ratios; ours within (ncat/64 + 8) 2^-53: 8 ncat + 64 covers both
        const double t = u * tot;
        const double D = (8.0 * (double)ncat + 64.0) * 0x1.0p-53 * tot;
        double carry = 0.0;
        serial = true;
        for (int b0 = 0; b0 < ncat; b0 += 64) {
            const int c = b0 + lane;
            const double w = c < ncat ? cats.w(c) : 0.0;
            const double incl = wave_incl_scan_f64(w);
            const double h = carry + incl, l = carry + (incl - w);
            const bool near = c < ncat && (fabs(t - h) <= D || fabs(t - l) <= D);
            if (__ballot(near) != 0ull) break;
            const unsigned long long in = __ballot(c < ncat && l < t && t < h);
            if (in != 0ull) {
                pick = b0 + __ffsll((long long)in) - 1;
                serial = false;
                break;
            }
            carry = lane_read_f64(h, 63);
        }
    }
    if (serial) {
        // one lane replays List.sum and the running acc exactly
        int p = -1;
        if (lane == 0) {
            double sum = 0.0;
            for (int c = 0; c < ncat; ++c) sum = sum + cats.w(c);
            double acc = 0.0;
            for (int c = 0; c < ncat; ++c) {
                const double w = cats.w(c) / sum;
                if (acc <= u && u <= acc + w) {
                    p = c;
                    break;
                }
                acc = acc + w;
            }
            atomicAdd(&a.fallbacks[1], 1ull);
        }
        pick = __shfl(p, 0, 64);
        if (pick < 0) pk.status = 2;  // list index past the end (.fs:752)
    }
    pk.cat = pick;
    return pk;
}

// Decode category `cat` of a scored target into (cnt, positions in F# cons order,
// PWMS); lane 0 writes.
__device__ __forceinline__ void decode(const Slot &sl, int K, int cat, int32_t *cnt_out,
                                       int32_t *pos_out, double *pwms_out, int lane) {
    if (lane != 0) return;
    if (cat < K) {
        *cnt_out = 0;
        *pwms_out = sl.G[cat];
        return;
    }
    int q = cat - K, i = 0;
    *pwms_out = sl.wgt[q];
    while (q >= 0) {
        pos_out[i++] = sl.last[q];
        q = sl.parent[q];
    }
    *cnt_out = i;
}

}  // namespace

// Aggregates of a list snapshot: C[a][j] over every listed segment, T[a] = Σ over
// list entries of (comp(s_m) − comp(seg))[a].  256 threads, one sequence each.
extern "C" __global__ void __launch_bounds__(256) gs_multi_agg_kernel(MultiArgs a, int64_t *out) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    unsigned long long *acc = (unsigned long long *)lds;
    const int A = a.A, W = a.W, cells = A * W + A;
    for (int c = threadIdx.x; c < cells; c += blockDim.x) acc[c] = 0ull;
    __syncthreads();
    for (int n = blockIdx.x * blockDim.x + threadIdx.x; n < a.n_local; n += gridDim.x * blockDim.x) {
        const uint8_t *s = a.seq + a.doff[n];
        const int cnt = a.cnt_in[n];
        for (int i = 0; i < cnt; ++i) {
            const int p = a.pos_in[(int64_t)n * a.cap_in + i];
            for (int x = 0; x < A; ++x)
                atomicAdd(&acc[A * W + x], (unsigned long long)a.comp[(int64_t)n * (a.E + 1) + x]);
            for (int j = 0; j < W; ++j) {
                const int e = s[p + j];
                if (e < A) {
                    atomicAdd(&acc[e * W + j], 1ull);
                    atomicAdd(&acc[A * W + e], ~0ull);  // -1
                }
            }
        }
    }
    __syncthreads();
    for (int c = threadIdx.x; c < cells; c += blockDim.x)
        if (acc[c]) atomicAdd((unsigned long long *)&out[c], acc[c]);
}

// One synchronous sweep (.fs:935-970): every target independently against the
// snapshot aggregates.  One wavefront per workgroup, persistent over targets.
extern "C" __global__ void __launch_bounds__(64) gs_multi_sweep_kernel(MultiArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    double *tab = (double *)(lds + a.o_tab);
    double *pcv = (double *)(lds + a.o_pcv);
    uint8_t *sseq = lds + a.o_seq;
    const int lane = threadIdx.x;
    const Slot sl = slot_of(a, blockIdx.x);
    const int AW = a.A * a.W;
    const int64_t *C = a.agg, *T = a.agg + AW;
    for (int i = blockIdx.x; i < a.n_targets; i += gridDim.x) {
        const int n = a.targets ? a.targets[i] : i;
        const int L = a.len[n];
        const int64_t gidx = a.global_offset + n;
        __syncthreads();
        stage(a.seq + a.doff[n], L, sseq, lane);
        __syncthreads();
        const int cnt = a.cnt_in[n];
        const int32_t *pos = a.pos_in + (int64_t)n * a.cap_in;
        const double u = a.u ? a.u[n] : uniform(a.seed, a.stream, (uint64_t)gidx);
        const Pick pk = score_target(a, n, L, sseq, cnt, pos, C, T, tab, pcv, sl, false, u, lane);
        if (pk.status == kMultiErrArena) {
            if (lane == 0) a.ovf_list[atomicAdd(a.ovf_count, 1)] = n;
            continue;
        }
        if (pk.status) {
            if (lane == 0) raise_err(a, gidx, pk.status);
            continue;
        }
        decode(sl, pk.K, pk.cat, a.cnt_out + n, a.pos_out + (int64_t)n * a.cap_out,
               a.pwms_out + n, lane);
    }
}

// Greedy Gauss–Seidel passes (.fs:885-929) in one workgroup (one wavefront):
// targets in order against the live acc (cnt_out/pos_out/pwms_out, in/out), the
// head of the descending sort kept when its PWMS is strictly larger (.fs:923);
// passes repeat until one leaves every Positions list unchanged (.fs:888).
extern "C" __global__ void __launch_bounds__(64) gs_multi_greedy_kernel(MultiArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    double *tab = (double *)(lds + a.o_tab);
    double *pcv = (double *)(lds + a.o_pcv);
    uint8_t *sseq = lds + a.o_seq;
    int64_t *agg = (int64_t *)(lds + a.o_agg);
    __shared__ int32_t newpos[kMultiMaxAmount];
    __shared__ int32_t newcnt;
    __shared__ double newpw;
    const int lane = threadIdx.x;
    const int A = a.A, W = a.W, AW = A * W;
    const Slot sl = slot_of(a, 0);
    for (int c = lane; c < AW + A; c += 64) agg[c] = a.agg[c];
    __syncthreads();
    int passes = 0;
    bool stop = false;
    while (!stop) {
        bool changed = false;
        for (int n = 0; n < a.n_local && !stop; ++n) {
            const int L = a.len[n];
            __syncthreads();
            stage(a.seq + a.doff[n], L, sseq, lane);
            __syncthreads();
            int32_t *lst = a.pos_out + (int64_t)n * a.cap_out;
            const int cnt = a.cnt_out[n];
            const Pick pk = score_target(a, n, L, sseq, cnt, lst, agg, agg + AW, tab, pcv, sl, true,
                                         0.0, lane);
            if (pk.status) {
                if (lane == 0) raise_err(a, a.global_offset + n, pk.status);
                stop = true;
                break;
            }
            decode(sl, pk.K, pk.cat, &newcnt, newpos, &newpw, lane);
            __syncthreads();
            if (!(newpw > a.pwms_out[n])) continue;  // tmp.PWMS > acc.[n].PWMS (.fs:923)
            bool same = newcnt == cnt;
            for (int i = 0; same && i < cnt; ++i) same = newpos[i] == lst[i];
            changed |= !same;
            // move the target's contribution from the old list to the new one
            if (lane < W) {
                for (int i = 0; i < cnt; ++i) {
                    const int e = sseq[lst[i] + lane];
                    if (e < A) {
                        atomicAdd((unsigned long long *)&agg[e * W + lane], ~0ull);
                        atomicAdd((unsigned long long *)&agg[AW + e], 1ull);
                    }
                }
                for (int i = 0; i < newcnt; ++i) {
                    const int e = sseq[newpos[i] + lane];
                    if (e < A) {
                        atomicAdd((unsigned long long *)&agg[e * W + lane], 1ull);
                        atomicAdd((unsigned long long *)&agg[AW + e], ~0ull);
                    }
                }
            }
            if (lane < A) {
                const int64_t ce = a.comp[(int64_t)n * (a.E + 1) + lane];
                atomicAdd((unsigned long long *)&agg[AW + lane],
                          (unsigned long long)(ce * (int64_t)(newcnt - cnt)));
            }
            __syncthreads();
            if (lane < newcnt) lst[lane] = newpos[lane];
            if (lane == 0) {
                a.cnt_out[n] = newcnt;
                a.pwms_out[n] = newpw;
            }
            __threadfence_block();
            __syncthreads();
        }
        if (stop) break;
        ++passes;
        if (!changed || passes >= a.max_passes) stop = true;
    }
    if (lane == 0) *a.passes_out = passes;
}

hipError_t gs_multi_agg_launch(const MultiArgs &a, int64_t *out, int n_cu, hipStream_t s) {
    if (a.n_local <= 0) return hipSuccess;
    const int grid = std::max(1, std::min((a.n_local + 255) / 256, n_cu * 4));
    const size_t lds = 8 * (size_t)(a.A * a.W + a.A);
    hipLaunchKernelGGL(gs_multi_agg_kernel, dim3(grid), dim3(256), lds, s, a, out);
    return hipGetLastError();
}

hipError_t gs_multi_sweep_launch(const MultiArgs &a, int grid, size_t lds, hipStream_t s) {
    hipLaunchKernelGGL(gs_multi_sweep_kernel, dim3(grid), dim3(64), lds, s, a);
    return hipGetLastError();
}

hipError_t gs_multi_greedy_launch(const MultiArgs &a, size_t lds, hipStream_t s) {
    hipLaunchKernelGGL(gs_multi_greedy_kernel, dim3(1), dim3(64), lds, s, a);
    return hipGetLastError();
}
