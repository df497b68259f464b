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
// ascending order.  Levels 1..M-1 live in a per-workgroup arena in HBM (product,
// log2 weight, last window, parent index); the last level — by far the largest
// (~K x |level M-1|) — is never stored but recomputed from its parents whenever it
// is walked.  A pick is decoded by walking parents, which yields the F# cons order
// (most recent position first).
//
// Per target:
//   1. hold-one-out from the snapshot aggregates (C, T) with every position of the
//      target's list removed (.fs:940-965, SURVEY §8(a) identities generalised to
//      lists: a sequence with p positions contributes p segments to C and
//      p·comp(s) − Σ comp(seg) to the background, exactly as Array.map2/concat do);
//   2. PCV, PPM, PWM in binary64 (.fs:115-120, .fs:255-261, .fs:282-287), every
//      window folded in binary64 in the reference's order (.fs:291-292, .fs:124);
//   3. sweep: rouletteWheelSelection (.fs:746-754) in two walks over the categories
//      (the total, then the prefix up to u): parallel binary64 sums and prefix scans
//      locate the pick; it is accepted only when u is farther than a rounding bound
//      from every CDF boundary, else one lane replays the reference's sequential
//      List.sum and running acc exactly;
//   4. greedy: List.sortByDescending |> List.head (.fs:917-920) = the first maximum
//      (NaN lowest).  Levels 1..M-1 are materialised (they are the parents); the last
//      level — by far the largest — is never stored: the workgroup scans its
//      products S_j * prod(parent) for the largest passing one, then takes binary64
//      logs only of the products within 2^-40 of it (log is monotone to within an
//      ulp, far inside that band), so the first maximum of log2 is decided exactly.
// The sweep runs one 64-lane wavefront per workgroup (many targets in flight); the
// greedy passes (Gauss–Seidel over the live positions) run in one persistent
// workgroup of several wavefronts that all score the current target, with the live
// aggregates and the window scores in LDS.
//
// Compiled with -ffp-contract=off: no FMA contraction.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "gs_common.h"
#include "gs_wave.h"

using namespace gs;

namespace {

constexpr int kMaxWaves = 16;
constexpr int kParentBlock = 512;  // parents staged in LDS per block of the greedy's scan

__device__ __forceinline__ int64_t wsum_i64(int64_t x) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
    return x;
}

__device__ __forceinline__ unsigned long long wave_min_u64(unsigned long long x) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        const unsigned long long y = __shfl_xor(x, d, 64);
        x = y < x ? y : x;
    }
    return x;
}

__device__ __forceinline__ void raise_err(const MultiArgs &a, int64_t gidx, int status) {
    atomicMin(a.err, ((unsigned long long)gidx << 4) | (unsigned long long)status);
}

// log2 as FSharpAux.Math.log2 (.fs:735-738): Math.Log(x) / Math.Log(2.0).
__device__ __forceinline__ double flog2_ref(double x) { return log(x) / kLn2; }

// (value key, index) with "largest key, then smallest index" as the order: the
// first maximum of a list.  Empty: (0, ~0).
struct Best {
    unsigned long long v, i;
};
__device__ __forceinline__ void best_take(Best &b, unsigned long long v, unsigned long long i) {
    if (v > b.v || (v == b.v && i < b.i)) {
        b.v = v;
        b.i = i;
    }
}
// Workgroup-wide reduction (all threads; red: LDS [kMaxWaves]).
__device__ Best block_best(Best b, Best *red) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const unsigned long long mv = wave_max_u64(b.v);
    const unsigned long long mi = wave_min_u64(b.v == mv ? b.i : ~0ull);
    __syncthreads();
    if (lane == 0) red[wave] = Best{mv, mi};
    __syncthreads();
    Best r = red[0];
    for (int w = 1; w < nw; ++w) best_take(r, red[w].v, red[w].i);
    return r;
}

struct Slot {
    double *S, *G, *prod, *wgt;
    int32_t *last, *parent;
};

__device__ __forceinline__ Slot slot_of(const MultiArgs &a, int idx, unsigned char *lds) {
    Slot s;
    double *b = a.scratch + (int64_t)idx * a.slot_doubles;
    if (a.o_S >= 0) {
        s.S = (double *)(lds + a.o_S);
        s.G = s.S + a.kmax;
    } else {
        s.S = b;
        s.G = b + a.kmax;
    }
    s.prod = b + 2 * (int64_t)a.kmax;
    s.wgt = s.prod + a.arena_cap;
    s.last = (int32_t *)(s.wgt + a.arena_cap);
    s.parent = s.last + a.arena_cap;
    return s;
}

// Stage the target's sequence into LDS (16-byte chunks; the upload pads each
// sequence to 16 bytes plus a 64-byte tail, so the last chunk stays in bounds).
__device__ __forceinline__ void stage(const uint8_t *g, int L, uint8_t *sseq) {
    for (int i = threadIdx.x * 16; i < L; i += blockDim.x * 16)
        *(uint4 *)(sseq + i) = *(const uint4 *)(g + i);
}

// Steps 1-2 for target n (every thread of the workgroup): PCV, PWM table and the
// window scores S_k, G_k.  C/T: aggregates of the snapshot including the target's
// own list (cnt, pos[0..cnt)); sseq: its staged sequence.  Returns 0 or 3 (the
// Checked int32 background sum overflows, .fs:117).
__device__ int prepare_target(const MultiArgs &a, int n, int L, const uint8_t *sseq, int cnt,
                              const int32_t *pos, const int64_t *C, const int64_t *T, double *tab,
                              double *pcv, const Slot &sl, int *flag) {
    const int A = a.A, W = a.W, E = a.E;
    const int K = L - W + 1;
    const int tid = threadIdx.x, NT = blockDim.x;
    // ---- hold-one-out background and PCV (.fs:945-954, .fs:115-120): wave 0 ----
    if (tid < 64) {
        int64_t bgc = 0;
        if (tid < E) {
            const int64_t ce = a.comp[(int64_t)n * (E + 1) + tid];
            bgc = ce;
            if (tid < A) {
                bgc += T[tid];
                for (int i = 0; i < cnt; ++i) {
                    const int p = pos[i];
                    int64_t sc = 0;
                    for (int j = 0; j < W; ++j) sc += sseq[p + j] == tid;
                    bgc -= ce - sc;  // createFCVWithout of the target's own segment
                }
            }
        }
        if (a.pcv_fixed) {
            if (tid < E) pcv[tid] = a.pcv_fixed[tid];
            if (tid == 0) *flag = 0;
        } else {
            const int64_t tot = wsum_i64(bgc);
            const double sum = (double)tot + a.apc;
            if (tid < E) pcv[tid] = tid < A ? ((double)bgc + a.pc) / sum : (double)bgc;
            if (tid == 0) *flag = tot > 0x7fffffffll ? 3 : 0;
        }
    }
    __syncthreads();
    if (*flag) return *flag;
    // ---- PWM of the others (.fs:955-965, .fs:255-261, .fs:282-287) ----
    for (int c = tid; c < E * W; c += NT) {
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
    // ---- every window, the reference's left folds (.fs:291-292, .fs:124) ----
    for (int k = tid; k < K; k += NT) {
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
    return 0;
}

// Levels lo_level..hi_level of the combinations (.fs:727-742) appended to the arena
// by ONE wavefront (lane = its lane), each level from the previous one.  Returns the
// arena size, or -1 when it overflows; *lv_lo/*lv_hi: range of the last level built.
__device__ int build_levels(const MultiArgs &a, const Slot &sl, int K, int top, int lane,
                            int *lv_lo, int *lv_hi) {
    const int W = a.W;
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
    int lo = 0, hi = 0;
    if (top >= 1) {
        // level 1: (log2(S_k * 1.0), [k]) for log2(S_k * 1.0) > cutOff (.fs:735-738)
        for (int k0 = 0; k0 < K && !ovf; k0 += 64) {
            const int k = k0 + lane;
            bool pass = false;
            double pr = 0.0, lv = 0.0;
            if (k < K) {
                pr = sl.S[k] * 1.0;
                lv = flog2_ref(pr);
                pass = lv > a.cutoff;
            }
            append(pass, pr, lv, k, -1);
        }
        hi = total;
    }
    // level m from level m-1: children j > last + W with log2(S_j * prod) > cutOff
    for (int m = 2; m <= top && !ovf && lo < hi; ++m) {
        for (int pb = lo; pb < hi && !ovf; pb += 64) {
            // parents 64 at a time into lane registers (arena writes above are this
            // wavefront's own, ordered by the fence)
            __threadfence_block();
            double mp = 0.0;
            int ml = 0;
            if (pb + lane < hi) {
                mp = sl.prod[pb + lane];
                ml = sl.last[pb + lane];
            }
            const int nb = min(64, hi - pb);
            for (int i = 0; i < nb && !ovf; ++i) {
                const double pq = lane_read_f64(mp, i);
                const int lq = __builtin_amdgcn_readlane(ml, i);
                for (int j0 = lq + W + 1; j0 < K && !ovf; j0 += 64) {
                    const int j = j0 + lane;
                    bool pass = false;
                    double pr = 0.0, lv = 0.0;
                    if (j < K) {
                        pr = sl.S[j] * pq;  // fst x * prob
                        lv = flog2_ref(pr);
                        pass = lv > a.cutoff;
                    }
                    append(pass, pr, lv, j, pb + i);
                }
            }
        }
        lo = hi;
        hi = total;
    }
    __threadfence_block();
    *lv_lo = lo;
    *lv_hi = hi;
    return ovf ? -1 : total;
}

// The last combination level, never stored: for every parent q in [plo, phi) (-1:
// the root, product 1.0) in order, its children j >= last(q) + W + 1 in ascending
// order, 64 per step; fn(pass, weight, q, j) per lane, wave-uniform calls, until it
// returns false (wave-uniformly).  Parents
// are loaded 64 at a time into lane registers and broadcast (no serial global loads).
template <class F>
__device__ __forceinline__ void for_last_level(const MultiArgs &a, const Slot &sl, int K, int plo,
                                               int phi, int lane, F fn) {
    const int W = a.W;
    for (int pb = plo; pb < phi; pb += 64) {
        const int myq = pb + lane;
        double mp = 1.0;
        int ml = -W - 1;
        if (myq >= 0 && myq < phi) {
            mp = sl.prod[myq];
            ml = sl.last[myq];
        }
        const int nb = min(64, phi - pb);
        for (int i = 0; i < nb; ++i) {
            const double pq = lane_read_f64(mp, i);
            const int lq = __builtin_amdgcn_readlane(ml, i);
            for (int j0 = lq + W + 1; j0 < K; j0 += 64) {
                const int j = j0 + lane;
                bool pass = false;
                double lv = 0.0;
                if (j < K) {
                    const double p = sl.S[j] * pq;  // fst x * prob
                    if (!(p < a.thr_lo)) {
                        lv = flog2_ref(p);
                        pass = p > a.thr_hi || lv > a.cutoff;
                    }
                }
                if (!fn(pass, pass ? lv : 0.0, pb + i, j)) return;
            }
        }
    }
}

struct RPick {
    int c;   // category in [0, K + total), or -1: last level (q, j), or -2: overrun
    int q, j;
    double w;
};

// rouletteWheelSelection (.fs:746-754) over [G_0..G_{K-1}] ++ arena[0..total) ++ the
// last level (children of arena [plo, phi)), one wavefront.
__device__ RPick roulette(const MultiArgs &a, const Slot &sl, int K, int total, int plo, int phi,
                          double u, int lane) {
    const int nmat = K + total;
    auto w_of = [&](int c) { return c < K ? sl.G[c] : sl.wgt[c - K]; };
    double s = 0.0;
    bool bad = false;
    int nlast = 0;
    for (int c = lane; c < nmat; c += 64) {
        const double w = w_of(c);
        bad |= !(w >= 0.0 && w < INFINITY);
        s += w;
    }
    for_last_level(a, sl, K, plo, phi, lane, [&](bool pass, double w, int, int) {
        if (pass) {
            bad |= !(w >= 0.0 && w < INFINITY);
            s += w;
            ++nlast;
        }
        return true;
    });
    const double tot = wave_sum_f64(s);
    const int ncat = nmat + wave_sum_i32(nlast);
    RPick pk{-2, -1, -1, 0.0};
    bool serial = __ballot(bad) != 0ull || !(tot > 0.0 && tot < INFINITY);
    if (!serial) {
        // the reference's boundaries acc_c are within (2 ncat + 2) 2^-53 of the exact
        // prefix ratios; ours within (ncat/64 + 8) 2^-53: 8 ncat + 64 covers both
        const double t = u * tot;
        const double D = (8.0 * (double)ncat + 64.0) * 0x1.0p-53 * tot;
        double carry = 0.0;
        int state = 0;  // 0 searching, 1 found, 2 undecided
        // one step of 64 consecutive categories (real: lanes holding a category)
        auto step = [&](bool real, double w) -> int {
            const double incl = wave_incl_scan_f64(real ? w : 0.0);
            const double h = carry + incl, l = carry + (incl - (real ? w : 0.0));
            const bool near = real && (fabs(t - h) <= D || fabs(t - l) <= D);
            carry = lane_read_f64(h, 63);
            if (__ballot(near) != 0ull) return -2;
            const unsigned long long in = __ballot(real && l < t && t < h);
            return in ? __ffsll((long long)in) - 1 : -1;
        };
        for (int b0 = 0; b0 < nmat && state == 0; b0 += 64) {
            const int c = b0 + lane;
            const int r = step(c < nmat, c < nmat ? w_of(c) : 0.0);
            if (r == -2) state = 2;
            if (r >= 0) {
                state = 1;
                pk.c = b0 + r;
            }
        }
        if (state == 0)
            for_last_level(a, sl, K, plo, phi, lane, [&](bool pass, double w, int q, int j) {
                const int r = step(pass, w);
                if (r == -2) state = 2;
                if (r >= 0) {
                    state = 1;
                    pk.c = -1;
                    pk.q = q;
                    pk.j = __shfl(j, r, 64);
                    pk.w = __shfl(w, r, 64);
                }
                return state == 0;
            });
        serial = state != 1;
    }
    if (serial) {
        // one lane replays List.sum and the running acc exactly, in category order
        pk.c = -2;
        if (lane == 0) {
            double sum = 0.0;
            for (int c = 0; c < nmat; ++c) sum = sum + w_of(c);
            for (int q = plo; q < phi; ++q) {
                const double pq = q < 0 ? 1.0 : sl.prod[q];
                for (int j = (q < 0 ? 0 : sl.last[q] + a.W + 1); j < K; ++j) {
                    const double p = sl.S[j] * pq;
                    const double lv = flog2_ref(p);
                    if (lv > a.cutoff) sum = sum + lv;
                }
            }
            double acc = 0.0;
            bool done = false;
            for (int c = 0; c < nmat && !done; ++c) {
                const double w = w_of(c) / sum;
                if (acc <= u && u <= acc + w) {
                    pk.c = c;
                    done = true;
                }
                acc = acc + w;
            }
            for (int q = plo; q < phi && !done; ++q) {
                const double pq = q < 0 ? 1.0 : sl.prod[q];
                for (int j = (q < 0 ? 0 : sl.last[q] + a.W + 1); j < K && !done; ++j) {
                    const double lv = flog2_ref(sl.S[j] * pq);
                    if (!(lv > a.cutoff)) continue;
                    const double w = lv / sum;
                    if (acc <= u && u <= acc + w) {
                        pk.c = -1;
                        pk.q = q;
                        pk.j = j;
                        pk.w = lv;
                        done = true;
                    }
                    acc = acc + w;
                }
            }
            atomicAdd(&GS_STAT(a)[1], 1ull);
        }
        pk.c = __shfl(pk.c, 0, 64);
        pk.q = __shfl(pk.q, 0, 64);
        pk.j = __shfl(pk.j, 0, 64);
        pk.w = __shfl(pk.w, 0, 64);
    }
    return pk;
}

// Write a category's (cnt, positions in F# cons order, PWMS): `last` = the newest
// position (or -1 for a background category) followed by the arena chain from q.
__device__ __forceinline__ void emit(const Slot &sl, int last, int q, double pwms, int32_t *cnt_out,
                                     int32_t *pos_out, double *pwms_out) {
    int i = 0;
    if (last >= 0) pos_out[i++] = last;
    while (q >= 0) {
        pos_out[i++] = sl.last[q];
        q = sl.parent[q];
    }
    *cnt_out = i;
    *pwms_out = pwms;
}

// Passing test of a product against the cut-off (.fs:735): certain by the
// thresholds, else the reference's log2.
__device__ __forceinline__ bool passes(const MultiArgs &a, double p) {
    return p > a.thr_hi || (!(p < a.thr_lo) && flog2_ref(p) > a.cutoff);
}

struct GPick {
    int level;   // 0 background, 1 arena entry, 2 last level (virtual)
    int idx;     // background window / arena index / parent arena index (-1 = root)
    int j;       // last level: newest window
    double pwms;
};

// The greedy's head of the stable descending sort (.fs:917-920), every thread of
// the workgroup.  Returns status 0 / kMultiErrArena.
__device__ int greedy_pick(const MultiArgs &a, const Slot &sl, int K, GPick &out, Best *red,
                           int *shared_i, double *ppar, int32_t *lpar) {
    const int tid = threadIdx.x, NT = blockDim.x, lane = tid & 63, wave = tid >> 6;
    const int nw = NT >> 6, W = a.W, M = a.M;
    // levels 1..M-1 (the last level's parents), built by wavefront 0
    if (wave == 0) {
        int lo = 0, hi = 0;
        const int total = build_levels(a, sl, K, M - 1, lane, &lo, &hi);
        if (lane == 0) {
            shared_i[0] = total;
            shared_i[1] = lo;
            shared_i[2] = hi;
        }
    }
    __syncthreads();
    const int total = shared_i[0];
    if (total < 0) return kMultiErrArena;
    const int plo = M == 1 ? -1 : shared_i[1], phi = M == 1 ? 0 : shared_i[2];
    // the first maximum of the materialised categories: backgrounds, then the arena
    Best bm{0ull, ~0ull};
    for (int c = tid; c < K + total; c += NT)
        best_take(bm, order_key(c < K ? sl.G[c] : sl.wgt[c - K]), (unsigned long long)c);
    bm = block_best(bm, red);
    // the last level: products S_j * prod(parent) (root: 1.0), children j >= last + W + 1
    // in (parent, j) order.  Parents are staged into LDS in blocks of kParentBlock
    // and dealt round-robin to the wavefronts, each scoring its parents' children
    // 64 at a time; the order key (parent + 1, j) keeps the category order.
    auto scan = [&](bool band, double pband, Best &b) {
        for (int pb = plo; pb < phi; pb += kParentBlock) {
            const int nb = min(kParentBlock, phi - pb);
            __syncthreads();
            for (int i = tid; i < nb; i += NT) {
                const int q = pb + i;
                ppar[i] = q < 0 ? 1.0 : sl.prod[q];
                lpar[i] = q < 0 ? -W - 1 : sl.last[q];
            }
            __syncthreads();
            for (int i = wave; i < nb; i += nw) {
                const double pq = ppar[i];
                const unsigned long long qk = (unsigned long long)(pb + i + 1) << 32;
                for (int j = lpar[i] + W + 1 + lane; j < K; j += 64) {
                    const double p = sl.S[j] * pq;  // fst x * prob
                    if (!band) {
                        if (passes(a, p)) best_take(b, order_key(p), qk | (unsigned)j);
                    } else if (p >= pband && passes(a, p)) {
                        best_take(b, order_key(flog2_ref(p)), qk | (unsigned)j);
                    }
                }
            }
        }
    };
    Best bp{0ull, ~0ull};
    scan(false, 0.0, bp);
    bp = block_best(bp, red);
    Best bl{0ull, ~0ull};
    if (bp.i != ~0ull) {
        // the largest passing product P*: every product below P*(1 - 2^-40) has a log2
        // at least 1.3e-12 below log2 P*, beyond the logs' ulp errors
        const int bq = (int)(bp.i >> 32) - 1, bj = (int)(bp.i & 0xffffffffu);
        const double pstar = sl.S[bj] * (bq < 0 ? 1.0 : sl.prod[bq]);
        scan(true, pstar * (1.0 - 0x1.0p-40), bl);
        bl = block_best(bl, red);
    }
    // first maximum over [backgrounds ++ arena] ++ last level (category order)
    if (bl.i != ~0ull && (bm.i == ~0ull || bl.v > bm.v)) {
        const int q = (int)(bl.i >> 32) - 1, j = (int)(bl.i & 0xffffffffu);
        out.level = 2;
        out.idx = q;
        out.j = j;
        out.pwms = flog2_ref(sl.S[j] * (q < 0 ? 1.0 : sl.prod[q]));
    } else {
        const int c = (int)bm.i;
        out.level = c < K ? 0 : 1;
        out.idx = c < K ? c : c - K;
        out.j = -1;
        out.pwms = c < K ? sl.G[c] : sl.wgt[c - K];
    }
    return 0;
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
    __shared__ int flag;
    const int lane = threadIdx.x;
    const Slot sl = slot_of(a, blockIdx.x, lds);
    const int AW = a.A * a.W;
    const int64_t *C = a.agg, *T = a.agg + AW;
    for (int i = blockIdx.x; i < a.n_targets; i += gridDim.x) {
        const int n = a.targets ? a.targets[i] : i;
        const int L = a.len[n];
        const int K = L - a.W + 1;
        const int64_t gidx = a.global_offset + n;
        __syncthreads();
        stage(a.seq + a.doff[n], L, sseq);
        __syncthreads();
        const int cnt = a.cnt_in[n];
        const int32_t *pos = a.pos_in + (int64_t)n * a.cap_in;
        const int st = prepare_target(a, n, L, sseq, cnt, pos, C, T, tab, pcv, sl, &flag);
        if (st) {
            if (lane == 0) raise_err(a, gidx, st);
            continue;
        }
        // levels 1..M-1 (the last level's parents) in the arena; the last level virtual
        int lo, hi;
        const int total = build_levels(a, sl, K, a.M - 1, lane, &lo, &hi);
        if (total < 0) {
            if (lane == 0) a.ovf_list[atomicAdd(a.ovf_count, 1)] = n;
            continue;
        }
        const int plo = a.M == 1 ? -1 : lo, phi = a.M == 1 ? 0 : hi;
        const double u = a.u ? a.u[n] : uniform(a.seed, a.stream, (uint64_t)gidx);
        const RPick pk = roulette(a, sl, K, total, plo, phi, u, lane);
        if (pk.c == -2) {
            if (lane == 0) raise_err(a, gidx, 2);  // list index past the end (.fs:752)
            continue;
        }
        if (lane == 0) {
            int32_t *po = a.pos_out + (int64_t)n * a.cap_out;
            if (pk.c == -1)
                emit(sl, pk.j, pk.q, pk.w, a.cnt_out + n, po, a.pwms_out + n);
            else
                emit(sl, -1, pk.c < K ? -1 : pk.c - K, pk.c < K ? sl.G[pk.c] : sl.wgt[pk.c - K],
                     a.cnt_out + n, po, a.pwms_out + n);
        }
    }
}

// Greedy Gauss–Seidel passes (.fs:885-929), speculatively: visits are scored in
// parallel against the live aggregates (gs_multi_spec_score_kernel, one workgroup per
// visit), then committed in visit order up to and including the first one that moves
// its Positions list (gs_multi_spec_commit_kernel); the visits after it are scored
// again next step against the updated aggregates.  A visit is only ever committed
// from a score against exactly the aggregates the sequential loop would use (every
// earlier visit of the step left them unchanged), so the passes are the reference's.
// The head of the descending sort is kept when its PWMS is strictly larger (.fs:923);
// passes repeat until one leaves every Positions list unchanged (.fs:888).
extern "C" __global__ void __launch_bounds__(1024) gs_multi_spec_score_kernel(MultiArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    double *tab = (double *)(lds + a.o_tab);
    double *pcv = (double *)(lds + a.o_pcv);
    uint8_t *sseq = lds + a.o_seq;
    int64_t *agg = (int64_t *)(lds + a.o_agg);
    __shared__ int flag;
    __shared__ int shared_i[4];
    __shared__ Best red[kMaxWaves];
    __shared__ double ppar[kParentBlock];
    __shared__ int32_t lpar[kParentBlock];
    const SpecCtl ctl = *a.spec_ctl;
    const int tid = threadIdx.x;
    const int n = ctl.base + (int)blockIdx.x;
    if (ctl.done || n >= a.n_local) return;
    const int A = a.A, W = a.W, AW = A * W;
    const Slot sl = slot_of(a, blockIdx.x, lds);
    for (int c = tid; c < AW + A; c += blockDim.x) agg[c] = a.agg_rw[c];
    const int L = a.len[n];
    const int K = L - W + 1;
    stage(a.seq + a.doff[n], L, sseq);
    __syncthreads();
    const int32_t *lst = a.pos_out + (int64_t)n * a.cap_out;
    const int cnt = a.cnt_out[n];
    int st = prepare_target(a, n, L, sseq, cnt, lst, agg, agg + AW, tab, pcv, sl, &flag);
    GPick pk{};
    if (!st) st = greedy_pick(a, sl, K, pk, red, shared_i, ppar, lpar);
    if (tid == 0) {
        SpecRes &r = a.spec_res[blockIdx.x];
        r.status = st;
        if (!st) {
            emit(sl, pk.level == 2 ? pk.j : -1, pk.level == 0 ? -1 : pk.idx, pk.pwms, &r.cnt,
                 r.pos, &r.pw);
            r.accept = r.pw > a.pwms_out[n];  // tmp.PWMS > acc.[n].PWMS (.fs:923)
            bool same = r.cnt == cnt;
            for (int i = 0; same && i < cnt; ++i) same = r.pos[i] == lst[i];
            r.moved = r.accept && !same;
        }
    }
}

extern "C" __global__ void __launch_bounds__(64) gs_multi_spec_commit_kernel(MultiArgs a) {
    SpecCtl *ctl = a.spec_ctl;
    const SpecCtl c0 = *ctl;
    if (c0.done) return;
    const int lane = threadIdx.x;
    const int A = a.A, W = a.W, AW = A * W;
    const int base = c0.base, nres = min(a.spec_slots, a.n_local - base);
    // the first visit that moves (or failed): everything before it stands
    int first = nres;
    for (int w0 = 0; w0 < nres; w0 += 64) {
        const int w = w0 + lane;
        const bool f = w < nres && (a.spec_res[w].moved || a.spec_res[w].status);
        const unsigned long long m = __ballot(f);
        if (m) {
            first = w0 + __ffsll((long long)m) - 1;
            break;
        }
    }
    for (int w = lane; w < first; w += 64)
        if (a.spec_res[w].accept) a.pwms_out[base + w] = a.spec_res[w].pw;  // same list
    int nbase = base + nres, changed = c0.changed;
    if (first < nres) {
        const SpecRes &r = a.spec_res[first];
        const int n = base + first;
        if (r.status) {  // raised against the reference's aggregates: the loop throws here
            if (lane == 0) {
                raise_err(a, a.global_offset + n, r.status);
                ctl->done = 1;
            }
            return;
        }
        // move the target's contribution from its old list to the new one
        int32_t *lst = a.pos_out + (int64_t)n * a.cap_out;
        const int cnt = a.cnt_out[n];
        const uint8_t *s = a.seq + a.doff[n];
        unsigned long long *C = (unsigned long long *)a.agg_rw, *T = C + AW;
        if (lane < W) {
            for (int i = 0; i < cnt; ++i) {
                const int e = s[lst[i] + lane];
                if (e < A) {
                    atomicAdd(&C[e * W + lane], ~0ull);
                    atomicAdd(&T[e], 1ull);
                }
            }
            for (int i = 0; i < r.cnt; ++i) {
                const int e = s[r.pos[i] + lane];
                if (e < A) {
                    atomicAdd(&C[e * W + lane], 1ull);
                    atomicAdd(&T[e], ~0ull);
                }
            }
        }
        if (lane < A) {
            const int64_t ce = a.comp[(int64_t)n * (a.E + 1) + lane];
            atomicAdd(&T[lane], (unsigned long long)(ce * (int64_t)(r.cnt - cnt)));
        }
        __syncthreads();
        if (lane < r.cnt) lst[lane] = r.pos[lane];
        if (lane == 0) {
            a.cnt_out[n] = r.cnt;
            a.pwms_out[n] = r.pw;
        }
        changed = 1;
        nbase = n + 1;
    }
    if (lane == 0) {
        SpecCtl c = c0;
        c.base = nbase;
        c.changed = changed;
        if (nbase >= a.n_local) {  // a pass ends (.fs:887-889)
            ++c.pass;
            if (!c.changed || c.pass >= a.max_passes)
                c.done = 1;
            else {
                c.base = 0;
                c.changed = 0;
            }
        }
        *ctl = c;
    }
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

// `steps` speculative steps (score + commit each), enqueued without host syncs; the
// kernels return at once when the passes are done.
hipError_t gs_multi_spec_launch(const MultiArgs &a, int threads, size_t lds, int steps,
                                hipStream_t s) {
    for (int i = 0; i < steps; ++i) {
        hipLaunchKernelGGL(gs_multi_spec_score_kernel, dim3(a.spec_slots), dim3(threads), lds, s, a);
        hipLaunchKernelGGL(gs_multi_spec_commit_kernel, dim3(1), dim3(64), 0, s, a);
    }
    return hipGetLastError();
}

// ---- the star greedy's hand-over to the speculative list path (gs_api.cpp) ----
extern "C" __global__ void __launch_bounds__(256) gs_single_to_lists_kernel(const int32_t *pos,
                                                                             int32_t n, int32_t *cnt,
                                                                             int32_t *lst) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const int p = pos[i];
        cnt[i] = p >= 0;
        lst[i] = p;
    }
}

extern "C" __global__ void __launch_bounds__(256) gs_lists_to_single_kernel(const int32_t *cnt,
                                                                             const int32_t *lst,
                                                                             int32_t n, int32_t *pos) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        pos[i] = cnt[i] > 0 ? lst[i] : -1;
}

// number of i with a[i] != b[i], added to *out
extern "C" __global__ void __launch_bounds__(256) gs_count_diff_kernel(const int32_t *a,
                                                                        const int32_t *b, int32_t n,
                                                                        int32_t *out) {
    int d = 0;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        d += a[i] != b[i];
    d = wave_sum_i32(d);
    if ((threadIdx.x & 63) == 0 && d) atomicAdd(out, d);
}

hipError_t gs_single_lists_launch(const int32_t *pos, int32_t n, int32_t *cnt, int32_t *lst,
                                  int to_lists, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const int grid = std::min((n + 255) / 256, 1024);
    if (to_lists)
        hipLaunchKernelGGL(gs_single_to_lists_kernel, dim3(grid), dim3(256), 0, s, pos, n, cnt, lst);
    else
        hipLaunchKernelGGL(gs_lists_to_single_kernel, dim3(grid), dim3(256), 0, s, cnt, lst, n,
                           (int32_t *)pos);
    return hipGetLastError();
}

hipError_t gs_count_diff_launch(const int32_t *a, const int32_t *b, int32_t n, int32_t *out,
                                hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const int grid = std::min((n + 255) / 256, 1024);
    hipLaunchKernelGGL(gs_count_diff_kernel, dim3(grid), dim3(256), 0, s, a, b, n, out);
    return hipGetLastError();
}
