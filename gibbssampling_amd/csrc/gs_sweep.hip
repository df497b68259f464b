// gs_sweep.hip — fused Gibbs sweep kernel for gfx950 (MI355X).
//
// A workgroup is 4 independent 64-lane wavefronts; each wavefront grid-strides
// over this rank's sequences.  Per sequence n (MotifSampler.
// findBestMotifIndicesByWithStartPositions, .fs:935-970, motifAmount = 1):
//   1. stage the encoded sequence into the wavefront's LDS slice (16-byte loads,
//      prefetched one sequence ahead).  Its symbol histogram (createFCVOf,
//      .fs:60-62) is static and precomputed at upload time;
//   2. hold-one-out background counts and PCV from the snapshot aggregates
//      (createFCVWithout/fuseFrequencyVectors/increaseInPlaceFCVOf/
//      createNormalizedPCVOfFCV, .fs:945-954) — integer exact;
//   3. log tables: log2 PWM = log2 PPM - log2 PCV (.fs:955-965).  The PPM and its
//      binary32 log2 are built once per workgroup (global counts, and counts
//      minus one for the sequence's own segment); per sequence only E logs of the
//      PCV remain.  With |alphabet| <= 16 the logs are paired into one table per
//      two motif columns indexed by the pair code s[i] + E*s[i+1];
//   4. certified scan: every W-mer window (.fs:759-777) is scored as a binary32
//      log2 sum under a rigorous per-sequence error bound.  The cut-off test
//      (.fs:735-738) is decided from the bound; the rare window inside the band
//      is marked and afterwards folded exactly in binary64 (the reference's
//      left fold of PWM / PCV factors, for which the exact table is built then);
//   5. roulette pick (.fs:746-754): a lane-level then window-level wavefront
//      prefix sum of the approximate weights; the pick is accepted only when u
//      is farther than the combined approximation + rounding bound from every
//      CDF boundary that decides it.  The picked window's weight is then folded
//      exactly (binary64, reference order); its log2 (.fs:737) is taken once per
//      64 sequences, one lane each.  An undecided pick rescans the sequence in
//      binary64 and certifies against rounding alone, or — still undecided —
//      one lane redoes the reference's sequential sums exactly;
//   6. the picked segment is folded into per-wavefront aggregates of the new
//      snapshot, flushed to XCD-replicated global accumulators once per
//      workgroup: the next sweep's count matrix and background totals.
//
// Compiled with -ffp-contract=off: no FMA contraction.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "gs_common.h"
#include "gs_wave.h"

using namespace gs;

namespace {

constexpr int kWavesPerBlock = 4;
typedef float f2 __attribute__((ext_vector_type(2)));

// In-kernel phase stamps, diagnostic build only (make STAMPS=1): never in the
// shipped library; their run time is not quoted, only the phase shares.
#ifdef GS_STAMPS
#define STAMP_DECL                               \
    unsigned long long st_acc[kStampSlots] = {0}; \
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
            for (int i_ = 0; i_ < kStampSlots - 1; ++i_)                         \
                atomicAdd(&a.stamps[i_], st_acc[i_]);                            \
            atomicAdd(&a.stamps[kStampSlots - 1], (unsigned long long)(nseq));   \
        }                                                                        \
    } while (0)
#elif defined(GS_MARKS)
// static instruction accounting (tools/isa_phases.py): phase labels in the ISA
#define STAMP_DECL
#define STAMP(i) asm volatile(";GSMARK stamp" #i ::: "memory")
#define GS_MARK(s) asm volatile(";GSMARK " s ::: "memory")
#define STAMP_FLUSH(nseq) \
    do {                  \
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
#ifndef GS_MARK
#define GS_MARK(s) \
    do {           \
    } while (0)
#endif

__device__ __forceinline__ void raise_error(const SweepArgs &a, int code, int64_t gidx) {
    atomicCAS(a.err_code, 0, code);
    atomicMin(a.err_index, (unsigned long long)gidx);
}

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
        // VGPRs at the peak (this fold is off the certified scan's hot path)
        __builtin_amdgcn_sched_barrier(0);
    }
    // materialise both folds here: otherwise the G fold is sunk below the caller's
    // log2 branch and every table operand stays live across it (VGPRs, occupancy)
    asm volatile("" ::"v"(S), "v"(G));
}

// Pairwise (tree) sum of the NG group terms: depth ceil(log2 NG), so each term's
// rounding error is bounded by depth * (sum of |terms|) * 2^-24.
template <int NG>
__device__ __forceinline__ f2 tree_sum(f2 *v) {
#pragma unroll
    for (int s = 1; s < NG; s *= 2) {
#pragma unroll
        for (int i = 0; i + s < NG; i += 2 * s) v[i] += v[i + s];
    }
    return v[0];
}

template <int NG>
constexpr int tree_depth() {
    int d = 0;
    for (int s = 1; s < NG; s *= 2) ++d;
    return d;
}

// Approximate (log2 S_k, log2 G_k) in binary32.  H = 2: codes[i] = s[i] + E*s[i+1]
// and ltab = [E*E][gt_stride(WM)] pair sums; H = 1: codes = symbols and ltab =
// [E][lt_stride(WM)].  Code-major with odd strides: the group offset g*8 is a
// ds_read immediate, different codes land in different banks.  Groups past the
// motif hold (0, 0).
template <int WM, int H>
__device__ __forceinline__ f2 window_logs(const uint8_t *codes, const unsigned char *ltab, int k) {
    constexpr int ND = WM / 4 + 1, NG = WM / H;
    constexpr int RS = (H == 2 ? gt_stride(WM) : lt_stride(WM)) * 8;
    const int kb = k & ~3, off = k & 3;
    uint32_t d[ND];
#pragma unroll
    for (int i = 0; i < ND; ++i) d[i] = *(const uint32_t *)(codes + kb + 4 * i);
    f2 v[NG];
#pragma unroll
    for (int i = 0; i < WM / 4; ++i) {
        const uint32_t x = __builtin_amdgcn_alignbyte(d[i + 1], d[i], off);
#pragma unroll
        for (int t = 0; t < 4; t += H) {
            const int g = (4 * i + t) / H;
            const uint32_t c = (x >> (8 * t)) & 0xffu;
            v[g] = *(const f2 *)(ltab + c * RS + g * 8);
        }
    }
    return tree_sum<NG>(v);
}

// Certified-scan view of the sequence's windows.
struct FastView {
    const uint8_t *lcodes, *sseq;
    const unsigned char *ltab, *tab;
    float hiS, loS;  // the cut-off band [loS, hiS] in binary32
    double cutoff;
};

enum { kFail = 0, kPass = 1, kUnsure = 2 };

// Window k in the certified scan: approximate background weight gw = 2^log2 G~
// and log2 S~; the class says whether S certainly passes the cut-off, certainly
// fails it, or lies in the band.  flag: a log outside the error model's range.
template <int WM, int H>
__device__ __forceinline__ int fast_window(const FastView &c, int k, double &gw, float &fs,
                                           bool &flag) {
    const f2 lg = window_logs<WM, H>(c.lcodes, c.ltab, k);
    fs = lg.x;
    const float fg = lg.y;
    flag |= !(fg > -1000.0f && fg < 1000.0f);
    gw = fexp2(fg);
    return (fs > c.hiS && fs < 1000.0f) ? kPass : (fs < c.loS ? kFail : kUnsure);
}

// A window in the band: the reference's binary64 fold decides (.fs:735-738).
template <int WM>
__device__ __forceinline__ float resolve_window(const FastView &c, int k) {
    double S, G;
    window_products<WM>(c.sseq, c.tab, k, S, G);
    const double l2 = log(S * 1.0) / kLn2;
    return l2 > c.cutoff ? (float)l2 : -INFINITY;
}

// Exact view: the reference's binary64 G_k and, when it passes the cut-off,
// log2 S_k (.fs:735-738, .fs:759-777).
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

// Certified roulette pick (.fs:746-754) over per-lane blocks of windows: lane l
// scored windows [l*R, l*R + nv_l) into the sums sG (background weights) and sM
// (motif weights, lcat categories).  ev(k, g, m) re-evaluates window k exactly as
// the scan did (m = -inf: not a category).  Weights are non-negative and each is
// within its share of eabs (the summed absolute error bound) of the reference's.
// Returns 0 (background category pk), 1 (motif category pk), or < 0 when the
// pick is not certified (the caller falls back): -1 total not separated from its
// error bound, -2 no candidate lane, -3 u within the bound of a deciding CDF
// boundary, -4 u between two lanes' blocks.
template <class Eval>
__device__ int certified_pick(const Eval &ev, int K, int R, int lane, double u, double sG,
                              double sM, int lcat, int npass, double eabs_g, double eabs_m_per,
                              double eabs_m_rel, int &pk) {
    const double inclG = wave_incl_scan_f64(sG);
    const double inclM = wave_incl_scan_f64(sM);
    const double totG = lane_read_f64(inclG, 63), totM = lane_read_f64(inclM, 63);
    const double total = totG + totM;
    const double eabs = totG * eabs_g + (double)npass * eabs_m_per + totM * eabs_m_rel;
    if (!(total > 4.0 * eabs) || !(total < INFINITY)) return -1;  // also NaN, total <= 0
    // rounding of the reference's sequential sums and of ours (wavefront scans,
    // one division each), relative to the total; SA = total (weights >= 0)
    const double ncat = (double)(K + npass + 2);
    const double delta =
        (8.0 * ncat + 64.0) * 0x1.0p-53 + eabs / total * (1.0 + (total + eabs) / (total - eabs));
    const double inv = 1.0 / total;
    const int nv = min(max(K - lane * R, 0), R);
    const bool phaseG = !(u > totG * inv + delta);
    // lane level: the first lane whose block range may contain u
    double lo, hi;
    if (phaseG) {
        lo = (inclG - sG) * inv;
        hi = inclG * inv;
    } else {
        lo = (totG + (inclM - sM)) * inv;
        hi = (totG + inclM) * inv;
    }
    const bool cand = (phaseG ? nv > 0 : lcat > 0) && u >= lo - delta && u <= hi + delta;
    const unsigned long long b = __ballot(cand);
    if (!b) return -2;
    const int f = __ffsll((long long)b) - 1;
    double base = lane_read_f64(lo, f);
    const int nf = __builtin_amdgcn_readlane(nv, f);
    // window level inside lane f's block, 64 windows at a time
    for (int c0 = 0; c0 < nf; c0 += 64) {
        const int t = c0 + lane;
        double w = 0.0;
        bool is_cat = false;
        if (t < nf) {
            double g, m;
            ev(f * R + t, g, m);
            const double x = phaseG ? g : m;
            is_cat = phaseG || x != -INFINITY;
            if (is_cat) w = x * inv;
        }
        const double incl = wave_incl_scan_f64(w);
        const double l0 = base + (incl - w), h0 = base + incl;
        const bool no = !is_cat || u < l0 - delta || u > h0 + delta;
        const bool yes = !no && u >= l0 + delta && u <= h0 - delta;
        const unsigned long long bb = __ballot(!no);
        if (bb) {
            const int first = __ffsll((long long)bb) - 1;
            if (!__builtin_amdgcn_readlane((int)yes, first)) return -3;
            pk = f * R + c0 + first;
            return phaseG ? 0 : 1;
        }
        base = base + lane_read_f64(incl, 63);
    }
    return -4;
}

}  // namespace

// Register budget: GS_WAVES_PER_EU (build flag) asks the allocator for that many
// resident waves per SIMD (512 / n VGPRs each).
#ifdef GS_WAVES_PER_EU
#define GS_SWEEP_ATTR __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(GS_WAVES_PER_EU, 8)))
#else
#define GS_SWEEP_ATTR __launch_bounds__(256)
#endif

template <int WM, int H>
__global__ void GS_SWEEP_ATTR gs_sweep_kernel(SweepArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar loads
    constexpr int NG = WM / H, WS = tab_stride(WM), LS = lt_stride(WM), GS = gt_stride(WM);

    const int A = a.A, E = a.E, W = a.W, AW = A * W, CS = E + 1, E2 = E * E;
    // workgroup-shared
    int32_t *cg = (int32_t *)(lds + a.o_cg);          // [A*W] global counts C
    int64_t *T = (int64_t *)(lds + a.o_T);            // [A+1] others' background totals, sum
    double *ppmG = (double *)(lds + a.o_ppmG);        // [A*W] (C + pc)/den
    double *ppmM = (double *)(lds + a.o_ppmM);        // [A*W] (C - 1 + pc)/den: own segment
    float *lppmG = (float *)(lds + a.o_lppmG);        // [A*W] log2 of the above, binary32
    float *lppmM = (float *)(lds + a.o_lppmM);
    unsigned int *bmax = (unsigned int *)(lds + a.o_bmax);  // max finite |log2 PPM|
    // wavefront slice
    unsigned char *wl = lds + a.o_wave + wid * a.wave_bytes;
    unsigned char *tab = wl + a.w_tab;                // [E][WS] double2 exact (PWM, PCV), lazy
    float2 *lt = (float2 *)(wl + a.w_lt);             // [E][LS] (log2 PWM, log2 PCV)
    unsigned char *gt = wl + a.w_gt;                  // H = 2: [E*E][GS] pair sums
    uint8_t *cseq = (uint8_t *)(wl + a.w_code);       // H = 2: pair codes
    int32_t *aggC = (int32_t *)(wl + a.w_aggC);       // [A*W]
    int64_t *aggM = (int64_t *)(wl + a.w_aggM);       // [A]
    double *pcv = (double *)(wl + a.w_pcv);           // [64] by encoded symbol
    float *lpcv = (float *)(wl + a.w_lpcv);           // [64] log2 PCV
    double2 *wfac = (double2 *)(wl + a.w_wfac);       // [WM] factors of the picked window
    int32_t *misc = (int32_t *)(wl + a.w_misc);
    uint8_t *sseq = (uint8_t *)(wl + a.w_seq);
    const uint8_t *lcodes = H == 2 ? cseq : sseq;
    const unsigned char *ltab = H == 2 ? gt : (const unsigned char *)lt;
    const bool certified = a.scan == kScanCertified;
    const uint32_t magicE = 0xffffffffu / (uint32_t)E + 1u;  // x / E for x < 2^16
    const uint32_t magicW = 0xffffffffu / (uint32_t)W + 1u;
    STAMP_DECL
    int nseq_done = 0;

    // The loads that start the pipeline are all issued before the prologue's
    // barrier (which waits for them anyway): the sticky error flag of earlier
    // sweeps, this wavefront's first 64 descriptors, and the first sequence and
    // its composition (address from scalar loads).
    const int err0 = __hip_atomic_load(a.err_code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // This wavefront's sequences are n0 + i*wstride, i < cnt.  Their descriptors
    // (length, offset, snapshot position, uniform) are loaded 64 at a time into
    // lane registers and their results kept there and stored 64 at a time, so the
    // only vector memory operations inside the loop are the one-ahead prefetches
    // of the next sequence and its composition (vmcnt waits are in order: a
    // descriptor load behind a prefetch or a store would otherwise wait for it).
    const int wstride = gridDim.x * kWavesPerBlock;
    const int n0 = blockIdx.x * kWavesPerBlock + wid;
    const int cnt = n0 < a.n_local ? (a.n_local - 1 - n0) / wstride + 1 : 0;
    int b_len = 0, b_pos = -1, r_pos = -1;
    int64_t b_off = 0;
    double b_u = 0.0, r_pw = 0.0;
    bool r_log = false;  // r_pw holds S of a motif pick: log2 taken at the batch end
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
    // one-sequence-ahead prefetch (sequences up to 1024 symbols) and composition
    uint4 pf = make_uint4(0, 0, 0, 0);
    int cpf = 0;
    if (cnt > 0) {
        const int L0 = a.len[n0];
        const int64_t o0 = a.doff[n0];
        if (L0 <= 1024 && lane * 16 < L0) pf = *(const uint4 *)(a.seq + o0 + lane * 16);
        if (lane < CS) cpf = a.comp[(int64_t)n0 * CS + lane];
    }
    load_batch(0);

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
    if (tid == 0) *bmax = 0u;
    if (blockIdx.x == 0 && a.agg_zero)
        for (int i = tid; i < kRepl * a.stride; i += 256) a.agg_zero[i] = 0;
    __syncthreads();
    // an earlier sweep raised an error: its snapshot is void, nothing to do (a
    // wavefront that exits leaves the workgroup barriers below)
    if (__builtin_amdgcn_readfirstlane(err0) != 0) return;
    if (a.mode == 0) {
        float mx = 0.0f;
        for (int c = tid; c < AW; c += 256) {
            const double g = ((double)cg[c] + a.pc) / a.den;  // normalizePPM (.fs:257-260)
            const double m = ((double)(cg[c] - 1) + a.pc) / a.den;
            ppmG[c] = g;
            ppmM[c] = m;
            const float lg = flog2(g), lm = flog2(m);
            lppmG[c] = lg;
            lppmM[c] = lm;
            // finite entries only (a count-minus-one cell of a zero count is NaN and
            // never used: own-segment cells have C >= 1)
            if (fabsf(lg) < INFINITY) mx = fmaxf(mx, fabsf(lg));
            if (fabsf(lm) < INFINITY) mx = fmaxf(mx, fabsf(lm));
        }
        mx = wave_max_nonneg_f32(mx);
        if (lane == 0) atomicMax(bmax, __float_as_uint(mx));
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
        // columns past the motif: exact factors 1.0, log terms 0 (never rewritten)
        for (int c = lane; c < E * WS; c += 64)
            if (c % WS >= W) *(double2 *)(tab + c * 16) = make_double2(1.0, 1.0);
        for (int c = lane; c < E * LS; c += 64)
            if (c % LS >= W) lt[c] = make_float2(0.0f, 0.0f);
        if (lane < WM && lane >= W) wfac[lane] = make_double2(1.0, 1.0);
    }
    __syncthreads();

    const int64_t sumT = a.mode == 0 ? T[A] : 0;  // Σ_a T[a], set in the prologue
    const float tppm = a.mode == 0 ? __uint_as_float(*bmax) : 0.0f;
    // exact (PWM, PCV) table of the current sequence, built on demand
    auto build_tab = [&](int p) {
        const int pp = p >= 0 ? p : 0;
        for (int c = lane; c < E * W; c += 64) {
            const int e = (int)__umulhi((uint32_t)c, magicW), j = c - e * W;
            const double pe = pcv[e];
            const bool own = (p >= 0) & (sseq[pp + j] == e);
            const double pm = (own ? ppmM : ppmG)[(e < A ? e : 0) * W + j];
            *(double2 *)(tab + (e * WS + j) * 16) = make_double2(e < A ? pm / pe : 0.0, pe);
        }
        wave_sync();
    };
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
        // createFCVOf (.fs:60-62), precomputed: lane e < E holds the count of symbol e
        const int my_comp = lane < E ? cpf : 0;
        const int na = __builtin_amdgcn_readlane(cpf, E);  // symbols outside the alphabet
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
            if (lane < CS) cpf = a.comp[(int64_t)(n + wstride) * CS + lane];
        }
        // zero tail: unrolled window reads past L see symbol 0 (a valid table row)
        for (int i = L + lane; i < L + WM + 76; i += 64) sseq[i] = 0;
        wave_sync();
        const int alpha_tot = L - na;
        STAMP(1);

        int newp = p;
        if (a.mode == 0) {
            // ---- hold-one-out background (integer exact) ----
            const int pp = p >= 0 ? p : 0;
            const int sj0 = sseq[pp + (lane < W ? lane : 0)];
            const int sj = (p >= 0 && lane < W) ? sj0 : 0xff;
            int my_segc = 0;
            for (int x = 0; x < A; ++x) {
                const int c = popc64(__ballot(sj == x));
                if (lane == x) my_segc = c;
            }
            const int seg_alpha = popc64(__ballot(sj < A));
            const int64_t bgc = lane < A ? T[lane] + (p >= 0 ? my_segc : my_comp) : 0;
            // Σ over the 49 slots: alphabet part + the sequence's own other symbols
            const int64_t tot = sumT + (p >= 0 ? seg_alpha : alpha_tot) + na;
            if (tot > 2147483647LL) {  // Checked Array.sum (.fs:117)
                if (lane == 0) raise_error(a, 3, gidx);
                goto seq_end;
            }
            // PCV (.fs:119); outside the alphabet the raw count (Q3)
            const double sbg = (double)tot + a.apc;
            const double pe = lane < A ? ((double)bgc + a.pc) / sbg : (double)my_comp;
            bool exact = !certified;
            float lq = 0.0f;
            if (!exact) lq = flog2(pe);
            if (lane < E) {
                pcv[lane] = pe;
                lpcv[lane] = lq;
            }
            // a zero PCV of an alphabet symbol makes PWM entries +inf / NaN: binary64 only
            exact = exact || __ballot(lane < A && !(pe > 0.0)) != 0;
            const float tG = wave_max_nonneg_f32(lane < E && fabsf(lq) < INFINITY ? fabsf(lq) : 0.0f);
            wave_sync();
            STAMP(2);
            FastView fv{};
            double epsS = 0.0, eabs_g = 0.0;
            if (!exact) {
                // ---- log table lt[e][j] = (log2 PPM' - log2 PCV, log2 PCV), j < W ----
                // (branch-free: clamped indices and selects keep every load unmasked)
                for (int c = lane; c < E * W; c += 64) {
                    const int e = (int)__umulhi((uint32_t)c, magicW), j = c - e * W;
                    const float le = lpcv[e];
                    const bool own = (p >= 0) & (sseq[pp + j] == e);
                    const float lp = (own ? lppmM : lppmG)[(e < A ? e : 0) * W + j];
                    // PWM 0 outside the alphabet
                    lt[e * LS + j] = make_float2(e < A ? lp - le : -INFINITY, le);
                }
                // ---- per-sequence error bounds ----
                // entries: |log2 PPM'| <= tppm, |log2 PCV| <= tG, |lt.x| <= tS; each
                // log carries kLog2AbsErr + |log| 2^-24, the subtraction |lt.x| 2^-24.
                // The pair table and the tree sum add <= levels * (W tS) 2^-24.
                const double tS = (double)tppm + (double)tG;
                constexpr double lv = (double)((H == 2) + tree_depth<NG>()) * 0x1.0p-24;
                const double eS = 2.0 * kLog2AbsErr + 2.0 * tS * 0x1.0p-24;
                const double eG = kLog2AbsErr + (double)tG * 0x1.0p-24;
                epsS = (double)W * (eS + tS * lv) + 1e-9;
                const double epsG = (double)W * (eG + (double)tG * lv) + 1e-9;
                if (!(epsS < 0.015625) || !(epsG < 0.015625)) exact = true;
                // |G~ - G| <= G~ ((2^epsG - 1) + kExp2RelErr)(1 + 3%) for epsG < 1/64
                eabs_g = 0.75 * epsG + 1.1 * kExp2RelErr;
                // binary32 thresholds of the cut-off band, widened by more than the
                // conversion's rounding (|x| 2^-24) so the band only grows
                const double ch = a.cutoff + epsS, cl = a.cutoff - epsS;
                fv.hiS = (float)(ch + fabs(ch) * 0x1.0p-22 + 1e-30);
                fv.loS = (float)(cl - fabs(cl) * 0x1.0p-22 - 1e-30);
                fv.lcodes = lcodes;
                fv.sseq = sseq;
                fv.ltab = ltab;
                fv.tab = tab;
                fv.cutoff = a.cutoff;
                wave_sync();
                if (H == 2) {
                    // pair tables gt[e0 + E*e1][g] = lt[e0][2g] + lt[e1][2g+1]; groups
                    // past the motif sum the zero padding columns
                    for (int c = lane; c < E2 * NG; c += 64) {
                        const int code = c / NG, g = c - code * NG;
                        const int e1 = (int)__umulhi((uint32_t)code, magicE);
                        const int e0 = code - e1 * E;
                        const float2 x0 = lt[e0 * LS + 2 * g], x1 = lt[e1 * LS + 2 * g + 1];
                        *(float2 *)(gt + (code * GS + g) * 8) = make_float2(x0.x + x1.x, x0.y + x1.y);
                    }
                    // pair codes, four per lane step: per byte s[i] + E*s[i+1] <= E*E-1 <
                    // 256, so the 32-bit multiply-add carries nothing across bytes
                    for (int i = lane * 4; i < L + WM + 68; i += 256) {
                        const uint32_t d0 = *(const uint32_t *)(sseq + i);
                        const uint32_t d1 = *(const uint32_t *)(sseq + i + 4);
                        *(uint32_t *)(cseq + i) =
                            d0 + (uint32_t)E * __builtin_amdgcn_alignbyte(d1, d0, 1);
                    }
                    wave_sync();
                }
            }
            STAMP(3);
            // ---- score every window (.fs:759-782); lane owns windows [k_lo, k_hi) ----
            // Only the lane sums are kept: the pick re-evaluates the one block it needs.
            const int R = (K + 63) >> 6;
            const int k_lo = lane * R;
            const int k_hi = min(K, k_lo + R);
            int kind = -1, pk = -1;  // kind 0 = background category, 1 = motif category
            double pw = 0.0;
            bool pw_log = false;
            bool tab_ready = false;
            if (!exact) {
                double sG = 0.0, sM = 0.0;
                bool flag = false;    // score outside the error model: exact rescan
                int lcat = 0;
                uint32_t unsure = 0;  // windows k_lo + r inside the cut-off band
                for (int k = k_lo; k < k_hi; ++k) {
                    double gw;
                    float fs;
                    const int cls = fast_window<WM, H>(fv, k, gw, fs, flag);
                    sG = sG + gw;
                    if (cls == kPass) {
                        sM = sM + (double)fs;
                        flag |= !(fs >= 0.0f);
                        ++lcat;
                    } else if (cls == kUnsure) {
                        const int r = k - k_lo;
                        if (r < 32)
                            unsure |= 1u << r;
                        else
                            flag = true;
                    }
                }
                STAMP(4);
                if (__ballot(unsure != 0) && !__ballot(flag)) {
                    build_tab(p);
                    tab_ready = true;
                    while (unsure) {
                        const int r = __builtin_ctz(unsure);
                        unsure &= unsure - 1;
                        const float m = resolve_window<WM>(fv, k_lo + r);
                        if (m != -INFINITY) {
                            sM = sM + (double)m;
                            flag |= !(m >= 0.0f) || !(m < INFINITY);
                            ++lcat;
                        }
                    }
                }
                const int npass = wave_sum_i32(lcat);
                STAMP(5);
                int why = 2;  // diagnostic counter of the rescan reason
                if (!__ballot(flag)) {
                    auto ev = [&](int k, double &g, double &m) {
                        float fs;
                        bool unused = false;
                        const int cls = fast_window<WM, H>(fv, k, g, fs, unused);
                        m = cls == kPass ? (double)fs
                                         : cls == kUnsure ? (double)resolve_window<WM>(fv, k)
                                                          : -INFINITY;
                    };
                    // |M~ - M| <= epsS above the band, |M~| 2^-24 for band windows
                    kind = certified_pick(ev, K, R, lane, u, sG, sM, lcat, npass, eabs_g, epsS,
                                          0x1.0p-23, pk);
                    why = kind < 0 ? 3 - kind : 0;
                }
                STAMP(6);
                if (kind >= 0) {
                    // the picked window's factors (lane j: column j), then the
                    // reference's left folds, uniform over the wavefront
                    // (columns j >= W of wfac hold 1.0 from the prologue)
                    if (lane < W) {
                        const int e = sseq[pk + lane];
                        const double pe_e = pcv[e];
                        const bool own = (p >= 0) & (sseq[pp + lane] == e);
                        const double pm = (own ? ppmM : ppmG)[(e < A ? e : 0) * W + lane];
                        wfac[lane] = make_double2(e < A ? pm / pe_e : 0.0, pe_e);
                    }
                    wave_sync();
                    double S = 1.0, G = 1.0;
#pragma unroll
                    for (int j = 0; j < WM; ++j) {
                        const double2 f = wfac[j];
                        S = S * f.x;
                        G = G * f.y;
                        if ((j & 3) == 3) __builtin_amdgcn_sched_barrier(0);  // 4 loads in flight
                    }
                    if (kind == 0) {
                        pw = G;
                    } else if (S > a.thr_hi) {
                        pw = S;  // certainly log2 S > cutOff: log2 taken at the batch end
                        pw_log = true;
                    } else {
                        pw = log(S * 1.0) / kLn2;
                        if (!(pw > a.cutoff)) {  // cannot happen when the bound holds
                            kind = -1;
                            why = 3;
                        }
                    }
                }
                if (kind < 0) {
                    exact = true;
                    if (lane == 0) {
                        atomicAdd(&a.fallbacks[0], 1ull);
                        atomicAdd(&a.fallbacks[why], 1ull);
                    }
                }
            }
            STAMP(7);
            if (exact) {
                // ---- exact scan: binary64 folds for every window ----
                if (!tab_ready) build_tab(p);
                auto ev = [&](int k, double &g, double &m) {
                    exact_eval<WM>(sseq, tab, a.thr_lo, a.cutoff, k, g, m);
                };
                double sG = 0.0, sM = 0.0;
                bool neg = false;
                int lcat = 0;
                for (int k = k_lo; k < k_hi; ++k) {
                    double G, M;
                    ev(k, G, M);
                    sG = sG + G;
                    neg |= !(G >= 0.0);
                    if (M != -INFINITY) {
                        sM = sM + M;
                        neg |= !(M >= 0.0);
                        ++lcat;
                    }
                }
                const int npass = wave_sum_i32(lcat);
                kind = -1;
                pw_log = false;
                if (!__ballot(neg))
                    kind = certified_pick(ev, K, R, lane, u, sG, sM, lcat, npass, 0.0, 0.0, 0.0, pk);
                if (kind < 0) {
                    // exact sequential restatement of .fs:747-754 on one lane, the
                    // windows re-evaluated in the reference's order: two summing
                    // passes (backgrounds, then motif scores) and two walking passes
                    if (lane == 0) {
                        atomicAdd(&a.fallbacks[1], 1ull);
                        double s = 0.0, acc = 0.0;
                        int rk = -1, rp = -1;
                        for (int pass = 0; pass < 4 && rk < 0; ++pass) {
                            for (int k = 0; k < K && rk < 0; ++k) {
                                double G, M;
                                ev(k, G, M);
                                const double x = (pass & 1) ? M : G;
                                if ((pass & 1) && M == -INFINITY) continue;
                                if (pass < 2) {
                                    s = s + x;
                                } else {
                                    const double w = x / s;
                                    if (acc <= u && u <= acc + w) {
                                        rk = pass - 2;
                                        rp = k;
                                    }
                                    acc = acc + w;
                                }
                            }
                        }
                        misc[0] = rk;
                        misc[1] = rp;
                    }
                    wave_sync();
                    kind = misc[0];
                    pk = misc[1];
                }
                if (kind >= 0) {
                    double G, M;
                    ev(pk, G, M);
                    pw = kind == 0 ? G : M;
                }
            }
            if (kind < 0) {  // every category missed: the reference's list index overruns
                if (lane == 0) raise_error(a, 2, gidx);
                goto seq_end;
            }
            newp = kind == 0 ? -1 : pk;
            if (lane == jb) {  // results wait in lane registers, stored 64 at a time
                r_pos = newp;
                r_pw = pw;
                r_log = pw_log;
            }
        }
        STAMP(8);
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
        STAMP(9);
    seq_end:
        if (jb == 63 || it + 1 == cnt) {
            if (a.mode == 0 && lane <= jb) {
                // log2 of the batch's motif picks (.fs:737), one lane per sequence
                if (r_log) r_pw = log(r_pw * 1.0) / kLn2;
                const int nb = n0 + (it - jb + lane) * wstride;
                a.pos_out[nb] = r_pos;
                a.pwms_out[nb] = r_pw;
            }
            r_log = false;
            if (jb == 63 && it + 1 < cnt) load_batch(it + 1);
        }
        STAMP(10);
    }
    (void)nseq_done;
    // ---- flush: sum the 4 wavefronts' aggregates, one atomic per cell ----
    __syncthreads();
    STAMP(11);
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

// Static per-sequence symbol histograms (createFCVOf, .fs:60-62): one wavefront
// per sequence, LDS counters by encoded symbol, plus the non-alphabet total.
__global__ void __launch_bounds__(256) gs_composition_kernel(const uint8_t *seq, const int64_t *doff,
                                                             const int32_t *len, int32_t n_local,
                                                             int32_t A, int32_t E, int32_t *comp) {
    __shared__ int32_t cnt[4][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int CS = E + 1;
    for (int n = blockIdx.x * 4 + w; n < n_local; n += gridDim.x * 4) {
        cnt[w][lane] = 0;
        wave_sync();
        const uint8_t *s = seq + doff[n];
        const int L = len[n];
        for (int i = lane; i < L; i += 64) atomicAdd(&cnt[w][s[i]], 1);
        wave_sync();
        const int v = lane < E ? cnt[w][lane] : 0;
        int na = (lane >= A && lane < E) ? v : 0;
        for (int o = 32; o > 0; o >>= 1) na += __shfl_xor(na, o);
        if (lane < E) comp[(int64_t)n * CS + lane] = v;
        if (lane == E) comp[(int64_t)n * CS + E] = na;
        wave_sync();
    }
}

// Measures the binary32 transcendental errors the certified scan budgets for
// (kLog2AbsErr, kExp2RelErr): flog2 on 2^24 points of [0.5, 1) against the
// binary64 log, and v_exp_f32 on every multiple of 2^-24 in [0, 1).
__global__ void __launch_bounds__(256) gs_fastmath_kernel(unsigned int *out) {
    const int n = 1 << 24;
    float el = 0.0f, ee = 0.0f;
    for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
        const double v = 0.5 + ((double)i + 0.37) * 0x1.0p-25;
        el = fmaxf(el, (float)fabs((double)flog2(v) - log(v) / kLn2));
        const float x = (float)i * 0x1.0p-24f;
        const double ex = exp2((double)x);
        ee = fmaxf(ee, (float)(fabs((double)__builtin_amdgcn_exp2f(x) - ex) / ex));
    }
    el = wave_max_nonneg_f32(el);
    ee = wave_max_nonneg_f32(ee);
    if ((threadIdx.x & 63) == 0) {
        atomicMax(&out[0], __float_as_uint(el));
        atomicMax(&out[1], __float_as_uint(ee));
    }
}

// Host-side launch helpers (the C-ABI translation unit stays free of kernel code).
#define GS_FOR_EACH_WM(X) X(4) X(8) X(12) X(16) X(20) X(24) X(28) X(32) X(40) X(48) X(56) X(64)

static const void *sweep_kernel_ptr(int wm, int h) {
    switch (wm) {
#define GS_CASE(N) \
    case N:        \
        return h == 2 ? (const void *)&gs_sweep_kernel<N, 2> : (const void *)&gs_sweep_kernel<N, 1>;
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

hipError_t gs_sweep_occupancy(int *blocks_per_cu, int W, int E, size_t lds_bytes) {
    const void *k = sweep_kernel_ptr(gs_sweep_wm(W), scan_group(E));
    if (!k) return hipErrorInvalidValue;
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, k, 256, lds_bytes);
}

hipError_t gs_sweep_launch(const SweepArgs &a, int grid, size_t lds_bytes, hipStream_t stream) {
    const void *k = sweep_kernel_ptr(gs_sweep_wm(a.W), scan_group(a.E));
    if (!k) return hipErrorInvalidValue;
    SweepArgs args = a;
    void *params[] = {&args};
    return hipLaunchKernel(k, dim3(grid), dim3(256), params, lds_bytes, stream);
}

hipError_t gs_fastmath_launch(unsigned int *out, hipStream_t stream) {
    hipLaunchKernelGGL(gs_fastmath_kernel, dim3(1024), dim3(256), 0, stream, out);
    return hipGetLastError();
}

hipError_t gs_composition_launch(const uint8_t *seq, const int64_t *doff, const int32_t *len,
                                 int32_t n_local, int32_t A, int32_t E, int32_t *comp, int n_cu,
                                 hipStream_t stream) {
    if (n_local <= 0) return hipSuccess;
    const int grid = std::max(1, std::min((n_local + 3) / 4, n_cu * 8));
    hipLaunchKernelGGL(gs_composition_kernel, dim3(grid), dim3(256), 0, stream, seq, doff, len,
                       n_local, A, E, comp);
    return hipGetLastError();
}
