// gs_sweep.hip — fused Gibbs sweep kernel for gfx950 (MI355X).
//
// A workgroup is 4 independent 64-lane wavefronts; each wavefront is split into
// G = 64/GL lane groups of GL = 16, 32 or 64 lanes, and each group scores its
// own sequence: short sequences share a wavefront so that every wave
// instruction of the per-sequence work serves several sequences.  Per sequence
// n (MotifSampler.findBestMotifIndicesByWithStartPositions, .fs:935-970,
// motifAmount = 1):
//   1. stage the encoded sequence into the group's LDS slice (16-byte loads,
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
//      log2 sum under a rigorous per-sequence error bound; the cut-off test
//      (.fs:735-738) is decided from the bound;
//   5. roulette pick (.fs:746-754): a lane-level then window-level segmented
//      prefix sum of the approximate weights; the pick is accepted only when u
//      is farther than the combined approximation + rounding bound from every
//      CDF boundary that decides it.  The picked window's weight is then folded
//      exactly (binary64, the reference's order); its log2 (.fs:737) is taken
//      once per 64 sequences, one lane each.  A sequence whose cut-off test or
//      pick the bound cannot settle is rescanned by the whole wavefront in
//      binary64 (the reference's folds for every window) and its pick certified
//      against rounding alone, or — still undecided — one lane redoes the
//      reference's sequential sums exactly;
//   6. the picked segment is added to per-wavefront aggregates of the new
//      snapshot (LDS atomics), flushed to XCD-replicated global accumulators
//      once per workgroup: the next sweep's count matrix and background totals.
//
// Compiled with -ffp-contract=off: no FMA contraction.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>

#include "gs_bgregime.h"
#include "gs_common.h"
#include "gs_fold.h"
#include "gs_pick.h"
#include "gs_stamps.h"
#include "gs_wave.h"

using namespace gs;

namespace {

typedef float f2 __attribute__((ext_vector_type(2)));

// A kernel argument read where it is used: a scalar load from the kernarg segment
// (volatile, so it is not hoisted to the kernel entry).  The arguments of rare paths
// and of the epilogue are read so, which keeps them out of the SGPRs of the
// per-sequence loop (the general kernel spilled ~120 SGPRs to VGPR lanes).
// The pointer is laundered through an empty asm at each use so the load cannot be
// hoisted; it stays in the constant address space, so the load is an s_load.
typedef const __attribute__((address_space(4))) SweepArgs KSweepArgs;
__device__ __forceinline__ KSweepArgs *kargs() {
    uint64_t p = (uint64_t)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(p));
    return (KSweepArgs *)p;
}
#define KA(f) (kargs()->f)

// log2 of a binary64 value as the certified scan's tables take it, out of line: its
// polynomial constants stay out of the per-sequence loop's registers (the rare
// sequences without a motif on the four-symbol path)
__device__ __noinline__ double log2_ool(double x) { return log2(x); }

__device__ __forceinline__ void raise_error(const SweepArgs &a, int code, int64_t gidx) {
    (void)a;
    atomicCAS(KA(err_code), 0, code);
    atomicMin(KA(err_index), (unsigned long long)gidx);
}

// Pairwise (tree) sum of the NG group terms: depth ceil(log2 NG), so each term's
// rounding error is bounded by depth * (sum of |terms|) * 2^-24.
template <int NG, class T>
__device__ __forceinline__ T tree_sum(T *v) {
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

// Table entry of the certified scan: the motif term log2 PWM' of one column (or the
// sum of two, H = 2) in the sequence's fixed point (a non-negative integer: the term
// less its column's clamp floor, in units of 2^-sc), and the background term log2
// PCV in binary32.
__device__ __forceinline__ uint2 tab_entry(const unsigned char *tab, uint32_t row_bytes, int g) {
    return *(const uint2 *)(tab + row_bytes + g * 8);
}

// Pair-table entry (code x, column pair g).  Code-major rows of RS bytes, or (GM, the
// four-symbol path's 16 codes) group-major rows of 16 entries = 128 B: the 16 lanes of
// a group read one row, i.e. one half of the 64 banks, and the odd group of each 32-lane
// half of the wavefront has its table 128 B further mod 256 (gs_engine.cpp carve), so
// the two groups that share a ds_read_b64 lane group never share a bank.
// (GM: the staged codes are the codes x 8, i.e. already the row offset in bytes: one
// v_add_u32_sdwa per address)
template <bool GM, int RS>
__device__ __forceinline__ uint2 pair_entry(const unsigned char *tab, uint32_t x, int g) {
    return GM ? *(const uint2 *)(tab + x + g * 128) : tab_entry(tab, x * RS, g);
}

// codes x 8 of a staged chunk (codes < 16: no carry into the next byte)
__device__ __forceinline__ uint4 codes_x8(uint4 v) {
    return make_uint4(v.x << 3, v.y << 3, v.z << 3, v.w << 3);
}

// (log2 S~_k, log2 G~_k) of window k: the motif part an exact integer sum (the
// sequence's fixed point), the background part a binary32 tree sum.  H = 2: codes[i]
// = s[i] + E*s[i+1] and ltab = [E*E][gt_stride(WM)] pair sums; H = 1: codes =
// symbols and ltab = [E][lt_stride(WM)].  Code-major with odd strides: the group
// offset g*8 is a ds_read immediate, different codes land in different banks.
// Groups past the motif hold (0, 0).
template <int WM, int H, bool GM = false>
__device__ __forceinline__ void window_logs(const uint8_t *codes, const unsigned char *ltab, int k,
                                            uint32_t &ls, float &lg) {
    constexpr int ND = WM / 4 + 1, NG = WM / H;
    constexpr int RS = (H == 2 ? gt_stride(WM) : lt_stride(WM)) * 8;
    const int kb = k & ~3, off = k & 3;
    uint32_t d[ND];
#pragma unroll
    for (int i = 0; i < ND; ++i) d[i] = *(const uint32_t *)(codes + kb + 4 * i);
    uint32_t vs[NG];
    float vg[NG];
#pragma unroll
    for (int i = 0; i < WM / 4; ++i) {
        const uint32_t x = __builtin_amdgcn_alignbyte(d[i + 1], d[i], off);
#pragma unroll
        for (int t = 0; t < 4; t += H) {
            const int g = (4 * i + t) / H;
            const uint2 v = pair_entry<GM, RS>(ltab, (x >> (8 * t)) & 0xffu, g);
            vs[g] = v.x;
            vg[g] = __uint_as_float(v.y);
        }
    }
    ls = 0u;
#pragma unroll
    for (int g = 0; g < NG; ++g) ls += vs[g];
    lg = tree_sum<NG>(vg);
}

// The same for two windows of one lane: their background sums share packed
// binary32 adds (.x: k0, .y: k1), their motif sums three-operand integer adds.
template <int WM, int H, bool GM = false>
__device__ __forceinline__ void window_logs2(const uint8_t *codes, const unsigned char *ltab, int k0,
                                             int k1, uint32_t &s0, uint32_t &s1, f2 &lg) {
    constexpr int ND = WM / 4 + 1, NG = WM / H;
    constexpr int RS = (H == 2 ? gt_stride(WM) : lt_stride(WM)) * 8;
    const int kb0 = k0 & ~3, off0 = k0 & 3, kb1 = k1 & ~3, off1 = k1 & 3;
    uint32_t d0[ND], d1[ND];
#pragma unroll
    for (int i = 0; i < ND; ++i) {
        d0[i] = *(const uint32_t *)(codes + kb0 + 4 * i);
        d1[i] = *(const uint32_t *)(codes + kb1 + 4 * i);
    }
    uint32_t v0[NG], v1[NG];
    f2 vg[NG];
#pragma unroll
    for (int i = 0; i < WM / 4; ++i) {
        const uint32_t x0 = __builtin_amdgcn_alignbyte(d0[i + 1], d0[i], off0);
        const uint32_t x1 = __builtin_amdgcn_alignbyte(d1[i + 1], d1[i], off1);
#pragma unroll
        for (int t = 0; t < 4; t += H) {
            const int g = (4 * i + t) / H;
            const uint2 a0 = pair_entry<GM, RS>(ltab, (x0 >> (8 * t)) & 0xffu, g);
            const uint2 a1 = pair_entry<GM, RS>(ltab, (x1 >> (8 * t)) & 0xffu, g);
            v0[g] = a0.x;
            v1[g] = a1.x;
            vg[g] = f2{__uint_as_float(a0.y), __uint_as_float(a1.y)};
        }
    }
    s0 = 0u;
    s1 = 0u;
#pragma unroll
    for (int g = 0; g < NG; ++g) {
        s0 += v0[g];
        s1 += v1[g];
    }
    lg = tree_sum<NG>(vg);
}

// The same for four consecutive windows k .. k+3 of one lane, k a multiple of 4 (H = 2):
// the lane's codes are read once as dwords and every table address is a compile-time
// byte of them, so all 4 * WM/2 table reads are in flight together.  Sums as
// window_logs (the pick's re-evaluation gives the same values).
template <int WM>
struct QuadCodes {
    static constexpr int ND = (WM + 1) / 4 + 1;
    uint32_t d[ND];
};
template <int WM>
__device__ __forceinline__ QuadCodes<WM> quad_codes(const uint8_t *codes, int k) {
    QuadCodes<WM> q;
#pragma unroll
    for (int i = 0; i < QuadCodes<WM>::ND; ++i) q.d[i] = *(const uint32_t *)(codes + k + 4 * i);
    return q;
}
// windows k + O and k + O + 1 (O = 0 or 2) of the quad
template <int WM, int O, bool GM>
__device__ __forceinline__ void window_logs_q(const QuadCodes<WM> &q, const unsigned char *ltab,
                                              uint32_t &s0, uint32_t &s1, f2 &lg) {
    constexpr int NG = WM / 2;
    constexpr int RS = gt_stride(WM) * 8;
    uint32_t v0[NG], v1[NG];
    f2 vg[NG];
#pragma unroll
    for (int g = 0; g < NG; ++g) {
        const int b0 = O + 2 * g, b1 = O + 1 + 2 * g;
        const uint32_t x0 = (q.d[b0 >> 2] >> (8 * (b0 & 3))) & 0xffu;
        const uint32_t x1 = (q.d[b1 >> 2] >> (8 * (b1 & 3))) & 0xffu;
        const uint2 a0 = pair_entry<GM, RS>(ltab, x0, g);
        const uint2 a1 = pair_entry<GM, RS>(ltab, x1, g);
        v0[g] = a0.x;
        v1[g] = a1.x;
        vg[g] = f2{__uint_as_float(a0.y), __uint_as_float(a1.y)};
    }
    s0 = 0u;
    s1 = 0u;
#pragma unroll
    for (int g = 0; g < NG; ++g) {
        s0 += v0[g];
        s1 += v1[g];
    }
    lg = tree_sum<NG>(vg);
}

// Certified-scan view of one group's sequence (per lane: the lane's group).  A
// window's motif log is log2 S~ = ls * unit + base (ls the integer sum); the cut-off
// band in those integers is [loU, hiU].
struct FastView {
    const uint8_t *lcodes;
    const unsigned char *ltab;
    uint32_t hiU, loU;
    double unit, base;
};

enum { kFail = 0, kPass = 1, kUnsure = 2 };

__device__ __forceinline__ int classify(const FastView &c, uint32_t ls) {
    return ls > c.hiU ? kPass : (ls < c.loU ? kFail : kUnsure);
}

// Alphabets of more than 16 symbols (H = 1), round 6: a window's log2 S = log2 M - log2 G
// with log2 M = sum_j log2 PPM'[s_{k+j}][j] and log2 G = sum_j log2 PCV[s_{k+j}].  The
// motif part reads the group's table of binary32 log2 PPM' (4-byte entries, code-major
// rows of mt_stride(WM), the own segment's count-minus-one cells patched in for the
// sequence: PCV-free, so the table is the workgroup's, patched in W cells instead of
// rebuilt in E x W), a binary32 tree sum; the background part is the difference of two
// int32 prefix sums of the positions' fixed-point log2 PCV (exact, in any order: the
// pick's re-evaluation gives the scan's values bit for bit).  DESIGN.md §5.2.
template <int WM>
__device__ __forceinline__ float window_m1(const uint8_t *codes, const unsigned char *mt, int k) {
    constexpr int ND = WM / 4 + 1;
    constexpr int RS = mt_stride(WM) * 4;
    const int kb = k & ~3, off = k & 3;
    uint32_t d[ND];
#pragma unroll
    for (int i = 0; i < ND; ++i) d[i] = *(const uint32_t *)(codes + kb + 4 * i);
    float v[WM];
#pragma unroll
    for (int i = 0; i < WM / 4; ++i) {
        const uint32_t x = __builtin_amdgcn_alignbyte(d[i + 1], d[i], off);
#pragma unroll
        for (int t = 0; t < 4; ++t) v[4 * i + t] = *(const float *)(mt + ((x >> (8 * t)) & 0xffu) * RS + (4 * i + t) * 4);
    }
    return tree_sum<WM>(v);
}

// 2^x for a binary64 |x| < 1000: v_exp_f32 on the fractional part (rounded to binary32:
// 2^-25 absolute, 0.35 ulp of the result), the exact power of two by v_ldexp_f64
__device__ __forceinline__ double fexp2_d(double x) {
    const double fl = floor(x);
    return ldexp((double)__builtin_amdgcn_exp2f((float)(x - fl)), (int)fl);
}

struct FastViewF {
    const uint8_t *lcodes;
    const unsigned char *mt;  // the group's motif table (log2 PPM', own cells patched)
    const int32_t *pfx;       // prefix sums of the positions' log2 PCV, units 2^-sP
    double unitP;             // 2^-sP
    int W;
    double hiS, loS;          // the cut-off band [loS, hiS]
};

// window k: (log2 S~ in fs, G~ in gw), its cut-off class; flag: outside the model's range
template <int WM>
__device__ __forceinline__ int fast_window_f(const FastViewF &c, int k, double &gw, double &fs,
                                             bool &flag) {
    const float fm = window_m1<WM>(c.lcodes, c.mt, k);
    const int32_t gi = (int32_t)((uint32_t)c.pfx[k + c.W] - (uint32_t)c.pfx[k]);
    const double lg = (double)gi * c.unitP;
    fs = (double)fm - lg;
    flag |= !(lg > -1000.0 && lg < 1000.0);
    gw = fexp2_d(lg);
    return (fs > c.hiS && fs < 1000.0) ? kPass : (fs < c.loS ? kFail : kUnsure);
}

}  // namespace

// Register budget: GS_WAVES_PER_EU (build flag) asks the allocator for that many
// resident waves per SIMD (512 / n VGPRs each).
#ifdef GS_WAVES_PER_EU
#define GS_SWEEP_ATTR __launch_bounds__(64 * sweep_waves(H)) __attribute__((amdgpu_waves_per_eu(GS_WAVES_PER_EU, 8)))
#else
// three resident waves per SIMD for the pair-table scan (config 2: 2,500 wavefronts
// on 1,024 SIMDs are all resident at once)
#define GS_SWEEP_ATTR __launch_bounds__(64 * sweep_waves(H)) __attribute__((amdgpu_waves_per_eu(H == 2 ? 3 : 1, 8)))
#endif

struct SweepResult {  // per batch slot, in LDS until the batch's results are stored
    int32_t pos, log;  // log != 0: pw holds S of a motif pick, log2 still to take
    double pw;
};

// Is this the last workgroup of the launch to get here?  Two-level done counter
// (`done`: 128-byte lines, [0] the top, [32 (1 + g)] group g = blockIdx % kRepl's), so
// that no address takes more than gridDim / 8 + 8 of the serialised same-address
// atomics; both levels reset themselves for the next launch.  Every workgroup calls it
// once, at its end, after its flush; the last one returns with an acquire, so it sees
// every other workgroup's flush (gs_common.h GS_DONE_FENCE: no L2 writeback).  (s_last: an LDS word no longer read by then, outside
// the workgroup tables the last workgroup rebuilds.)
__device__ __forceinline__ bool wg_is_last(unsigned int *done, int *s_last, int tid) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
        GS_DONE_FENCE(__ATOMIC_RELEASE);
        const int grp = blockIdx.x % kRepl;
        const unsigned int ng = (gridDim.x - grp + kRepl - 1) / kRepl;  // workgroups of the group
        const unsigned int ngroups = min(gridDim.x, (unsigned int)kRepl);
        bool last = false;
        if (atomicAdd(&done[32 * (1 + grp)], 1u) == ng - 1) {
            atomicExch(&done[32 * (1 + grp)], 0u);
            GS_DONE_FENCE(__ATOMIC_ACQ_REL);
            last = atomicAdd(&done[0], 1u) == ngroups - 1;
            if (last) atomicExch(&done[0], 0u);
        }
        *s_last = last;
    }
    __syncthreads();
    const bool last = *s_last != 0;
    if (last) GS_DONE_FENCE(__ATOMIC_ACQUIRE);
    return last;
}

// The workgroup tables of a snapshot on the four-symbol path (gs_common.h ek4_layout,
// [0, o_wave) of the workgroup's LDS), built from the kRepl aggregate replicas `rep`:
// the counts C and backgrounds T summed, PPM = (C + pc)/den and the own-segment cells
// (C - 1 + pc)/den (normalizePPM .fs:257-260) with their binary64 log2, and the
// hold-one-out PCV logs of every motif-bearing sequence, log2(T[a] + s + pc) for the
// segment's count s = 0..W of symbol a, then log2(sum T + W + A pc)
// (createNormalizedPCVOfFCV .fs:119).  The same operations as every sweep used to do
// in its prologue, now once a sweep: built by the previous sweep's last workgroup (the
// handoff) or by gs_sweep_tables_kernel, and copied by every workgroup.  `coherent`:
// the replicas were written by other workgroups of the running launch (read at agent
// scope, past the other XCDs' L2s).
template <int WM>
__device__ void ek4_build_tables(unsigned char *lds, const int64_t *rep, int stride, double pc,
                                 double den, double apc, bool coherent, int tid, int nthr) {
    constexpr Ek4Layout L4 = ek4_layout(WM, 16);
    constexpr int W = WM, AW = 4 * W, cells = AW + 4, nT = 4 * (W + 1);
    int32_t *cg = (int32_t *)(lds + L4.o_cg);
    int64_t *T = (int64_t *)(lds + L4.o_T);
    double *ppmG = (double *)(lds + L4.o_ppmG), *ppmM = (double *)(lds + L4.o_ppmM);
    double *lppmG = (double *)(lds + L4.o_lppmG), *lppmM = lppmG + AW;
    double *lTab = (double *)(lds + L4.o_lT);
    // (the alignment padding and the unused bmax slots: the image is copied whole)
    for (int i = tid; i < L4.o_wave / 4; i += nthr)
        if (i >= L4.o_bmax / 4 && i < L4.o_lT / 4) ((uint32_t *)lds)[i] = 0u;
    for (int c = tid; c < cells; c += nthr) {
        int64_t v = 0;
        if (rep) {
#pragma unroll
            for (int r = 0; r < kRepl; ++r) {
                const int64_t *p = rep + (int64_t)r * stride + c;
                // (coherent: an atomic, performed where the flushes were)
                v += coherent ? (int64_t)atomicAdd((unsigned long long *)p, 0ull) : *p;
            }
        }
        if (c < AW)
            cg[c] = (int32_t)v;
        else
            T[c - AW] = v;
    }
    __syncthreads();
    // sum T: exact (integers below 2^53, any order)
    const double q = (double)T[0] + (double)T[1] + (double)T[2] + (double)T[3];
    for (int c = tid; c < AW + nT + 1; c += nthr) {
        if (c < AW) {
            const int32_t cc = cg[c];
            const double g = ((double)cc + pc) / den;
            const double m = ((double)(cc - 1) + pc) / den;
            ppmG[c] = g;
            ppmM[c] = m;
            // binary64 log2 (< 1e-12 absolute error); a count-minus-one cell of a zero
            // count is negative and never used (own-segment cells: C >= 1)
            lppmG[c] = log2(g);
            lppmM[c] = m > 0.0 ? log2(m) : -INFINITY;
        } else {
            const int t = c - AW;
            if (t < nT) {
                const int e = t / (W + 1);
                lTab[t] = log2((double)(T[e] + (t - e * (W + 1))) + pc);
            } else {
                lTab[t] = log2((q + (double)W) + apc);
            }
        }
    }
    __syncthreads();
}

template <int WM>
__device__ __forceinline__ void ek4_store_tables(const unsigned char *lds, unsigned char *out, int tid,
                                                 int nthr) {
    constexpr int nv = ek4_layout(WM, 16).o_wave / 16;
    for (int i = tid; i < nv; i += nthr) ((uint4 *)out)[i] = ((const uint4 *)lds)[i];
}

// The sweep's end, every workgroup once, after its flush (the error exit too): with a
// done counter the last workgroup builds the next sweep's workgroup tables from the
// replicas it accumulated (EK = 4, ftab_out) and/or folds agg_out's kRepl replicas into
// replica 0 (the others re-zeroed), so that one (A W + A)-cell vector is all a
// multi-GPU sweep all-reduces.
// (s_last: the first word of the wavefront slices, dead after the flush)
template <int WM, int EK>
__device__ __forceinline__ void sweep_epilogue(const SweepArgs &a, unsigned char *lds, int *s_last,
                                               int tid) {
    unsigned int *const done = KA(done);
    if (!done) return;
    if (!wg_is_last(done, s_last, tid)) return;
    int64_t *const agg_out = KA(agg_out);
#ifdef GS_FTAB
    if constexpr (EK == 4) {
        unsigned char *const ftab_out = KA(ftab_out);
        if (ftab_out) {
            ek4_build_tables<WM>(lds, agg_out, a.stride, a.pc, a.den, a.apc, true, tid, blockDim.x);
            ek4_store_tables<WM>(lds, ftab_out, tid, blockDim.x);
        }
    }
#endif
    if (!KA(fold)) return;
    for (int c = tid; c < a.cells; c += blockDim.x) {
        int64_t v = 0;
#pragma unroll
        for (int r = 1; r < kRepl; ++r)
            v += (int64_t)atomicExch((unsigned long long *)&agg_out[(int64_t)r * a.stride + c], 0ull);
        if (v != 0) atomicAdd((unsigned long long *)&agg_out[c], (unsigned long long)v);
    }
}

// One group's binary64 rescan for H = 1 (more than 16 symbols), out of line: the
// cold path's registers (its exact table build, the wavefront-wide certified pick, the
// serial replay, the binary64 logs) stay out of the sweep loop's, which runs 12
// wavefronts a workgroup at <= 170 VGPRs (the inline form spilled).  The group gg's
// sequence (its symbols in the group's slice), length Lx, snapshot position px and
// uniform ux; the reference's folds for every window (.fs:759-777), the pick certified
// against rounding alone, else the reference's sequential sums (.fs:747-754) on one
// lane.  Returns the category kind (0 background, 1 motif, < 0 none), the window and
// its exact weight, uniform over the wavefront.  The kernel arguments through the
// kernarg segment (ka): the by-value struct is not copied.
struct RxOut {
    int kk, pkk;
    double xw;
};
template <int WM>
__device__ __attribute__((noinline)) RxOut rescan_group_h1(KSweepArgs *ka_in, int gg, int Lx, int px, double ux) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    // (the segment pointer made wave-uniform: its fields are scalar loads)
    const uint64_t pv = (uint64_t)ka_in;
    KSweepArgs *ka = (KSweepArgs *)(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(pv >> 32)) << 32) |
                                    (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)pv));
    constexpr int WS = tab_stride(WM);
    const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int A = ka->A, E = ka->E, W = ka->W;
    unsigned char *const wl = lds + ka->o_wave + wid * ka->wave_bytes;
    const unsigned char *gx = wl + ka->w_group + gg * ka->group_bytes;
    const uint8_t *sx = (const uint8_t *)(gx + ka->g_seq);
    const double *pcvx = (const double *)(gx + ka->g_pcv);
    unsigned char *tab = wl + ka->w_tab;
    const double *ppmG = (const double *)(lds + ka->o_ppmG), *ppmM = (const double *)(lds + ka->o_ppmM);
    int32_t *misc = (int32_t *)(wl + ka->w_misc);
    const uint32_t magicW = 0xffffffffu / (uint32_t)W + 1u;
    const double cutoff = ka->cutoff;
    const int Kx = Lx - W + 1;
    const int ppx = px >= 0 ? px : 0;
    for (int c = lane; c < E * W; c += 64) {
        const int e = magic_div((uint32_t)c, (uint32_t)W, magicW), j = c - e * W;
        const double pe_e = pcvx[e];
        const bool own = (px >= 0) & (sx[ppx + j] == e);
        const double pm = (own ? ppmM : ppmG)[(e < A ? e : 0) * W + j];
        *(double2 *)(tab + (e * WS + j) * 16) = make_double2(e < A ? pm / pe_e : 0.0, pe_e);
    }
    if (ka->w_tab == ka->w_lt)  // (the padding columns: the motif tables were there)
        for (int c = lane; c < E * WS; c += 64)
            if (c % WS >= W) *(double2 *)(tab + c * 16) = make_double2(1.0, 1.0);
    wave_sync();
    const double thr_lo = ka->thr_lo;
    auto evx = [&](int k, double &g, double &m) { exact_eval<WM, true>(sx, tab, thr_lo, cutoff, k, g, m); };
    const int Rx = (Kx + 63) >> 6;
    const int kx_lo = lane * Rx, kx_hi = min(Kx, kx_lo + Rx);
    double xG = 0.0, xM = 0.0;
    bool neg = false;
    int xcat = 0;
    for (int k = kx_lo; k < kx_hi; ++k) {
        double g, m;
        evx(k, g, m);
        xG = xG + g;
        neg |= !(g >= 0.0);
        if (m != -INFINITY) {
            xM = xM + m;
            neg |= !(m >= 0.0);
            ++xcat;
        }
    }
    const int xpass = wave_sum_i32(xcat);
    int pkk = -1;
    const bool ok = __ballot(neg) == 0;
    int kk = certified_pick<64>(evx, ok, Kx, Rx, lane, ux, xG, xM, xcat, xpass, 0.0, 0.0, 0.0, pkk);
    if (kk < 0) {
        // exact sequential restatement of .fs:747-754 on one lane, the windows
        // re-evaluated in the reference's order: two summing passes (backgrounds, then
        // motif scores), two walking passes
        if (lane == 0) {
            atomicAdd(&(ka->fallbacks + (blockIdx.x % kRepl) * kStatStride)[1], 1ull);
            double sacc = 0.0, acc = 0.0;
            int rk = -1, rp = -1;
            for (int pass = 0; pass < 4 && rk < 0; ++pass) {
                for (int k = 0; k < Kx && rk < 0; ++k) {
                    double g, m;
                    evx(k, g, m);
                    const double x = (pass & 1) ? m : g;
                    if ((pass & 1) && m == -INFINITY) continue;
                    if (pass < 2) {
                        sacc = sacc + x;
                    } else {
                        const double w = x / sacc;
                        if (acc <= ux && ux <= acc + w) {
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
        kk = misc[0];
        pkk = misc[1];
    }
    double xw = 0.0;
    if (kk >= 0) {
        double g, m;
        evx(pkk, g, m);
        xw = kk == 0 ? g : m;
    }
    wave_sync();  // the shared exact table is rebuilt for the next group
    return RxOut{kk, pkk, xw};
}

// EK = 4: the alphabet is exactly four symbols and the data holds no other (DNA):
// E is a compile-time constant, a symbol is its pair code's low two bits, and the
// per-sequence table build runs with static trip counts (every LDS read of a lane
// issued before the first is consumed).  EK = 0: E from the arguments.
template <int WM, int H, int GL, int EK>
__global__ void GS_SWEEP_ATTR gs_sweep_kernel(SweepArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    constexpr int G = 64 / GL;
    // sweep_waves(H) wavefronts, fewer when the LDS of that many does not fit
    const int kWavesPerBlock = blockDim.x >> 6, kSweepThreads = blockDim.x;
    constexpr int NG = WM / H, WS = tab_stride(WM), LS = lt_stride(WM), GS = gt_stride(WM);
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar loads
    const int gi = lane / GL, li = lane & (GL - 1), gbase = lane & ~(GL - 1);

    static_assert(EK == 0 || (EK == 4 && H == 2), "EK = 4 is the pair-table DNA path");
    // EK = 4 kernels run for W == WM only (gs_sweep_ek): the motif width is static too
    const int A = EK ? EK : a.A, E = EK ? EK : a.E, W = EK ? WM : a.W, AW = A * W, CS = E + 1,
              E2 = E * E;
    // LDS offsets: compile-time constants on the four-symbol path (gs_common.h
    // ek4_layout, the host carve's), else the host carve's arguments
    constexpr Ek4Layout L4 = ek4_layout(WM, GL);
    const int o_cg = EK ? L4.o_cg : a.o_cg, o_T = EK ? L4.o_T : a.o_T;
    const int o_ppmG = EK ? L4.o_ppmG : a.o_ppmG, o_ppmM = EK ? L4.o_ppmM : a.o_ppmM;
    const int o_lppmG = EK ? L4.o_lppmG : a.o_lppmG, o_bmax = EK ? L4.o_bmax : a.o_bmax;
    const int o_lT = EK ? L4.o_lT : a.o_lT, o_wave = EK ? L4.o_wave : a.o_wave;
    const int w_aggC = EK ? L4.w_aggC : a.w_aggC, w_aggT = EK ? L4.w_aggT : a.w_aggT;
    const int w_tab = EK ? L4.w_tab : a.w_tab, w_res = EK ? L4.w_res : a.w_res;
    const int w_misc = EK ? L4.w_misc : a.w_misc, w_group = EK ? L4.w_group : a.w_group;
    const int g_lt = EK ? L4.g_lt : a.g_lt, g_gt = EK ? L4.g_gt : a.g_gt;
    const int g_seq = EK ? L4.g_seq : a.g_seq, g_pcv = EK ? L4.g_pcv : a.g_pcv;
    const int g_lpcv = EK ? L4.g_lpcv : a.g_lpcv, g_cnt = EK ? L4.g_lpcv : a.g_cnt;
    const int g_cmax = EK ? L4.g_cmax : a.g_cmax, g_wfac = EK ? L4.g_cmax : a.g_wfac;
    // workgroup-shared
    int32_t *cg = (int32_t *)(lds + o_cg);          // [A*W] global counts C
    int64_t *T = (int64_t *)(lds + o_T);            // [A+1] others' background totals, sum
    double *ppmG = (double *)(lds + o_ppmG);        // [A*W] (C + pc)/den
    double *ppmM = (double *)(lds + o_ppmM);        // [A*W] (C - 1 + pc)/den: own segment
    double *lppmG = (double *)(lds + o_lppmG);      // H = 2: [A*W] log2 of ppmG, binary64,
    double *lppmM = lppmG + A * W;                  //        then [A*W] log2 of ppmM
    float *flppmG = (float *)(lds + o_lppmG);       // H = 1: [A*W] log2 ppmG, binary32,
    float *flppmM = flppmG + A * W;                 //        then [A*W] log2 ppmM
    unsigned int *bmax = (unsigned int *)(lds + o_bmax);  // H = 1: [waves] max finite |log2 PPM|
    // EK = 4: [4][W+1] log2(T[a] + s + pc) for own-segment counts s = 0..W, then
    // log2(sum T + W + A pc): the hold-one-out PCV logs of every motif-bearing sequence
    double *lTab = (double *)(lds + o_lT);
    // wavefront slice
    unsigned char *wl = lds + o_wave + wid * a.wave_bytes;
    int32_t *aggC = (int32_t *)(wl + w_aggC);       // [A*W]
    int64_t *aggT = (int64_t *)(wl + w_aggT);       // [A] background outside segments
    unsigned char *tab = wl + w_tab;                // [E][WS] exact (PWM, PCV): rescans
    SweepResult *res = (SweepResult *)(wl + w_res);  // [64] batch results
    int32_t *misc = (int32_t *)(wl + w_misc);
    // this lane's group slice
    unsigned char *gsl = wl + w_group + gi * a.group_bytes;
    // [E][LS] (log2 PWM fixed, log2 PCV): EK = 0 in the wavefront's contiguous block
    uint2 *lt = (uint2 *)(EK ? gsl + g_lt : wl + a.w_lt + gi * a.lt_bytes);
    unsigned char *gt = gsl + g_gt;                 // H = 2: [E*E][GS] pair sums
    // the group's sequence: H = 2 as pair codes s[i] + E*s[i+1] (precomputed at upload,
    // a.pseq), H = 1 as symbols; sym() recovers symbol s[i] from either (a symbol < E
    // is its own residue)
    // (EK = 4: the odd group's sequence 64 B further, so the two groups of a 32-lane half
    // read their codes from different banks)
    uint8_t *sseq = (uint8_t *)(gsl + g_seq + (EK ? (gi & 1) * 64 : 0));
    double *pcv = (double *)(gsl + g_pcv);          // [GL] by encoded symbol
    double *lpcv = (double *)(gsl + g_lpcv);        // [GL] log2 PCV, binary64
    // [WM] during the table build: (column maximum of log2 PWM', log2 PPM' of the own
    // segment's cell) per column (aliases wfac)
    double2 *cmax = (double2 *)(gsl + g_cmax);
    int32_t *scnt = (int32_t *)(gsl + g_cnt);       // [GL] own-segment symbol counts
    double2 *wfac = (double2 *)(gsl + g_wfac);      // [WM] factors of the picked window
    // EK = 4: the scan reads a second copy of the codes, x 8 (pair_entry), right after
    // the sequence's slot (its span: Lmax + WM + 96 bytes and the odd group's 64)
    uint8_t *scode8 = EK ? sseq + ((a.Lmax + WM + 96 + 15) & ~15) + 64 : sseq;
    const uint8_t *lcodes = scode8;
    const unsigned char *ltab = H == 2 ? gt : (const unsigned char *)lt;
    // EK = 4 runs the certified sweep only (mode 0, no caller's PCV): the other modes
    // take the EK = 0 kernel (gs_sweep_ek)
    const int mode = EK ? 0 : a.mode;
    const bool certified = EK ? true : a.scan == kScanCertified;
    const double *const pcv_fixed = EK ? nullptr : a.pcv_fixed;
    const uint32_t magicE = 0xffffffffu / (uint32_t)E + 1u;  // x / E for x < 2^16
    const uint32_t magicW = 0xffffffffu / (uint32_t)W + 1u;
    auto sym = [&](uint32_t x) -> int {
        if constexpr (EK == 4)
            return (int)(x & 3u);
        else if constexpr (H == 2)
            return (int)(x - (uint32_t)E * (uint32_t)magic_div(x, (uint32_t)E, magicE));
        else
            return (int)x;
    };
    const uint8_t *gseq = H == 2 ? a.pseq : a.seq;  // what is staged
    STAMP_DECL
    const int tl_w = blockIdx.x * kWavesPerBlock + wid;  // (timeline marks: stamps build)
    (void)tl_w;
    TLINE(tl_w, 0);
    TLF(tl_w, 0);
    int nseq_done = 0;

    // The loads that start the pipeline are all issued before the prologue's
    // barrier (which waits for them anyway): the sticky error flag of earlier
    // sweeps, this wavefront's first 64 descriptors, then each group's first
    // sequence and composition.
    TLP(tl_w, 0);
    const int err0 = __hip_atomic_load(a.err_code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // EK = 4: the snapshot's workgroup tables (C, T, PPM, PPM', their logs, the PCV log
    // table: ek4_build_tables) are built by every workgroup from the replicas (default),
    // or come finished (a.ftab_in, gs_set_tuning ftab_mode 1 / 2: a table kernel before
    // the sweep, or the previous sweep's last workgroup): one 16-byte load a thread.
    // Measured (config 2, profiles/r6/ftab_ab.jsonl): the tables given cost the kernel
    // 0.65 us less, but building them once costs more than that wherever it is done, so
    // the finished tables are a build of their own (-DGS_FTAB, libgibbs_hip_ftab.so).
#ifdef GS_FTAB  // (a build of its own: the runtime branch cost the default prologue 0.7 us)
    const bool useF = EK == 4 && a.ftab_in != nullptr;
#else
    constexpr bool useF = false;
#endif
    // (issued before the descriptor-dependent sequence loads, stored to LDS before the
    // prologue's barrier)
    constexpr int kFtV = EK == 4 ? L4.o_wave / 16 : 1, kFtPer = (kFtV + 255) / 256;
    uint4 ftv[kFtPer];
    if (EK == 4 && useF) {
        const uint4 *const ft = (const uint4 *)a.ftab_in;
#pragma unroll
        for (int i = 0; i < kFtPer; ++i)
            if (i * 256 + tid < kFtV) ftv[i] = ft[i * 256 + tid];
        __builtin_amdgcn_sched_barrier(0);
    }
    // EK = 4 (256 threads, at most 132 cells): this thread's aggregate replicas are
    // loaded before the descriptor-dependent sequence loads, so that the prologue's
    // sums wait for one round trip, overlapping the sequences'.  Thread c < cells sums
    // cell c; thread 64 + t the T cell of PCV log-table entry t (t < 4 (W + 1)), or
    // T cell t - 4 (W + 1) for the quad that sums them (log2 of the PCV denominator).
    // With AW <= 64 the count-minus-one PPM cells (normalizePPM's own-segment cells) are
    // the fourth wavefront's: thread 192 + c loads cell c's replicas too, so that no
    // wavefront takes two binary64 logs and divisions before the prologue's barrier.
    constexpr bool kSplitM = EK == 4 && 4 * WM <= 64;
    int64_t rc[kRepl], rt[kRepl], rm[kSplitM ? kRepl : 1];
    const int nT = 4 * (W + 1), tt = tid - 64;
    const bool hasC = EK == 4 && tid < a.cells, hasT = EK == 4 && tt >= 0 && tt < nT + 4;
    const bool hasM = kSplitM && tid >= 192 && tid - 192 < AW;
    const int acell = tt < nT ? tt / (W + 1) : tt - nT;
    if constexpr (EK == 4) {
#pragma unroll
        for (int r = 0; r < kRepl; ++r) rc[r] = rt[r] = 0;
#pragma unroll
        for (int r = 0; r < (kSplitM ? kRepl : 1); ++r) rm[r] = 0;
        if (!useF && a.agg_in) {
            if (hasC)
#pragma unroll
                for (int r = 0; r < kRepl; ++r) rc[r] = a.agg_in[(int64_t)r * a.stride + tid];
            if (hasT)
#pragma unroll
                for (int r = 0; r < kRepl; ++r) rt[r] = a.agg_in[(int64_t)r * a.stride + AW + acell];
            if constexpr (kSplitM) {
                if (hasM)
#pragma unroll
                    for (int r = 0; r < kRepl; ++r) rm[r] = a.agg_in[(int64_t)r * a.stride + tid - 192];
            }
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    TLP(tl_w, 1);
    const uint64_t rng_stream = a.stream;
    // This wavefront's sequences ("slots") are n0 + s*wstride, s < cnt; iteration
    // it scores slots it*G + gi.  Descriptors (length, offset, snapshot position,
    // uniform) of 64 slots at a time sit in lane registers; results wait in LDS
    // and are stored 64 at a time, so the only vector memory operations of an
    // iteration are the one-ahead prefetches of each group's next sequence.
    // Slots are a contiguous range per wavefront (wstride 1), and wavefronts are
    // numbered XCD-major (workgroup b runs on XCD b % 8): neighbouring sequences —
    // and the cache lines of their descriptors and compositions — are read by one
    // XCD's L2 instead of by all eight (cfg2 PMC traffic per launch 4.96 -> 3.16 MB).
    constexpr int wstride = 1;
    const int xcd = blockIdx.x % kRepl, q8 = gridDim.x / kRepl, r8 = gridDim.x % kRepl;
    const int lblock = xcd * q8 + min(xcd, r8) + (int)(blockIdx.x / kRepl);
    const int nwaves = gridDim.x * kWavesPerBlock, lwave = lblock * kWavesPerBlock + wid;
    const int qn = a.wq, rn = a.wr;  // n_local / nwaves and its remainder (host)
    (void)nwaves;
    const int n0 = lwave * qn + min(lwave, rn);
    const int cnt = qn + (lwave < rn ? 1 : 0);
    const int nit = (cnt + G - 1) / G;
    // H = 1 (kDyn): the workgroup's wavefronts share its range [wn0, wn0 + wcnt) by
    // units of G sequences (one iteration), handed out by a workgroup counter in LDS:
    // the SIMD arbiter serves a CU's wavefronts in age order, so static shares leave a
    // 12-wavefront workgroup's end to its youngest wavefronts (config 5: wavefronts
    // 0-3 / 4-7 / 8-11 finished their shares at 102 / 114 / 130 us).  A wavefront's
    // first two units are wid and wid + waves, every next one the counter's; a unit's
    // descriptors are loaded two units ahead, its sequence one ahead.
    constexpr bool kDyn = H == 1;
    const int wb0 = lblock * kWavesPerBlock, wb1 = wb0 + kWavesPerBlock;
    const int wn0 = wb0 * qn + min(wb0, rn);
    const int wcnt = wb1 * qn + min(wb1, rn) - wn0;
    const int nunits = (wcnt + G - 1) / G;
    unsigned int *const wctr = (unsigned int *)(lds + o_bmax) + 15;  // (bmax: <= 12 slots used)
    // a unit's descriptors for this lane's group (none past the range)
    auto unit_desc = [&](int unit, int &ln, int64_t &of, int &ps) {
        const int k = unit * G + gi;
        const bool v = unit < nunits && k < wcnt;
        const int nb = wn0 + k;
        const unsigned long long oob = __ballot(v && (unsigned)nb >= (unsigned)a.n_local);
        if (oob && lane == 0)  // audit, gs_stats [13]
            atomicAdd(&(KA(fallbacks) + (blockIdx.x % kRepl) * kStatStride)[13],
                      (unsigned long long)__popcll(oob));
        if (v) {
            ln = a.len[nb];
            of = a.doff[nb];
            ps = a.pos_in[nb];
        }
    };
    int cu = wid, nu = wid + kWavesPerBlock;  // (kDyn) this and the next unit
    int c_len = 0, c_pos = -1, n_len = 0, n_pos = -1;
    int64_t c_off = 0, n_off = 0;
    int b_len = 0, b_pos = -1;
    int64_t b_off = 0;
    double b_u = 0.0;
    auto load_batch = [&](int base) {
        const int i = base + lane;
        const int nb = n0 + i * wstride;
        const unsigned long long oob = __ballot(i < cnt && (unsigned)nb >= (unsigned)a.n_local);
        if (oob && lane == 0)  // audit, gs_stats [13] (as the first descriptors' below)
            atomicAdd(&(KA(fallbacks) + (blockIdx.x % kRepl) * kStatStride)[13],
                      (unsigned long long)__popcll(oob));
        if (i < cnt) {
            b_len = a.len[nb];
            b_off = a.doff[nb];
            b_pos = a.pos_in[nb];
            if (mode == 0)
                b_u = a.u_in ? a.u_in[nb]
                             : uniform(a.seed, rng_stream, (uint64_t)(a.global_offset + nb));
        }
    };
    // the groups' first sequences: their descriptors are the first vector loads of
    // the wavefront (lane g loads slot g's; the vmcnt wait for them precedes every
    // other load's), then each group takes its own by a lane permute — one round trip
    // instead of a chain of dependent scalar loads per group
    uint4 pf = make_uint4(0, 0, 0, 0);
    int cpf = 0;
    if constexpr (kDyn) {
        unit_desc(cu, c_len, c_off, c_pos);
        unit_desc(nu, n_len, n_off, n_pos);
        if (cu < nunits && cu * G + gi < wcnt) {
            if (c_len <= 16 * GL && li * 16 < c_len) pf = *(const uint4 *)(gseq + c_off + li * 16);
            if (li < CS) cpf = a.comp[(int64_t)(wn0 + cu * G + gi) * CS + li];
        }
        if (tid == 0) *wctr = 2u * (unsigned)kWavesPerBlock;  // (read after the prologue's barrier)
    } else {
        int dl = 0;
        int64_t dof = 0;
        int Ln;
        int64_t on;
        if (a.seq_stride > 0) {
            // every sequence of the same length, a fixed stride apart: no descriptor
            // round trip before the first sequences' loads
            Ln = a.Lmax;
            on = (int64_t)(n0 + gi * wstride) * a.seq_stride;
        } else {
            // lane g < G reads slot g's descriptor, for the slots this wavefront has (an
            // empty shard or a short wavefront reads none past its range)
            const bool rd = lane < G && lane < cnt;
            const int ng = n0 + lane * wstride;
            if (rd) {
                dl = a.len[ng];
                dof = a.doff[ng];
            }
            // audit (gs_stats [13]): a descriptor index outside [0, n_local) would be a
            // read before or past the arrays; the tests require none
            const unsigned long long oob = __ballot(rd && (unsigned)ng >= (unsigned)a.n_local);
            if (oob && lane == 0)
                atomicAdd(&(KA(fallbacks) + (blockIdx.x % kRepl) * kStatStride)[13],
                          (unsigned long long)__popcll(oob));
            Ln = bperm_i32(dl, gi);
            on = bperm_i64(dof, gi);
        }
        if (gi < cnt) {
            if (Ln <= 16 * GL && li * 16 < Ln) pf = *(const uint4 *)(gseq + on + li * 16);
            if (li < CS) cpf = a.comp[(int64_t)(n0 + gi * wstride) * CS + li];
        }
    }
    if constexpr (!kDyn) load_batch(0);
    TLP(tl_w, 2);

    // ---- prologue: aggregates of the snapshot (sum of the replicas) ----
    int64_t csum0 = 0;  // EK = 4: this thread's cell (c = tid)
    if (EK == 4 && !useF) {
#pragma unroll
        for (int r = 0; r < kRepl; ++r) csum0 += rc[r];
        TLP(tl_w, 3);
        if (hasC) {
            if (tid < AW)
                cg[tid] = (int32_t)csum0;
            else
                T[tid - AW] = csum0;
        }
        // log2 PCV = log2(T[a] + s + pc) - log2(sum T + W + A pc) for a motif-bearing
        // sequence with s symbols a in its segment (createNormalizedPCVOfFCV .fs:119
        // of the hold-one-out background): 4 (W + 1) + 1 binary64 logs per workgroup
        // (the second wavefront: the first takes the PPM logs) instead of four per
        // sequence.  The PCV rounding is below 2^-52 in the log.
        int64_t v = 0;
#pragma unroll
        for (int r = 0; r < kRepl; ++r) v += rt[r];
        double q = (hasT && tt >= nT) ? (double)v : 0.0;  // exact: integers below 2^53
        q += __shfl_xor(q, 1);
        q += __shfl_xor(q, 2);
        if (hasT && tt <= nT)
            lTab[tt] = tt < nT ? log2((double)(v + (tt - acell * (W + 1))) + a.pc)
                               : log2((q + (double)W) + a.apc);
        TLP(tl_w, 4);
    }
    if (EK == 4 && useF) {
        TLP(tl_w, 3);
#pragma unroll
        for (int i = 0; i < kFtPer; ++i)
            if (i * 256 + tid < kFtV) ((uint4 *)lds)[i * 256 + tid] = ftv[i];
        TLP(tl_w, 4);
    }
    for (int c = EK ? a.cells : tid; c < a.cells; c += kSweepThreads) {
        int64_t s = 0;
        if (a.agg_in) {
#pragma unroll
            for (int r = 0; r < kRepl; ++r) s += a.agg_in[(int64_t)r * a.stride + c];
        }
        if (c < AW)
            cg[c] = (int32_t)s;
        else
            T[c - AW] = s;  // background of the motif-bearing sequences outside their segments
    }
    TLINE(tl_w, 1);
    for (int c = lane; c < AW; c += 64) aggC[c] = 0;
    if (lane < A) aggT[lane] = 0;
    if (blockIdx.x == 0) {
        int64_t *const agg_zero = KA(agg_zero);
        if (agg_zero)
            for (int i = tid; i < kRepl * a.stride; i += kSweepThreads) agg_zero[i] = 0;
    }
    if (mode == 0) {
        // normalizePPM (.fs:257-260): PPM = (C + pc)/den, and (C - 1 + pc)/den for the
        // own segment's cells (a cell's count is the one this thread summed above)
        float mx = 0.0f;
        if (kSplitM && !useF) {
            if (tid < AW) {
                const double g = ((double)(int32_t)csum0 + a.pc) / a.den;
                ppmG[tid] = g;
                lppmG[tid] = log2(g);
            }
            if (hasM) {
                int64_t mc = 0;
#pragma unroll
                for (int r = 0; r < kRepl; ++r) mc += rm[r];
                const double m = ((double)((int32_t)mc - 1) + a.pc) / a.den;
                ppmM[tid - 192] = m;
                lppmM[tid - 192] = m > 0.0 ? log2(m) : -INFINITY;
            }
        }
        // (the finished tables: in LDS already)
        for (int c = (kSplitM || useF) ? AW : tid; c < AW; c += kSweepThreads) {
            const int32_t cc = EK ? (int32_t)csum0 : cg[c];  // (EK = 4: c = tid, one pass)
            const double g = ((double)cc + a.pc) / a.den;
            const double m = ((double)(cc - 1) + a.pc) / a.den;
            ppmG[c] = g;
            ppmM[c] = m;
            if constexpr (H == 2) {
                // binary64 log2 (< 1e-12 absolute error here); a count-minus-one cell
                // of a zero count is negative and never used (own-segment cells: C >= 1)
                lppmG[c] = log2(g);
                lppmM[c] = m > 0.0 ? log2(m) : -INFINITY;
            } else {
                const float lg = flog2(g), lm = flog2(m);
                flppmG[c] = lg;
                flppmM[c] = lm;
                // finite entries only (a count-minus-one cell of a zero count is NaN and
                // never used: own-segment cells have C >= 1)
                if (fabsf(lg) < INFINITY) mx = fmaxf(mx, fabsf(lg));
                if (fabsf(lm) < INFINITY) mx = fmaxf(mx, fabsf(lm));
            }
        }
        // H = 1: each wavefront's largest |log2 PPM| into its own slot (no init race)
        if (H == 1) {
            mx = wave_max_nonneg_f32(mx);
            if (lane == 0) bmax[wid] = __float_as_uint(mx);
        }
        // columns past the motif: exact factors 1.0, log terms 0 (rewritten only after a
        // rescan whose exact table shares the log tables' LDS)
        for (int c = lane; c < E * WS; c += 64)
            if (c % WS >= W) *(double2 *)(tab + c * 16) = make_double2(1.0, 1.0);
        if constexpr (EK == 0 && H == 2)  // (the four-symbol layout has no single-column table)
            for (int c = li; c < E * LS; c += GL)
                if (c % LS >= W) lt[c] = make_uint2(0u, 0u);
        for (int j = li; j < WM; j += GL)
            if (j >= W) wfac[j] = make_double2(1.0, 1.0);
    }
    TLP(tl_w, 5);
    // an earlier sweep raised an error: its snapshot is void, nothing to do but the
    // done count (the whole workgroup decides together, at the prologue's barrier)
    if (__syncthreads_or(err0 != 0)) {
        sweep_epilogue<WM, EK>(a, lds, (int *)(lds + o_wave), tid);
        return;
    }
    TLINE(tl_w, 2);
    TLF(tl_w, 1);
    TLP(tl_w, 6);

    // Σ_a T[a] (exact: integers far below 2^53)
    const int64_t sumT = (int64_t)wave_sum_f64(lane < A ? (double)T[lane] : 0.0);
    // background error-bound coefficients: |log2 PCV| <= tG, each
    // binary32 entry carries kLog2AbsErr + tG 2^-24, the pair table and the tree sum
    // add <= levels * (W tG) 2^-24.  (The motif part's bound is per sequence, below.)
    constexpr double lv = (double)((H == 2) + tree_depth<NG>()) * 0x1.0p-24;
    const double epsG0 = (double)W * kLog2AbsErr + 1e-9;
    // H = 1: binary32 motif terms, |log2 PPM'| <= tppm, |lt.x| <= tS = tppm + tG; each
    // log carries kLog2AbsErr + |log| 2^-24, the subtraction |lt.x| 2^-24, the tree
    // sum <= levels * (W tS) 2^-24
    float tppm = 0.0f;
    if (H == 1 && mode == 0)
        for (int w = 0; w < kWavesPerBlock; ++w) tppm = fmaxf(tppm, __uint_as_float(bmax[w]));
    // H = 1: the group's motif table, the workgroup's log2 PPM (binary32) by code-major
    // rows, -inf off the alphabet (PWM 0), 0 in the columns past the motif; the own
    // segment's cells are patched in per sequence (and out after it)
    constexpr int MRS = mt_stride(WM);
    float *const mtab = (float *)(H == 1 ? wl + a.w_lt + gi * a.lt_bytes : wl);
    int32_t *const pfx = (int32_t *)(H == 1 ? wl + a.w_pfx + gi * a.pfx_bytes : wl);
    auto mtab_fill = [&]() {
        for (int c = li; c < E * MRS; c += GL) {
            const int e = c / MRS, j = c - e * MRS;
            mtab[c] = j < W ? (e < A ? flppmG[e * W + j] : -INFINITY) : 0.0f;
        }
    };
    if (H == 1 && mode == 0 && certified) {
        mtab_fill();
        wave_sync();
    }
    const double epsS0 = (double)W * (2.0 * kLog2AbsErr + ((double)tppm) * (2.0 * 0x1.0p-24 + lv)) + 1e-9;
    const double epsS1 = (double)W * (2.0 * 0x1.0p-24 + lv);  // epsS = epsS0 + epsS1 * tG
    const double epsG1 = (double)W * (0x1.0p-24 + lv);        // epsG = epsG0 + epsG1 * tG
    STAMP(0);

    for (int it = 0; kDyn ? cu < nunits : it < nit; ++it) {
        const int s = kDyn ? cu * G + gi : it * G + gi;  // this group's slot (kDyn: in the workgroup's range)
        const bool act = s < (kDyn ? wcnt : cnt);
        const int bsl = s & 63;
        int Lr, pr;
        int64_t off;
        double u = 0.0;
        int n;
        if constexpr (kDyn) {
            Lr = c_len, pr = c_pos, off = c_off;
            n = wn0 + s;
            if (mode == 0 && act)
                u = a.u_in ? a.u_in[n] : uniform(a.seed, rng_stream, (uint64_t)(a.global_offset + n));
        } else {
            // (every lane permutes: ds_bpermute reads 0 from a lane that is switched off,
            // and the source lanes belong to other groups)
            Lr = bperm_i32(b_len, bsl), pr = bperm_i32(b_pos, bsl);
            off = bperm_i64(b_off, bsl);
            u = bperm_f64(b_u, bsl);
            n = n0 + s * wstride;
        }
        const int L = act ? Lr : W;
        const int p = act ? pr : -1;
        const int K = L - W + 1;
        const int64_t gidx = a.global_offset + n;
        // kDyn: the unit after next, its descriptors (used at the next iteration's prefetch)
        int nn = 0, x_len = 0, x_pos = -1;
        int64_t x_off = 0;
        if constexpr (kDyn) {
            if (lane == 0) nn = (int)atomicAdd(wctr, 1u);
            nn = __builtin_amdgcn_readfirstlane(nn);
            unit_desc(nn, x_len, x_off, x_pos);
        }
        ++nseq_done;
        if (act) {
            // 16-byte chunks; the bytes of the last chunk past L are zeroed here
            if (L <= 16 * GL) {
                if (li * 16 < L) {
                    const uint4 v = keep_bytes(pf, L - li * 16);
                    *(uint4 *)(sseq + li * 16) = v;
                    if constexpr (EK == 4) *(uint4 *)(scode8 + li * 16) = codes_x8(v);
                }
            } else {
                const uint8_t *g = gseq + off;
                for (int i = li * 16; i < L; i += GL * 16) {
                    const uint4 v = keep_bytes(*(const uint4 *)(g + i), L - i);
                    *(uint4 *)(sseq + i) = v;
                    if constexpr (EK == 4) *(uint4 *)(scode8 + i) = codes_x8(v);
                }
            }
        }
        // createFCVOf (.fs:60-62), precomputed: group lane e < E holds the count of e
        const int my_comp = li < E ? cpf : 0;
        // symbols outside the alphabet (none on the four-symbol path)
        const int na = EK ? 0 : bperm_i32(cpf, gbase + E);
        // ---- one-ahead prefetch of each group's next sequence ----
        if constexpr (kDyn) {
            const int kn = nu * G + gi;
            // (the lane's offsets laundered: the per-lane 64-bit addresses are formed here,
            // not hoisted out of the loop into registers it cannot spare)
            int lo16 = li * 16, lc = li;
            asm volatile("" : "+v"(lo16), "+v"(lc));
            if (nu < nunits && kn < wcnt) {
                if (n_len <= 16 * GL && lo16 < n_len) pf = *(const uint4 *)(gseq + n_off + lo16);
                if (lc < CS) cpf = a.comp[(int64_t)(wn0 + kn) * CS + lc];
            }
        } else {
            const int sn = s + G;
            if ((((it + 1) * G) & 63) == 0 && (it + 1) * G < cnt) load_batch((it + 1) * G);
            const int bn = sn & 63;
            const int Ln = bperm_i32(b_len, bn);
            const int64_t on = bperm_i64(b_off, bn);
            if (sn < cnt) {
                if (Ln <= 16 * GL && li * 16 < Ln) pf = *(const uint4 *)(gseq + on + li * 16);
                if (li < CS) cpf = a.comp[(int64_t)(n0 + sn * wstride) * CS + li];
            }
        }
        // zero tail: unrolled window reads past L see symbol 0 (a valid table row)
        for (int i = ((L + 15) & ~15) + li * 16; i < L + WM + 76; i += GL * 16) {
            *(uint4 *)(sseq + i) = make_uint4(0, 0, 0, 0);
            if constexpr (EK == 4) *(uint4 *)(scode8 + i) = make_uint4(0, 0, 0, 0);
        }
        if constexpr (EK == 0) scnt[li] = 0;
        wave_sync();
        STAMP(1);

        int newp = p;
        bool keep = act;  // this group's pick is folded into the aggregates
        if (mode == 0) {
            // ---- hold-one-out background (integer exact) ----
            const int pp = p >= 0 ? p : 0;
            int segc, seg_alpha;
            if constexpr (EK == 4) {
                // lane e < 4 counts symbol e in the own segment (a symbol is its pair
                // code's low two bits): W/4 unaligned dwords, matching bytes by mask
                // and popcount — no LDS atomics, no counter round trip
                segc = 0;
                if (act && p >= 0 && li < 4) {
                    const int b0 = pp & ~3, sh = pp & 3;
                    uint32_t d[WM / 4 + 1];
#pragma unroll
                    for (int i = 0; i <= WM / 4; ++i) d[i] = *(const uint32_t *)(sseq + b0 + 4 * i);
                    const uint32_t pat = (uint32_t)li * 0x01010101u;
#pragma unroll
                    for (int i = 0; i < WM / 4; ++i) {
                        const uint32_t m = (__builtin_amdgcn_alignbyte(d[i + 1], d[i], sh) & 0x03030303u) ^ pat;
                        segc += 4 - __builtin_popcount((m | (m >> 1)) & 0x01010101u);
                    }
                }
                seg_alpha = W;  // every segment symbol is in the alphabet
            } else {
                if (act && p >= 0)
                    for (int j = li; j < W; j += GL) atomicAdd(&scnt[sym(sseq[pp + j])], 1);
                wave_sync();
                segc = li < E ? scnt[li] : 0;
                seg_alpha = seg_last_i32<GL>(seg_scan_i32<GL>(li < A ? segc : 0), lane);
            }
            const int64_t bgc = li < A ? T[li] + (p >= 0 ? segc : my_comp) : 0;
            // Σ over the 49 slots: alphabet part + the sequence's own other symbols
            const int64_t tot = sumT + (p >= 0 ? seg_alpha : L - na) + na;
            if (act && !pcv_fixed && tot > 2147483647LL) {  // Checked Array.sum (.fs:117)
                if (li == 0) raise_error(a, 3, gidx);
                keep = false;
            }
            // PCV (.fs:119); outside the alphabet the raw count (Q3).  The ...ByPCV
            // variants (.fs:828-853) take the caller's vector instead.
            const double sbg = (double)tot + a.apc;
            const double pe = pcv_fixed ? pcv_fixed[li < E ? li : 0]
                                          : (li < A ? ((double)bgc + a.pc) / sbg : (double)my_comp);
            float lq;
            if constexpr (H == 2) {
                double lq64 = 0.0;
                if constexpr (EK == 4) {
                    // motif-bearing (tot = sum T + W): the workgroup's table, log2(bgc + pc)
                    // - log2(sbg) (the rounding of PCV's division is < 2^-52 in the log)
                    if (certified && li < E)
                        lq64 = (p >= 0 && !pcv_fixed) ? lTab[li * (W + 1) + segc] - lTab[4 * (W + 1)]
                                                        : log2_ool(pe);
                } else {
                    lq64 = certified && li < E ? log2(pe) : 0.0;
                }
                lq = (float)lq64;
                if (li < E) lpcv[li] = lq64;
            } else {
                lq = certified ? flog2(pe) : 0.0f;
                if (li < E) ((float *)lpcv)[li] = lq;
            }
            if (li < E) pcv[li] = pe;
            // a zero PCV of an alphabet symbol makes PWM entries +inf / NaN: binary64
            const unsigned long long zero_pcv = seg_ballot<GL>(li < A && !(pe > 0.0), lane);
            bool fast = keep && certified && zero_pcv == 0;
            const float tG = __int_as_float(seg_last_i32<GL>(
                seg_scan_max_i32<GL>(__float_as_int(li < E && fabsf(lq) < INFINITY ? fabsf(lq) : 0.0f)),
                lane));
            // H = 1: the symbols' log2 PCV in fixed point 2^-sP (int32, after the binary32
            // logs: a window's W of them within 2^30, W tG 2^sP < 2^30), rounded within
            // 2^-(sP+1) each
            int sP = 0;
            if constexpr (H == 1) {
                sP = min(30, 29 - ilogb((double)W * (double)tG + 1.0));
                if (li < E)
                    ((int32_t *)lpcv)[GL + li] = fabsf(lq) < INFINITY ? (int32_t)rint(ldexp((double)lq, sP)) : 0;
            }
            wave_sync();
            STAMP(2);
            TLF(tl_w, 2);
            TLP(tl_w, 7);
            const double epsG = epsG0 + epsG1 * (double)tG + (H == 1 ? (double)W * ldexp(1.0, -sP - 1) : 0.0);
            fast = fast && epsG < 0.015625 && fabs(a.cutoff) < 1000.0;
            // |G~ - G| <= G~ ((2^epsG - 1) + kExp2RelErr)(1 + 3%) for epsG < 1/64
            const double eabs_g = 0.75 * epsG + 1.1 * kExp2RelErr;
            double epsS;
            FastView fv;
            FastViewF fvf;
            bool patched = false;  // H = 1: the own segment's cells are in the group's motif table
            if constexpr (H == 2) {
                // ---- motif terms t[e][j] = log2 PPM' - log2 PCV in fixed point ----
                // Column j's terms are clamped below at Fc_j = cutOff - 1 - (Smax - cmax_j)
                // (Smax = sum of the column maxima): a window with a term at or below it
                // scores at most cutOff - 1 and certainly fails (.fs:735), whatever the
                // term.  Stored is round((max(t, Fc_j) - Fc_j) 2^sc) >= 0, so a window's
                // integer sum is at most W (Smax - cutOff + 1) 2^sc < 2^32 (sc chosen so)
                // and exact; log2 S~ = sum 2^-sc + sum_j Fc_j, within
                // epsS = W (2^-(sc+1) + 4e-12) + 1e-9 of the reference's log2 S (the
                // binary64 logs and differences, the reference's own folds and log).
                double csum = 0.0;
                constexpr int NJ = (WM + GL - 1) / GL;  // columns per lane (EK path)
                double mj[NJ];
                if constexpr (EK == 4) {
                    // the column maxima with every read of the lane issued at once
                    const double lq0 = lpcv[0], lq1 = lpcv[1], lq2 = lpcv[2], lq3 = lpcv[3];
#pragma unroll
                    for (int q = 0; q < NJ; ++q) {
                        const int j = li + q * GL;
                        mj[q] = -INFINITY;
                        if (fast && j < W) {
                            const int o = p >= 0 ? sym(sseq[pp + j]) : -1;
                            const double lo = o >= 0 ? lppmM[o * W + j] : -INFINITY;
                            const double t0 = (o == 0 ? lo : lppmG[0 * W + j]) - lq0;
                            const double t1 = (o == 1 ? lo : lppmG[1 * W + j]) - lq1;
                            const double t2 = (o == 2 ? lo : lppmG[2 * W + j]) - lq2;
                            const double t3 = (o == 3 ? lo : lppmG[3 * W + j]) - lq3;
                            const double m = fmax(fmax(fmax(fmax(-INFINITY, t0), t1), t2), t3);
                            mj[q] = m;
                            cmax[j] = make_double2(m, lo);
                            csum = csum + m;
                        }
                    }
                } else if (fast) {
                    for (int j = li; j < W; j += GL) {
                        const int o = p >= 0 ? sym(sseq[pp + j]) : -1;
                        // the own segment's cell (C - 1 counts, C >= 1): normalizePPM .fs:257-260
                        const double lo = o >= 0 && o < A ? lppmM[o * W + j] : -INFINITY;
                        double m = -INFINITY;
                        for (int e = 0; e < A; ++e)
                            m = fmax(m, (e == o ? lo : lppmG[e * W + j]) - lpcv[e]);
                        cmax[j] = make_double2(m, lo);
                        csum = csum + m;
                    }
                }
                const double smax = seg_last_f64<GL>(seg_scan_f64<GL>(csum), lane);
                // near binary64 overflow of S (.fs:291-292): the exact rescan
                fast = fast && !(smax > 900.0);
                const bool nopass = !(smax > a.cutoff - 1.0);  // no window can pass (also -inf)
                int sc = 30;
                double sumFc = 0.0;
                if (!nopass) {
                    const double width = (double)W * (smax - a.cutoff + 1.0);
                    int ex;
                    (void)frexp(width + 1.0, &ex);  // width + 1 < 2^ex
                    sc = min(30, 32 - ex);
                    sumFc = (double)W * (a.cutoff - 1.0) - (double)(W - 1) * smax;
                }
                fast = fast && sc >= 8;
                const double scale = ldexp(1.0, sc);
                epsS = (double)W * (ldexp(1.0, -sc - 1) + 4e-12) + 1e-9 + 1e-11;
                if constexpr (EK == 4) {
                    // column j's clamp floor Fc_j = cutOff - 1 - (Smax - cmax_j), kept in
                    // place of cmax_j for the table build
#pragma unroll
                    for (int q = 0; q < NJ; ++q) {
                        const int j = li + q * GL;
                        if (fast && !nopass && j < W) cmax[j].x = a.cutoff - 1.0 - (smax - mj[q]);
                    }
                }
                fv.lcodes = lcodes;
                fv.ltab = ltab;
                fv.unit = ldexp(1.0, -sc);
                fv.base = sumFc;
                {
                    const double x = (a.cutoff + epsS - sumFc) * scale;
                    const double y = (a.cutoff - epsS - sumFc) * scale;
                    fv.hiU = nopass || !(x < 4294967290.0) ? 0xffffffffu : (uint32_t)floor(x) + 1u;
                    fv.loU = nopass ? 0xffffffffu : (y <= 1.0 ? 0u : (uint32_t)ceil(y) - 1u);
                }
                wave_sync();
                TLF(tl_w, 3);
                if constexpr (EK == 4) {
                    // ---- pair table directly: lane entry (code, g), code = e0 + 4 e1 ----
                    // gt[code][g] = (t[e0][2g] + t[e1][2g+1] fixed, lq[e0] + lq[e1] binary32),
                    // columns past the motif (0, 0); t as the generic path's lt below
                    if (fast) {
                        constexpr int NE = (16 * NG + GL - 1) / GL;
#pragma unroll
                        for (int q = 0; q < NE; ++q) {
                            const int idx = li + q * GL;
                            if (idx < 16 * NG) {
                                const int code = idx & 15, g = idx >> 4;
                                uint32_t sv[2];
                                float bgv[2];
#pragma unroll
                                for (int h = 0; h < 2; ++h) {
                                    const int e = h ? code >> 2 : code & 3, j = 2 * g + h;
                                    sv[h] = 0u;
                                    bgv[h] = 0.0f;
                                    if (j < W) {
                                        const double le = lpcv[e];
                                        bgv[h] = (float)le;
                                        if (!nopass) {
                                            const double2 cf = cmax[j];  // (Fc_j, own cell's log2 PPM')
                                            const bool own = (p >= 0) & (sym(sseq[pp + j]) == e);
                                            const double t = (own ? cf.y : lppmG[e * W + j]) - le;
                                            sv[h] = (uint32_t)rint((fmax(t, cf.x) - cf.x) * scale);
                                        }
                                    }
                                }
                                *(uint2 *)(gt + g * 128 + code * 8) =
                                    make_uint2(sv[0] + sv[1], __float_as_uint(bgv[0] + bgv[1]));
                            }
                        }
                    }
                } else if (fast) {
                    // ---- log table lt[e][j] = (t fixed, log2 PCV binary32), j < W ----
                    for (int c = li; c < E * W; c += GL) {
                        const int e = magic_div((uint32_t)c, (uint32_t)W, magicW), j = c - e * W;
                        const double le = lpcv[e];
                        uint32_t sv = 0u;
                        if (!nopass) {
                            const double2 cm = cmax[j];
                            const double fc = a.cutoff - 1.0 - (smax - cm.x);
                            const bool own = (p >= 0) & (sym(sseq[pp + j]) == e);
                            // PWM 0 off the alphabet: -inf, clamped
                            const double t = e < A ? (own ? cm.y : lppmG[e * W + j]) - le : -INFINITY;
                            sv = (uint32_t)rint((fmax(t, fc) - fc) * scale);
                        }
                        lt[e * LS + j] = make_uint2(sv, __float_as_uint((float)le));
                    }
                }
            } else {
                // log2 S~ = log2 M~ (binary32 tree sum of log2 PPM') - log2 G~ (exact
                // fixed-point sum of binary32 log2 PCV): within the bound of the round-3
                // form (its log-table entries were the differences of the same two logs)
                // plus the fixed point's rounding
                epsS = epsS0 + epsS1 * (double)tG + (double)W * ldexp(1.0, -sP - 1);
                fast = fast && epsS < 0.015625;
                fvf.hiS = a.cutoff + epsS;
                fvf.loS = a.cutoff - epsS;
                fvf.lcodes = lcodes;
                fvf.mt = (const unsigned char *)mtab;
                fvf.pfx = pfx;
                fvf.unitP = ldexp(1.0, -sP);
                fvf.W = W;
                // the own segment's count-minus-one cells (normalizePPM .fs:257-260, the
                // target's own segment counted in C), out again after the pick
                patched = fast && p >= 0;
                if (patched)
                    for (int j = li; j < W; j += GL) {
                        const int o = sseq[pp + j];
                        if (o < A) mtab[o * MRS + j] = flppmM[o * W + j];
                    }
                if (fast) {
                    // prefix sums P[i] of the positions' fixed-point log2 PCV (wrapping
                    // int32: a window's difference P[k + W] - P[k] is exact), lane li
                    // summing positions [li Q, li Q + Q)
                    const int32_t *bq = (const int32_t *)lpcv + GL;
                    const int Q = (L + GL - 1) / GL, i0 = li * Q;
                    uint32_t loc = 0u;
                    for (int t = 0; t < Q; ++t) {
                        const int i = i0 + t;
                        if (i < L) loc += (uint32_t)bq[sseq[i]];
                    }
                    uint32_t run = seg_scan_u32<GL>(loc) - loc;
                    for (int t = 0; t < Q; ++t) {
                        const int i = i0 + t;
                        if (i < L) {
                            run += (uint32_t)bq[sseq[i]];
                            pfx[i + 1] = (int32_t)run;
                        }
                    }
                    if (li == 0) pfx[0] = 0;
                }
            }
            wave_sync();
            if (H == 2 && EK == 0 && fast) {
                // pair tables gt[e0 + E*e1][g] = lt[e0][2g] + lt[e1][2g+1]; groups
                // past the motif sum the zero padding columns
                for (int c = li; c < E2 * NG; c += GL) {
                    const int code = c / NG, g = c - code * NG;
                    const int e1 = magic_div((uint32_t)code, (uint32_t)E, magicE);
                    const int e0 = code - e1 * E;
                    const uint2 x0 = lt[e0 * LS + 2 * g], x1 = lt[e1 * LS + 2 * g + 1];
                    *(uint2 *)(gt + (code * GS + g) * 8) =
                        make_uint2(x0.x + x1.x, __float_as_uint(__uint_as_float(x0.y) + __uint_as_float(x1.y)));
                }
            }
            wave_sync();
            STAMP(3);
            TLF(tl_w, 4);
            // ---- score every window (.fs:759-782); group lane li owns [li*R, li*R+R) ----
            // Only the lane sums are kept: the pick re-evaluates the one block it needs.
            // (16-lane groups of the pair tables: blocks of a multiple of 4 windows, so
            // that a lane's windows go four at a time from 4-aligned codes; the block
            // ends stay within the zero tail, K + 4 GL + WM < L + WM + 76)
            constexpr bool kQuad = H == 2 && GL == 16;
            const int R = kQuad ? (((K + GL - 1) / GL + 3) & ~3) : (K + GL - 1) / GL;
            const int k_lo = li * R;
            const int Rmax = wave_max_i32(fast ? R : 0);
            double sG = 0.0, sM = 0.0;
            bool flag = false;  // a window in the band or outside the error model: rescan
            int lcat = 0;
            // two windows per step: their LDS lookups overlap (the loop is latency-bound)
            if constexpr (kQuad) {
                // branch-free but for the (rare) windows that pass the cut-off; a window
                // past the lane's block adds +0.0 (the sums are >= +0.0: exact)
                auto take = [&](int kk, int rr, uint32_t so, float lgo) {
                    const bool ok = rr < R && kk < K;
                    const bool xo = !(lgo > -1000.0f && lgo < 1000.0f);
                    const double go = fexp2(lgo);
                    const int co = classify(fv, so);
                    sG = sG + (ok ? go : 0.0);
                    if (ok && co == kPass) {
                        const double fo = (double)so * fv.unit + fv.base;
                        sM = sM + fo;
                        flag |= !(fo >= 0.0);
                        ++lcat;
                    }
                    flag |= ok && (xo || co == kUnsure);
                };
                for (int r = 0; r < Rmax; r += 4) {
                    const int k0 = k_lo + r;
                    const QuadCodes<WM> q = quad_codes<WM>(lcodes, k0);
                    uint32_t s0, s1, s2, s3;
                    f2 l01, l23;
                    window_logs_q<WM, 0, EK == 4>(q, ltab, s0, s1, l01);
                    take(k0, r, s0, l01.x);
                    take(k0 + 1, r + 1, s1, l01.y);
                    __builtin_amdgcn_sched_barrier(0);  // 12 table reads in flight at a time
                    window_logs_q<WM, 2, EK == 4>(q, ltab, s2, s3, l23);
                    take(k0 + 2, r + 2, s2, l23.x);
                    take(k0 + 3, r + 3, s3, l23.y);
                }
            } else if constexpr (H == 2) {
                for (int r = 0; r < Rmax; r += 2) {
                    const int k0 = k_lo + r, k1 = k0 + 1;
                    uint32_t s0, s1;
                    f2 lg;
                    window_logs2<WM, H, EK == 4>(lcodes, ltab, k0, k1, s0, s1, lg);
                    const bool x0 = !(lg.x > -1000.0f && lg.x < 1000.0f);
                    const bool x1 = !(lg.y > -1000.0f && lg.y < 1000.0f);
                    const double g0 = fexp2(lg.x), g1 = fexp2(lg.y);
                    const int c0 = classify(fv, s0), c1 = classify(fv, s1);
                    if (r < R && k0 < K) {
                        sG = sG + g0;
                        if (c0 == kPass) {
                            const double f0 = (double)s0 * fv.unit + fv.base;
                            sM = sM + f0;
                            flag |= !(f0 >= 0.0);
                            ++lcat;
                        }
                        flag |= x0 || c0 == kUnsure;
                    }
                    if (r + 1 < R && k1 < K) {
                        sG = sG + g1;
                        if (c1 == kPass) {
                            const double f1 = (double)s1 * fv.unit + fv.base;
                            sM = sM + f1;
                            flag |= !(f1 >= 0.0);
                            ++lcat;
                        }
                        flag |= x1 || c1 == kUnsure;
                    }
                }
            } else {
                for (int r = 0; r < Rmax; r += 2) {
                    const int k0 = k_lo + r, k1 = k0 + 1;
                    double g0, g1, f0, f1;
                    bool x0 = false, x1 = false;
                    const int c0 = fast_window_f<WM>(fvf, k0, g0, f0, x0);
                    const int c1 = fast_window_f<WM>(fvf, k1, g1, f1, x1);
                    if (r < R && k0 < K) {
                        sG = sG + g0;
                        if (c0 == kPass) {
                            sM = sM + f0;
                            flag |= !(f0 >= 0.0);
                            ++lcat;
                        }
                        flag |= x0 || c0 == kUnsure;
                    }
                    if (r + 1 < R && k1 < K) {
                        sG = sG + g1;
                        if (c1 == kPass) {
                            sM = sM + f1;
                            flag |= !(f1 >= 0.0);
                            ++lcat;
                        }
                        flag |= x1 || c1 == kUnsure;
                    }
                }
            }
            const unsigned long long flagged = seg_ballot<GL>(flag, lane);
            fast = fast && flagged == 0;
            const int npass = seg_last_i32<GL>(seg_scan_i32<GL>(lcat), lane);
            STAMP(4);
            TLINE(tl_w, 3);
            TLF(tl_w, 5);
            int pk = -1;
            auto ev = [&](int k, double &g, double &m) {
                if constexpr (H == 2) {
                    uint32_t ls;
                    float lg;
                    window_logs<WM, H, EK == 4>(lcodes, ltab, k, ls, lg);
                    g = fexp2(lg);
                    m = classify(fv, ls) == kPass ? (double)ls * fv.unit + fv.base : -INFINITY;
                } else {
                    double fs;
                    bool unused = false;
                    m = fast_window_f<WM>(fvf, k, g, fs, unused) == kPass ? fs : -INFINITY;
                }
            };
            // |M~ - M| <= epsS above the band; M~'s own rounding: 2^-52 relative (H = 2,
            // the fixed-point sum), 2^-23 (H = 1, binary32)
            int kind = certified_pick<GL>(ev, fast, K, R, lane, u, sG, sM, lcat, npass, eabs_g,
                                          epsS, H == 2 ? 0x1.0p-52 : 0x1.0p-23, pk);
            STAMP(5);
            TLINE(tl_w, 4);
            // ---- the picked window's exact weight ----
            // factors of column j (group lane j, padding columns hold 1.0), then the
            // reference's left folds, uniform over the group
            if (kind >= 0) {
                for (int j = li; j < W; j += GL) {
                    const int e = sym(sseq[pk + j]);
                    const double pe_e = pcv[e];
                    const bool own = (p >= 0) & (sym(sseq[pp + j]) == e);
                    const double pm = (own ? ppmM : ppmG)[(e < A ? e : 0) * W + j];
                    wfac[j] = make_double2(e < A ? pm / pe_e : 0.0, pe_e);
                }
            }
            wave_sync();
            double pw = 0.0;
            bool pw_log = false;
            {
                double S = 1.0, Gp = 1.0;
#pragma unroll
                for (int j = 0; j < WM; ++j) {
                    const double2 f = wfac[j];
                    S = S * f.x;
                    Gp = Gp * f.y;
                    if ((j & 3) == 3) __builtin_amdgcn_sched_barrier(0);  // 4 loads in flight
                }
                if (kind == 0) {
                    pw = Gp;
                } else if (kind == 1) {
                    if (S > KA(thr_hi)) {
                        pw = S;  // certainly log2 S > cutOff: log2 taken at the batch end
                        pw_log = true;
                    } else {
                        pw = (H == 1 ? log_ool(S * 1.0) : log(S * 1.0)) / kLn2;
                        if (!(pw > a.cutoff)) kind = -6;  // cannot happen when the bound holds
                    }
                }
            }
            // statistics of undecided groups (one lane per group)
            if (keep && kind < 0 && li == 0) {
                atomicAdd(&(KA(fallbacks) + (blockIdx.x % kRepl) * kStatStride)[0], 1ull);
                const int why = !fast ? 2 : kind == -6 ? 3 : 3 - kind;
                atomicAdd(&(KA(fallbacks) + (blockIdx.x % kRepl) * kStatStride)[why], 1ull);
            }
            STAMP(6);
            // ---- binary64 rescans, one group at a time on the whole wavefront ----
            unsigned long long todo = __ballot(keep && kind < 0 && li == 0);
            const bool any_rx = todo != 0ull;
            while (todo) {
                const int src = __ffsll((long long)todo) - 1;
                todo &= todo - 1;
                const int gg = src / GL;
                const int Lx = __builtin_amdgcn_readlane(L, src);
                const int px = __builtin_amdgcn_readlane(p, src);
                const double ux = lane_read_f64(u, src);
                if constexpr (H == 1) {
                    const RxOut r = rescan_group_h1<WM>(kargs(), gg, Lx, px, ux);
                    if (gi == gg) {
                        kind = r.kk;
                        pk = r.pkk;
                        pw = r.xw;
                        pw_log = false;
                    }
                    continue;
                }
                const int Kx = Lx - W + 1;
                const unsigned char *gx = wl + w_group + gg * a.group_bytes;
                uint8_t *sx = (uint8_t *)(gx + g_seq + (EK ? (gg & 1) * 64 : 0));
                const double *pcvx = (const double *)(gx + g_pcv);
                const int ppx = px >= 0 ? px : 0;
                if constexpr (H == 2) {
                    // the binary64 folds read symbols: the group's pair codes become
                    // their residues in place (every later reader takes sym() of them)
                    for (int i = lane; i < Lx + WM + 16; i += 64) sx[i] = (uint8_t)sym(sx[i]);
                    wave_sync();
                }
                for (int c = lane; c < E * W; c += 64) {
                    const int e = magic_div((uint32_t)c, (uint32_t)W, magicW), j = c - e * W;
                    const double pe_e = pcvx[e];
                    const bool own = (px >= 0) & (sx[ppx + j] == e);
                    const double pm = (own ? ppmM : ppmG)[(e < A ? e : 0) * W + j];
                    *(double2 *)(tab + (e * WS + j) * 16) = make_double2(e < A ? pm / pe_e : 0.0, pe_e);
                }
                if (EK == 0 && a.w_tab == a.w_lt)  // (the padding columns: the log tables' zeros were there)
                    for (int c = lane; c < E * WS; c += 64)
                        if (c % WS >= W) *(double2 *)(tab + c * 16) = make_double2(1.0, 1.0);
                wave_sync();
                const double thr_lo = KA(thr_lo);
                auto evx = [&](int k, double &g, double &m) {
                    exact_eval<WM, H == 1>(sx, tab, thr_lo, a.cutoff, k, g, m);
                };
                const int Rx = (Kx + 63) >> 6;
                const int kx_lo = lane * Rx, kx_hi = min(Kx, kx_lo + Rx);
                double xG = 0.0, xM = 0.0;
                bool neg = false;
                int xcat = 0;
                for (int k = kx_lo; k < kx_hi; ++k) {
                    double g, m;
                    evx(k, g, m);
                    xG = xG + g;
                    neg |= !(g >= 0.0);
                    if (m != -INFINITY) {
                        xM = xM + m;
                        neg |= !(m >= 0.0);
                        ++xcat;
                    }
                }
                const int xpass = wave_sum_i32(xcat);
                int kk = -1, pkk = -1;
                const bool ok = __ballot(neg) == 0;
                kk = certified_pick<64>(evx, ok, Kx, Rx, lane, ux, xG, xM, xcat, xpass, 0.0, 0.0,
                                        0.0, pkk);
                if (kk < 0) {
                    // exact sequential restatement of .fs:747-754 on one lane, the
                    // windows re-evaluated in the reference's order: two summing
                    // passes (backgrounds, then motif scores), two walking passes
                    if (lane == 0) {
                        atomicAdd(&(KA(fallbacks) + (blockIdx.x % kRepl) * kStatStride)[1], 1ull);
                        double sacc = 0.0, acc = 0.0;
                        int rk = -1, rp = -1;
                        for (int pass = 0; pass < 4 && rk < 0; ++pass) {
                            for (int k = 0; k < Kx && rk < 0; ++k) {
                                double g, m;
                                evx(k, g, m);
                                const double x = (pass & 1) ? m : g;
                                if ((pass & 1) && m == -INFINITY) continue;
                                if (pass < 2) {
                                    sacc = sacc + x;
                                } else {
                                    const double w = x / sacc;
                                    if (acc <= ux && ux <= acc + w) {
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
                    kk = misc[0];
                    pkk = misc[1];
                }
                double xw = 0.0;
                if (kk >= 0) {
                    double g, m;
                    evx(pkk, g, m);
                    xw = kk == 0 ? g : m;
                }
                if (gi == gg) {
                    kind = kk;
                    pk = pkk;
                    pw = xw;
                    pw_log = false;
                }
                wave_sync();  // the shared exact table is rebuilt for the next group
            }
            if constexpr (H == 1) {
                // the group's motif table: the exact table of a rescan overwrote every
                // group's (refilled), else the own segment's cells out again
                if (any_rx && a.w_tab == a.w_lt) {
                    mtab_fill();
                } else if (patched) {
                    for (int j = li; j < W; j += GL) {
                        const int o = sseq[pp + j];
                        if (o < A) mtab[o * MRS + j] = flppmG[o * W + j];
                    }
                }
                wave_sync();
            }
            if (EK == 0 && H == 2 && any_rx && a.w_tab == a.w_lt) {
                // the exact table shared the groups' log tables: their padding columns
                // (zeros past W, written once in the prologue) again
                uint2 *lt_all = (uint2 *)(wl + a.w_lt);
                const int per = a.lt_bytes >> 3;
                for (int c = lane; c < G * per; c += 64) {
                    const int r = c % per;
                    if (r < E * LS && r % LS >= W) lt_all[c] = make_uint2(0u, 0u);
                }
                wave_sync();
            }
            STAMP(7);
            TLINE(tl_w, 5);
            TLF(tl_w, 6);
            if (keep && kind < 0) {  // every category missed: the list index overruns
                if (li == 0) raise_error(a, 2, gidx);
                keep = false;
            }
            newp = kind == 0 ? -1 : pk;
            if (keep && li == 0) {
                if constexpr (kDyn) {  // stored now (.fs:737's log2 for a motif pick)
                    KA(pos_out)[n] = newp;
                    KA(pwms_out)[n] = pw_log ? log_ool(pw * 1.0) / kLn2 : pw;  // (H = 1: the log out of line)
                } else {
                    res[bsl] = SweepResult{newp, pw_log ? 1 : 0, pw};
                }
            }
        }
        STAMP(8);
        // ---- fold the chosen segment into the next snapshot's aggregates ----
        // C[a][j] += segment; T[a] += composition - segment (the background outside
        // the segment, createFCVWithout + fuseFrequencyVectors of .fs:945-952)
        if (keep && newp >= 0) {
            for (int j = li; j < W; j += GL) {
                const int sy = sym(sseq[newp + j]);
                if (sy < A) {
                    atomicAdd(&aggC[sy * W + j], 1);
                    atomicAdd((unsigned long long *)&aggT[sy], ~0ull);  // -1
                }
            }
            if (li < A) atomicAdd((unsigned long long *)&aggT[li], (unsigned long long)my_comp);
        }
        wave_sync();
        STAMP(9);
        // ---- results of a full batch (or the last one): log2, then 64 stores ----
        if (!kDyn && ((((it + 1) * G) & 63) == 0 || (it + 1) * G >= cnt)) {
            const int i = ((it * G) & ~63) + lane;
            if (mode == 0 && i < cnt) {
                const SweepResult r = res[lane];
                const double v = r.log ? log(r.pw * 1.0) / kLn2 : r.pw;  // .fs:737
                const int nb = n0 + i * wstride;
#ifndef GS_DIAG_NOOUT  // (traffic attribution builds only: the results are not stored)
                KA(pos_out)[nb] = r.pos;
                KA(pwms_out)[nb] = v;
#else
                asm volatile("" ::"v"(r.pos), "v"(v));
#endif
            }
        }
        STAMP(10);
        TLINE(tl_w, 6);
        if constexpr (kDyn) {
            cu = nu, c_len = n_len, c_off = n_off, c_pos = n_pos;
            nu = nn, n_len = x_len, n_off = x_off, n_pos = x_pos;
        }
    }
    (void)nseq_done;
    // is this snapshot in the all-background state (gs_bgregime.h)?  The host sweeps
    // the rest of the chain with gs_sweep_bg_kernel once it is.  Evaluated at the end
    // (workgroup 0, dispatched first), on the snapshot tables still in LDS; ppmG is
    // its scratch
    if (blockIdx.x == 0 && mode == 0 && KA(bg_note)) {
        __syncthreads();
        const bool bg = bg_regime(cg, T, A, W, a.pc, a.den, a.apc, KA(Lmax), KA(cmin), a.cutoff, ppmG, tid);
        if (tid == 0) *KA(bg_note) = bg ? 1 : 0;
    }
    // ---- flush: sum the 4 wavefronts' aggregates, one atomic per cell ----
    __syncthreads();
    STAMP(11);
    STAMP_FLUSH(nseq_done);
    int64_t *dst = KA(agg_out) + (int64_t)(blockIdx.x % kRepl) * a.stride;
    for (int c = tid; c < a.cells; c += kSweepThreads) {
        int64_t v = 0;
#pragma unroll
        for (int w = 0; w < kWavesPerBlock; ++w) {
            const unsigned char *ow = lds + o_wave + w * a.wave_bytes;
            v += c < AW ? (int64_t)((const int32_t *)(ow + w_aggC))[c]
                        : ((const int64_t *)(ow + w_aggT))[c - AW];
        }
        // (with a done counter returning atomics: its vmcnt wait sees them performed)
#ifdef GS_DIAG_NOFLUSH  // (traffic attribution builds only: the aggregates are not flushed)
        v = 0;
#endif
        if (v != 0) {
            if (KA(done))
                GS_FLUSH_ADD((unsigned long long *)&dst[c], (unsigned long long)v);
            else
                atomicAdd((unsigned long long *)&dst[c], (unsigned long long)v);
        }
    }
    TLINE(tl_w, 7);
    TLF(tl_w, 7);
    sweep_epilogue<WM, EK>(a, lds, (int *)(lds + o_wave), tid);
}

#ifndef GS_FOR_EACH_WM  // (a single WM for quick resource checks: -D'GS_FOR_EACH_WM(X)=X(12)')
#define GS_FOR_EACH_WM(X) X(4) X(8) X(12) X(16) X(20) X(24) X(28) X(32) X(40) X(48) X(56) X(64)
#endif
#ifdef GS_SWEEP_EK4_UNIT
// This translation unit (gs_sweep_ek4.hip) instantiates the EK = 4 kernels only, so
// the two halves compile in parallel.
template <int WM>
static const void *sweep_ek4_for(int gl) {
    if (gl == 16) return (const void *)&gs_sweep_kernel<WM, 2, 16, 4>;
    if (gl == 32) return (const void *)&gs_sweep_kernel<WM, 2, 32, 4>;
    if (gl == 64) return (const void *)&gs_sweep_kernel<WM, 2, 64, 4>;
    return nullptr;
}
// The four-symbol sweep's workgroup tables of the snapshot in `rep` (kRepl replicas,
// null: zero aggregates), one workgroup: the first sweep of a chain, and every sweep
// whose previous one could not hand them over (a communicator's all-reduce follows the
// sweep kernel; stream captures).
template <int WM>
__global__ void __launch_bounds__(256) gs_sweep_tables_kernel(const int64_t *rep, int32_t stride, double pc,
                                                              double den, double apc, unsigned char *out) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    ek4_build_tables<WM>(lds, rep, stride, pc, den, apc, false, threadIdx.x, blockDim.x);
    ek4_store_tables<WM>(lds, out, threadIdx.x, blockDim.x);
}

hipError_t gs_sweep_tables_launch(int W, const int64_t *rep, int32_t stride, double pc, double den,
                                  double apc, unsigned char *out, hipStream_t stream) {
    const size_t bytes = (size_t)ek4_layout(W, 16).o_wave;
    switch (W) {
#define GS_CASE(N)                                                                                   \
    case N:                                                                                          \
        hipLaunchKernelGGL(gs_sweep_tables_kernel<N>, dim3(1), dim3(256), bytes, stream, rep, stride, \
                           pc, den, apc, out);                                                       \
        return hipGetLastError();
        GS_CASE(4) GS_CASE(8) GS_CASE(12) GS_CASE(16) GS_CASE(20) GS_CASE(24) GS_CASE(28) GS_CASE(32)
#undef GS_CASE
    }
    return hipErrorInvalidValue;
}

// (W <= 32 only: the host never selects the four-symbol kernel above)
const void *gs_sweep_ek4_ptr(int wm, int gl) {
    switch (wm) {
#define GS_CASE(N) \
    case N:        \
        return sweep_ek4_for<N>(gl);
        GS_CASE(4) GS_CASE(8) GS_CASE(12) GS_CASE(16) GS_CASE(20) GS_CASE(24) GS_CASE(28) GS_CASE(32)
#undef GS_CASE
    }
    return nullptr;
}
#else
const void *gs_sweep_ek4_ptr(int wm, int gl);  // gs_sweep_ek4.hip

// Sets a device counter in stream order (the graph chain's first sweep index).
__global__ void gs_set_u64_kernel(unsigned long long *p, unsigned long long v, unsigned int *z) {
    *p = v;
    *z = 0u;
}

// Uniforms of `sweeps` consecutive sweeps from the device sweep counter *ctr:
// u[k][n] = uniform(seed, stream_sweep(*ctr + k), global_offset + n) — the values
// the sweep kernel draws itself — for a replayed graph whose launch arguments
// repeat.  The last workgroup to finish advances *ctr by `sweeps`.
__global__ void __launch_bounds__(256) gs_uniforms_kernel(double *u, int32_t n_local,
                                                          int64_t global_offset, uint64_t seed,
                                                          int32_t sweeps, unsigned long long *ctr,
                                                          unsigned int *done) {
    const unsigned long long t0 =
        __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int64_t total = (int64_t)sweeps * n_local;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t k = i / n_local, n = i - k * n_local;
        u[i] = uniform(seed, stream_sweep(t0 + (uint64_t)k), (uint64_t)(global_offset + n));
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();
        if (atomicAdd(done, 1u) == gridDim.x - 1) {
            atomicExch(done, 0u);
            atomicAdd(ctr, (unsigned long long)sweeps);
        }
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

template <int WM>
static const void *sweep_kernel_for(int h, int gl, int ek) {
    if (h == 2 && ek == 4) {
        return gs_sweep_ek4_ptr(WM, gl);
    } else if (h == 2) {
        if (gl == 16) return (const void *)&gs_sweep_kernel<WM, 2, 16, 0>;
        if (gl == 32) return (const void *)&gs_sweep_kernel<WM, 2, 32, 0>;
        if (gl == 64) return (const void *)&gs_sweep_kernel<WM, 2, 64, 0>;
    } else {  // more than 16 symbols: groups of >= 32 lanes (E + 1 <= GL)
        if (gl == 32) return (const void *)&gs_sweep_kernel<WM, 1, 32, 0>;
        if (gl == 64) return (const void *)&gs_sweep_kernel<WM, 1, 64, 0>;
    }
    return nullptr;
}

int gs_sweep_wm(int W);

// The four-symbol kernel (EK = 4): four symbols and no other in the data, the
// certified sweep (mode 0) without a caller's PCV, W a multiple of 4 up to 32 (its
// motif width is the template's WM) and 4 wavefronts a workgroup (its prologue gives
// every thread one aggregate cell).  The host carve decides (gs_engine.cpp launch_sweep)
// and lays the LDS out for it (gs_common.h ek4_layout).
int gs_sweep_ek(const SweepArgs &a) { return a.ek; }  // chosen by the host carve

static const void *sweep_kernel_ptr(int wm, int h, int gl, int ek) {
    switch (wm) {
#define GS_CASE(N) \
    case N:        \
        return sweep_kernel_for<N>(h, gl, ek);
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

// Lanes per sequence: the smallest group that holds the composition vector
// (E + 1 lanes) and prefetches the longest sequence in one 16-byte load per lane.
int gs_sweep_group_lanes(int E, int Lmax) {
    int gl = 16;
    while (gl < 64 && (E + 1 > gl || Lmax > 16 * gl)) gl *= 2;
    if (scan_group(E) == 1 && gl < 32) gl = 32;
    return gl;
}

hipError_t gs_sweep_occupancy(int *blocks_per_cu, const SweepArgs &a, int waves, size_t lds_bytes) {
    const void *k = sweep_kernel_ptr(gs_sweep_wm(a.W), scan_group(a.E), a.gl, gs_sweep_ek(a));
    if (!k) return hipErrorInvalidValue;
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, k, 64 * waves, lds_bytes);
}

// start / stop (nullable): events stamped by the dispatch itself (hipExtLaunchKernel),
// so the measured time is the kernel's, without the event packets around it.
hipError_t gs_sweep_launch(const SweepArgs &a, int grid, size_t lds_bytes, hipStream_t stream,
                           hipEvent_t start, hipEvent_t stop) {
    const void *k = sweep_kernel_ptr(gs_sweep_wm(a.W), scan_group(a.E), a.gl, gs_sweep_ek(a));
    if (!k) return hipErrorInvalidValue;
    SweepArgs args = a;
    const int nwaves = grid * a.waves;  // the kernel's slot ranges: n_local split evenly
    args.wq = a.n_local / nwaves;
    args.wr = a.n_local % nwaves;
    void *params[] = {&args};
    const int threads = 64 * a.waves;
    if (!start && !stop)  // plain launch (also the form a stream capture records)
        return hipLaunchKernel(k, dim3(grid), dim3(threads), params, lds_bytes, stream);
    return hipExtLaunchKernel(k, dim3(grid), dim3(threads), params, lds_bytes, stream, start,
                              stop, 0);
}

hipError_t gs_set_counter_launch(unsigned long long *p, unsigned long long v, unsigned int *z,
                                 hipStream_t stream) {
    hipLaunchKernelGGL(gs_set_u64_kernel, dim3(1), dim3(1), 0, stream, p, v, z);
    return hipGetLastError();
}

hipError_t gs_uniforms_launch(double *u, int32_t n_local, int64_t global_offset, uint64_t seed,
                              int32_t sweeps, unsigned long long *ctr, unsigned int *done,
                              int n_cu, hipStream_t stream) {
    const int64_t total = (int64_t)sweeps * n_local;
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((total + 255) / 256, n_cu * 4));
    hipLaunchKernelGGL(gs_uniforms_kernel, dim3(grid), dim3(256), 0, stream, u, n_local,
                       global_offset, seed, sweeps, ctr, done);
    return hipGetLastError();
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
#endif  // GS_SWEEP_EK4_UNIT
