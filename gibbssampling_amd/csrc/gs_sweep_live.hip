// gs_sweep_live.hip — the synchronous Gibbs sweep of a live chain on gfx950.
//
// MotifSampler.findBestMotifIndicesByWithStartPositions (.fs:935-970) with
// motifAmount = 1, for alphabets of at most 4 symbols with no other symbol in the
// data and motifs of at most 16 columns (the packed layout of gs_sweep_dna.hip),
// shaped for the chain the reference runs: getPWMOfRandomStarts' output swept
// (.fs:1035-1037, .fs:993-995), where every target keeps a motif and a few of its
// windows pass the cut-off (.fs:735).
//
// Per target (one lane, or G lanes each owning a 16-aligned range of windows):
//  1. hold-one-out background and PCV in binary64 (.fs:945-954, .fs:109-120);
//  2. FILTER: every window's score against an upper-bound table shared by the
//     workgroup, U_k = sum of ceil-rounded int16 entries of log2 PPM - log2 PCV_ref
//     (the global counts: the own segment's count-minus-one cells only lower the
//     score), one 16-byte pair-table row per position slid into a ring of packed
//     int16 partial sums; a per-target shift W max_e (log2 PCV_ref - log2 PCV_n)
//     turns it into a bound of the reference's log2 S_k.  One bit a window (above
//     the target's threshold) goes into the lane's candidate masks in LDS, the
//     sequence words with them;
//  3. REFINE every candidate: log2 S_k in fixed point (int64, 2^-29) from a
//     workgroup pair table indexed by (own segment pair, window pair) -- log2 PPM or
//     log2 PPM' per column (.fs:255-260, .fs:955-965) less the reference PCV, int32
//     entries -- and the target's PCV log difference times the window's symbol
//     counts: within 3e-7 of the reference's log2 S_k; a window within that of the
//     cut-off (.fs:735) goes to the exact rescan.  The passing weights are summed per
//     32-window chunk into LDS;
//  4. PICK (.fs:746-754): the background categories' total is bounded by K pmax^W;
//     u times the motif total is located among the chunk sums, then among the
//     windows of that one chunk (refined again, identically), certified against
//     every rounding as in gs_pick.h; the picked window's weight is the reference's
//     binary64 fold of PPM'/PCV, then log2 (.fs:283-292, .fs:737);
//  5. whatever the bound cannot settle (a pick near a CDF boundary or among the
//     backgrounds, a target without a passing window) is rescanned exactly in
//     binary64 by the whole wavefront right after its tile (rescan_target); the last
//     workgroup (a done counter) reduces the aggregate replicas into one vector and
//     adds the rank's symbol totals (compsum) to T.
//
// Compiled with -ffp-contract=off: no FMA contraction.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "gs_bgregime.h"
#include "gs_common.h"
#include "gs_fold.h"
#include "gs_pick.h"
#include "gs_stamps.h"
#include "gs_wave.h"

using namespace gs;

// A kernel argument read where it is used: a scalar load from the kernarg segment,
// the pointer laundered through an empty asm so the load is not hoisted to the entry.
// The epilogue's and the rare paths' arguments are read so, which keeps them out of
// the SGPRs of the tile loop (216 SGPRs spilled to VGPR lanes before).
typedef const __attribute__((address_space(4))) DnaArgs KDnaArgs;
__device__ __forceinline__ KDnaArgs *kargs_dna() {
    uint64_t p = (uint64_t)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(p));
    return (KDnaArgs *)p;
}
#define KD(f) (kargs_dna()->f)

namespace {

typedef short s2 __attribute__((ext_vector_type(2)));

// Timing experiments only (make variant VFLAGS=-DGS_EXP=n, never the shipped
// library): phases skipped, bit 1 refine, 2 pick and fold, 4 aggregates, 8 scan,
// 16 the post-scan PCV, 32 the fold, 64 the output stores; no target is rescanned.
#ifndef GS_EXP
#define GS_EXP 0
#endif

// LDS carve (bytes): workgroup tables, then one slice per wavefront
// (live_slice_bytes: the lanes' candidate lists, or the exact rescan's staging)
constexpr int O_C = 0;          // int32 [A*W] counts C of the snapshot
constexpr int O_T = 256;        // int64 [4] T, [4] = sum
constexpr int O_PPM = 304;      // double2 [16 j][4 e]: (C + pc)/den, (C - 1 + pc)/den
constexpr int O_L64 = 1328;     // double [16 j][4 e][2]: their log2
constexpr int O_LPG = 2352;     // double [4]: log2 of the tables' reference PCV
constexpr int O_COARSE = 2384;  // uint4 [16 codes]: int16 pairs (g, g + 4), units 2^-cs
constexpr int O_MISC = 2640;    // int32 [16]: [0] cs, [1] table fault, [2] max pair bound, [3] max
                                // refinement entry, [8] last workgroup
constexpr int O_STAT = 2704;    // uint32 [12]: the workgroup's gs_stats counts
constexpr int O_PREF = 2768;    // double [4] the reference PCV, [4] its reciprocal
constexpr int O_WAGG = 2832;    // per wavefront: int32 C[64], int64 T[4]  (288 B)
constexpr int WAGG_BYTES = 288;
constexpr int O_RT = O_WAGG + kLiveWaves * WAGG_BYTES;  // int32 [8 groups][17 own pairs][16 pairs]
constexpr int RT_G = 17 * 16;   // entries per group (own pair 16: no own segment)
constexpr int O_WAVE = (O_RT + 8 * RT_G * 4 + 255) & ~255;  // 256-aligned: lane arrays at ds offsets
static_assert(O_RT % 16 == 0 && O_WAVE % 256 == 0, "carve");

constexpr int32_t kEntryMax = 4095;  // |filter entry| (units 2^-cs): 8 of them fit an int16

__device__ __forceinline__ uint32_t pk_add(uint32_t x, uint32_t y) {
    return __builtin_bit_cast(uint32_t, __builtin_bit_cast(s2, x) + __builtin_bit_cast(s2, y));
}

// Quad DPP permute (quad_perm control CTRL) of an int; every lane has a source.
template <int CTRL>
__device__ __forceinline__ int qperm_i32(int v) {
    return __builtin_amdgcn_mov_dpp(v, CTRL, 0xf, 0xf, false);
}
// Lane q of the lane's aligned group of G = 2 or 4 lanes, in every lane of the group.
template <int G>
__device__ __forceinline__ int64_t grp_bcast_i64(int64_t x, int q) {
    const int lo = (int)(uint32_t)x, hi = (int)(uint32_t)((uint64_t)x >> 32);
    int l2, h2;
    if constexpr (G == 4) {
        // quad_perm [q, q, q, q] (q static after unrolling)
        switch (q) {
            case 0: l2 = qperm_i32<0x00>(lo); h2 = qperm_i32<0x00>(hi); break;
            case 1: l2 = qperm_i32<0x55>(lo); h2 = qperm_i32<0x55>(hi); break;
            case 2: l2 = qperm_i32<0xAA>(lo); h2 = qperm_i32<0xAA>(hi); break;
            default: l2 = qperm_i32<0xFF>(lo); h2 = qperm_i32<0xFF>(hi); break;
        }
    } else {
        // pairs: quad_perm [0, 0, 2, 2] or [1, 1, 3, 3]
        if (q == 0) {
            l2 = qperm_i32<0xA0>(lo);
            h2 = qperm_i32<0xA0>(hi);
        } else {
            l2 = qperm_i32<0xF5>(lo);
            h2 = qperm_i32<0xF5>(hi);
        }
    }
    return (int64_t)(((uint64_t)(uint32_t)h2 << 32) | (uint32_t)l2);
}

// The window completed by a ring step: the low int16 of the register it was born in
// plus the high int16 of the register born 8 positions later, sign-extended.
__device__ __forceinline__ int half_sum(uint32_t lo_reg, uint32_t hi_reg) {
    int r;
    asm("v_add_u16_sdwa %0, %1, %2 dst_sel:WORD_0 dst_unused:UNUSED_SEXT src0_sel:WORD_0 "
        "src1_sel:WORD_1"
        : "=v"(r)
        : "v"(lo_reg), "v"(hi_reg));
    return r;
}

// count of symbol e among the first W symbols of a packed word (wmask: 2W bits)
__device__ __forceinline__ int sym_count(uint32_t x, int e, uint32_t wmask) {
    const uint32_t y = ~(x ^ (0x55555555u * (uint32_t)e));
    return __popc(y & (y >> 1) & 0x55555555u & wmask);
}

__device__ __forceinline__ uint32_t funnel(uint32_t hi, uint32_t lo, int sh) {
    return __builtin_amdgcn_alignbit(hi, lo, (uint32_t)sh);
}

__device__ __forceinline__ void raise_error(const DnaArgs &a, int code, int64_t gidx) {
    atomicCAS(KD(err_code), 0, code);
    atomicMin(KD(err_index), (unsigned long long)gidx);
}

__device__ __forceinline__ uint4 load_words(const uint32_t *p) {
    uint4 v;
    __builtin_memcpy(&v, p, 16);  // 4-byte aligned 16-byte load
    return v;
}

// ---- the filter ring ----------------------------------------------------------
// Register i (mod 16) is born at position i with the row's dword 0 (groups 0 and 4);
// the rows of later positions add their groups g (dword g & 3) into the register of
// window i - 2g.  Low int16: groups 0..3 of window i; high int16: groups 4..7 of
// window i - 8.  Window i - 14 is complete after position i.
struct Ring {
    uint32_t c[16];
};
constexpr int PD = 2;  // table rows in flight (64 % PD == 0)
struct Pipe {
    uint4 c[PD];
};

// pair code * 16 of position P of a chunk whose words are ww[1..4] (ww[5], ww[6]:
// the next chunk's first words)
template <int P>
__device__ __forceinline__ uint32_t pair16(const uint32_t (&ww)[7]) {
    constexpr int rr = P & 15, wi = (P >> 4) + 1;
    uint32_t v;
    if constexpr (rr >= 2)
        v = funnel(ww[wi + 1], ww[wi], 2 * rr - 4);
    else
        v = funnel(ww[wi], ww[wi - 1], 28 + 2 * rr);
    return v & 0xF0u;
}

// The workgroup tables by LDS address (the kernels have no static LDS: the dynamic
// block starts at address 0, checked in the prologue), so that the table's offset
// folds into the load's immediate.
__device__ __forceinline__ uint4 lds_load_u4(uint32_t addr) {
#if defined(__HIP_DEVICE_COMPILE__)
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    const v4u x = *(__attribute__((address_space(3))) const v4u *)(size_t)addr;
    return make_uint4(x.x, x.y, x.z, x.w);
#else
    (void)addr;
    return make_uint4(0u, 0u, 0u, 0u);
#endif
}

template <int P>
__device__ __forceinline__ void fetch(Pipe &pp, const uint32_t (&ww)[7], const unsigned char *) {
    pp.c[P % PD] = lds_load_u4(O_COARSE + pair16<P>(ww));
}

template <int R>
__device__ __forceinline__ int ring_add(Ring &g, const Pipe &pp) {
    const uint4 cq = pp.c[R % PD];
    constexpr int i0 = R & 15;
    g.c[i0] = cq.x;
    g.c[(i0 - 2) & 15] = pk_add(g.c[(i0 - 2) & 15], cq.y);
    g.c[(i0 - 4) & 15] = pk_add(g.c[(i0 - 4) & 15], cq.z);
    g.c[(i0 - 6) & 15] = pk_add(g.c[(i0 - 6) & 15], cq.w);
    return half_sum(g.c[(i0 - 14) & 15], g.c[(i0 - 6) & 15]);
}

// Per-lane LDS arrays of the wavefront's slice, [entry][64 lanes].
struct LaneArrays {
    uint32_t *mask;   // [nmw] x 4 B: bit i of entry d = window 32 d + i is a candidate
    uint32_t *words;  // [nw] x 4 B: the lane's sequence words from its first window's
    int64_t *bsum;    // [nb] x 8 B: 32-window chunk sums of the passing weights (2^-kFx)
};

// Positions R .. R1 - 1 of a 64-position chunk: windows kq + R (kq = 64 q - 14)
// complete at steps R; each window shifts one bit into cm (set: U_k > thr, a
// candidate), and every 32nd window (R % 32 == 13) stores the mask of the last 32
// windows (window 32 d at bit 31).
template <int R, int R1>
__device__ __forceinline__ void scan_range(Ring &g, Pipe &pp, uint32_t &cm, const uint32_t (&ww)[7],
                                           const unsigned char *coarse, int thr, int kq,
                                           uint32_t *mask, int nmw) {
    if constexpr (R < R1) {
        const int sc = ring_add<R>(g, pp);
        fetch<R + PD>(pp, ww, coarse);
        cm = __builtin_amdgcn_alignbit(cm, (uint32_t)(thr - sc), 31u);
        if constexpr ((R & 31) == 13) {
            const int d = ((kq + R + 1) >> 5) - 1;  // the mask just completed
            if (d >= 0 && d < nmw) mask[64 * d] = cm;
        }
        scan_range<R + 1, R1>(g, pp, cm, ww, coarse, thr, kq, mask, nmw);
    }
}

// log2 S of window `win` (W packed symbols) for the target, in units of 2^-kFx
// (int64): the refinement table's entries of the window's pairs (int32, units
// 2^-kRt, scaled up by a 32 x 32 -> 64 multiply-add each) less base0 (W times symbol
// 0's difference against the table's reference PCV; nbase = -base0) and the
// window's counts of symbols 1..3 times the target's PCV log differences dn relative
// to symbol 0's (int32; negated: ndn).  Group g's entry sits at byte O_RT + g RT_G 4
// + tb + 4 (16 o + c): c the window's pair code, o the own segment's (gwE / gwO: the
// own pair codes of the even / odd groups, shifted into the high nibbles of bytes, 0
// without an own segment, whose row tb = 1024 points past the own rows).  Exact
// integer sums: within kFxErr of the reference's log2 S_k (8 entries rounded to
// 2^-kRt, base0 and dn to 2^-kFx with dn times at most 16 symbols, the binary64 logs
// and folds: 2.4e-7 + 1.5e-8 + 1e-13).  kFx = 29 keeps |dn| < 2 in an int32: in the
// all-background snapshot (T = 0) a target's PCV is its own composition, far from the
// reference PCV.
constexpr int kFx = 29;
constexpr int kRt = 24;
constexpr double kFxErr = 3e-7;

// a * b + c: 32 x 32 -> 64-bit signed multiply-add
__device__ __forceinline__ int64_t mad_i64_i32(int a, int b, int64_t c) {
    int64_t r;
    uint64_t carry;
    asm("v_mad_i64_i32 %0, %1, %2, %3, %4" : "=v"(r), "=s"(carry) : "v"(a), "v"(b), "v"(c));
    return r;
}

template <int NGT>
__device__ __forceinline__ int64_t refine(uint32_t win, uint32_t gwE, uint32_t gwO, uint32_t tb,
                                          uint32_t m5, int ndn1, int ndn2, int ndn3, int64_t nbase) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const uint32_t E = (win & 0x0F0F0F0Fu) | gwE, O = ((win >> 4) & 0x0F0F0F0Fu) | gwO;
    int v[NGT];
#pragma unroll
    for (int g = 0; g < NGT; ++g) {
        const uint32_t byte = __builtin_amdgcn_ubfe((g & 1) ? O : E, 8 * (g >> 1), 8);
        v[g] = *(const int32_t *)(lds + O_RT + g * RT_G * 4 + tb + 4 * byte);
    }
    const uint32_t b0 = win & m5, b1 = (win >> 1) & m5;
    const int c3 = __popc(b0 & b1), c1 = __popc(b0) - c3, c2 = __popc(b1) - c3;
    int64_t s = mad_i64_i32(c3, ndn3, mad_i64_i32(c2, ndn2, mad_i64_i32(c1, ndn1, nbase)));
#pragma unroll
    for (int g = 0; g < NGT; ++g) s = mad_i64_i32(v[g], 1 << (kFx - kRt), s);
    return s;
}

// The picked window's weight: the reference's binary64 left fold of PPM'/PCV
// (.fs:283-292), then log2 (.fs:737).  The W quotients are independent (issued
// together), the products in column order; columns past W multiply by 1.0, exactly.
template <int WM>
__device__ __forceinline__ double picked_weight(uint32_t win, uint32_t gw, bool has_own, int W,
                                             double p0, double p1, double p2, double p3) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const double2 *sPPM = (const double2 *)(lds + O_PPM);
    double q[WM];
#pragma unroll
    for (int j = 0; j < WM; ++j) {
        q[j] = 1.0;
        if (j < W) {
            const int e = (int)((win >> (2 * j)) & 3u);
            const bool own = has_own && (int)((gw >> (2 * j)) & 3u) == e;
            const double2 pp = sPPM[j * 4 + e];
            const double pe = e == 0 ? p0 : e == 1 ? p1 : e == 2 ? p2 : p3;
            q[j] = (own ? pp.y : pp.x) / pe;
        }
    }
    double S = 1.0;
#pragma unroll
    for (int j = 0; j < WM; ++j) S = S * q[j];
    return log(S * 1.0) / kLn2;
}

// Exact binary64 rescan of target sq (wave-uniform) by the whole wavefront: the
// reference's folds for every window (.fs:759-777), the pick certified against
// rounding alone, else one lane replays the reference's sequential sums
// (.fs:747-754).  Writes pos_out / pwms_out (or raises the overrun error) and adds
// the new segment to the wavefront's aggregates.  Staging in the wavefront's slice:
// the unpacked sequence at 0, the (PWM, PCV) table at tab_off, scratch after it.
// BYREF: the kernel arguments through `a` (a function called out of line has no
// kernarg segment pointer of its own: the caller passes the segment, ArgT =
// KDnaArgs); else by KD (scalar loads where used).
template <int WM, bool BYREF = false, class ArgT = DnaArgs>
__device__ void rescan_target(const ArgT &a, int sq, uint64_t rng_stream, unsigned char *wslice,
                              int tab_off, const double2 *sPPM, const int64_t *sT, int64_t sumT,
                              int lane, int32_t *waggC, int64_t *waggT) {
    const int A = a.A, W = a.W;
    const uint32_t wmask = W >= 16 ? 0xffffffffu : ((1u << (2 * W)) - 1u);
    const int Lx = a.len[sq], px = a.pos_in[sq];
    const int64_t wox = a.pkoff[sq];
    const int64_t gx = a.global_offset + sq;
    const double ux = a.u_in ? a.u_in[sq] : uniform(a.seed, rng_stream, (uint64_t)gx);
    uint32_t gwx = 0;
    if (px >= 0) {
        const uint32_t *q = a.pk + wox + (px >> 4);
        gwx = funnel(q[1], q[0], 2 * (px & 15)) & wmask;
    }
    uint8_t *sx = wslice;
    constexpr int WS = tab_stride(WM);
    unsigned char *tab = wslice + tab_off;
    double *mpcv = (double *)(wslice + tab_off + 4 * WS * 16);
    int32_t *mres = (int32_t *)(wslice + tab_off + 4 * WS * 16 + 32);
    // hold-one-out PCV (.fs:945-954)
    if (lane < A) {
        const int64_t tot = sumT + (px >= 0 ? W : Lx);
        const int64_t bgc =
            sT[lane] + (px >= 0 ? sym_count(gwx, lane, wmask) : a.comp[(int64_t)sq * (A + 1) + lane]);
        mpcv[lane] = ((double)bgc + a.pc) / ((double)tot + a.apc);
    }
    // unpack the sequence: one word (16 symbols) per lane step
    const int nwx = (Lx + 15) >> 4;
    for (int i = lane; i < nwx; i += 64) {
        const uint32_t v = a.pk[wox + i];
        uint32_t d[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            uint32_t x = 0;
#pragma unroll
            for (int b = 0; b < 4; ++b) x |= ((v >> (2 * (4 * t + b))) & 3u) << (8 * b);
            d[t] = x;
        }
        *(uint4 *)(sx + 16 * i) = keep_bytes(make_uint4(d[0], d[1], d[2], d[3]), Lx - 16 * i);
    }
    for (int i = 16 * nwx + 16 * lane; i < Lx + WM + 96; i += 16 * 64)
        *(uint4 *)(sx + i) = make_uint4(0, 0, 0, 0);
    wave_sync();
    // (PWM, PCV) [e][WS], columns past W (1, 1)
    for (int c = lane; c < A * WS; c += 64) {
        const int e = c / WS, j = c - e * WS;
        double2 v = make_double2(1.0, 1.0);
        if (j < W) {
            const bool own = px >= 0 && (int)((gwx >> (2 * j)) & 3u) == e;
            const double2 pp = sPPM[j * 4 + e];
            const double pe = mpcv[e];
            v = make_double2((own ? pp.y : pp.x) / pe, pe);
        }
        *(double2 *)(tab + (e * WS + j) * 16) = v;
    }
    wave_sync();
    const double thr_lo = BYREF ? a.thr_lo : KD(thr_lo);
    auto evx = [&](int k, double &gg, double &mm) {
        exact_eval<WM>(sx, tab, thr_lo, a.cutoff, k, gg, mm);
    };
    const int Kx = Lx - W + 1;
    const int Rx = (Kx + 63) >> 6;
    const int kx_lo = lane * Rx, kx_hi = min(Kx, kx_lo + Rx);
    double xG = 0.0, xM = 0.0;
    bool neg = false;
    int xcat = 0;
    for (int k = kx_lo; k < kx_hi; ++k) {
        double gg, mm;
        evx(k, gg, mm);
        xG = xG + gg;
        neg |= !(gg >= 0.0);
        if (mm != -INFINITY) {
            xM = xM + mm;
            neg |= !(mm >= 0.0);
            ++xcat;
        }
    }
    const int xpass = wave_sum_i32(xcat);
    int pkk = -1;
    const bool okx = __ballot(neg) == 0;
    int kk = certified_pick<64>(evx, okx, Kx, Rx, lane, ux, xG, xM, xcat, xpass, 0.0, 0.0, 0.0, pkk);
    if (kk < 0) {
        // the reference's sequential sums (.fs:747-754) on one lane
        if (lane == 0) {
            atomicAdd(&((BYREF ? a.fallbacks : KD(fallbacks)) + (blockIdx.x % kRepl) * kStatStride)[1], 1ull);
            double sacc = 0.0, acc = 0.0;
            int rk = -1, rp = -1;
            for (int pass = 0; pass < 4 && rk < 0; ++pass) {
                for (int k = 0; k < Kx && rk < 0; ++k) {
                    double gg, mm;
                    evx(k, gg, mm);
                    const double x = (pass & 1) ? mm : gg;
                    if ((pass & 1) && mm == -INFINITY) continue;
                    if (pass < 2) {
                        sacc = sacc + x;
                    } else {
                        const double wgt = x / sacc;
                        if (acc <= ux && ux <= acc + wgt) {
                            rk = pass - 2;
                            rp = k;
                        }
                        acc = acc + wgt;
                    }
                }
            }
            mres[0] = rk;
            mres[1] = rp;
        }
        wave_sync();
        kk = mres[0];
        pkk = mres[1];
    }
    double xw = 0.0;
    if (kk >= 0) {
        double gg, mm;
        evx(pkk, gg, mm);
        xw = kk == 0 ? gg : mm;
    }
    if (kk < 0) {
        if (lane == 0) {
            // every category missed (.fs:752)
            atomicCAS(BYREF ? a.err_code : KD(err_code), 0, 2);
            atomicMin(BYREF ? a.err_index : KD(err_index), (unsigned long long)gx);
            (BYREF ? a.pos_out : KD(pos_out))[sq] = -1;
        }
    } else {
        const int newp = kk == 0 ? -1 : pkk;
        if (lane == 0) {
            (BYREF ? a.pos_out : KD(pos_out))[sq] = newp;
            (BYREF ? a.pwms_out : KD(pwms_out))[sq] = xw;
        }
        if (newp >= 0) {
            // the new segment into the wavefront's aggregates
            const int e = lane < W ? sx[newp + lane] : 0;
            if (lane < W) atomicAdd(&waggC[e * W + lane], 1);
            if (lane < A) {
                int sc = 0;
                for (int j = 0; j < W; ++j) sc += sx[newp + j] == lane ? 1 : 0;
                waggT[lane] += (int64_t)(a.comp[(int64_t)sq * (A + 1) + lane] - sc);
            }
        }
    }
    wave_sync();  // the staging area is rewritten for the next target
}

// The exact rescan out of line (a cold path: its registers stay out of the tile loop's,
// round 6: the live kernel's too, as the long sweep's); the kernel arguments through the
// kernarg segment the kernel passes (made wave-uniform here, so its fields are scalar
// loads; a reference to the kernel's by-value argument would copy the whole struct to
// scratch).
template <int WM>
__device__ __attribute__((noinline)) void rescan_ool(KDnaArgs *ka_in, int sq, uint64_t rng_stream,
                                                     unsigned char *wslice, int tab_off, const double2 *sPPM,
                                                     const int64_t *sT, int64_t sumT, int lane, int32_t *waggC,
                                                     int64_t *waggT) {
    const uint64_t pv = (uint64_t)ka_in;
    const uint64_t pu = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(pv >> 32)) << 32) |
                        (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)pv);
    KDnaArgs *ka = (KDnaArgs *)pu;
    rescan_target<WM, true, KDnaArgs>(*ka, sq, rng_stream, wslice, tab_off, sPPM, sT, sumT, lane, waggC, waggT);
}


// A target without a passing window (its group's ntot is 0): its categories are the K
// background products alone (.fs:759-784), the reference's binary64 folds of PCV over
// the windows (.fs:123-124), here by incremental products (two multiplies a window);
// the group's total, then u times it located among the windows in order, certified
// with gs_sweep_bg.hip's margins; the picked window's weight is its exact fold.  Out
// of line: a cold path (the chain from uniform starts, high cut-offs) kept off the hot
// loops' registers.
struct BgPick {
    bool ok;
    double pw;
};
template <int G>
__device__ __attribute__((noinline)) BgPick bg_pick(const uint32_t *words, uint32_t wmask, int W, int K, int nwin,
                                                   bool bgo, double u, int part, int gbase, double p0, double p1,
                                                   double p2, double p3) {
    const double pc4[4] = {p0, p1, p2, p3};
    auto pcv_of = [&](uint32_t e) {
        const double lo = (e & 1u) ? pc4[1] : pc4[0], hi = (e & 1u) ? pc4[3] : pc4[2];
        return (e & 2u) ? hi : lo;
    };
    double inv[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) inv[e] = 1.0 / pc4[e];
    auto inv_of = [&](uint32_t e) {
        const double lo = (e & 1u) ? inv[1] : inv[0], hi = (e & 1u) ? inv[3] : inv[2];
        return (e & 2u) ? hi : lo;
    };
    // the 16 symbols from position q of the lane's range (words from its first window's)
    auto sym16 = [&](int q) {
        return funnel(words[64 * ((q >> 4) + 1)], words[64 * (q >> 4)], 2 * (q & 15));
    };
    auto fold_pcv = [&](int k) {  // the reference's fold of window k (exact)
        const uint32_t wk = sym16(k) & wmask;
        double g = 1.0;
        for (int j = 0; j < W; ++j) g = g * pcv_of((wk >> (2 * j)) & 3u);
        return g;
    };
    // windows [0, n) in order, by 16-window blocks (the entering and leaving symbols of
    // a block from two funnel shifts): window k's product from window k - 1's, times
    // PCV of the symbol entering and 1 / PCV of the one leaving (three roundings a
    // step: the bound below); visit(k, g) returns true to stop
    auto walk_bg = [&](int n, auto &&visit) {
        double g = fold_pcv(0);
        for (int b = 0; b < n; b += 16) {
            // (block 0: window R leaves position R - 1, bits 2R of the first word shifted up)
            const uint32_t in = sym16(b + W - 1), out = b > 0 ? sym16(b - 1) : words[0] << 2;
            for (int R = 0; R < 16 && b + R < n; ++R) {
                if (b + R > 0)
                    g = g * pcv_of(__builtin_amdgcn_ubfe(in, 2 * R, 2)) * inv_of(__builtin_amdgcn_ubfe(out, 2 * R, 2));
                if (visit(b + R, g)) return;
            }
        }
    };
    double Bl = 0.0;
    if (bgo && nwin > 0) walk_bg(nwin, [&](int, double g) {
            Bl = Bl + g;
            return false;
        });
    double incl = Bl;
    if constexpr (G > 1) {
#pragma unroll
        for (int dd = 1; dd < G; dd <<= 1) {
            const double v = __shfl_up(incl, dd, 64);
            if (part >= dd) incl = incl + v;
        }
    }
    const double Bpre = incl - Bl;
    const double Tt = G > 1 ? __shfl(incl, gbase + G - 1, 64) : Bl;
    // each product within (5W + 3K + 20) 2^-53 of the reference's fold, the sums' and
    // the group scan's roundings, the roulette's own: gs_sweep_bg.hip's margins
    const double rel = (double)(5 * W + 3 * K + 20) * 0x1.0p-53 * (1.0 + 0x1.0p-10);
    const double eb = Tt * rel + Tt * (double)(4 * G + 64) * 0x1.0p-53;
    const double ncb = (double)(K + 2);
    const bool okb = bgo && Tt > 4.0 * eb && Tt < INFINITY;
    const double d2 = (8.0 * ncb + 64.0) * 0x1.0p-53 + eb / Tt * (1.0 + (Tt + eb) / (Tt - eb));
    const double Ub = u * Tt, Db = d2 * Tt, Tb = Ub - Db;
    BgPick r{false, 0.0};
    if (okb && Bpre + Bl >= Tb && (part == 0 || Bpre < Tb)) {
        double P = Bpre;
        walk_bg(nwin, [&](int k, double g) {
            const double lo = P;
            P = P + g;
            if (P < Tb) return false;
            r.ok = Ub >= lo + Db && Ub <= P - Db;
            r.pw = fold_pcv(k);  // the picked category's weight: the exact fold
            return true;
        });
    }
    return r;
}

// The target's hold-one-out PCV (.fs:945-954, .fs:109-120: createNormalizedPCVOfFCV)
// and tn = its log2 less the tables' reference log2 PCV_ref: log2(1 + r) of r =
// PCV / PCV_ref - 1 by its series to r^6 when |r| < 2^-7 (truncation below 2^-45,
// inside the refinement's budget), else log2; bad: a PCV that is not positive or a
// log out of range.  (Called before the scan for the target's filter threshold and
// again after it: recomputed rather than held in registers across the scan.)
__device__ __forceinline__ void target_pcv(const DnaArgs &a, const int64_t *sT, const double *sLPG,
                                           const double *sPref, int sq, int p, uint32_t gw,
                                           uint32_t wmask, int64_t tot, double (&pcv)[4], double (&tn)[4],
                                           bool &bad) {
    const double sbg = (double)tot + a.apc;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        pcv[e] = 1.0;
        tn[e] = 0.0;
        if (e < a.A) {
            const int64_t bgc = sT[e] + (p >= 0 ? sym_count(gw, e, wmask) : a.comp[(int64_t)sq * (a.A + 1) + e]);
            pcv[e] = ((double)bgc + a.pc) / sbg;
            const double r = (pcv[e] - sPref[e]) * sPref[4 + e];
            double t;
            if (fabs(r) < 0x1.0p-7) {
                double q = 1.0 / 5.0 - r * (1.0 / 6.0);
                q = 1.0 / 4.0 - r * q;
                q = 1.0 / 3.0 - r * q;
                q = 0.5 - r * q;
                q = 1.0 - r * q;
                t = r * q * (1.0 / kLn2);
            } else {
                t = log2(pcv[e]) - sLPG[e];
            }
            bad |= !(pcv[e] > 0.0) || !(fabs(t + sLPG[e]) < 60.0);
            tn[e] = t;
        }
    }
}

// The snapshot's aggregates into LDS (C int32, T int64, T's sum) and the binary64
// PPM pairs (C + pc)/den, (C - 1 + pc)/den: normalizePPM (.fs:257-260) and its
// count-minus-one cells (.fs:955-965), layout [j][e]; with logs (sL64 non-null) their
// log2.  Every thread of the workgroup (one barrier inside, one at the end).
__device__ __forceinline__ void snapshot_tables(const DnaArgs &a, int32_t *sC, int64_t *sT, double2 *sPPM,
                                                double *sL64, int32_t *sMisc, int tid) {
    const int A = a.A, W = a.W, AW = A * W;
    for (int c = tid; c < a.cells; c += blockDim.x) {
        const int64_t v = a.agg_in ? a.agg_in[c] : 0;
        if (c < AW)
            sC[c] = (int32_t)v;
        else
            sT[c - AW] = v;
    }
    __syncthreads();
    if (tid < 64) {
        const int j = tid >> 2, e = tid & 3;
        double2 pp = make_double2(1.0, 1.0);
        double l0 = 0.0, l1 = 0.0;
        if (j < W && e < A) {
            const int Cc = sC[e * W + j];
            pp.x = ((double)Cc + a.pc) / a.den;
            pp.y = ((double)(Cc - 1) + a.pc) / a.den;
            if (sL64) {
                l0 = log2(pp.x);
                // own cells have C >= 1 (the target's own segment is counted in C)
                l1 = Cc >= 1 ? log2(pp.y) : l0;
                if (!(l0 < INFINITY) || !(l1 < INFINITY) || l0 != l0 || l1 != l1) sMisc[1] = 1;
            }
        }
        sPPM[tid] = pp;
        if (sL64) {
            sL64[2 * tid] = l0;
            sL64[2 * tid + 1] = l1;
        }
    } else if (tid == 64) {
        int64_t s = 0;
        for (int e2 = 0; e2 < A; ++e2) s += sT[e2];
        sT[4] = s;
    }
    __syncthreads();
}

// The in-kernel exchange (gs_exchange_open), by the last workgroup of a sweep: thread c
// < cells holds this rank's partial v of cell c.  Its two 32-bit halves go into every
// rank's buffer (slot [parity][this rank]) as two 8-byte words, each tagged with the
// sweep's flag in its upper half (the LL form: a word is either the old one or the new
// one whole, so its flag proves its half arrived -- no release or acquire fence, no
// L2 writeback or invalidation).  The stores and the polls are system-scope atomics
// (written through to, and read from, memory whatever the buffer's caching).  Thread c
// then polls cell c's words of every other rank in its own buffer, eight at a time, until
// every flag is the sweep's (bounded: 0.5 s of the 100 MHz real-time counter, then the
// exchange error), and agg_out[c] = the sum over the ranks (integers modulo 2^64:
// any order gives the same sums).  Two parities: a rank writes slot set s & 1 of sweep
// s only after every rank's words of sweep s - 1 arrived, i.e. after every rank
// finished reading the slots of sweep s - 2.
__device__ __attribute__((noinline)) void xch_reduce(KDnaArgs *ka_in, int tid, int cells, int64_t v,
                                                    int64_t *agg_out, int *s_seq) {  // s_seq: 3 LDS ints
    // (out of line: the epilogue's registers stay out of the tile loop's; the segment
    // pointer made wave-uniform, so its fields are scalar loads)
    const uint64_t pv = (uint64_t)ka_in;
    KDnaArgs *ka = (KDnaArgs *)(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(pv >> 32)) << 32) |
                                (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)pv));
    int64_t *const *const xpeer = ka->xpeer;
    const int n = ka->xranks, me = ka->xrank;
    // this sweep's number: the count the workgroup read in its prologue (s_seq[0..1]),
    // plus one, stored back for the next sweep (stream-ordered sweeps: one writer)
    const unsigned long long sq = (((unsigned long long)(uint32_t)s_seq[1] << 32) | (uint32_t)s_seq[0]) + 1ull;
    if (tid == 0) {
        *ka->xseq = sq;
        s_seq[2] = 0;  // (a rank late)
    }
    __syncthreads();
    const int par = (int)(sq & 1ull);
    const uint64_t flag = (uint64_t)(sq % 0xFFFFFFFFull + 1ull) << 32;  // in [1, 2^32 - 1]: never the zeroed buffer's
    bool late = false;
    if (tid < cells) {
        const uint64_t lo = flag | (uint32_t)(uint64_t)v, hi = flag | (uint32_t)((uint64_t)v >> 32);
        const int64_t mine = ((int64_t)par * kXchRanks + me) * (2 * kXchStride) + 2 * tid;
        for (int q = 0; q < n; ++q) {
            uint64_t *w = (uint64_t *)xpeer[q] + mine;
            __hip_atomic_store(w, lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(w + 1, hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        const uint64_t *x = (const uint64_t *)xpeer[me] + (int64_t)par * kXchRanks * (2 * kXchStride) + 2 * tid;
        uint64_t s = (uint64_t)v;  // (this rank's own partial: not polled back)
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        for (int q0 = 0; q0 < n && !late; q0 += 4) {
            // ranks q0 .. q0 + 3: their eight words loaded together, reloaded until all arrived
            uint64_t wv[8];
            unsigned pend = 0xffu;
#pragma unroll
            for (int k = 0; k < 8; ++k)
                if (q0 + (k >> 1) >= n || q0 + (k >> 1) == me) pend &= ~(1u << k);
            while (pend) {
#pragma unroll
                for (int k = 0; k < 8; ++k)
                    if (pend & (1u << k))
                        wv[k] = __hip_atomic_load(x + (int64_t)(q0 + (k >> 1)) * (2 * kXchStride) + (k & 1),
                                                  __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
#pragma unroll
                for (int k = 0; k < 8; ++k)
                    if ((pend & (1u << k)) && (wv[k] & 0xFFFFFFFF00000000ull) == flag) {
                        s += (k & 1) ? (wv[k] << 32) : (wv[k] & 0xFFFFFFFFull);
                        pend &= ~(1u << k);
                    }
                if (!pend) break;
                if (__builtin_amdgcn_s_memrealtime() - t0 > 50000000ull) {  // 0.5 s at 100 MHz
                    late = true;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        agg_out[tid] = (int64_t)s;
    }
    // (not __syncthreads_or: its static LDS word would move the dynamic LDS off 0,
    // which the kernels' table check refuses)
    if (late) s_seq[2] = 1;
    __syncthreads();
    if (s_seq[2] != 0 && tid == 0) {
        atomicCAS(ka->err_code, 0, 5);  // the exchange timed out (GS_E_RCCL)
        atomicMin(ka->err_index, (unsigned long long)ka->global_offset);
    }
}

}  // namespace

template <int WM, int G>
#ifndef GS_LIVE_WAVES_PER_EU
#define GS_LIVE_WAVES_PER_EU 4
#endif
__global__ void __launch_bounds__(64 * kLiveWaves, GS_LIVE_WAVES_PER_EU) gs_sweep_live_kernel(DnaArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int A = a.A, W = a.W;
    const int AW = A * W, cells = a.cells;
    int32_t *sC = (int32_t *)(lds + O_C);
    int64_t *sT = (int64_t *)(lds + O_T);
    double2 *sPPM = (double2 *)(lds + O_PPM);
    double *sL64 = (double *)(lds + O_L64);
    double *sLPG = (double *)(lds + O_LPG);
    int32_t *sMisc = (int32_t *)(lds + O_MISC);
    const unsigned char *coarse = lds + O_COARSE;
    const int slice = a.live_slice;
    unsigned char *wslice = lds + O_WAVE + wid * slice;
    int32_t *waggC = (int32_t *)(lds + O_WAGG + wid * WAGG_BYTES);
    int64_t *waggT = (int64_t *)(lds + O_WAGG + wid * WAGG_BYTES + 256);
    // the lanes' arrays in the wavefront's slice
    const int rn_max = live_rn_max(a.Lmax, W, G);
    const int nmw = live_nmw(rn_max), nw = live_nw(rn_max);
    LaneArrays la;
    la.mask = (uint32_t *)wslice + lane;
    la.words = la.mask + 64 * nmw;
    la.bsum = (int64_t *)(wslice + 256 * (nmw + nw)) + lane;

    STAMP_DECL
    const int tl_w = blockIdx.x * (blockDim.x >> 6) + wid;  // (timeline marks: stamps build)
    (void)tl_w;
    TLINE(tl_w, 0);
    const int err0 = __hip_atomic_load(a.err_code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t rng_stream = a.sweep_ctr ? stream_sweep(*a.sweep_ctr) : 0;

    // ---- prologue: the snapshot's aggregates and the workgroup tables ----
    if (lane < 64) waggC[lane] = 0;
    if (lane < 4) waggT[lane] = 0;
    if (tid < 12) ((uint32_t *)(lds + O_STAT))[tid] = 0u;
    // (slots 10, 11: the exchange count so far, read now so the last workgroup's
    // exchange starts without a global round trip; xch_reduce)
    if (tid < 16) sMisc[tid] = (tid == 10 || tid == 11) && KD(xpeer) ? (int)(uint32_t)(*KD(xseq) >> (tid == 11 ? 32 : 0)) : 0;
    snapshot_tables(a, sC, sT, sPPM, sL64, sMisc, tid);
    // a void snapshot (an error raised by an earlier sweep): no tiles, but every
    // workgroup still reaches the done counter below
    const bool void_snap = __builtin_amdgcn_readfirstlane(err0) != 0;
    // is this snapshot in the all-background state (gs_bgregime.h)?  (scratch:
    // wavefront 1's slice, free until the tile loop)
    if (blockIdx.x == 0 && KD(bg_note)) {
        const bool bg = bg_regime(sC, sT, A, W, a.pc, a.den, a.apc, KD(Lmax), KD(cmin), a.cutoff,
                                  (double *)(lds + O_WAVE + slice), tid);
        if (tid == 0) *KD(bg_note) = bg ? 1 : 0;
    }
    if (tid < 4) {
        // the tables' reference PCV: every target's hold-one-out PCV is this plus a
        // small per-target difference
        const double sbg = (double)sT[4] + (double)W + a.apc;
        const double v = tid < A ? ((double)sT[tid] + a.pc + (double)W / (double)A) / sbg : 1.0;
        ((double *)(lds + O_PREF))[tid] = v;
        ((double *)(lds + O_PREF))[4 + tid] = 1.0 / v;
        const double l = log2(v);
        if (!(fabs(l) < 60.0)) sMisc[1] = 1;
        sLPG[tid] = l;
    }
    __syncthreads();
    // filter table: code c = s + 4 s', group g = columns 2g, 2g + 1; entries rounded
    // up (an upper bound of every target's log2 PWM' pair against the reference PCV)
    double tg = 0.0;
    if (tid < 128) {
        const int c = tid >> 3, g = tid & 7, lo = c & 3, hi = c >> 2;
        const int j0 = 2 * g, j1 = 2 * g + 1;
        if (j0 < W) tg += lo < A ? sL64[(j0 * 4 + lo) * 2] - sLPG[lo] : -1.0e6;
        if (j1 < W) tg += hi < A ? sL64[(j1 * 4 + hi) * 2] - sLPG[hi] : -1.0e6;
        if (tg != tg) sMisc[1] = 1;
        const float mx = wave_max_nonneg_f32((float)fmax(tg, 0.0) * 1.001f);
        if (lane == 0) atomicMax(&sMisc[2], __float_as_int(mx));
    }
    // refinement table: group g, own-segment pair o (16: none), window pair c: the sum
    // over the group's columns j < W of (log2 PPM' where the window's symbol is the
    // own segment's, else log2 PPM) less log2 PCV_ref, in units of 2^-kRt; entries
    // below -64 are raised to -64 (such a window cannot pass: checked below)
    {
        float vmax = 0.0f;  // the largest entry (a wave max, one LDS atomic a wavefront)
        for (int i = tid; i < 8 * RT_G; i += blockDim.x) {
            const int g = i / RT_G, r = i - g * RT_G, o = r >> 4, c = r & 15;
            double v = 0.0;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int j = 2 * g + h, sy = (c >> (2 * h)) & 3, oy = (o >> (2 * h)) & 3;
                if (j < W) v += sy < A ? sL64[(j * 4 + sy) * 2 + (o < 16 && oy == sy ? 1 : 0)] - sLPG[sy] : -1.0e300;
            }
            if (v != v || v > 60.0) sMisc[1] = 1;
            vmax = fmaxf(vmax, (float)fmax(v, 0.0) * 1.001f);
            ((int32_t *)(lds + O_RT))[i] = (int32_t)rint(ldexp(fmax(v, -64.0), kRt));
        }
        vmax = wave_max_nonneg_f32(vmax);
        if (lane == 0 && vmax > 0.0f) atomicMax(&sMisc[3], __float_as_int(vmax));
    }
    {
        // the 8 entries of a window, at most kEntryMax each, fit an int16; negative
        // entries are clamped up to -kEntryMax (still an upper bound)
        const float mx = __int_as_float(sMisc[2]);
        int cs = 8;
        while (cs > -8 && mx * ldexpf(1.0f, cs) > (float)(kEntryMax - 2)) --cs;
        if (tid < 128) {
            const int c = tid >> 3, g = tid & 7;
            const double q = fmin(fmax(ceil(ldexp(tg, cs)), -(double)kEntryMax), (double)kEntryMax);
            ((short *)(lds + O_COARSE))[c * 8 + (g & 3) * 2 + (g >> 2)] = (short)(int)q;
        }
        if (tid == 0) sMisc[0] = cs;
    }
    __syncthreads();
    const int cs = __builtin_amdgcn_readfirstlane(sMisc[0]);
    // a window with a raised entry scores at most -64 + 7 (largest entry): below the
    // cut-off, as its true score is
    // (a negative cut-off lets negative weights pass: the certified pick assumes
    // non-negative ones, so every target goes to the exact rescan)
    const bool table_fault = sMisc[1] != 0 || !(fabs(a.cutoff) < 1000.0) || a.cutoff < 0.0 ||
#if defined(__HIP_DEVICE_COMPILE__)
                             (uint32_t)(size_t)(__attribute__((address_space(3))) unsigned char *)lds != 0u ||
#endif
                             !(-64.0 + 7.0 * (double)__int_as_float(sMisc[3]) < a.cutoff - 1.0);
    const int64_t sumT = sT[4];
    STAMP(0);
    TLINE(tl_w, 1);

    // ---- this wavefront's tiles: contiguous, workgroups numbered XCD-major ----
    constexpr int SPT = 64 / G;  // targets per tile
    const int ntiles = (a.n_local + SPT - 1) / SPT;
    const int xcd = blockIdx.x % kRepl, q8 = gridDim.x / kRepl, r8 = gridDim.x % kRepl;
    const int lblock = xcd * q8 + min(xcd, r8) + (int)(blockIdx.x / kRepl);
    const int nwv = blockDim.x >> 6;  // wavefronts of this workgroup (at most kLiveWaves)
    const int nwaves = gridDim.x * nwv;
    const int qn = ntiles / nwaves, rn = ntiles % nwaves;
    (void)lblock;
    // Tiles are handed out by kWorkPools work counters (as gs_sweep_long.hip): static
    // shares left the sweep's end to the wavefronts the SIMD arbiter serves last.  Pool
    // P (XCD blockIdx % 8, half (blockIdx / 8) & 1) owns tiles [t0, t0 + tcnt) in
    // proportion to its wavefronts; a wavefront's first tile is its rank in the pool,
    // each next one a device-scope atomic issued at the start of the tile before and
    // read after its filter scan (then its descriptors are requested).
    const int half = (int)(blockIdx.x / kRepl) & 1;
    int t0, tcnt, nwp;
    {
        const int nbx = q8 + (xcd < r8 ? 1 : 0);
        const int r0 = xcd * q8 + min(xcd, r8) + (half ? (nbx + 1) >> 1 : 0);
        const int rc = half ? nbx >> 1 : (nbx + 1) >> 1;
        const int lw0 = r0 * nwv, lw1 = (r0 + rc) * nwv;
        t0 = lw0 * qn + min(lw0, rn);
        tcnt = void_snap ? 0 : lw1 * qn + min(lw1, rn) - t0;
        nwp = rc * nwv;
    }
    const int wrank = ((int)(blockIdx.x / kRepl) >> 1) * nwv + wid;
    unsigned int *const wctr = KD(done) + 32 * (1 + 2 * xcd + half);
    const int tab_off = live_tab_off(a.Lmax, WM);
    const int part = lane % G, gbase = lane - part;
    const uint32_t wmask = W >= 16 ? 0xffffffffu : ((1u << (2 * W)) - 1u);
    // gs_stats counts go straight into the workgroup's LDS counters (rare events: no
    // per-wavefront registers held across the tile loop)
    uint32_t *sStat = (uint32_t *)(lds + O_STAT);

    // the next tile's descriptors are requested while this one is swept
    struct Desc {
        int L, p;
        int64_t wo;
    };
    auto load_desc = [&](int tile) {
        const int seq = tile * SPT + lane / G;
        const int sq = min(seq, a.n_local - 1);
        // audit (gs_stats [13]): a descriptor index outside [0, n_local); the tests
        // require none (wave-uniform calls: all lanes active)
        const unsigned long long oob = __ballot((unsigned)sq >= (unsigned)a.n_local);
        if (oob && lane == 0)
            atomicAdd(&(KD(fallbacks) + (blockIdx.x % kRepl) * kStatStride)[13], (unsigned long long)__popcll(oob));
        Desc d;
        d.L = a.len[sq];
        d.p = seq < a.n_local ? a.pos_in[sq] : -1;
        d.wo = a.pkoff[sq];
        return d;
    };
    // (no descriptor is read by a wavefront without tiles: an empty shard has none)
    Desc nx{0, -1, 0};
    int tc = wrank < tcnt ? wrank : tcnt;  // pool-relative tile index
    if (tc < tcnt) nx = load_desc(t0 + tc);
    int ntdone = 0;
    while (tc < tcnt) {
        ++ntdone;
        const int tile = t0 + tc;
        const Desc dd = nx;
        // (the next tile, read after the scan; a pool with no more tiles than wavefronts
        // needs no counter: every wavefront's one tile is its rank)
        int gpend = tcnt;
        if (tcnt > nwp && lane == 0) gpend = (int)atomicAdd(wctr, 1u);
        const int seq = tile * SPT + lane / G;
        const bool act = seq < a.n_local;
        const int sq = act ? seq : a.n_local - 1;
        const int64_t gidx = a.global_offset + sq;
        const int L = dd.L;
        const int p = dd.p;
        const int64_t wo = dd.wo;
        uint32_t gw = 0;  // the target's own segment (snapshot position p)
        if (p >= 0) {
            const uint32_t *q = a.pk + wo + (p >> 4);
            gw = funnel(q[1], q[0], 2 * (p & 15)) & wmask;
        }
        const bool lead = part == 0;
        bool keep = act;

        // ---- hold-one-out background; no symbol outside the alphabet ----
        const int64_t tot = sumT + (p >= 0 ? W : L);
        if (act && tot > 2147483647LL) {  // Checked Array.sum (.fs:117)
            if (lead) raise_error(a, 3, gidx);
            keep = false;
        }
#if defined(GS_LIVE_DEBUG)
        bool bad = table_fault;
#else
        bool bad = table_fault || a.live_force;
#endif
        // the filter's per-target shift W max_e (log2 PCV_ref - log2 PCV): a bound from
        // binary32 arithmetic (each log within 2^-12 of the reference's binary64 one)
        double shift;
        {
            const float sbgf = (float)((double)tot + a.apc);
            float sh = -INFINITY;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                if (e < A) {
                    const int64_t bgc = sT[e] + (p >= 0 ? sym_count(gw, e, wmask) : a.comp[(int64_t)sq * (A + 1) + e]);
                    const float pf = ((float)bgc + (float)a.pc) / sbgf;
                    const float lf = __builtin_amdgcn_logf(pf);
                    bad |= !(pf > 0.0f) || !(fabsf(lf) < 60.0f);
                    sh = fmaxf(sh, (float)sLPG[e] - lf);
                }
            }
            shift = (double)sh + 0x1.0p-12;
        }
        const int K = L - W + 1;
        const int Rn = G == 1 ? K : ((((K + G - 1) / G) + 15) & ~15);
        const int x0 = min(part * Rn, K), x1 = min(K, x0 + Rn);
        const int nwin = x1 - x0;
        bad |= nwin > rn_max;  // the slice's arrays hold rn_max windows a lane
        // U_k 2^-cs + W shift >= the reference's log2 S_k for every window (binary64
        // logs, folds and sums inside 1e-9)
        const double thd = ldexp(a.cutoff - (double)W * shift - 1e-8, cs);
        const int thr = bad ? -2147483647 : (int)fmin(fmax(floor(thd), -2147483647.0), 2147483646.0);
        STAMP(1);

        // ---- filter scan: every window of the lane's range, one ring step a position;
        // candidate bits into the lane's masks, the words into its word array ----
        // 16-position blocks: window nwin - 1 completes at position nwin + 13
        const int nblk = (nwin + 14 + 15) >> 4;
        const bool scan = keep && !bad;
        const int nblk_max = __builtin_amdgcn_readfirstlane(-wave_min_i32(-(scan && !(GS_EXP & 8) ? nblk : 0)));
        const int nch_max = (nblk_max + 3) >> 2;
        {
            Ring rg;
#pragma unroll
            for (int i = 0; i < 16; ++i) rg.c[i] = 0u;
            const uint32_t *wp = a.pk + wo + (x0 >> 4);
            uint32_t ww[7];
            const uint4 cur = load_words(wp);
            ww[0] = 0u;
            ww[1] = cur.x;
            ww[2] = cur.y;
            ww[3] = cur.z;
            ww[4] = cur.w;
            Pipe pp;
            fetch<0>(pp, ww, coarse);
            if constexpr (PD > 1) fetch<1>(pp, ww, coarse);
            if constexpr (PD > 2) fetch<2>(pp, ww, coarse);
            if constexpr (PD > 3) fetch<3>(pp, ww, coarse);
            static_assert(PD <= 4, "initial fetches");
            uint32_t cm = 0;
            for (int q = 0; q < nch_max; ++q) {
                const uint4 nxt = load_words(wp + 4 * (q + 1));
                ww[5] = nxt.x;
                ww[6] = nxt.y;
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    if (4 * q + i < nw) la.words[64 * (4 * q + i)] = ww[1 + i];
                const int kq = 64 * q - 14, nbq = nblk_max - 4 * q;
                scan_range<0, 16>(rg, pp, cm, ww, coarse, thr, kq, la.mask, nmw);
                if (nbq > 1) {
                    scan_range<16, 32>(rg, pp, cm, ww, coarse, thr, kq, la.mask, nmw);
                    if (nbq > 2) {
                        scan_range<32, 48>(rg, pp, cm, ww, coarse, thr, kq, la.mask, nmw);
                        if (nbq > 3) scan_range<48, 64>(rg, pp, cm, ww, coarse, thr, kq, la.mask, nmw);
                    }
                }
                ww[0] = ww[4];
                ww[1] = nxt.x;
                ww[2] = nxt.y;
                ww[3] = nxt.z;
                ww[4] = nxt.w;
            }
#pragma unroll
            for (int i = 0; i < 4; ++i)
                if (4 * nch_max + i < nw) la.words[64 * (4 * nch_max + i)] = ww[1 + i];
            // the trailing partial mask: its last window, ke = 16 nblk_max - 15 (ke % 32
            // is 1 or 17, never 31: not stored above), at bit 0
            const int ke = 16 * nblk_max - 15, dt = ke >> 5;
            if (nblk_max > 0 && dt < nmw) la.mask[64 * dt] = cm << (31 - (ke & 31));
        }
        STAMP(2);
        TLINE(tl_w, 2);

        // the next tile and its descriptors
        const int tnext = tcnt > nwp ? min(nwp + __builtin_amdgcn_readlane(gpend, 0), tcnt) : tcnt;
        if (tnext < tcnt) nx = load_desc(t0 + tnext);
        // ---- refine every candidate; the passing weights into the block sums ----
        // the target's PCV again (opaque copies of its inputs: not kept from before the scan)
        double pcv[4], tn[4];
        if (GS_EXP & 16) {
#pragma unroll
            for (int e = 0; e < 4; ++e) pcv[e] = 0.25, tn[e] = 0.0;
        } else {
            int sq2 = sq, p2 = p;
            uint32_t gw2 = gw;
            int64_t tot2 = tot;
            asm volatile("" : "+v"(sq2), "+v"(p2), "+v"(gw2), "+v"(tot2));
            bool bad2 = false;
            target_pcv(a, sT, sLPG, (const double *)(lds + O_PREF), sq2, p2, gw2, wmask, tot2, pcv, tn, bad2);
            bad |= bad2;  // (its scan, if any, is not used)
        }
        // the lane's refinement rows: the own segment's pair codes per group
        const uint32_t gwE = p >= 0 && !(GS_EXP & 128) ? (gw & 0x0F0F0F0Fu) << 4 : 0u;
        const uint32_t gwO = p >= 0 && !(GS_EXP & 128) ? gw & 0xF0F0F0F0u : 0u;
        const uint32_t tb = p >= 0 && !(GS_EXP & 128) ? 0u : 1024u;
        const uint32_t m5 = 0x55555555u & wmask;
        // the PCV log differences in units of 2^-kFx (int32: |difference| < 2, else
        // the exact rescan)
        int ndn[4] = {0, 0, 0, 0};
#pragma unroll
        for (int e = 1; e < 4; ++e) {
            const double x = ldexp(tn[e] - tn[0], kFx);
            bad |= !(fabs(x) < 0x1.0p30);
            ndn[e] = bad ? 0 : -(int)rint(x);
        }
        const int64_t nbase = bad ? 0 : -(int64_t)rint(ldexp((double)W * tn[0], kFx));
        // the cut-off band: a refined score within kFxErr of the cut-off is folded
        const int64_t thi = (int64_t)ceil(ldexp(a.cutoff + kFxErr, kFx));
        const int64_t tlo = (int64_t)floor(ldexp(a.cutoff - kFxErr, kFx));
        const int nd = (nwin + 31) >> 5, nb = nd;  // chunk sums: one a mask word
        // the last mask word's windows past nwin are not the lane's
        const uint32_t tailm = (nwin & 31) ? (1u << (nwin & 31)) - 1u : 0xffffffffu;
        for (int i = 0; i < nb; ++i) la.bsum[64 * i] = 0;
        int npass = 0;
        bool unsure = false;
        {
            // one candidate a round for every lane that has one left: the round's work
            // is not branched on (a lane without one refines window 0 and adds nothing);
            // the passing weights go into the 32-window chunk sums by LDS atomics
            bool live = scan && nd > 0 && !(GS_EXP & 1);
            int d = -1;
            uint32_t m = 0;
            // the lane's next mask word is requested one word ahead: moving to it waits
            // for no LDS round trip unless the current word yielded nothing
            uint32_t mnx = live ? la.mask[0] : 0u;
            auto advance = [&]() {
                while (live && m == 0u) {
                    ++d;
                    live = d < nd;
                    if (live) {
                        m = __builtin_bitreverse32(mnx) & (d == nd - 1 ? tailm : 0xffffffffu);
                        mnx = d + 1 < nd ? la.mask[64 * (d + 1)] : 0u;
                    }
                }
            };
            advance();
            // two candidates a round (independent chains of LDS reads in flight)
            while (__ballot(live) != 0ull) {
                const bool live1 = live;
                const int k1 = live1 ? 32 * d + __builtin_ctz(m) : 0;
                m &= m - 1u;
                advance();
                const bool live2 = live;
                const int k2 = live2 ? 32 * d + __builtin_ctz(m) : 0;
                m &= m - 1u;
                advance();
                const uint32_t win1 =
                    funnel(la.words[64 * ((k1 >> 4) + 1)], la.words[64 * (k1 >> 4)], 2 * (k1 & 15)) & wmask;
                const uint32_t win2 =
                    funnel(la.words[64 * ((k2 >> 4) + 1)], la.words[64 * (k2 >> 4)], 2 * (k2 & 15)) & wmask;
                const int64_t mk1 = refine<WM / 2>(win1, gwE, gwO, tb, m5, ndn[1], ndn[2], ndn[3], nbase);
                const int64_t mk2 = refine<WM / 2>(win2, gwE, gwO, tb, m5, ndn[1], ndn[2], ndn[3], nbase);
                const bool pass1 = live1 && mk1 > thi, pass2 = live2 && mk2 > thi;
                // within the bound of the cut-off (|score - cutOff| <= kFxErr): the
                // exact rescan decides
                unsure |= (live1 && !pass1 && mk1 >= tlo) || (live2 && !pass2 && mk2 >= tlo);
                __hip_atomic_fetch_add(&la.bsum[64 * (k1 >> 5)], pass1 ? mk1 : (int64_t)0, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);
                __hip_atomic_fetch_add(&la.bsum[64 * (k2 >> 5)], pass2 ? mk2 : (int64_t)0, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);
                npass += (pass1 ? 1 : 0) + (pass2 ? 1 : 0);
            }
        }
        int64_t Ml = 0;  // the lane's motif total (2^-kFx)
        for (int i = 0; i < nb; ++i) Ml += la.bsum[64 * i];
        STAMP(3);
        TLINE(tl_w, 3);

        // ---- the target's totals over its G lanes ----
        int64_t MtotI = Ml, OpreI = 0;
        int ntot = npass;
        bool badg = bad || unsure;
        if constexpr (G == 2 || G == 4) {
            // a target's lanes are an aligned pair or quad: quad DPP permutes (VALU
            // latency, no LDS crossbar round trip)
            ntot += qperm_i32<0xB1>(ntot);  // lane ^ 1
            int bi = badg ? 1 : 0;
            bi |= qperm_i32<0xB1>(bi);
            if constexpr (G == 4) {
                ntot += qperm_i32<0x4E>(ntot);  // lane ^ 2
                bi |= qperm_i32<0x4E>(bi);
            }
            badg = bi != 0;
#pragma unroll
            for (int q = 0; q < G - 1; ++q) {
                const int64_t v = grp_bcast_i64<G>(Ml, q);
                if (q < part) OpreI += v;
            }
            MtotI = grp_bcast_i64<G>(OpreI + Ml, G - 1);
        } else if constexpr (G > 1) {
#pragma unroll
            for (int dd = 1; dd < G; dd <<= 1) {
                ntot += __shfl_xor(ntot, dd, 64);
                badg |= __shfl_xor((int)badg, dd, 64) != 0;
            }
#pragma unroll
            for (int q = 0; q < G - 1; ++q) {
                const int64_t v = __shfl(Ml, gbase + q, 64);
                if (q < part) OpreI += v;
            }
            MtotI = __shfl(OpreI + Ml, gbase + G - 1, 64);
        }
        // binary64 from here: the totals (exact integers below 2^53 here) in log2 units
        const double Mtot = ldexp((double)MtotI, -kFx);
        // each weight within kFxErr of the reference's
        const double etot = (double)ntot * kFxErr;

        // ---- certified pick (.fs:746-754) ----
        const double u = a.u_in ? a.u_in[sq] : uniform(a.seed, rng_stream, (uint64_t)gidx);
        // backgrounds first: their total lies in [0, Bhi] (each G_k <= pmax^W); each
        // motif weight within its bound, the sums within 2^-50 of their terms'
        double pmax = 0.0;
#pragma unroll
        for (int e = 0; e < 4; ++e)
            if (e < A) pmax = fmax(pmax, pcv[e]);
        double pmw = 1.0;
        for (int j = 0; j < W; ++j) pmw = pmw * pmax;
        const double Bhi = (double)K * pmw * (1.0 + 1e-12);
        const double eabs = Bhi + etot + Mtot * 0x1.0p-50;
        const double ncat = (double)(K + ntot + 2);
        bool ok = keep && !badg && ntot > 0 && Mtot > 4.0 * eabs && Mtot < INFINITY;
        const double delta =
            (8.0 * ncat + 64.0) * 0x1.0p-53 + eabs / Mtot * (1.0 + (Mtot + eabs) / (Mtot - eabs));
        ok = ok && u > delta;  // not in the background block
        const double U = u * Mtot, D = delta * Mtot, Tg = U - D, Th = U + D;
        // the boundaries in the sums' own units (2^-kFx): for an integer X below 2^53,
        // X 2^-kFx >= Tg exactly when X >= ceil(Tg 2^kFx) (scaling by 2^kFx is exact)
        const int64_t TgI = ok ? (int64_t)ceil(ldexp(Tg, kFx)) : 0;
        const int64_t TlI = ok ? (int64_t)floor(ldexp(Tg, kFx)) : 0;
        const int64_t ThI = ok ? (int64_t)ceil(ldexp(Th, kFx)) : 0;
        const bool mine = !(GS_EXP & 2) && ok && OpreI < TgI && OpreI + Ml >= TgI;
        bool found = false, cert = false;
        int pk = -1;
        uint32_t win = 0;
        if (mine) {
            // the chunk (32 windows) whose upper boundary first reaches U - D
            int64_t PI = OpreI;
            int bb = nb - 1;
            for (int i = 0; i < nb; ++i) {
                const int64_t v = la.bsum[64 * i];
                if (PI + v >= TgI) {
                    bb = i;
                    break;
                }
                PI += v;
            }
            // its windows in order (its mask word), refined again (identically): from the
            // chunk's nearer end by passing mass (round 6: half the re-refinements on
            // average).  Every sum is an exact integer, so walking down from the chunk's
            // end (its sum, as accumulated) gives the same boundaries: the pick is the
            // first passing window whose interval reaches U - D either way
            uint32_t mm = __builtin_bitreverse32(la.mask[64 * bb]) & (bb == nd - 1 ? tailm : 0xffffffffu);
            const int64_t Pend = PI + la.bsum[64 * bb];
            const bool desc = TgI - PI > Pend - TgI;
            int64_t P = desc ? Pend : PI;
            auto next_k = [&]() {  // the next candidate of the walk, its bit cleared
                const int b = desc ? 31 - __builtin_clz(mm) : __builtin_ctz(mm);
                mm &= ~(1u << b);
                return 32 * bb + b;
            };
            // two candidates an iteration (their refinements overlap)
            while (mm != 0u && !found) {
                const int k1 = next_k();
                const bool has2 = mm != 0u;
                const int k2 = has2 ? next_k() : k1;
                const uint32_t w1 =
                    funnel(la.words[64 * ((k1 >> 4) + 1)], la.words[64 * (k1 >> 4)], 2 * (k1 & 15)) & wmask;
                const uint32_t w2 =
                    funnel(la.words[64 * ((k2 >> 4) + 1)], la.words[64 * (k2 >> 4)], 2 * (k2 & 15)) & wmask;
                const int64_t mk1 = refine<WM / 2>(w1, gwE, gwO, tb, m5, ndn[1], ndn[2], ndn[3], nbase);
                const int64_t mk2 = refine<WM / 2>(w2, gwE, gwO, tb, m5, ndn[1], ndn[2], ndn[3], nbase);
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    if (h == 1 && (found || !has2)) break;
                    const int64_t mk = h ? mk2 : mk1;
                    if (mk > thi) {
                        // this window's interval [lo, hi) reaches U - D; certified when it
                        // holds all of [U - D, U + D]
                        const int64_t lo = desc ? P - mk : P, hi = desc ? P : P + mk;
                        if (desc ? lo < TgI : hi >= TgI) {
                            found = true;
                            cert = lo <= TlI && hi >= ThI;
                            pk = x0 + (h ? k2 : k1);
                            win = h ? w2 : w1;
                        }
                        P = desc ? lo : hi;
                    }
                }
            }
        }
        STAMP(4);
        TLINE(tl_w, 4);
        // the picked window's weight: the reference's binary64 fold
        double pw = 0.0;
        bool win_ok = false;
        if (found && cert) {
            pw = (GS_EXP & 32) ? 2.0 : picked_weight<WM>(win, gw, p >= 0, W, pcv[0], pcv[1], pcv[2], pcv[3]);
            win_ok = pw > a.cutoff;
        }
        // ---- a target without a passing window: its categories are the K background
        // products alone (.fs:759-784), each the reference's binary64 fold of PCV over
        // the window (.fs:123-124); the group's total, then u times it located among
        // the windows in order, certified as in gs_sweep_bg.hip ----
        const bool bgo = keep && !badg && ntot == 0;
        if (__ballot(bgo) != 0ull) {
            const BgPick r = bg_pick<G>(la.words, wmask, W, K, nwin, bgo, u, part, gbase, pcv[0], pcv[1],
                                        pcv[2], pcv[3]);
            if (r.ok) {
                win_ok = true;  // a background category: Positions [], PWMS its product
                pk = -1;
                pw = r.pw;
            }
        }
        // the group's result: from the part that held the pick
        if constexpr (G > 1) {
            const unsigned long long bb = __ballot(win_ok);
            const unsigned long long gm = (bb >> gbase) & ((1ull << G) - 1ull);
            const int src = gm ? gbase + __ffsll((long long)gm) - 1 : gbase;
            const int pk_s = __shfl(pk, src, 64);
            const double pw_s = __shfl(pw, src, 64);
            const uint32_t win_s = (uint32_t)__shfl((int)win, src, 64);
            win_ok = gm != 0;
            pk = pk_s;
            pw = pw_s;
            win = win_s;
        }
        STAMP(5);
        TLINE(tl_w, 5);
        const bool need_fb = keep && !win_ok && !GS_EXP;
        if (__ballot(need_fb && lead) != 0ull) {  // (wave-uniform; rare)
            // why (gs_stats [2..6], [10..12]): a score out of range / NaN / no passing
            // window / total not separated / u among the backgrounds / not certified
            const bool lf = need_fb && lead;
            bool uns_g = unsure, bad_g = bad;
            if constexpr (G > 1) {
#pragma unroll
                for (int d = 1; d < G; d <<= 1) {
                    uns_g |= __shfl_xor((int)uns_g, d, 64) != 0;
                    bad_g |= __shfl_xor((int)bad_g, d, 64) != 0;
                }
            }
            const int why = bad_g ? 0 : uns_g ? 5 : ntot == 0 ? 7
                          : !(Mtot > 4.0 * eabs) ? 2 : !(u > delta) ? 3 : 4;
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                const int cnt = __popcll(__ballot(lf && why == r));
                if (cnt && lane == 0) atomicAdd(&sStat[1 + r], (uint32_t)cnt);
            }
        }
        STAMP(7);
        if (keep && !need_fb && lead && !(GS_EXP & 64)) {
            KD(pos_out)[sq] = pk;
            KD(pwms_out)[sq] = pw;
        }
        // targets the bound could not settle: on the exact rescan's list
        const unsigned long long fbm = __ballot(need_fb && lead);
        if (fbm != 0ull && lane == 0) atomicAdd(&sStat[0], (uint32_t)__popcll(fbm));
        STAMP(8);

        // ---- aggregates of the new snapshot: C[a][j] += segment; T[a] = the rank's
        // symbol totals (added once, by the last workgroup's reduction) less every kept
        // segment's symbols and the whole composition of every target left without
        // one here (rescan_target adds composition - segment for those that keep one) ----
        {
            const bool km = lead && keep && !need_fb && pk >= 0 && !(GS_EXP & 4);
            const uint32_t nsw = win;
            const unsigned long long Km = __ballot(km);
            const unsigned long long Fm = __ballot(lead && act && !km);
            if (Km != 0) {
                int cv = 0, segtot[4] = {0, 0, 0, 0};
                for (int j = 0; j < W; ++j) {
                    const unsigned long long b0 = __ballot(km && ((nsw >> (2 * j)) & 1u));
                    const unsigned long long b1 = __ballot(km && ((nsw >> (2 * j + 1)) & 1u));
                    const int c3 = __popcll(b0 & b1), c2 = __popcll(b1 & ~b0), c1 = __popcll(b0 & ~b1);
                    const int c0 = __popcll(Km) - c1 - c2 - c3;
                    segtot[0] += c0;
                    segtot[1] += c1;
                    segtot[2] += c2;
                    segtot[3] += c3;
                    cv = lane == j ? c0 : cv;
                    cv = lane == W + j ? c1 : cv;
                    cv = lane == 2 * W + j ? c2 : cv;
                    cv = lane == 3 * W + j ? c3 : cv;
                }
                if (lane < AW && cv) atomicAdd(&waggC[lane], cv);
                if (lane == 0) {
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        if (e < A && segtot[e]) waggT[e] -= segtot[e];
                }
            }
            STAMP(9);
            if (Fm != 0) {
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    if (e < A) {
                        const int cmp = (lead && act && !km) ? a.comp[(int64_t)sq * (A + 1) + e] : 0;
                        const int t = wave_sum_i32(cmp);
                        if (lane == 0 && t) waggT[e] -= t;
                    }
                }
            }
        }
        wave_sync();
        STAMP(10);
        // ---- targets the bound could not settle: the whole wavefront rescans each
        // exactly (binary64 folds of every window) in its slice, whose lane arrays
        // are dead by now; the new segment goes into the wavefront's aggregates ----
        for (unsigned long long fm = fbm; fm != 0ull; fm &= fm - 1ull) {
            const int sqx = __builtin_amdgcn_readfirstlane(__shfl(sq, __ffsll((long long)fm) - 1, 64));
            rescan_ool<WM>(kargs_dna(), sqx, rng_stream, wslice, tab_off, sPPM, sT, sumT, lane, waggC, waggT);
        }
        STAMP(6);
        TLINE(tl_w, 6);
        tc = tnext;
    }
    // gs_stats: the wavefronts' counts, summed in LDS by the tile loop; one device
    // atomic per nonzero counter and workgroup (after the barrier below)
    STAMP_FLUSH(ntdone);

    // ---- flush: the workgroup's sums into replica blockIdx % 8, one atomic a cell;
    // the last workgroup (a done counter) reduces the replicas ----
    __syncthreads();
    if (tid < 9) {
        // sStat: [0] rescans, [1 + why]: why 0..4 -> stats 2..6, 5..7 -> stats 10..12
        const uint32_t v = sStat[tid];
        if (v) atomicAdd(&(KD(fallbacks) + (blockIdx.x % kRepl) * kStatStride)[tid == 0 ? 0 : tid <= 5 ? tid + 1 : tid + 4], (unsigned long long)v);
    }
    int64_t *dst = KD(rep) + (int64_t)(blockIdx.x % kRepl) * a.stride;
    for (int c = tid; c < cells; c += blockDim.x) {
        int64_t v = 0;
#pragma unroll
        for (int w2 = 0; w2 < nwv; ++w2) {
            const unsigned char *wa = lds + O_WAGG + w2 * WAGG_BYTES;
            v += c < AW ? (int64_t)((const int32_t *)wa)[c] : ((const int64_t *)(wa + 256))[c - AW];
        }
        if (v != 0) GS_FLUSH_ADD((unsigned long long *)&dst[c], (unsigned long long)v);  // (returning: gs_common.h)
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int &s_last = sMisc[8];
    if (tid == 0) {
        // two levels, so that no address takes more than gridDim / 8 + 8 of the
        // serialised same-address atomics: the workgroups of one replica group
        // (blockIdx % 8) count in done[1 + group], the last of them in done[0]
        GS_DONE_FENCE(__ATOMIC_RELEASE);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const int grp = blockIdx.x % kRepl;
        const unsigned int ng = (gridDim.x - grp + kRepl - 1) / kRepl;  // workgroups of the group
        const unsigned int ngroups = min(gridDim.x, (unsigned int)kRepl);
        bool last = false;
        unsigned int *const done = KD(done);
        if (atomicAdd(&done[1 + grp], 1u) == ng - 1) {
            atomicExch(&done[1 + grp], 0u);
            GS_DONE_FENCE(__ATOMIC_ACQ_REL);
            last = atomicAdd(&done[0], 1u) == ngroups - 1;
        }
        s_last = last;
    }
    __syncthreads();
    TLINE(tl_w, 7);
    if (!s_last) return;
    GS_DONE_FENCE(__ATOMIC_ACQUIRE);
    if (tid < kWorkPools) atomicExch(KD(done) + 32 * (1 + tid), 0u);  // the work counters
    // agg_out = the rank's symbol totals (T cells) plus the replicas, which are
    // re-zeroed for the next sweep
    const int64_t *const compsum = KD(compsum);
    int64_t *const rep = KD(rep);
    int64_t *const agg_out = KD(agg_out);
    int64_t xv = 0;  // (the exchange: thread c's cell, cells <= 68 < the workgroup)
    for (int c = tid; c < cells; c += blockDim.x) {
        int64_t v = c >= AW ? compsum[c - AW] : 0;
#pragma unroll
        for (int r = 0; r < kRepl; ++r)
            v += (int64_t)atomicExch((unsigned long long *)&rep[(int64_t)r * a.stride + c], 0ull);
        agg_out[c] = v;
        xv = v;
    }
    if (KD(xpeer)) xch_reduce(kargs_dna(), tid, cells, xv, agg_out, sMisc + 10);
    if (tid == 0) {
        atomicExch(KD(done), 0u);
        unsigned long long *const ctr = KD(sweep_ctr);
        if (ctr) atomicAdd(ctr, 1ull);
    }
}

#ifndef GS_SWEEP_LONG_UNIT  // (gs_sweep_long.hip includes this file for its helpers)
// WM: the motif width rounded up to 8, 12 or 16 (the refinement's pair groups are
// WM / 2, the fold's and the exact rescan's columns WM); G: lanes per target
#define GS_LIVE_FOR_EACH(X) \
    X(8, 1) X(8, 2) X(8, 4) X(8, 8) X(12, 1) X(12, 2) X(12, 4) X(12, 8) X(16, 1) X(16, 2) X(16, 4) X(16, 8)

static const void *live_kernel_ptr(int wm, int g) {
#define GS_CASE(W_, G_) \
    if (wm == W_ && g == G_) return (const void *)&gs_sweep_live_kernel<W_, G_>;
    GS_LIVE_FOR_EACH(GS_CASE)
#undef GS_CASE
    return nullptr;
}

int gs_live_wm(int W) { return W <= 8 ? 8 : W <= 12 ? 12 : 16; }

int gs_live_lds_bytes(int Lmax, int W, int G, int waves) {
    return O_WAVE + waves * live_slice_bytes(Lmax, W, G, gs_live_wm(W));
}

hipError_t gs_live_occupancy(int *blocks_per_cu, int W, int G, int Lmax, int waves) {
    const void *k = live_kernel_ptr(gs_live_wm(W), G);
    if (!k) return hipErrorInvalidValue;
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, k, 64 * waves,
                                                        (size_t)gs_live_lds_bytes(Lmax, W, G, waves));
}

// The live sweep: grid workgroups of `waves` wavefronts; start / stop: events
// around the dispatch (profiling), or null.
hipError_t gs_live_launch(const DnaArgs &a, int G, int grid, int waves, hipStream_t stream, hipEvent_t start,
                          hipEvent_t stop) {
    const void *k = live_kernel_ptr(gs_live_wm(a.W), G);
    if (!k || waves < 1 || waves > kLiveWaves) return hipErrorInvalidValue;
    DnaArgs args = a;
    args.live_slice = live_slice_bytes(a.Lmax, a.W, G, gs_live_wm(a.W));
    const size_t lds = (size_t)gs_live_lds_bytes(a.Lmax, a.W, G, waves);
    void *params[] = {&args};
    if (!start) return hipLaunchKernel(k, dim3(grid), dim3(64 * waves), params, lds, stream);
    return hipExtLaunchKernel(k, dim3(grid), dim3(64 * waves), params, lds, stream, start, stop, 0);
}
#endif  // GS_SWEEP_LONG_UNIT
