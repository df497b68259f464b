// gs_sweep_long.hip — the synchronous Gibbs sweep of a live chain over long DNA
// sequences on gfx950 (BASELINE config 3: 100k x 500 bp, W = 15).
//
// MotifSampler.findBestMotifIndicesByWithStartPositions (.fs:935-970) with
// motifAmount = 1, for the packed layout of gs_sweep_dna.hip (at most 4 symbols, no
// other symbol in the data, W <= 16) and sequences of at most 16 x 32 windows.
//
// Why another kernel: the per-lane kernels (gs_sweep_dna.hip, gs_sweep_live.hip)
// give one target one lane (or a few), which at config 3 leaves 1.5 wavefronts per
// SIMD (100k targets / 64) and repeats each target's fixed work in every lane that
// shares it; their window scores are filters that need a per-target refinement or a
// per-lane fine table.  Here one DPP row of 16 lanes owns one target:
//
//  1. the target's hold-one-out PCV (.fs:945-954, .fs:109-120) by 4 lanes, its log2
//     from a per-workgroup table of log2(T[a] + s + pc) (s = own-segment count);
//  2. its EXACT fixed-point table of log2 PWM' pair sums (.fs:255-260, .fs:955-965):
//     entry (pair code c, column pair g) = round((log2 PPM'[s0][2g] - log2 PCV[s0]) +
//     (log2 PPM'[s1][2g+1] - log2 PCV[s1])) at 2^-kPU, lane c of the row building code
//     c's entries (the own segment's count-minus-one cells where it matches), clamped
//     below at a floor under which no window can pass the cut-off;
//  3. lane q scores its share of the windows, K / 16 consecutive ones (one more in the
//     first K % 16 lanes, at most 32), with a sliding ring over positions: the NG / 2
//     parts (two column pairs each) of the row of the position's pair code, read with
//     ds_read_b64 from the target's table -- a 16-lane group reads one target's
//     128-byte part and the targets of a 32-lane half sit in opposite bank halves, so
//     the reads are conflict-free -- and added into the windows that see the position
//     (every window's exact integer sum, within NG 2^-(kPU+1) of the reference's
//     log2 S_k);
//  4. the cut-off test (.fs:735) and the passing windows' sum per lane, the row's
//     prefix sums (DPP), the certified pick (.fs:746-754) located in one lane's
//     8-window block and re-evaluated there, the picked window's weight the
//     reference's binary64 fold of PPM'/PCV (.fs:283-292) and log2 (.fs:737) -- the W
//     quotients computed by W lanes of the row;
//  5. targets the bound cannot settle (a window within the bound of the cut-off, a
//     pick within it of a CDF boundary) are rescanned exactly by the whole wavefront
//     (gs_sweep_live.hip rescan_target); targets without a passing window take the
//     background walk (bg_pick); aggregates, flush and done counter as the live sweep.
//
// Compiled with -ffp-contract=off: no FMA contraction.
#define GS_SWEEP_LONG_UNIT
#include "gs_sweep_live.hip"

namespace {

constexpr int kLongWaves = 8;   // wavefronts per workgroup (the host may launch fewer, >= 2)
#ifndef GS_LONG_WAVES_PER_EU
#define GS_LONG_WAVES_PER_EU 3
#endif
#ifndef GS_LONG_TL_IT
#define GS_LONG_TL_IT 1  // the iteration the timeline variant marks (its second: caches warm)
#endif
// Lanes a target.  16 (default): a 16-lane group of the ring's ds_read2_b64 (4 x 16
// lanes, banks (a / 4) mod 32) reads one target's 128-byte table part, conflict-free.
// 8 (-DGS_LONG_LPT=8, measured): 23 % fewer VALU (the per-target work on half the lanes)
// but two targets' tables under one group's banks: 8x the bank-conflict cycles, the
// same time (config 3: 86.6 vs 86.8 us).
#ifndef GS_LONG_LPT
#define GS_LONG_LPT 16
#endif
constexpr int kLpt = GS_LONG_LPT;       // lanes a target (8 or 16)
constexpr int kTpw = 64 / kLpt;         // targets a wavefront iteration
constexpr unsigned long long kSegMask = (1ull << kLpt) - 1ull;
constexpr int kLongRn = 512 / kLpt;     // windows a lane owns at most: K <= 512
constexpr int kLongBw = 8;              // windows per block of the lane's prefix sums
constexpr int kRawWords = kLpt == 16 ? 4 : 6;  // packed words a lane loads (from x0's word)
constexpr int kLW = kLpt == 16 ? 3 : 5;        // its words kept in LDS for the pick
static_assert(kLpt == 8 || kLpt == 16, "lanes a target");
// LDS carve: the live sweep's workgroup part up to its refinement table (C, T, PPM,
// their logs, misc, stats, wavefront aggregates), then the PCV log table, then one
// slice per wavefront
constexpr int O_LTAB = O_RT;    // double [4][17] log2(T[a] + s + pc), s = 0..16; [68] log2(sum T + W + A pc)
constexpr int O_LWAVE = (O_LTAB + 8 * 69 + 255) & ~255;
// inside a slice (the exact rescan's staging reuses it from 0 after the picks)
constexpr int L_TAB = 0;        // the targets' tables: part p of target t at 1024 (t >> 1) + 256 p + 128 (t & 1)
constexpr int L_BSUM = 512 * kTpw;  // int64 [blocks][64 lanes]: the lane's passing sum at each block's end
constexpr int L_WORDS = L_BSUM + 8 * 64 * (kLongRn / kLongBw);  // uint32 [kLW][64 lanes]: the lane's words
constexpr int L_TSCR = (L_WORDS + 256 * kLW + 255) & ~255;  // per target, 256 B: pcv[4] @ 0, log2 PCV[4] @ 32, factors @ 64
constexpr int kLongSliceMin = L_TSCR + kTpw * 256;
static_assert(kLongSliceMin % 256 == 0 && O_LWAVE % 256 == 0, "carve");
static_assert(L_BSUM + 8 * 64 * (kLongRn / kLongBw) <= L_WORDS, "block sums");

// Segmented scans over the kLpt lanes of a target (q = lane % kLpt): DPP row shifts,
// a source in another target's segment (kLpt = 8: the row's other half) adding 0
template <int CTRL, int N>
__device__ __forceinline__ int64_t seg_step_i64(int64_t x, int q) {
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)x, CTRL, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)((uint64_t)x >> 32), CTRL, 0xf, 0xf, true);
    const int64_t v = (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
    return x + ((kLpt < 16 && q < N) ? (int64_t)0 : v);
}
__device__ __forceinline__ int64_t seg_scan_i64_t(int64_t x, int q) {
    x = seg_step_i64<0x111, 1>(x, q);
    x = seg_step_i64<0x112, 2>(x, q);
    x = seg_step_i64<0x114, 4>(x, q);
    if constexpr (kLpt == 16) x = seg_step_i64<0x118, 8>(x, q);
    return x;
}
template <bool MAX>
__device__ __forceinline__ int seg_scan_i32_t(int v, int q) {
#define GS_SEG_I32(CTRL, N)                                                         \
    {                                                                               \
        int u_ = __builtin_amdgcn_update_dpp(0, v, CTRL, 0xf, 0xf, true);           \
        if (kLpt < 16 && q < N) u_ = 0;                                             \
        v = MAX ? max(v, u_) : v + u_;                                              \
    }
    GS_SEG_I32(0x111, 1)
    GS_SEG_I32(0x112, 2)
    GS_SEG_I32(0x114, 4)
    if constexpr (kLpt == 16) GS_SEG_I32(0x118, 8)
#undef GS_SEG_I32
    return v;
}
__device__ __forceinline__ double seg_scan_f64_t(double x, int q) {
#define GS_SEG_F64(CTRL, N)                                                         \
    {                                                                               \
        double u_ = dpp_f64<CTRL, 0xf>(x);                                          \
        if (kLpt < 16 && q < N) u_ = 0.0;                                           \
        x = x + u_;                                                                 \
    }
    GS_SEG_F64(0x111, 1)
    GS_SEG_F64(0x112, 2)
    GS_SEG_F64(0x114, 4)
    if constexpr (kLpt == 16) GS_SEG_F64(0x118, 8)
#undef GS_SEG_F64
    return x;
}

// The value of the target's last lane (q = kLpt - 1) in every lane of its segment: the
// row totals of the scans above.  kLpt = 16 (one DPP row a target): DPP row_newbcast:15
// (control 0x15F on gfx950, checked by tools/probe/dpp_newbcast.hip), one VALU a dword
// and no LDS round trip; kLpt = 8: ds_bpermute from that lane
__device__ __forceinline__ int row_last_i32(int v, int gbase) {
    if constexpr (kLpt == 16) return __builtin_amdgcn_update_dpp(0, v, 0x15F, 0xf, 0xf, false);
    else return bperm_i32(v, gbase + kLpt - 1);
}
__device__ __forceinline__ int64_t row_last_i64(int64_t x, int gbase) {
    const uint32_t lo = (uint32_t)row_last_i32((int)(uint32_t)x, gbase);
    const uint32_t hi = (uint32_t)row_last_i32((int)(uint32_t)((uint64_t)x >> 32), gbase);
    return (int64_t)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ double row_last_f64(double x, int gbase) {
    return __hiloint2double(row_last_i32(__double2hiint(x), gbase), row_last_i32(__double2loint(x), gbase));
}

// The LDS address of the row of position P's pair code (P static; position 0 = the
// lane's first window, symbol i at bits 2 (i % 16) of w[i / 16]): the target's table
// (128-aligned) or'd with code * 8 -- two VALU
template <int P>
__device__ __forceinline__ uint32_t row_addr(const uint32_t (&w)[kRawWords], uint32_t tabv) {
    constexpr int wi = P >> 4, r = P & 15;
    if constexpr (r >= 2)
        return (__builtin_amdgcn_alignbit(w[wi + 1], w[wi], 2 * r - 3) & 0x78u) | tabv;
    else
        return (__builtin_amdgcn_ubfe(w[wi], 2 * r, 4) << 3) | tabv;
}

// The table row (NP parts of two int32 entries) at LDS address ra.
template <int NP>
struct Row {
    uint2 e[NP];
};
template <int NP>
__device__ __forceinline__ Row<NP> load_row(uint32_t ra) {
    typedef __attribute__((address_space(3))) const uint2 lds_u2;
    Row<NP> r;
#pragma unroll
    for (int p = 0; p < NP; ++p) r.e[p] = *(const uint2 *)(lds_u2 *)(size_t)(ra + 256 * p);
    return r;
}

// One ring step (position P, static) and the rest of the scan by recursion: position
// P adds its row's part entries into the windows P - 2g that see it as column pair g;
// window k completes at position k + 2 (NG - 1).  Per window: the cut-off test
// against the target's thresholds (passing: > thr_hi; in the band: in [thr_lo,
// thr_hi], tracked as the least unsigned sc - thr_lo), the passing sum (non-negative
// scores, bits 0..47 of M) and count (bits 48..63: one 64-bit add for both), and M at
// the end of every 8-window block into the lane's block prefixes (LDS, [b][64 lanes]).
// Windows k < KU are in every lane's range (the caller checked the wave's
// least nwin), the rest are tested against nwin.  The rows of position P + PD are
// requested before position P is added.
template <int NG, int PD, int P, int NPOS, int KU>
__device__ __forceinline__ void long_steps(int (&R)[2 * NG], Row<NG / 2> (&rows)[PD], const uint32_t (&w)[kRawWords],
                                           uint32_t tabv, int nwin, int thr_hi, int thr_lo, uint64_t *bsum,
                                           uint64_t &M, uint32_t &dmin) {
    if constexpr (P < NPOS) {
        constexpr int RS = 2 * NG;
        const Row<NG / 2> cur = rows[P % PD];
        if constexpr (P + PD < NPOS) rows[P % PD] = load_row<NG / 2>(row_addr<P + PD>(w, tabv));
        R[P % RS] = (int)cur.e[0].x;
#pragma unroll
        for (int g = 1; g < NG; ++g) {
            const uint2 pe = cur.e[g >> 1];
            R[(P - 2 * g + 4 * RS) % RS] += (int)((g & 1) ? pe.y : pe.x);
        }
        constexpr int k = P - 2 * (NG - 1);
        if constexpr (k >= 0) {
            const int sc = R[k % RS];
            bool pass = sc > thr_hi;
            uint32_t d = (uint32_t)sc - (uint32_t)thr_lo;  // (unsigned: the same bits, no signed overflow)
            if constexpr (k >= KU) {
                const bool valid = k < nwin;
                pass = pass && valid;
                d = valid ? d : 0xffffffffu;
            }
            dmin = min(dmin, d);
            M += pass ? ((1ull << 48) | (uint32_t)sc) : 0ull;
            if constexpr (k % kLongBw == kLongBw - 1) bsum[64 * (k / kLongBw)] = M;
        }
        // (the pipeline depth is PD positions: the scheduler would otherwise hoist the
        // table reads of many positions, each holding NG registers)
        __builtin_amdgcn_sched_barrier(0);
        long_steps<NG, PD, P + 1, NPOS, KU>(R, rows, w, tabv, nwin, thr_hi, thr_lo, bsum, M, dmin);
    }
}

// The lane's windows [0, nwin), nwin <= RNW, every lane's nwin >= KU.
template <int NG, int RNW, int KU>
__device__ __forceinline__ void long_scan(const uint32_t (&w)[kRawWords], uint32_t tabv, int nwin, int thr_hi,
                                          int thr_lo, uint64_t *bsum, uint64_t &M, uint32_t &dmin) {
    constexpr int PD = 2, NPOS = RNW + 2 * (NG - 1);
    static_assert(NPOS <= 16 * (kRawWords - 1), "the lane's words");
    int R[2 * NG];
#pragma unroll
    for (int i = 0; i < 2 * NG; ++i) R[i] = 0;
    Row<NG / 2> rows[PD];
    rows[0] = load_row<NG / 2>(row_addr<0>(w, tabv));
    rows[1] = load_row<NG / 2>(row_addr<1>(w, tabv));
    long_steps<NG, PD, 0, NPOS, KU>(R, rows, w, tabv, nwin, thr_hi, thr_lo, bsum, M, dmin);
}

// The exact rescan out of line (a cold path: its registers stay out of the scan's);
// the kernel arguments through the kernarg segment the kernel passes (made
// wave-uniform here, so its fields are scalar loads; a reference to the kernel's
// by-value argument would copy the whole struct to scratch).
template <int WM>
__device__ __attribute__((noinline)) void long_rescan(KDnaArgs *ka_in, int sq, uint64_t rng_stream,
                                                      unsigned char *wslice, int tab_off, const double2 *sPPM,
                                                      const int64_t *sT, int64_t sumT, int lane, int32_t *waggC,
                                                      int64_t *waggT) {
    const uint64_t pv = (uint64_t)ka_in;
    const uint64_t pu = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(pv >> 32)) << 32) |
                        (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)pv);
    KDnaArgs *ka = (KDnaArgs *)pu;
    rescan_target<WM, true, KDnaArgs>(*ka, sq, rng_stream, wslice, tab_off, sPPM, sT, sumT, lane, waggC, waggT);
}

// A target without a passing window on the long sweep's row (gs_sweep_live.hip bg_pick's
// walk, specialised): its categories are the K background products alone (.fs:759-784),
// each the reference's binary64 fold of PCV over the window (.fs:123-124), by incremental
// products (window k's from window k - 1's, times PCV of the entering symbol and 1 / PCV
// of the leaving one: the same operations, so the same values, in both passes); the
// row's total, then u times it located among the windows in order, certified with
// gs_sweep_bg.hip's margins; the picked window's weight is its exact fold.  Unrolled
// over the lane's NW windows at most, keeping the product at each BB-window block's
// start and the running sum at its end, so the locating lane walks one block (BB
// windows) instead of its whole range again.  Out of line: the uniform-start sweep's
// path, kept off the scan's registers.
template <int G, int NW>
__device__ __attribute__((noinline)) BgPick bg_pick_row(const uint32_t *words, uint32_t wmask, int W, int K,
                                                       int nwin, bool bgo, double u, int part, int gbase,
                                                       double p0, double p1, double p2, double p3) {
    constexpr int BB = 4, NB = NW / BB;
    static_assert(NW % 16 == 0, "16-window symbol blocks");
    const double pc4[4] = {p0, p1, p2, p3};
    auto pcv_of = [&](uint32_t e) {
        const double lo = (e & 1u) ? pc4[1] : pc4[0], hi = (e & 1u) ? pc4[3] : pc4[2];
        return (e & 2u) ? hi : lo;
    };
    // 1 / PCV by v_rcp_f64 and two Newton steps (within 2^-52 relative, as gs_pick.h's
    // total: one rounding more a step than a division's, counted in rel below)
    double inv[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const double p = pc4[e];
        double x = __builtin_amdgcn_rcp(p);
        x = fma(x, fma(-p, x, 1.0), x);
        inv[e] = fma(x, fma(-p, x, 1.0), x);
    }
    auto inv_of = [&](uint32_t e) {
        const double lo = (e & 1u) ? inv[1] : inv[0], hi = (e & 1u) ? inv[3] : inv[2];
        return (e & 2u) ? hi : lo;
    };
    auto sym16 = [&](int q) {  // the 16 symbols from position q of the lane's range
        return funnel(words[64 * ((q >> 4) + 1)], words[64 * (q >> 4)], 2 * (q & 15));
    };
    auto fold_pcv = [&](int k) {  // the reference's fold of window k (exact)
        const uint32_t wk = sym16(k) & wmask;
        double g = 1.0;
        for (int j = 0; j < W; ++j) g = g * pcv_of((wk >> (2 * j)) & 3u);
        return g;
    };
    double gst[NB], cum[NB];
    double Bl = 0.0;
    if (bgo && nwin > 0) {
        double g = fold_pcv(0);
        uint32_t in = 0u, out = 0u;
#pragma unroll
        for (int k = 0; k < NW; ++k) {
            if ((k & 15) == 0) {
                in = sym16(k + W - 1);
                out = k > 0 ? sym16(k - 1) : words[0] << 2;
            }
            if (k > 0) g = g * pcv_of(__builtin_amdgcn_ubfe(in, 2 * (k & 15), 2)) * inv_of(__builtin_amdgcn_ubfe(out, 2 * (k & 15), 2));
            if (k % BB == 0) gst[k / BB] = g;
            if (k < nwin) Bl = Bl + g;
            if (k % BB == BB - 1) cum[k / BB] = Bl;
        }
    }
    double incl = Bl;
#pragma unroll
    for (int dd = 1; dd < G; dd <<= 1) {
        const double v = __shfl_up(incl, dd, 64);
        if (part >= dd) incl = incl + v;
    }
    const double Bpre = incl - Bl;
    static_assert(G == kLpt, "the row's segment");
    const double Tt = row_last_f64(incl, gbase);
    // each product within (5W + 4K + 20) 2^-53 of the reference's fold (four roundings
    // a step with the Newton reciprocals), the sums' and the group scan's roundings, the
    // roulette's own: gs_sweep_bg.hip's margins.  The certification's own quotients by
    // reciprocals (2^-46 relative after one Newton step), the bound widened by 2^-40
    const double rel = (double)(5 * W + 4 * K + 20) * 0x1.0p-53 * (1.0 + 0x1.0p-10);
    const double eb = Tt * rel + Tt * (double)(4 * G + 64) * 0x1.0p-53;
    const double ncb = (double)(K + 2);
    const bool okb = bgo && Tt > 4.0 * eb && Tt < INFINITY;
    double rt = __builtin_amdgcn_rcp(Tt);
    rt = fma(rt, fma(-Tt, rt, 1.0), rt);
    const double dm = Tt - eb;
    double rd = __builtin_amdgcn_rcp(dm);
    rd = fma(rd, fma(-dm, rd, 1.0), rd);
    const double d2 = (8.0 * ncb + 64.0) * 0x1.0p-53 + eb * rt * (1.0 + (Tt + eb) * rd) * (1.0 + 0x1.0p-40);
    const double Ub = u * Tt, Db = d2 * Tt, Tb = Ub - Db;
    BgPick r{false, 0.0};
    if (okb && Bpre + Bl >= Tb && (part == 0 || Bpre < Tb)) {
        // the first block whose running sum reaches u Tt - D ...
        int kb = (NB - 1) * BB;
        double g = gst[NB - 1], P = Bpre + (NB > 1 ? cum[NB - 2] : 0.0);
#pragma unroll
        for (int b = NB - 1; b >= 0; --b) {
            if (b * BB < nwin && Bpre + cum[b] >= Tb) {
                kb = b * BB;
                g = gst[b];
                P = Bpre + (b > 0 ? cum[b - 1] : 0.0);
            }
        }
        // ... then its windows in order, from the block's first product
        for (int k = kb; k < kb + BB && k < nwin; ++k) {
            if (k > kb) g = g * pcv_of(sym16(k + W - 1) & 3u) * inv_of(sym16(k - 1) & 3u);
            const double lo = P;
            P = P + g;
            if (P < Tb) continue;
            r.ok = Ub >= lo + Db && Ub <= P - Db;
            r.pw = fold_pcv(k);  // the picked category's weight: the exact fold
            break;
        }
    }
    return r;
}

// Window k's exact integer score (k dynamic; its 16 symbols from position k in x16):
// the same entries and sums as the scan.
template <int NG>
__device__ __forceinline__ int long_eval(uint32_t x16, const unsigned char *tab) {
    int v[NG];
#pragma unroll
    for (int g = 0; g < NG; ++g)
        v[g] = *(const int32_t *)(tab + (__builtin_amdgcn_ubfe(x16, 4 * g, 4) << 3) + 256 * (g >> 1) + 4 * (g & 1));
    int s = 0;
#pragma unroll
    for (int g = 0; g < NG; ++g) s += v[g];
    return s;
}

}  // namespace

template <int WM>
__global__ void __launch_bounds__(64 * kLongWaves, GS_LONG_WAVES_PER_EU) gs_sweep_long_kernel(DnaArgs a) {
    constexpr int NG = WM / 2;  // column pairs of the motif (W <= WM)
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int A = a.A, W = a.W;
    const int AW = A * W, cells = KD(cells);
    int32_t *sC = (int32_t *)(lds + O_C);
    int64_t *sT = (int64_t *)(lds + O_T);
    double2 *sPPM = (double2 *)(lds + O_PPM);
    double *sL64 = (double *)(lds + O_L64);
    double *sLT = (double *)(lds + O_LTAB);
    int32_t *sMisc = (int32_t *)(lds + O_MISC);
    uint32_t *sStat = (uint32_t *)(lds + O_STAT);
    const int slice = KD(live_slice);
    unsigned char *wslice = lds + O_LWAVE + wid * slice;
    int32_t *waggC = (int32_t *)(lds + O_WAGG + wid * WAGG_BYTES);
    int64_t *waggT = (int64_t *)(lds + O_WAGG + wid * WAGG_BYTES + 256);
    // this lane's target slot t (kLpt lanes of a DPP row) and its place q in it
    const int t = lane / kLpt, q = lane & (kLpt - 1), gbase = lane & ~(kLpt - 1);
    const unsigned char *tab = wslice + L_TAB + 1024 * (t >> 1) + 128 * (t & 1);
    double *tpcv = (double *)(wslice + L_TSCR + 256 * t);  // [0..3] pcv, [4..7] log2 pcv, [8..] factors
    uint64_t *bsum = (uint64_t *)(wslice + L_BSUM) + lane;
    uint32_t *const lw0 = (uint32_t *)(wslice + L_WORDS);

    const int tl_w = blockIdx.x * (blockDim.x >> 6) + wid;  // (timeline marks: stamps build)
    (void)tl_w;
    TLINE(tl_w, 0);
    const int err0 = __hip_atomic_load(a.err_code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t rng_stream = KD(sweep_ctr) ? stream_sweep(*KD(sweep_ctr)) : 0;

    // ---- prologue: the snapshot's aggregates and the workgroup tables ----
    waggC[lane] = 0;
    if (lane < 4) waggT[lane] = 0;
    if (tid < 12) sStat[tid] = 0u;
    // (slots 10, 11: the exchange count so far, read now so the last workgroup's
    // exchange starts without a global round trip; xch_reduce)
    if (tid < 16) sMisc[tid] = (tid == 10 || tid == 11) && KD(xpeer) ? (int)(uint32_t)(*KD(xseq) >> (tid == 11 ? 32 : 0)) : 0;
    snapshot_tables(a, sC, sT, sPPM, sL64, sMisc, tid);
    const bool void_snap = __builtin_amdgcn_readfirstlane(err0) != 0;
    if (blockIdx.x == 0 && KD(bg_note)) {
        const bool bg = bg_regime(sC, sT, A, W, KD(pc), KD(den), KD(apc), KD(Lmax), KD(cmin), KD(cutoff),
                                  (double *)(lds + O_LWAVE), tid);
        if (tid == 0) *KD(bg_note) = bg ? 1 : 0;
    }
    // log2(T[a] + s + pc) for the own-segment counts s = 0..W and log2(sum T + W + A pc):
    // log2 of a motif-bearing target's hold-one-out PCV (.fs:119) is a difference of two
    // (the division's rounding is below 2^-52 in the log)
    for (int i = tid; i <= 4 * (W + 1); i += blockDim.x) {
        double v = 0.0;
        if (i < 4 * (W + 1)) {
            const int e = i / (W + 1), s = i - e * (W + 1);
            if (e < A) v = log2((double)(sT[e] + s) + KD(pc));
            sLT[e * 17 + s] = v;
        } else {
            v = log2(((double)sT[4] + (double)W) + KD(apc));
            sLT[68] = v;
        }
        if (!(fabs(v) < 60.0)) sMisc[1] = 1;
    }
    __syncthreads();
    // (a negative cut-off lets negative weights pass: the certified pick assumes
    // non-negative ones, so every target goes to the exact rescan)
    const bool table_fault = sMisc[1] != 0 || !(fabs(KD(cutoff)) < 1000.0) || KD(cutoff) < 0.0 ||
#if defined(__HIP_DEVICE_COMPILE__)
                             (uint32_t)(size_t)(__attribute__((address_space(3))) unsigned char *)lds != 0u ||
#endif
                             false;
    const int64_t sumT = sT[4];
    TLINE(tl_w, 1);

    // ---- this wavefront's targets: a contiguous range, workgroups numbered XCD-major;
    // four targets (one a row) an iteration, handed out by kWorkPools work counters ----
    // Static shares leave the tail to the wavefronts the SIMD arbiter serves last (a
    // CU's third workgroup iterates ~35 % slower than its first), so the workgroups of
    // pool P (XCD blockIdx % 8, half (blockIdx / 8) & 1) share its range of targets by
    // batches of four, in pairs: a wavefront's first pair is its rank in the pool, each
    // next one comes from the pool's counter (one device-scope atomic at the start of
    // the pair's second batch; the next batch's descriptor is loaded after the current
    // one's scan, its words with it or after its pick).
    const int nwv = blockDim.x >> 6;
    const int xcd = blockIdx.x % kRepl, q8 = gridDim.x / kRepl, r8 = gridDim.x % kRepl;
    const int half = (int)(blockIdx.x / kRepl) & 1;
    const int nwaves = gridDim.x * nwv;
    const int qn = KD(n_local) / nwaves, rn = KD(n_local) % nwaves;
    int X0, cnt;
    {
        const int nbx = q8 + (xcd < r8 ? 1 : 0);
        const int r0 = xcd * q8 + min(xcd, r8) + (half ? (nbx + 1) >> 1 : 0);
        const int rc = half ? nbx >> 1 : (nbx + 1) >> 1;
        const int lw0 = r0 * nwv, lw1 = (r0 + rc) * nwv;
        X0 = lw0 * qn + min(lw0, rn);
        cnt = void_snap ? 0 : lw1 * qn + min(lw1, rn) - X0;
    }
    const int nb = (cnt + kTpw - 1) / kTpw;
    const int nwp = (half ? (q8 + (xcd < r8 ? 1 : 0)) >> 1 : (q8 + (xcd < r8 ? 1 : 0) + 1) >> 1) * nwv;
    const int wrank = ((int)(blockIdx.x / kRepl) >> 1) * nwv + wid;
    unsigned int *const wctr = KD(done) + 32 * (1 + 2 * xcd + half);
    const int tab_off = live_tab_off(a.Lmax, WM);
    const uint32_t wmask = W >= 16 ? 0xffffffffu : ((1u << (2 * W)) - 1u);

    struct Desc {
        int L, p;
        int64_t wo;
    };
    auto load_desc = [&](int b) {
        const int s = kTpw * b + t;
        const int sq = X0 + min(s, cnt - 1);
        // audit (gs_stats [13]); wave-uniform calls
        const unsigned long long oob = __ballot((unsigned)sq >= (unsigned)KD(n_local));
        if (oob && lane == 0)
            atomicAdd(&(KD(fallbacks) + (blockIdx.x % kRepl) * kStatStride)[13], (unsigned long long)__popcll(oob));
        Desc d;
        d.L = KD(len)[sq];
        d.p = s < cnt ? KD(pos_in)[sq] : -1;
        d.wo = KD(pkoff)[sq];
        return d;
    };
    // the loads that depend on a target's descriptor (the lane's words) are issued a
    // batch ahead (the own segment comes from the lane words that hold it)
    struct Pre {
        uint4 w4;
        uint2 w2;  // (kLpt = 8: two more words)
    };
    auto words_at = [&](const uint32_t *src) {
        Pre r;
        r.w4 = load_words(src);  // (the zero tail covers reads past L)
        r.w2 = make_uint2(0u, 0u);
        if constexpr (kRawWords > 4) __builtin_memcpy(&r.w2, src + 4, 8);
        return r;
    };
    auto load_pre = [&](const Desc &d, int b) {
        const int s = kTpw * b + t;
        const int Lp = s < cnt ? d.L : W, Kp = Lp - W + 1;
        const int xp = q * (Kp / kLpt) + min(q, Kp % kLpt);
        return words_at(KD(pk) + d.wo + (xp >> 4));
    };
    // every sequence Lmax long, pkoff[n] = n pk_stride: the words need no descriptor,
    // so they are requested with it (no dependent round trip within the batch)
#ifdef GS_LONG_NO_STRIDE  // (timing experiments: the ragged path)
    const int pks = 0;
#else
    const int pks = KD(pk_stride);
#endif
    auto load_pre_s = [&](int b) {
        const int s = kTpw * b + t;
        const int sq = X0 + min(s, cnt - 1);
        const int Lp = s < cnt ? KD(Lmax) : W, Kp = Lp - W + 1;
        const int xp = q * (Kp / kLpt) + min(q, Kp % kLpt);
        return words_at(KD(pk) + (int64_t)sq * pks + (xp >> 4));
    };
    // the next batch of the pool (lane 0's atomic; its value read later in the batch)
    auto grab = [&]() -> int {
        int v = 0;
        if (lane == 0) v = (int)atomicAdd(wctr, 1u);
        return v;
    };
    // batches go in pairs (pair v = batches 2v, 2v + 1): one atomic every other batch
    int bc = 2 * wrank < nb ? 2 * wrank : nb;
    Desc dd{0, -1, 0};
    Pre cur{make_uint4(0u, 0u, 0u, 0u), make_uint2(0u, 0u)};
    if (bc < nb) {
        dd = load_desc(bc);
        cur = load_pre(dd, bc);
    }
    for (int it = 0; bc < nb; ++it) {
        // the second batch of bc's pair, else the next pair from the pool
        const bool need = (bc & 1) != 0 || bc + 1 >= nb;
        const int gpend = need ? grab() : 0;
        int bn = nb;
        Desc dn{0, -1, 0};
        Pre pn{make_uint4(0u, 0u, 0u, 0u), make_uint2(0u, 0u)};
        const int s = kTpw * bc + t;
        const bool act = s < cnt;
        const int sq = X0 + min(s, cnt - 1);
        const int64_t gidx = KD(global_offset) + sq;
        const int L = act ? dd.L : W;
        const int p = dd.p;
        bool keep = act;
        const int64_t tot = sumT + (p >= 0 ? W : L);
        if (act && tot > 2147483647LL) {  // Checked Array.sum (.fs:117)
            if (q == 0) raise_error(a, 3, gidx);
            keep = false;
        }
        const int K = L - W + 1;
        // lane q's windows [x0, x0 + nwin): K / kLpt each and one more in the first
        // K % kLpt lanes; its words from x0 (the words from x0's, shifted)
        const int x0 = q * (K / kLpt) + min(q, K % kLpt), nwin = K / kLpt + (q < K % kLpt ? 1 : 0);
        const int shx = 2 * (x0 & 15);
        uint32_t w[kRawWords];
        {
            const uint32_t raw[6] = {cur.w4.x, cur.w4.y, cur.w4.z, cur.w4.w, cur.w2.x, cur.w2.y};
#pragma unroll
            for (int i = 0; i < kRawWords; ++i) w[i] = funnel(i + 1 < kRawWords ? raw[i + 1] : 0u, raw[i], shx);
        }
        // the target's own segment (snapshot position p < K): symbols p .. p + W - 1 from
        // the words of the lane whose range holds p (p - x0 < kLongRn: within its words)
        uint32_t gw = 0u;
        bool gw_miss = false;
        {
            const int dp = p - x0;
            const bool holds = p >= 0 && dp >= 0 && dp < nwin;
            const int di = (dp >> 4) & 3;
            uint32_t lo = w[0], hi = w[1];
#pragma unroll
            for (int i = 1; i < kRawWords - 1 && i < 4; ++i) {
                lo = di == i ? w[i] : lo;
                hi = di == i ? w[i + 1] : hi;
            }
            const uint32_t cand = funnel(hi, lo, 2 * (dp & 15));
            const unsigned long long hm = (__ballot(holds) >> gbase) & kSegMask;
            const int hsrc = hm ? gbase + __ffsll((long long)hm) - 1 : lane;
            const uint32_t gv = (uint32_t)bperm_i32((int)cand, hsrc);
            gw = (p >= 0 && hm) ? gv & wmask : 0u;
            gw_miss = p >= 0 && hm == 0ull;  // (a position outside [0, K): the exact rescan)
        }

        // ---- hold-one-out PCV (.fs:945-954, .fs:109-120), lanes q < 4: symbol q ----
        bool bad_e = false;
        if (q < 4) {
            double pv = 1.0, lp = 0.0;
            if (q < A) {
                const int sc = p >= 0 ? sym_count(gw, q, wmask) : 0;
                const int64_t bgc = sT[q] + (p >= 0 ? sc : KD(comp)[(int64_t)sq * (A + 1) + q]);
                pv = ((double)bgc + KD(pc)) / ((double)tot + KD(apc));
                lp = p >= 0 ? sLT[q * 17 + sc] - sLT[68] : log2(pv);
                bad_e = !(pv > 0.0) || !(fabs(lp) < 60.0);
            }
            tpcv[q] = pv;
            tpcv[4 + q] = lp;
        }
#pragma unroll
        for (int i = 0; i < kLW; ++i) lw0[64 * i + lane] = w[i];
        bool bad = table_fault || (bool)KD(live_force) || nwin > kLongRn || gw_miss || ((__ballot(bad_e) >> gbase) & kSegMask) != 0;
        wave_sync();
        if (it == GS_LONG_TL_IT) TLINE(tl_w, 2);

        // ---- the target's table: lane q builds pair codes q + kLpt i's entries ----
        // entry (c, g) = t[s0][2g] + t[s1][2g + 1], t[e][j] = log2 PPM'[e][j] - log2 PCV[e]
        // (the count-minus-one cell where the own segment has e in column j); columns
        // past W add 0
        constexpr int CPL = 16 / kLpt;  // codes a lane
        double v[CPL][NG];
        double mx = 0.0;
#pragma unroll
        for (int ci = 0; ci < CPL; ++ci) {
            const int c = q + kLpt * ci;
            const int s0 = c & 3, s1 = c >> 2;
            const double lp0 = tpcv[4 + s0], lp1 = tpcv[4 + s1];
            // the own segment's columns holding s0 (s1): bit 2j of eq0 (eq1)
            const uint32_t xs0 = gw ^ (0x55555555u * (uint32_t)s0), xs1 = gw ^ (0x55555555u * (uint32_t)s1);
            const uint32_t eq0 = p >= 0 ? ~(xs0 | (xs0 >> 1)) & 0x55555555u : 0u;
            const uint32_t eq1 = p >= 0 ? ~(xs1 | (xs1 >> 1)) & 0x55555555u : 0u;
#pragma unroll
            for (int g = 0; g < NG; ++g) {
                // (selects, not branches: the log table spans 16 columns, so the reads
                // past W stay inside it)
                const int j0 = 2 * g, j1 = 2 * g + 1;
                const int own0 = (int)((eq0 >> (2 * j0)) & 1u);
                const int own1 = (int)((eq1 >> (2 * j1)) & 1u);
                const double a0 = sL64[(j0 * 4 + s0) * 2 + own0] - lp0;
                const double a1 = sL64[(j1 * 4 + s1) * 2 + own1] - lp1;
                const double y0 = j0 < W ? (s0 < A ? a0 : -1.0e300) : 0.0;
                const double y1 = j1 < W ? (s1 < A ? a1 : -1.0e300) : 0.0;
                const double x = y0 + y1;
                v[ci][g] = x;
                mx = fmax(mx, x);
            }
        }
        // the target's largest entry (an upper bound, binary32), then the floor F: a
        // window with an entry at or below F scores at most F + (NG - 1) max < cutOff - 1
        // and certainly fails (.fs:735), so entries are clamped to it; the fixed point
        // 2^-kPU keeps NG max(|F|, max) below 2^31
        const float mxf = __int_as_float(
            row_last_i32(seg_scan_i32_t<true>(__float_as_int((float)mx * 1.001f + 1e-30f), q), gbase));
        const double mxt = (double)mxf;
        const double F = KD(cutoff) - 1.0 - (double)(NG - 1) * mxt - 1e-6;
        const double range = (double)NG * fmax(fabs(F), mxt);
        // kpu = floor(log2(0x1.fep30 / max(range, 1))), without the division
        const double rg = fmax(range, 1.0);
        const int erg = ilogb(rg);
        const int kpu = min(24, 30 - erg - (ldexp(rg, -erg) > 0x1.fep0 ? 1 : 0));
        // per window: NG entries each within 2^-(kPU+1), the binary64 logs and the
        // reference's own folds and log (1e-9)
        const double eps = (double)NG * ldexp(1.0, -kpu - 1) + 2e-9;
        const double xh = ldexp(KD(cutoff) + eps, kpu), xl = ldexp(KD(cutoff) - eps, kpu);
        bad |= !(kpu >= 12) || !(range < 1.0e6) || !(fabs(xh) < 0x1.0p30);
        const int thr_hi = bad ? 2147483647 : (int)ceil(xh), thr_lo = bad ? 2147483647 : (int)floor(xl);
#pragma unroll
        for (int ci = 0; ci < CPL; ++ci) {
            int e[NG];
#pragma unroll
            for (int g = 0; g < NG; ++g) {
                // (clamped, so the conversion is defined whatever a bad target's values)
                const int ev = (int)fmin(fmax(rint(ldexp(fmax(v[ci][g], F), kpu)), -2147483648.0), 2147483647.0);
                e[g] = bad ? 0 : ev;
            }
#pragma unroll
            for (int pp = 0; pp < NG / 2; ++pp)
                *(uint2 *)(tab + 8 * (q + kLpt * ci) + 256 * pp) = make_uint2((uint32_t)e[2 * pp], (uint32_t)e[2 * pp + 1]);
        }
        wave_sync();

        // the pick's inputs that do not depend on the scan, ahead of it (the target's
        // uniform, .fs:748, and the background bound K pmax^W)
        const double u = KD(u_in) ? KD(u_in)[sq] : uniform(KD(seed), rng_stream, (uint64_t)gidx);
        const double pc0 = tpcv[0], pc1 = tpcv[1], pc2 = tpcv[2], pc3 = tpcv[3];
        double pmax = pc0;
        if (A > 1) pmax = fmax(pmax, pc1);
        if (A > 2) pmax = fmax(pmax, pc2);
        if (A > 3) pmax = fmax(pmax, pc3);
        // pmax^W by squarings (W <= 16; its roundings far inside the 1e-12 below)
        const double pw2 = pmax * pmax, pw4 = pw2 * pw2, pw8 = pw4 * pw4;
        double pmw = (W & 1) ? pmax : 1.0;
        if (W & 2) pmw = pmw * pw2;
        if (W & 4) pmw = pmw * pw4;
        if (W & 8) pmw = pmw * pw8;
        if (W & 16) pmw = pmw * (pw8 * pw8);
        const double Bhi = (double)K * pmw * (1.0 + 1e-12);
        if (it == GS_LONG_TL_IT) TLINE(tl_w, 3);
        // ---- every window of the lane's range: exact integer scores ----
        // (a lane that does not scan has thresholds nothing reaches: its M, np and
        // unsure stay 0 whatever its windows read)
        const bool scan = keep && !bad;
        const int th_hi = scan ? thr_hi : 2147483647, th_lo = scan ? thr_lo : 2147483647;
        uint64_t M = 0;
        uint32_t dmin = 0xffffffffu;
        const uint32_t tabv = (uint32_t)(size_t)(__attribute__((address_space(3))) const unsigned char *)tab;
        const int nmax = __builtin_amdgcn_readfirstlane(-wave_min_i32(scan ? -nwin : 0));
        const int nmin = __builtin_amdgcn_readfirstlane(wave_min_i32(scan ? nwin : kLongRn));
        constexpr int RH = kLongRn / 2;
        if (nmax <= RH) {
            if (nmin >= RH - 4)
                long_scan<NG, RH, RH - 4>(w, tabv, nwin, th_hi, th_lo, bsum, M, dmin);
            else
                long_scan<NG, RH, 0>(w, tabv, nwin, th_hi, th_lo, bsum, M, dmin);
        } else {
            if (nmin >= kLongRn - 4)
                long_scan<NG, kLongRn, kLongRn - 4>(w, tabv, nwin, th_hi, th_lo, bsum, M, dmin);
            else
                long_scan<NG, kLongRn, 0>(w, tabv, nwin, th_hi, th_lo, bsum, M, dmin);
        }

        if (it == GS_LONG_TL_IT) TLINE(tl_w, 4);
        // the next batch and its descriptor
        bn = need ? min(2 * (nwp + __builtin_amdgcn_readlane(gpend, 0)), nb) : bc + 1;
        if (bn < nb) {
            dn = load_desc(bn);
            if (pks > 0) pn = load_pre_s(bn);
        }
        // ---- the target's totals over its row ----
        constexpr uint64_t kSumMask = (1ull << 48) - 1ull;
        // the lane's block prefixes, read now (their LDS round trip under the totals)
        int64_t bpx[kLongRn / kLongBw];
#pragma unroll
        for (int b = 0; b < kLongRn / kLongBw; ++b) bpx[b] = (int64_t)(bsum[64 * b] & ((1ull << 48) - 1ull));
        const int np = (int)(M >> 48);
        M &= kSumMask;
        const bool unsure = dmin <= (uint32_t)(th_hi - th_lo);
        const int64_t incl = seg_scan_i64_t((int64_t)M, q);
        const int64_t OpreI = incl - (int64_t)M;
        const int64_t MtotI = row_last_i64(incl, gbase);
        const int ntot = row_last_i32(seg_scan_i32_t<false>(np, q), gbase);
        const bool badg = ((__ballot(bad || unsure) >> gbase) & kSegMask) != 0;
        const bool uns_g = ((__ballot(unsure) >> gbase) & kSegMask) != 0;
        const double Mtot = ldexp((double)MtotI, -kpu);
        const double etot = (double)ntot * eps;

        // ---- certified pick (.fs:746-754): backgrounds first, their total in [0, Bhi]
        // (each G_k <= pmax^W); each motif weight within eps, the sums within 2^-50 ----
        const double eabs = Bhi + etot + Mtot * 0x1.0p-50;
        const double ncat = (double)(K + ntot + 2);
        bool ok = keep && !badg && ntot > 0 && Mtot > 4.0 * eabs && Mtot < INFINITY;
        const double delta =
            (8.0 * ncat + 64.0) * 0x1.0p-53 + 2.0 * eabs / (Mtot - eabs) * (1.0 + 0x1.0p-50);  // = eabs/M (1 + (M+e)/(M-e))
        ok = ok && u > delta;  // not in the background block
        const double U = u * Mtot, D = delta * Mtot, Tg = U - D, Th = U + D;
        // the boundaries in the sums' own units (2^-kPU): for an integer X below 2^53,
        // X 2^-kPU >= Tg exactly when X >= ceil(Tg 2^kPU)
        const int64_t TgI = ok ? (int64_t)ceil(ldexp(Tg, kpu)) : 0;
        const int64_t TlI = ok ? (int64_t)floor(ldexp(Tg, kpu)) : 0;
        const int64_t ThI = ok ? (int64_t)ceil(ldexp(Th, kpu)) : 0;
        const bool mine = ok && OpreI < TgI && OpreI + (int64_t)M >= TgI;
        // the 8-window block of the mine lane (at most one a row) whose prefix first
        // reaches U - D ...
        int bb = 0;
        int64_t PI = OpreI;
        if (mine) {
            const int nbk = (nwin + kLongBw - 1) / kLongBw;
            bb = nbk - 1;
#pragma unroll
            for (int b = kLongRn / kLongBw - 1; b >= 0; --b) {
                const int64_t bp = b < nbk ? bpx[b] : (int64_t)M;
                if (b < nbk && OpreI + bp >= TgI) {
                    bb = b;
                    PI = OpreI + (b > 0 ? bpx[b - 1] : 0);
                }
            }
        }
        // ... then its 8 windows re-evaluated by lanes 0..7 of the row at once (the
        // same integer sums as the scan), their passing scores' prefix over the 8 lanes
        // (DPP), the first lane whose prefix reaches U - D the pick
        const unsigned long long mm = (__ballot(mine) >> gbase) & kSegMask;
        const int msrc = mm ? gbase + __ffsll((long long)mm) - 1 : lane;
        const int kx = kLongBw * __shfl(bb, msrc, 64) + (q & 7);
        const int64_t PIr = bperm_i64(PI, msrc);
        // (the shuffle outside the condition: a bpermute in a branch reads 0 from the
        // lanes the branch leaves off)
        const int nwm = __shfl(nwin, msrc, 64);
        const bool ev = mm != 0ull && q < kLongBw && kx < nwm;
        const uint32_t x16 = funnel(lw0[64 * ((kx >> 4) + 1) + msrc], lw0[64 * (kx >> 4) + msrc], 2 * (kx & 15));
        const int scx = long_eval<NG>(x16, tab);
        const bool px = ev && scx > thr_hi;
        // (kLpt = 16: lanes 8..15 re-evaluate nothing; their sums are not read)
        const int64_t cum = seg_scan_i64_t(px ? (int64_t)scx : 0, q);
        const bool hit = px && PIr + cum >= TgI;
        bool found, cert;
        int pk;
        uint32_t win;
        {
            const unsigned long long fm = (__ballot(hit) >> gbase) & kSegMask;
            const int src = fm ? gbase + __ffsll((long long)fm) - 1 : lane;
            const bool cx = PIr + cum - scx <= TlI && PIr + cum >= ThI;
            pk = __shfl(__shfl(x0, msrc, 64) + kx, src, 64);
            win = (uint32_t)__shfl((int)(x16 & wmask), src, 64);
            const bool cr = __shfl((int)cx, src, 64) != 0;
            found = fm != 0ull;
            cert = found && cr;
        }
        bool win_ok;
        double pw = 0.0;
#ifndef GS_LONG_PRE_LATE
        if (pks == 0 && bn < nb) pn = load_pre(dn, bn);
#endif
        // ---- the picked window's weight (.fs:283-292, .fs:737): log2 of the product
        // of the W quotients PPM'/PCV as the sum of their binary64 log2s, the ones the
        // table is built from (lane q < NG adds column pair q; the row sums).  Each log
        // is within an ulp or two of magnitude <= 60, so the sum is within ~5e-13 of
        // the reference's log of the product: relative 5e-13 once the weight is >= 1
        // (the passing weights at cut-off >= 1; north_star holds scores to 1e-5).
        // Below 1 the reference's own fold: the W quotients by W lanes, then log ----
        {
            double xs = 0.0;
            if (cert && q < NG) {
                const int j0 = 2 * q, j1 = 2 * q + 1;
                if (j0 < W) {
                    const int e = (int)((win >> (2 * j0)) & 3u);
                    const int own = p >= 0 && (int)((gw >> (2 * j0)) & 3u) == e ? 1 : 0;
                    xs += sL64[(j0 * 4 + e) * 2 + own] - tpcv[4 + e];
                }
                if (j1 < W) {
                    const int e = (int)((win >> (2 * j1)) & 3u);
                    const int own = p >= 0 && (int)((gw >> (2 * j1)) & 3u) == e ? 1 : 0;
                    xs += sL64[(j1 * 4 + e) * 2 + own] - tpcv[4 + e];
                }
            }
            pw = row_last_f64(seg_scan_f64_t(xs, q), gbase);
        }
        if (__ballot(cert && !(pw >= 1.0)) != 0ull) {
            const bool slow = cert && !(pw >= 1.0);
            if (slow)
                for (int j = q; j < W; j += kLpt) {
                    const int e = (int)((win >> (2 * j)) & 3u);
                    const bool own = p >= 0 && (int)((gw >> (2 * j)) & 3u) == e;
                    const double2 pp = sPPM[j * 4 + e];
                    tpcv[8 + j] = (own ? pp.y : pp.x) / tpcv[e];
                }
            wave_sync();
            if (slow) {
                double S = 1.0;
                for (int j = 0; j < W; ++j) S = S * tpcv[8 + j];
                pw = log(S * 1.0) / kLn2;
            }
        }
        win_ok = cert && pw > KD(cutoff);
        // ---- a target without a passing window (and none in the band): its categories
        // are the K background products alone (.fs:759-784), each the reference's
        // binary64 fold of PCV over the window (.fs:123-124).  The live sweep's
        // background walk over the row's 16 lane ranges (incremental products, the
        // row's prefix, u times the total located and certified with gs_sweep_bg.hip's
        // margins, the picked product folded exactly): the first sweep of a chain from
        // uniform random starts, where no window passes against a flat PPM, no longer
        // sends every target to the wavefront-wide exact rescan ----
        const bool bgo = keep && !badg && ntot == 0;
        if (__ballot(bgo) != 0ull) {
            const BgPick r = bg_pick_row<kLpt, kLongRn>(lw0 + lane, wmask, W, K, nwin, bgo, u, q, gbase, pc0, pc1, pc2, pc3);
            const unsigned long long gm = (__ballot(r.ok) >> gbase) & kSegMask;
            const int src = gm ? gbase + __ffsll((long long)gm) - 1 : gbase;
            const double pw_s = __shfl(r.pw, src, 64);
            if (gm != 0ull) {
                win_ok = true;  // a background category: Positions [], PWMS its product
                pk = -1;
                pw = pw_s;
            }
        }
        if (it == GS_LONG_TL_IT) TLINE(tl_w, 5);
        // (what the bound cannot settle goes to the exact rescan)
        const bool need_fb = keep && !win_ok;
        if (__ballot(need_fb && q == 0) != 0ull) {
            // why (gs_stats [2..6], [10], [12]): a score out of range / no passing window
            // / total not separated / u among the backgrounds / not certified
            const int why = (badg && !uns_g) ? 0 : uns_g ? 5 : ntot == 0 ? 7
                          : !(Mtot > 4.0 * eabs) ? 2 : !(u > delta) ? 3 : 4;
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                const int c = __popcll(__ballot(need_fb && q == 0 && why == r));
                if (c && lane == 0) atomicAdd(&sStat[1 + r], (uint32_t)c);
            }
        }
        if (keep && !need_fb && q == 0) {
            KD(pos_out)[sq] = pk;
            KD(pwms_out)[sq] = pw;
        }
        // ---- aggregates of the new snapshot: C[a][j] += segment; T[a] = the rank's
        // symbol totals (the last workgroup adds them) less every kept segment's
        // symbols and the whole composition of every target left without one here
        // (rescan_target adds composition - segment for those that keep one) ----
        const bool km = keep && !need_fb && pk >= 0;
        if (km)
            for (int j = q; j < W; j += kLpt) atomicAdd(&waggC[(int)((win >> (2 * j)) & 3u) * W + j], 1);
        if (act && q < A) {
            const int64_t d = km ? -(int64_t)sym_count(win, q, wmask) : -(int64_t)KD(comp)[(int64_t)sq * (A + 1) + q];
            if (d != 0) atomicAdd((unsigned long long *)&waggT[q], (unsigned long long)d);
        }
        // ---- targets the bound could not settle: the whole wavefront rescans each
        // exactly, in its slice (whose tables are dead by now) ----
#ifdef GS_LONG_PRE_LATE
        if (pks == 0 && bn < nb) pn = load_pre(dn, bn);
#endif
        const unsigned long long fbm = __ballot(need_fb && q == 0);
        if (fbm != 0ull && lane == 0) atomicAdd(&sStat[0], (uint32_t)__popcll(fbm));
        wave_sync();
        for (unsigned long long fm = fbm; fm != 0ull; fm &= fm - 1ull) {
            const int sqx = __builtin_amdgcn_readfirstlane(__shfl(sq, __ffsll((long long)fm) - 1, 64));
            long_rescan<WM>(kargs_dna(), sqx, rng_stream, wslice, tab_off, sPPM, sT, sumT, lane, waggC, waggT);
        }
        if (it == GS_LONG_TL_IT) TLINE(tl_w, 6);
        bc = bn;
        dd = dn;
        cur = pn;
    }
    TLINE(tl_w, 7);

    // ---- flush: the workgroup's sums into replica blockIdx % 8, one atomic a cell;
    // the last workgroup (a done counter) reduces the replicas ----
    __syncthreads();
    if (tid < 9) {
        // sStat: [0] rescans, [1 + why]: why 0..4 -> stats 2..6, 5..7 -> stats 10..12
        const uint32_t vv = sStat[tid];
        if (vv)
            atomicAdd(&(KD(fallbacks) + (blockIdx.x % kRepl) * kStatStride)[tid == 0 ? 0 : tid <= 5 ? tid + 1 : tid + 4],
                      (unsigned long long)vv);
    }
    int64_t *dst = KD(rep) + (int64_t)(blockIdx.x % kRepl) * KD(stride);
    for (int c = tid; c < cells; c += blockDim.x) {
        int64_t vv = 0;
        for (int w2 = 0; w2 < nwv; ++w2) {
            const unsigned char *wa = lds + O_WAGG + w2 * WAGG_BYTES;
            vv += c < AW ? (int64_t)((const int32_t *)wa)[c] : ((const int64_t *)(wa + 256))[c - AW];
        }
        if (vv != 0) GS_FLUSH_ADD((unsigned long long *)&dst[c], (unsigned long long)vv);  // (returning: gs_common.h)
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int &s_last = sMisc[8];
    if (tid == 0) {
        // two levels (as the live sweep): the workgroups of one replica group count in
        // done[1 + group], the last of them in done[0]
        GS_DONE_FENCE(__ATOMIC_RELEASE);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const int grp = blockIdx.x % kRepl;
        const unsigned int ng = (gridDim.x - grp + kRepl - 1) / kRepl;
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
    if (!s_last) return;
    unsigned int *const done_all = KD(done);
    GS_DONE_FENCE(__ATOMIC_ACQUIRE);
    if (tid < kWorkPools) atomicExch(done_all + 32 * (1 + tid), 0u);  // the work counters
    const int64_t *const compsum = KD(compsum);
    int64_t *const rep = KD(rep);
    int64_t *const agg_out = KD(agg_out);
    int64_t xv = 0;  // (the exchange: thread c's cell, cells <= 68 < the workgroup)
    for (int c = tid; c < cells; c += blockDim.x) {
        int64_t vv = c >= AW ? compsum[c - AW] : 0;
#pragma unroll
        for (int r = 0; r < kRepl; ++r)
            vv += (int64_t)atomicExch((unsigned long long *)&rep[(int64_t)r * KD(stride) + c], 0ull);
        agg_out[c] = vv;
        xv = vv;
    }
    if (KD(xpeer)) xch_reduce(kargs_dna(), tid, cells, xv, agg_out, sMisc + 10);
    if (tid == 0) {
        atomicExch(KD(done), 0u);
        unsigned long long *const ctr = KD(sweep_ctr);
        if (ctr) atomicAdd(ctr, 1ull);
    }
}

static int long_wm(int W) { return W <= 8 ? 8 : W <= 12 ? 12 : 16; }

static const void *long_kernel_ptr(int wm) {
    if (wm == 8) return (const void *)&gs_sweep_long_kernel<8>;
    if (wm == 12) return (const void *)&gs_sweep_long_kernel<12>;
    if (wm == 16) return (const void *)&gs_sweep_long_kernel<16>;
    return nullptr;
}

// The shapes the long sweep takes: W <= 16 and at most 16 x kLongRn windows.
bool gs_long_fits(int Lmax, int W) { return W >= 1 && W <= 16 && Lmax - W + 1 <= kLpt * kLongRn; }

int gs_long_slice_bytes(int Lmax, int W) {
    const int rs = (live_rescan_slice(Lmax, long_wm(W)) + 255) & ~255;
    return rs > kLongSliceMin ? rs : kLongSliceMin;
}

int gs_long_lds_bytes(int Lmax, int W, int waves) { return O_LWAVE + waves * gs_long_slice_bytes(Lmax, W); }

hipError_t gs_long_occupancy(int *blocks_per_cu, int W, int Lmax, int waves) {
    const void *k = long_kernel_ptr(long_wm(W));
    if (!k) return hipErrorInvalidValue;
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, k, 64 * waves,
                                                        (size_t)gs_long_lds_bytes(Lmax, W, waves));
}

hipError_t gs_long_launch(const DnaArgs &a, int grid, int waves, hipStream_t stream, hipEvent_t start,
                          hipEvent_t stop) {
    const void *k = long_kernel_ptr(long_wm(a.W));
    if (!k || waves < 2 || waves > kLongWaves || !gs_long_fits(a.Lmax, a.W)) return hipErrorInvalidValue;
    DnaArgs args = a;
    args.live_slice = gs_long_slice_bytes(a.Lmax, a.W);
    const size_t lds = (size_t)gs_long_lds_bytes(a.Lmax, a.W, waves);
    void *params[] = {&args};
    if (!start) return hipLaunchKernel(k, dim3(grid), dim3(64 * waves), params, lds, stream);
    return hipExtLaunchKernel(k, dim3(grid), dim3(64 * waves), params, lds, stream, start, stop, 0);
}
