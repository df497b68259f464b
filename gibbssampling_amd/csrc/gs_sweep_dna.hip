// gs_sweep_dna.hip — the synchronous Gibbs sweep for small alphabets on gfx950.
//
// MotifSampler.findBestMotifIndicesByWithStartPositions (.fs:935-970) with
// motifAmount = 1, for alphabets of at most 4 symbols (DNA) and motifs of at most
// 16 columns, when no symbol outside the alphabet occurs in the data.
//
// Layout: one lane owns one sequence (G = 1) or 1/G of its windows; a wavefront
// holds 64/G sequences.  Sequences are 2-bit packed in HBM (16 symbols a word), so
// the pair code s[i] + 4 s[i+1] of any position is one funnel shift of two words.
//
// Scoring every window (.fs:759-777) is a sliding ring over positions: position
// i reads ONE 16-byte row (8 motif-column pairs) of a pair table indexed by its
// pair code and adds the 8 entries into the 8 windows that see position i as the
// first symbol of column pair g (window i - 2g).  Entries are int16, in two
// tables whose sum is the window's log2 score:
//   coarse[c][g]  (workgroup-shared): log2 PPM - log2 PCV of the global counts,
//                 rounded to 2^-cs (cs per sweep, 8 when the table fits);
//   fine[c][g]    (one copy per lane): the rest of the lane's exact binary32 log2
//                 PWM pair (its own hold-one-out PCV, .fs:945-954, its own
//                 segment's count-minus-one cells, .fs:955-965) rounded to 2^-m.
// Both are exact integer sums, so each window's score is known to within a
// per-sequence bound eps.  Cut-off tests (.fs:735) and the
// roulette pick (.fs:746-754) are taken only where the bound certifies them:
// the pick walks 16-window block sums kept during the scan, re-runs the ring
// over the one block that holds u, and folds the picked window's weight in
// binary64 exactly as the reference does.  Everything the bound cannot settle
// (and every sequence whose pick is a background category, including a run with
// no motif-bearing sequences) is rescanned exactly in binary64 by the whole
// wavefront, as in gs_sweep.hip.
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

namespace {

typedef short s2 __attribute__((ext_vector_type(2)));


// LDS carve (bytes): workgroup-shared tables, then one 16 KB slice per wavefront
// (the lanes' fine tables; the exact rescan's staging area afterwards).
constexpr int O_C = 0;          // int32 [A*W] global counts C
constexpr int O_T = 256;        // int64 [4] T, [4] = sum
constexpr int O_PPM = 304;      // double2 [16 j][4 e]: (C + pc)/den, (C - 1 + pc)/den
constexpr int O_OA = 1328;      // int32 [16 j][4 e]: log2 of their ratio (own-cell change), 2^-kFix
constexpr int O_LPG = 1584;     // double [4]: log2 of the table's PCV estimate
constexpr int O_UB = 1616;      // double: sum over columns of max_e log2 PPM (motif score bound)
constexpr int O_COARSE = 1840;  // uint4 [16 codes]: int16 pairs (g, g + 4)
constexpr int O_RES = 2096;     // int32 [16 codes][8 groups]: pair value - coarse, 2^-kFix
constexpr int O_MISC = 2608;    // [5] cs, [6] table fault, [7] max |pair value|
constexpr int O_WAGG = 2672;    // per wavefront: int32 C[64], int64 T[4]  (288 B)
constexpr int WAGG_BYTES = 288;
constexpr int O_STAT = 3840;    // uint32 [8]: the workgroup's gs_stats counts
constexpr int O_WAVE = 3904;
constexpr int kSmemBytes = O_WAVE + kDnaWaves * kDnaFineBytes;
// inside a wavefront slice, for the exact rescan
constexpr int F_SEQ = 0;        // the sequence's symbols, one byte each
constexpr int F_TAB = 8320;     // (PWM, PCV) [E][tab_stride(WM)]
constexpr int F_MISC = 9408;    // pcv[4] (doubles), pick results
static_assert(F_SEQ + kDnaMaxL + 16 + 96 <= F_TAB, "rescan staging");
static_assert(F_MISC + 64 <= kDnaFineBytes, "rescan scratch");
// Fixed point of the table terms: every log2 term a fine entry adds up is held as an
// int32 multiple of 2^-kFix: the residual (< 2^-4) and two own-cell and two PCV
// terms (each < 16, else the lane is rescanned), so the sum stays below 2^30
constexpr int kFix = 24;
constexpr int32_t kOaBad = (int32_t)0x80000000;  // own-cell term out of range

__device__ __forceinline__ uint32_t pk_add(uint32_t x, uint32_t y) {
    return __builtin_bit_cast(uint32_t, __builtin_bit_cast(s2, x) + __builtin_bit_cast(s2, y));
}

// The window completed by a ring step: low int16 of the register it was born in
// plus the high int16 of the register born 8 positions later, as a sign-extended
// int32 (one SDWA add: the sum of two entries of at most 4 x 4095 never wraps).
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
    atomicCAS(a.err_code, 0, code);
    atomicMin(a.err_index, (unsigned long long)gidx);
}

__device__ __forceinline__ uint4 load_words(const uint32_t *p) {
    uint4 v;
    __builtin_memcpy(&v, p, 16);  // 4-byte aligned 16-byte load
    return v;
}

// Ring state of one lane: the registers born at the last 16 positions (mod 16),
// coarse and fine tables, and the running results.
struct Ring {
    uint32_t c[16], f[16];
};

struct ScanAcc {
    int64_t M;     // sum of the passing windows' scores (units 2^-m)
    int32_t Mb;    // the same for the current 16-window block
    int32_t npass;
    bool unsure;   // a window in the cut-off band
};

// Table rows in flight: the two 16-byte rows of position P are requested PD ring
// steps before they are added (64 % PD == 0 so the slot of a position does not
// depend on its chunk).
constexpr int PD = 4;
constexpr int kChunkCk = 8;  // chunk prefixes kept in registers (lanes of <= 512 positions)
struct Pipe {
    uint4 c[PD], f[PD];
};

// Pair code * 16 of position P of a chunk whose words are ww[1..4], ww[0] the word
// before and ww[5] the first word of the next chunk (P < 64 + 14: ww[6] only
// feeds bits that are masked off).
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

template <int P>
__device__ __forceinline__ void fetch(Pipe &pp, const uint32_t (&ww)[7], const unsigned char *coarse,
                                      const unsigned char *fine_lane) {
    const uint32_t a16 = pair16<P>(ww);
    pp.c[P % PD] = *(const uint4 *)(coarse + a16);
    pp.f[P % PD] = *(const uint4 *)(fine_lane + (a16 << 6));
}

// Ring step R (static): the rows of position R go into the 4 windows they
// continue; returns the score of the window completed at this step (window
// R - 14 of the chunk) in units of 2^-m.
template <int R>
__device__ __forceinline__ int ring_add(Ring &g, const Pipe &pp, int sh) {
    const uint4 cq = pp.c[R % PD], fq = pp.f[R % PD];
    constexpr int i0 = R & 15;
    g.c[i0] = cq.x;
    g.c[(i0 - 2) & 15] = pk_add(g.c[(i0 - 2) & 15], cq.y);
    g.c[(i0 - 4) & 15] = pk_add(g.c[(i0 - 4) & 15], cq.z);
    g.c[(i0 - 6) & 15] = pk_add(g.c[(i0 - 6) & 15], cq.w);
    g.f[i0] = fq.x;
    g.f[(i0 - 2) & 15] = pk_add(g.f[(i0 - 2) & 15], fq.y);
    g.f[(i0 - 4) & 15] = pk_add(g.f[(i0 - 4) & 15], fq.z);
    g.f[(i0 - 6) & 15] = pk_add(g.f[(i0 - 6) & 15], fq.w);
    const int ch = half_sum(g.c[(i0 - 14) & 15], g.c[(i0 - 6) & 15]);
    const int fl = half_sum(g.f[(i0 - 14) & 15], g.f[(i0 - 6) & 15]);
    return (int)((uint32_t)ch << sh) + fl;
}

// One 64-position chunk of the scan (chunk q: its windows are 64q - 14 + R
// relative to the lane's first; kq = 64q - 14).  The rows of the chunk's first
// PD positions were requested by the previous chunk (or the prologue); this one
// requests the next chunk's.
template <int R = 0>
__device__ __forceinline__ void scan_chunk(Ring &g, Pipe &pp, ScanAcc &s, const uint32_t (&ww)[7],
                                           const unsigned char *coarse,
                                           const unsigned char *fine_lane, int sh, int thr_hi,
                                           int thr_lo, int kq, int nwin, int32_t *ckp_q) {
    if constexpr (R < 64) {
        const int sc = ring_add<R>(g, pp, sh);
        fetch<R + PD>(pp, ww, coarse, fine_lane);
        const bool valid = (uint32_t)(kq + R) < (uint32_t)nwin;
        const bool hi = sc > thr_hi, lo = sc >= thr_lo;
        const bool pass = valid && hi;
        s.npass += pass ? 1 : 0;
        s.Mb += pass ? sc : 0;
        s.unsure |= valid && (hi != lo);  // in the band: lo but not hi
        if constexpr ((R & 15) == 13) {
            // last window of a 16-window block: (64q + R - 14) / 16 = 4q + (R - 13) / 16 - 1
            if (kq + R >= 0) ckp_q[((R - 13) / 16 - 1) * 64] = s.Mb;
            s.M += s.Mb;
            s.Mb = 0;
        }
        scan_chunk<R + 1>(g, pp, s, ww, coarse, fine_lane, sh, thr_hi, thr_lo, kq, nwin, ckp_q);
    }
}

struct BlockScores {
    int v[16];
};

// The block re-run of the pick: 30 steps from the block's first position; the
// windows complete at steps 14..29 in order.  ww[0] word before, ww[1..3] words.
template <int R = 0>
__device__ __forceinline__ void rerun_block(Ring &g, Pipe &pp, const uint32_t (&ww)[7],
                                            const unsigned char *coarse,
                                            const unsigned char *fine_lane, int sh, int (&scs)[16]) {
    if constexpr (R < 30) {
        const int sc = ring_add<R>(g, pp, sh);
        if constexpr (R + PD < 30) fetch<R + PD>(pp, ww, coarse, fine_lane);
        if constexpr (R >= 14) scs[R - 14] = sc;
        rerun_block<R + 1>(g, pp, ww, coarse, fine_lane, sh, scs);
    }
}

// Its own function: inlined, its 30 steps would compete for registers with the
// scan's (the kernel went past 256 VGPRs).
struct Words7 {
    uint32_t w[7];
};

__device__ __noinline__ BlockScores rerun_scores(Words7 ww, uint32_t fine_off, int sh) {
    // LDS through the kernel's own dynamic array (address space 3: ds_read, not flat)
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const unsigned char *coarse = lds + O_COARSE, *fine_lane = lds + fine_off;
    Ring r2;
#pragma unroll
    for (int i = 0; i < 16; ++i) r2.c[i] = r2.f[i] = 0u;
    Pipe pp;
    fetch<0>(pp, ww.w, coarse, fine_lane);
    fetch<1>(pp, ww.w, coarse, fine_lane);
    fetch<2>(pp, ww.w, coarse, fine_lane);
    fetch<3>(pp, ww.w, coarse, fine_lane);
    BlockScores bs;
    rerun_block(r2, pp, ww.w, coarse, fine_lane, sh, bs.v);
    return bs;
}


// The picked window's weight: the reference's binary64 left fold of PPM'/PCV
// (.fs:283-292), then log2 (.fs:737).  Its own function: inlined at the end of
// the pick, the binary64 log and divisions raised the kernel past 256 VGPRs.
__device__ __forceinline__ double picked_weight(uint32_t win, uint32_t gw, bool has_own, int W,
                                             const double2 *sPPM, double p0, double p1, double p2,
                                             double p3) {
    double S = 1.0;
    for (int j = 0; j < W; ++j) {
        const int e = (int)((win >> (2 * j)) & 3u);
        const bool own = has_own && (int)((gw >> (2 * j)) & 3u) == e;
        const double2 pp = sPPM[j * 4 + e];
        const double pe = e == 0 ? p0 : e == 1 ? p1 : e == 2 ? p2 : p3;
        S = S * ((own ? pp.y : pp.x) / pe);
    }
    return log(S * 1.0) / kLn2;
}

// Background weights G_k = prod_j pcv[s[k+j]] (.fs:123-124, .fs:759-777) of the
// windows [x0, x0 + nwin) of the sequence at seqw, approximately and relative to
// 2^(W lref): g_k = 2^(lg_k 2^-f), lg_k the exact integer sum of lpq over the
// window's symbols (lpq[e] = log2 pcv[e] - lref rounded to 2^-f), slid one
// position a step; the binary32 fraction goes through v_exp_f32 and the integer
// part through v_ldexp_f64.  Error bound: bg_rel_err.  blk(t) at the start of
// each 16-window block (t relative to x0), fn(k, g) for every window in order; a
// lane leaves once fn returns true.
struct BgLut {
    int32_t l0, d1, d2, d3;  // lpq[s] = l0 + bit0 d1 + bit1 d2 + (s == 3) d3
};
__device__ __forceinline__ BgLut bg_lut(const int32_t (&q)[4]) {
    return BgLut{q[0], q[1] - q[0], q[2] - q[0], q[3] - q[2] - q[1] + q[0]};
}
// lpq of symbol r of w, less l0: sign-extended bit fields as masks (no lookups)
template <int R>
__device__ __forceinline__ int32_t bg_term(uint32_t w, const BgLut &t) {
    const int32_t m0 = (int32_t)(w << (31 - 2 * R)) >> 31, m1 = (int32_t)(w << (30 - 2 * R)) >> 31;
    return (m0 & t.d1) + (m1 & t.d2) + (m0 & m1 & t.d3);
}

template <int R = 0, class V>
__device__ __forceinline__ void bg_block(int &lg, bool &done, uint32_t nw, uint32_t ow, int b, int nwin,
                                         int x0, int f, int fw, const BgLut &t, V &v) {
    if constexpr (R < 16) {
        if (R > 0 || b > 0) lg += bg_term<R>(nw, t) - bg_term<R>(ow, t);
        if (!done && b + R < nwin) {
            const int xi = lg >> f;
            const uint32_t fr = __builtin_amdgcn_ubfe((uint32_t)lg, (uint32_t)(f - fw), (uint32_t)fw);
            const float fx = __builtin_ldexpf((float)fr, -fw);
            const double g = __builtin_ldexp((double)__builtin_amdgcn_exp2f(fx), xi);
            done = v.win(x0 + b + R, g);
        }
        bg_block<R + 1>(lg, done, nw, ow, b, nwin, x0, f, fw, t, v);
    }
}

template <class V>
__device__ __forceinline__ V bg_walk(const uint32_t *seqw, int x0, int nwin, int W, int f,
                                     const BgLut &t, V v) {
    auto word = [&](int i) -> uint32_t { return i >= 0 ? seqw[i] : 0u; };
    const int fw = min(f, 24);  // fraction bits kept (binary32 exact)
    int lg = 0;
    if (nwin > 0) {
        const uint32_t x = funnel(word((x0 >> 4) + 1), word(x0 >> 4), 2 * (x0 & 15));
        int acc = 0;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const int32_t m0 = -(int32_t)((x >> (2 * j)) & 1u), m1 = -(int32_t)((x >> (2 * j + 1)) & 1u);
            if (j < W) acc += t.l0 + (m0 & t.d1) + (m1 & t.d2) + (m0 & m1 & t.d3);
        }
        lg = acc;
    }
    // symbols entering (position k + W - 1) and leaving (k - 1) the window k
    const int pn0 = x0 + W - 1, po0 = x0 - 1;
    const int shn = 2 * (pn0 & 15), sho = 2 * (po0 & 15);
    const int in0 = pn0 >> 4, io0 = po0 >> 4;
    uint32_t n0 = word(in0), n1 = word(in0 + 1), o0 = word(io0), o1 = word(io0 + 1);
    bool done = false;
    for (int b = 0; b < nwin && !done; b += 16) {
        const uint32_t n2 = word(in0 + (b >> 4) + 2), o2 = word(io0 + (b >> 4) + 2);
        const uint32_t nw = funnel(n1, n0, shn), ow = funnel(o1, o0, sho);
        v.blk(b);
        bg_block(lg, done, nw, ow, b, nwin, x0, f, fw, t, v);
        n0 = n1;
        n1 = n2;
        o0 = o1;
        o1 = o2;
    }
    return v;
}

// bg_walk visitors (state by value: lambdas capturing locals by reference left
// them in scratch).  Pass 1: the lane's sum and its value at the starts of 8
// chunks of Cz windows (whole 16-window blocks).
struct BgSum {
    double B, pre[8];
    int ci, nck, Cz;
    __device__ __forceinline__ void blk(int t) {
        if (t == nck) {
#pragma unroll
            for (int i = 0; i < 8; ++i) pre[i] = i == ci ? B : pre[i];
            ++ci;
            nck += Cz;
        }
    }
    static constexpr bool kStops = false;  // never ends a walk early
    __device__ __forceinline__ bool win(int, double g) {
        B = B + g;
        return false;
    }
};
// Pass 2: from running sum P, the first window whose upper boundary reaches Tb;
// certified when Ub lies inside [lo + Db, hi - Db].
struct BgFind {
    double P, Tb, Ub, Db;
    int pk;
    bool found, cert;
    static constexpr bool kStops = true;
    __device__ __forceinline__ void blk(int) {}
    __device__ __forceinline__ bool win(int k, double g) {
        const double lo = P;
        P = P + g;
        const bool hit = P >= Tb;
        cert = hit && Ub >= lo + Db && Ub <= P - Db;
        pk = hit ? k : pk;
        found = hit;
        return hit;
    }
};

// The background walk of a wavefront whose lanes all skipped the motif scan (the
// all-background state of the chain: no motif category can pass, so the pick is a
// background window).  Their fine-table slots are free, so each lane keeps a ratio
// table there, [16 rows][64 lanes] binary64 (a lane's row r at 512 r + 8 lane: the
// 64 lanes of a read hit 64 distinct banks), row i + 4 o = pcv[i] (1 / pcv[o]),
// and -- when they fit -- the words of its window range, staged by 16-byte
// global->LDS copies ([quad][64 lanes][16 B] at kBgWordsOff).  Window x0 is
// pcv[0]^W times the product of its rows (s_j, 0); every next window is
// g_k = g_{k-1} R[s_{k-1+W}][s_{k-1}], one product and one table read a window
// instead of an integer log sum and an exp2.  Relative error of each g_k against
// the reference's fold: bg_fast_rel_err.
constexpr int kBgRows = 16;
constexpr int kBgWordsOff = kBgRows * 64 * 8;
constexpr int kBgQuads = (kDnaFineBytes - kBgWordsOff) / 1024;
static_assert(kBgQuads >= 4, "staged words");

__device__ __forceinline__ void bg_fast_table(double *rt, const double (&pcv)[4]) {
    double inv[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) inv[e] = 1.0 / pcv[e];
#pragma unroll
    for (int c = 0; c < 16; ++c) rt[c * 64] = pcv[c & 3] * inv[c >> 2];
}

// The staged words of a lane's range, addressed from the walk's first word: word(i)
// = word i (i >= -1; word -1 is prev0 when the walk starts at the staged range's
// first word).  Read-ahead past the staged quads returns words no window uses.
struct WordsLds {
    const unsigned char *base;  // the lane's staged quad 0 (slice + kBgWordsOff + 16 lane)
    int w0;                     // the walk's first word among the staged ones
    uint32_t prev0;             // word -1 of the staged range
    __device__ __forceinline__ uint32_t word(int i) const {
        const int k = w0 + i;
        if (k < 0) return prev0;
        return *(const uint32_t *)(base + min(k >> 2, kBgQuads - 1) * 1024 + (k & 3) * 4);
    }
};

// One 16-window block: the 16 table reads are issued before the first product
// (a product a window waited for its read otherwise); FULL: every window of the
// block is in the lane's range.
template <bool FULL, class V>
__device__ __forceinline__ void bg_fast_block(double &g, bool &done, uint32_t nw, uint32_t ow, int b,
                                              int nwin, int x0, const double *rt, V &v) {
    double r[16];
#pragma unroll
    for (int R = 0; R < 16; ++R) {
        const uint32_t ci = __builtin_amdgcn_ubfe(nw, 2 * R, 2), co = __builtin_amdgcn_ubfe(ow, 2 * R, 2);
        r[R] = rt[(ci | (co << 2)) * 64];
    }
#pragma unroll
    for (int R = 0; R < 16; ++R) {
        if (R > 0 || b > 0) g = g * r[R];
        if constexpr (V::kStops) {
            if (!done && (FULL || b + R < nwin)) done = v.win(x0 + b + R, g);
        } else {
            if (FULL || b + R < nwin) v.win(x0 + b + R, g);
        }
    }
}

// One 16-window block a step, W <= 16: block k reads words k - 1, k and k + 1 of
// the walk (in-symbols of its windows start at x0 + 16k + W - 1, out-symbols at
// x0 + 16k - 1); the word two blocks ahead is requested as a block starts.
template <class V>
__device__ __forceinline__ V bg_walk_fast(const WordsLds &src, int x0, int nwin, int W, double pw0,
                                          const double *rt, V v) {
    if (nwin <= 0) return v;
    uint32_t wa = src.word(-1), wb = src.word(0), wc = src.word(1);
    // window x0: pcv[0]^W times its rows (s_j, 0) = pcv[s_j] / pcv[0]
    double f[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) f[j] = rt[__builtin_amdgcn_ubfe(wb, 2 * j, 2) * 64];
    double g = pw0;
#pragma unroll
    for (int j = 0; j < 16; ++j)
        if (j < W) g = g * f[j];
    const int shn = 2 * (W - 1);
    bool done = false;
    for (int b = 0; b < nwin && !done; b += 16) {
        const uint32_t wd = src.word((b >> 4) + 2);
        const uint32_t nw = funnel(wc, wb, shn), ow = funnel(wb, wa, 30);
        v.blk(b);
        if (b + 16 <= nwin)
            bg_fast_block<true>(g, done, nw, ow, b, nwin, x0, rt, v);
        else
            bg_fast_block<false>(g, done, nw, ow, b, nwin, x0, rt, v);
        wa = wb;
        wb = wc;
        wc = wd;
    }
    return v;
}

// Relative error of bg_walk_fast's g_k (k - x0 < K steps) against the reference's
// fold: the first window's 4W + 1 roundings (rows: 1 / pcv[0] and the product;
// the multiplies; pcv[0]^W), per step three (1 / pcv, the table product, the
// multiply), the reference's own W.
__device__ __forceinline__ double bg_fast_rel_err(int W, int K) {
    return (double)(5 * W + 3 * K + 20) * 0x1.0p-53 * (1.0 + 0x1.0p-10);
}

// Relative error of bg_walk's g_k against the reference's binary64 fold G_k /
// 2^(W lref): the W roundings of lpq (2^-(f+1) each) and of the binary64 logs,
// the fraction's truncation to 24 bits, v_exp_f32 (kExp2RelErr), the fold's own
// W roundings; (1 + 2^-10) covers e^x - 1 <= x (1 + x) for these x.
__device__ __forceinline__ double bg_rel_err(int W, int f) {
    const double lg_err = (double)W * (__builtin_ldexp(1.0, -(f + 1)) + 0x1.0p-44) +
                          (f > 24 ? 0x1.0p-24 : 0.0);  // truncation to 24 fraction bits
    return (kLn2 * lg_err + kExp2RelErr + (double)W * 0x1.0p-52) * (1.0 + 0x1.0p-10);
}


// Exact binary64 rescan of sequence sq (wave-uniform) by the whole wavefront:
// the reference's folds for every window (.fs:759-777), the pick certified
// against rounding alone, else one lane replays the reference's sequential sums
// (.fs:747-754).  Writes pos_out / pwms_out (or raises the overrun error) and
// adds the new segment to the wavefront's aggregates.
// Mark of a sequence left to the exact rescan (pos_out, overwritten before the
// kernel ends).
constexpr int32_t kFbMark = (int32_t)0x80000000;

template <int WM>
__device__ __forceinline__ void rescan_seq(const DnaArgs &a, int sq, uint64_t rng_stream,
                                        unsigned char *wslice, const double2 *sPPM,
                                        const int64_t *sT, int64_t sumT, int lane,
                                        int32_t *waggC, int64_t *waggT STAMP_PARAMS) {
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
    uint8_t *sx = wslice + F_SEQ;
    unsigned char *tab = wslice + F_TAB;
    double *mpcv = (double *)(wslice + F_MISC);
    int32_t *mres = (int32_t *)(wslice + F_MISC + 32);
    // hold-one-out PCV (.fs:945-954), as in the scan
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
    STAMP(11);
    // (PWM, PCV) [e][tab_stride(WM)], columns past W (1, 1)
    constexpr int WS = tab_stride(WM);
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
    STAMP(12);
    auto evx = [&](int k, double &gg, double &mm) {
        exact_eval<WM>(sx, tab, a.thr_lo, a.cutoff, k, gg, mm);
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
    STAMP(13);
    int pkk = -1;
    const bool okx = __ballot(neg) == 0;
    int kk = certified_pick<64>(evx, okx, Kx, Rx, lane, ux, xG, xM, xcat, xpass, 0.0, 0.0, 0.0, pkk);
    if (kk < 0) {
        // the reference's sequential sums (.fs:747-754) on one lane
        if (lane == 0) {
            atomicAdd(&GS_STAT(a)[1], 1ull);
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
    STAMP(14);
    double xw = 0.0;
    if (kk >= 0) {
        double gg, mm;
        evx(pkk, gg, mm);
        xw = kk == 0 ? gg : mm;
    }
    if (kk < 0) {
        if (lane == 0) {
            raise_error(a, 2, gx);  // every category missed (.fs:752)
            a.pos_out[sq] = -1;
        }
    } else {
        const int newp = kk == 0 ? -1 : pkk;
        if (lane == 0) {
            a.pos_out[sq] = newp;
            a.pwms_out[sq] = xw;
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
    wave_sync();  // the staging area is rewritten for the next sequence
}

}  // namespace

template <int WM, int G>
__global__ void __launch_bounds__(64 * kDnaWaves) gs_sweep_dna_kernel(DnaArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    int A = a.A, W = a.W;
    const int AW = A * W, cells = a.cells;
    int32_t *sC = (int32_t *)(lds + O_C);
    int64_t *sT = (int64_t *)(lds + O_T);
    double2 *sPPM = (double2 *)(lds + O_PPM);
    int32_t *sOA = (int32_t *)(lds + O_OA);
    double *sLPG = (double *)(lds + O_LPG);
    const unsigned char *coarse = lds + O_COARSE;
    int32_t *sRes = (int32_t *)(lds + O_RES);
    float *sMisc = (float *)(lds + O_MISC);
    unsigned char *wslice = lds + O_WAVE + wid * kDnaFineBytes;
    int32_t *waggC = (int32_t *)(lds + O_WAGG + wid * WAGG_BYTES);
    int64_t *waggT = (int64_t *)(lds + O_WAGG + wid * WAGG_BYTES + 256);

    STAMP_DECL
    const int err0 = __hip_atomic_load(a.err_code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t rng_stream = a.sweep_ctr ? stream_sweep(*a.sweep_ctr) : 0;

    // ---- prologue: the snapshot's aggregates and the workgroup tables ----
    for (int c = tid; c < cells; c += blockDim.x) {
        const int64_t v = a.agg_in ? a.agg_in[c] : 0;
        if (c < AW)
            sC[c] = (int32_t)v;
        else
            sT[c - AW] = v;
    }
    if (lane < 64) waggC[lane] = 0;
    if (lane < 4) waggT[lane] = 0;
    if (tid < 8) ((uint32_t *)(lds + O_STAT))[tid] = 0u;
    if (tid < 8) sMisc[tid] = 0.0f;
    __syncthreads();
    if (__builtin_amdgcn_readfirstlane(err0) != 0) return;  // the snapshot is void
    const int mode = a.mode;
    // is this snapshot in the all-background state (gs_bgregime.h)?  The host sweeps
    // the rest of the chain with gs_sweep_bg_kernel once it is (scratch: wavefront
    // 1's slice, free until the tile loop)
    if (blockIdx.x == 0 && mode == 0 && a.bg_note) {
        const bool bg = bg_regime(sC, sT, A, W, a.pc, a.den, a.apc, a.Lmax, a.cmin, a.cutoff,
                                  (double *)(lds + O_WAVE + kDnaFineBytes), tid);
        if (tid == 0) *a.bg_note = bg ? 1 : 0;
    }

    if (mode == 0) {
        // binary64 log2 of the table cells, staged in wavefront 0's slice (free until
        // the tile loop)
        double *sLX = (double *)(lds + O_WAVE);
        if (tid < 64) {
            // normalizePPM (.fs:257-260) and its count-minus-one cells; layout [j][e]
            const int j = tid >> 2, e = tid & 3;
            double2 pp = make_double2(1.0, 1.0);
            double lx = 0.0;
            int32_t oa = 0;
            if (j < W && e < A) {
                const int Cc = sC[e * W + j];
                pp.x = ((double)Cc + a.pc) / a.den;
                pp.y = ((double)(Cc - 1) + a.pc) / a.den;
                lx = log2(pp.x);
                if (!(fabs(lx) < 60.0)) sMisc[6] = 1.0f;
                oa = kOaBad;  // own cells have C >= 1
                if (Cc >= 1) {
                    const double d = log2(pp.y) - lx;
                    if (fabs(d) < 16.0) oa = (int32_t)rint(ldexp(d, kFix));
                }
            }
            sPPM[tid] = pp;
            sLX[tid] = lx;
            sOA[tid] = oa;
            if (tid == 0) {
                int64_t s = 0;
                for (int e2 = 0; e2 < A; ++e2) s += sT[e2];
                sT[4] = s;
            }
        }
        __syncthreads();
        if (tid < 4) {
            // the table's PCV estimate: every lane's hold-one-out PCV is this plus
            // a small per-sequence difference the fine table takes up
            const double sbg = (double)sT[4] + (double)W + a.apc;
            const double v = tid < A ? ((double)sT[tid] + a.pc + (double)W / (double)A) / sbg : 1.0;
            const double l = log2(v);
            if (!(fabs(l) < 60.0)) sMisc[6] = 1.0f;
            sLPG[tid] = l;
        }
        if (tid == 4) {
            // max over windows of log2 PPM' <= sum over columns of max_e log2 PPM
            // (own cells only lower it): a sequence whose PCV puts even that below
            // the cut-off has no motif category
            double s = 0.0;
            for (int j = 0; j < W; ++j) {
                double mx = -INFINITY;
                for (int e = 0; e < A; ++e) mx = fmax(mx, sLX[j * 4 + e]);
                s += mx;
            }
            *(double *)(lds + O_UB) = s;
        }
        __syncthreads();
        // pair table of the global counts: code c = s + 4 s', group g = columns 2g, 2g+1
        double tg = 0.0;
        if (tid < 128) {
            const int c = tid >> 3, g = tid & 7, lo = c & 3, hi = c >> 2;
            const int j0 = 2 * g, j1 = 2 * g + 1;
            if (j0 < W && lo < A) tg += sLX[j0 * 4 + lo] - sLPG[lo];
            if (j1 < W && hi < A) tg += sLX[j1 * 4 + hi] - sLPG[hi];
            const float mx = wave_max_nonneg_f32((float)fabs(tg));
            if (lane == 0) atomicMax((unsigned int *)&sMisc[7], __float_as_uint(mx));
        }
        __syncthreads();
        int cs = 8;
        {
            const float mx = sMisc[7];  // <= 240: cs >= 4
            while (cs > 0 && mx * ldexpf(1.0f, cs) > 4000.0f) --cs;
        }
        if (tid < 128) {
            const int c = tid >> 3, g = tid & 7;
            const double q = rint(ldexp(tg, cs));
            sRes[tid] = (int32_t)rint(ldexp(tg - ldexp(q, -cs), kFix));
            // dword (g & 3) of the row holds groups (g & 3) and (g & 3) + 4
            ((short *)(lds + O_COARSE))[c * 8 + (g & 3) * 2 + (g >> 2)] = (short)(int)q;
        }
        if (tid == 0) ((int *)sMisc)[5] = cs;
        __syncthreads();
    }
    int cs = __builtin_amdgcn_readfirstlane(((const int *)sMisc)[5]);
    const bool table_fault = sMisc[6] != 0.0f;
    const int64_t sumT = mode == 0 ? sT[4] : 0;

    // ---- this wavefront's tiles: contiguous, workgroups numbered XCD-major ----
    constexpr int SPT = 64 / G;  // sequences per tile
    const int ntiles = (a.n_local + SPT - 1) / SPT;
    const int xcd = blockIdx.x % kRepl, q8 = gridDim.x / kRepl, r8 = gridDim.x % kRepl;
    const int lblock = xcd * q8 + min(xcd, r8) + (int)(blockIdx.x / kRepl);
    const int nwaves = gridDim.x * kDnaWaves, lwave = lblock * kDnaWaves + wid;
    const int qn = ntiles / nwaves, rn = ntiles % nwaves;
    const int t0 = lwave * qn + min(lwave, rn), tcnt = qn + (lwave < rn ? 1 : 0);
    const int part = lane % G, gbase = lane - part;
    int32_t *ckp = a.ckp + (int64_t)(blockIdx.x * kDnaWaves + wid) * a.maxblk * 64 + lane;
    unsigned char *fine_lane = wslice + lane * 16;
    int nfall = 0, nwhy[5] = {0, 0, 0, 0, 0}, nbgp = 0, nbgk = 0;
    STAMP(0);

    for (int ti = 0; ti < tcnt; ++ti) {
        // the workgroup tables are re-read every tile: keeping them in registers
        // across the loop would cost ~200 VGPRs (occupancy)
        asm volatile("" ::: "memory");
        // ... and so is every value derived from the launch's constants: hoisted out
        // of the loop they would hold ~150 registers across it
        W = *(const volatile int32_t *)&a.W;
        A = *(const volatile int32_t *)&a.A;
        cs = __builtin_amdgcn_readfirstlane(((const int *)sMisc)[5]);
        const int tile = t0 + ti;
        const int seq = tile * SPT + lane / G;
        const bool act = seq < a.n_local;
        const int sq = act ? seq : a.n_local - 1;
        const uint32_t wmask = W >= 16 ? 0xffffffffu : ((1u << (2 * W)) - 1u);
        const int64_t gidx = a.global_offset + sq;
        const int L = act ? a.len[sq] : W;
        const int p = act ? a.pos_in[sq] : -1;
        const int64_t wo = a.pkoff[sq];
        int cmp[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) cmp[e] = (act && e < A) ? a.comp[(int64_t)sq * (A + 1) + e] : 0;
        uint32_t gw = 0;  // the sequence's own segment (snapshot position p)
        if (p >= 0) {
            const uint32_t *q = a.pk + wo + (p >> 4);
            gw = funnel(q[1], q[0], 2 * (p & 15)) & wmask;
        }
        const bool lead = part == 0;
        int newp = p;
        bool keep = act;
        double pw = 0.0;
        bool need_fb = false;
        double pcv[4] = {1.0, 1.0, 1.0, 1.0};
        uint32_t nsw = gw;  // the new segment (mode 1: the snapshot's own)
        STAMP(1);

        if (mode == 0) {
            const double u = a.u_in ? a.u_in[sq] : uniform(a.seed, rng_stream, (uint64_t)gidx);
            // ---- hold-one-out background; E == A: no other symbols ----
            const int64_t tot = sumT + (p >= 0 ? W : L);
            if (act && tot > 2147483647LL) {  // Checked Array.sum (.fs:117)
                if (lead) raise_error(a, 3, gidx);
                keep = false;
            }
            const double sbg = (double)tot + a.apc;
            // (a negative cut-off lets negative weights pass, which the certified pick
            // does not model: every target to the exact rescan)
            bool bad = table_fault || !(fabs(a.cutoff) < 1000.0) || a.cutoff < 0.0;
            // the lane's PCV against the table's: dp[e] = log2 PCV - log2 PCV estimate
            int32_t dp[4] = {0, 0, 0, 0};
            double dmax = 0.0;
            double lpe[4] = {0.0, 0.0, 0.0, 0.0};  // log2 PCV
            double lpmin = INFINITY;
            bool pcv_bad = false;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                if (e < A) {
                    const int64_t bgc = sT[e] + (p >= 0 ? sym_count(gw, e, wmask) : cmp[e]);
                    pcv[e] = ((double)bgc + a.pc) / sbg;  // createNormalizedPCVOfFCV (.fs:119)
                    lpe[e] = log2(pcv[e]);
                    lpmin = fmin(lpmin, lpe[e]);
                    const double d = lpe[e] - sLPG[e];
                    pcv_bad |= !(pcv[e] > 0.0) || !(lpe[e] > -60.0);
                    bad |= !(fabs(d) < 16.0);
                    dmax = fmax(dmax, fabs(d));
                    dp[e] = fabs(d) < 16.0 ? (int32_t)rint(ldexp(d, kFix)) : 0;
                }
            }
            // no window of this sequence can pass the cut-off (log2 PWM' <= log2 PPM -
            // log2 PCV, columnwise maxima; the binary64 folds and logs are inside 1e-9):
            // no motif category, nothing to scan
            const double ub = *(const double *)(lds + O_UB) - (double)W * lpmin;
            const bool noscan = ub < a.cutoff - 1e-9 && !pcv_bad;
            const bool skip_all = __builtin_amdgcn_readfirstlane(__ballot(keep && !noscan) == 0);
            bad |= pcv_bad;
            // own cells: oa[j] = log2 (C - 1 + pc) - log2 (C + pc) at the segment's symbol
            int32_t oa[16];
            int32_t omax = 0;
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const int gj = (int)((gw >> (2 * j)) & 3u);
                const int32_t v = (p >= 0 && j < W) ? sOA[j * 4 + gj] : 0;
                bad |= v == kOaBad;
                oa[j] = v == kOaBad ? 0 : v;
                omax = max(omax, abs(oa[j]));
            }
            // fine scale 2^-m: the fine entries (own cells, PCV difference, coarse
            // rounding) must stay within +-4095 so 8 of them add up in int16
            const double fb = ldexp(1.0, -cs - 1) + 2.0 * dmax + 2.0 * ldexp((double)omax, -kFix) + 1e-6;
            int m = ilogb(4000.0 / fb);
            m = min(m, cs + 11);
            bad |= !(m >= cs);
            if (bad) m = cs;
            const int sh = m - cs, shf = kFix - m;
            const int32_t half = 1 << (shf - 1);
            STAMP(2);
            // ---- this lane's fine table: 16 rows of 8 int16, groups (g, g + 4) per dword ----
            int fqmax = 0;
#pragma unroll
            for (int c = 0; c < (skip_all ? 0 : 16); ++c) {
                const int lo = c & 3, hi = c >> 2;
                const int32_t dpair = dp[lo] + dp[hi];
                const uint4 r0 = *(const uint4 *)(sRes + c * 8), r1 = *(const uint4 *)(sRes + c * 8 + 4);
                const int32_t rr[8] = {(int32_t)r0.x, (int32_t)r0.y, (int32_t)r0.z, (int32_t)r0.w,
                                       (int32_t)r1.x, (int32_t)r1.y, (int32_t)r1.z, (int32_t)r1.w};
                int f[8];
#pragma unroll
                for (int g = 0; g < 8; ++g) {
                    const int j0 = 2 * g, j1 = 2 * g + 1;
                    const int o0 = (int)((gw >> (2 * j0)) & 3u), o1 = (int)((gw >> (2 * j1)) & 3u);
                    int32_t v = rr[g] + (o0 == lo ? oa[j0] : 0) + (o1 == hi ? oa[j1] : 0);
                    v -= j1 < W ? dpair : j0 < W ? dp[lo] : 0;
                    const int qi = (v + half) >> shf;
                    fqmax = max(fqmax, abs(qi));
                    f[g] = qi;
                }
                uint4 row;
                row.x = (uint32_t)(f[0] & 0xffff) | ((uint32_t)f[4] << 16);
                row.y = (uint32_t)(f[1] & 0xffff) | ((uint32_t)f[5] << 16);
                row.z = (uint32_t)(f[2] & 0xffff) | ((uint32_t)f[6] << 16);
                row.w = (uint32_t)(f[3] & 0xffff) | ((uint32_t)f[7] << 16);
                *(uint4 *)(fine_lane + c * 1024) = row;
                __builtin_amdgcn_sched_barrier(0);
            }
            // materialised before the scan: sunk to its use after it, the maximum
            // would keep all 128 table entries live across the scan
            asm volatile("" : "+v"(fqmax));
            bad |= fqmax > 4095;
            // per-window bound: NG fine entries, each the sum of five
            // terms rounded to 2^-kFix and rounded once to 2^-m; the binary64 logs
            // (inside W 2^-40) and the reference's own binary64 rounding (inside 1e-9)
            const int NG = (W + 1) / 2;
            double eps = (double)NG * (ldexp(1.0, -m - 1) + 5.0 * ldexp(1.0, -kFix - 1)) * (1.0 + 0x1.0p-10) +
                         (double)W * 0x1.0p-40 + 1e-9;
            const double ths = ldexp(a.cutoff + eps, m), tls = ldexp(a.cutoff - eps, m);
            const int thr_hi = (int)fmin(fmax(floor(ths), -2147483647.0), 2147483647.0);
            const int thr_lo = (int)fmin(fmax(ceil(tls), -2147483647.0), 2147483647.0);
            {
                int badi = bad ? 1 : 0;
                asm volatile("" : "+v"(badi), "+v"(eps));
                bad = badi != 0;
            }
            wave_sync();
            STAMP(3);

            // ---- scan: every window of the lane's range, one ring step a position ----
            const int K = L - W + 1;
            const int Rn = G == 1 ? K : ((((K + G - 1) / G) + 15) & ~15);
            const int x0 = min(part * Rn, K), x1 = min(K, x0 + Rn);
            const int nwin = x1 - x0;
            const int nch = (nwin + 14 + 63) >> 6;
            const int nch_max = skip_all ? 0 : __builtin_amdgcn_readfirstlane(
                -wave_min_i32(-(keep ? nch : 0)));
            Ring rg;
#pragma unroll
            for (int i = 0; i < 16; ++i) rg.c[i] = rg.f[i] = 0u;
            ScanAcc s{0, 0, 0, false};
            const uint32_t *wp = a.pk + wo + (x0 >> 4);
            uint32_t ww[7];
            uint4 cur = load_words(wp);
            ww[0] = x0 > 0 ? wp[-1] : 0u;
            ww[1] = cur.x;
            ww[2] = cur.y;
            ww[3] = cur.z;
            ww[4] = cur.w;
            Pipe pp;
            fetch<0>(pp, ww, coarse, fine_lane);
            fetch<1>(pp, ww, coarse, fine_lane);
            fetch<2>(pp, ww, coarse, fine_lane);
            fetch<3>(pp, ww, coarse, fine_lane);
            // the prefix sums at the last kChunkCk chunk ends stay in registers (a shift
            // queue: ck[i] = prefix through chunk nch_max - 1 - i, i.e. through block
            // 4q + 2), so the pick reads at most 4 block sums from memory
            int64_t ck[kChunkCk];
#pragma unroll
            for (int i = 0; i < kChunkCk; ++i) ck[i] = 0;
            const bool short_lanes = nch_max <= kChunkCk;  // wave-uniform
            for (int q = 0; q < nch_max; ++q) {
                const uint4 nxt = load_words(wp + 4 * (q + 1));
                ww[5] = nxt.x;
                ww[6] = nxt.y;
                scan_chunk(rg, pp, s, ww, coarse, fine_lane, sh, thr_hi, thr_lo, 64 * q - 14, nwin,
                           ckp + (int64_t)(4 * q) * 64);
                ww[0] = ww[4];
                ww[1] = nxt.x;
                ww[2] = nxt.y;
                ww[3] = nxt.z;
                ww[4] = nxt.w;
#pragma unroll
                for (int i = kChunkCk - 1; i > 0; --i) ck[i] = ck[i - 1];
                ck[0] = s.M;
            }
#ifdef GS_CUT_AFTER_SCAN
            a.pwms_out[sq] = (double)(s.M + s.npass + s.unsure + s.Mb);
            continue;
#endif
            // the trailing partial block
            if (nch_max > 0) ckp[(int64_t)(4 * nch_max - 1) * 64] = s.Mb;
            s.M += s.Mb;
            if (noscan) {
                // the bound is exact: whatever its (skipped or unchecked) scan found
                s.M = 0;
                s.npass = 0;
                s.unsure = false;
                bad = pcv_bad;
            }

            STAMP(4);
            // ---- the sequence's totals over its G lanes ----
            int64_t Mtot = s.M, Opre = 0;
            int npass = s.npass;
            bool uns = s.unsure, badg = bad;
            if constexpr (G > 1) {
#pragma unroll
                for (int d = 1; d < G; d <<= 1) {
                    Mtot += __shfl_xor(Mtot, d, 64);
                    npass += __shfl_xor(npass, d, 64);
                    uns |= __shfl_xor((int)uns, d, 64) != 0;
                    badg |= __shfl_xor((int)badg, d, 64) != 0;
                }
                // exclusive prefix of the parts' sums
#pragma unroll
                for (int q = 0; q < G - 1; ++q) {
                    const int64_t v = __shfl(s.M, gbase + q, 64);
                    if (q < part) Opre += v;
                }
            }
            // ---- certified pick (.fs:746-754) ----
            // backgrounds first: their total lies in [0, Bhi] (each G_k <= pmax^W)
            double pmax = 0.0;
#pragma unroll
            for (int e = 0; e < 4; ++e)
                if (e < A) pmax = fmax(pmax, pcv[e]);
            double pmw = 1.0;
            for (int j = 0; j < W; ++j) pmw = pmw * pmax;
            const double Bhi = (double)K * pmw * (1.0 + 1e-12);
            const double Tt = ldexp((double)Mtot, -m);
            const double eabs = Bhi + (double)npass * eps;
            const double ncat = (double)(K + npass + 2);
            bool ok = keep && !badg && !uns && npass > 0 && Tt > 4.0 * eabs && Tt < INFINITY;
            const double delta =
                (8.0 * ncat + 64.0) * 0x1.0p-53 + eabs / Tt * (1.0 + (Tt + eabs) / (Tt - eabs));
            ok = ok && u > delta;  // not in the background block
            // units of 2^-m: the first passing window j with U <= P_j + D, certified if
            // U lies inside [P_j - s_j + D, P_j - D]
            const double Mt = (double)Mtot;
            double U = u * Mt, D = delta * Mt;
            // ---- background categories (G_k, []) ahead of the motifs (.fs:759-784) ----
            // Where the bound Bhi cannot rule them out (no motif category, or u near
            // the background block), their weights are summed approximately (bg_walk,
            // exact integer log sums) and the pick is located among them or past them.
            const uint32_t *seqw = a.pk + wo;
            bool bg_found = false, bg_cert = false, bg_staged = false;
            int bg_pk = -1;
            const bool bgl = keep && !badg && !uns && !ok;
#ifdef GS_NO_BG
            if (false) {
#else
            if (__builtin_amdgcn_readfirstlane(__ballot(bgl) != 0)) {
#endif
                // skip_all (wave-uniform): no lane built a fine table, so the slots take
                // the ratio tables and staged words of bg_walk_fast, if every lane's
                // words fit (else the integer log walk, bg_walk)
                const int nbw = bgl ? nwin : 0;
                const int nqs = nbw > 0 ? (nbw + W - 2) / 64 + 1 : 0;  // quads with data
                const int nqs_w = __builtin_amdgcn_readfirstlane(-wave_min_i32(-nqs));
                const bool fast = skip_all && nqs_w <= kBgQuads;
                double *rt = (double *)wslice + lane;
                WordsLds wl{wslice + kBgWordsOff + 16 * lane, 0, 0u};
                double pw0 = 1.0;
                if (fast) {
                    // the words of the lane's range, 16 bytes a lane per copy
                    const uint32_t *src = a.pk + wo + (x0 >> 4);
                    for (int i = 0; i < nqs_w; ++i)
                        __builtin_amdgcn_global_load_lds(
                            (const __attribute__((address_space(1))) void *)(src + 4 * i),
                            (__attribute__((address_space(3))) void *)(wslice + kBgWordsOff + 1024 * i), 16,
                            0, 0);
                    if (x0 > 0) wl.prev0 = src[-1];
                    bg_fast_table(rt, pcv);
                    for (int j = 0; j < W; ++j) pw0 = pw0 * pcv[0];
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                }
                double lref = -INFINITY;
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    if (e < A) lref = fmax(lref, lpe[e]);
                const double spread = (double)W * (lref - lpmin);
                // lpq in units 2^-f with W max|lpq| <= 2^30; f >= 16 and no underflow
                const int f = min(28, ilogb(0x1.0p30 / fmax(spread, 0x1.0p-20)));
                const bool bgbad = !fast && (!(f >= 16) || !(spread < 900.0));
                int32_t lpq[4] = {0, 0, 0, 0};
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    if (e < A && !bgbad) lpq[e] = (int32_t)rint(ldexp(lpe[e] - lref, f));
                const BgLut lut = bg_lut(lpq);
                const int fw = bgbad ? 16 : f;
                if (fast) lref = 0.0;  // absolute weights
                // pass 1: the lane's sum, with the running sum at the starts of 8 chunks
                // of whole 16-window blocks; then the sequence's total and the lane's prefix
                const int nb = bgl && !bgbad ? nwin : 0;
                const int Cz = max(16, ((nb + 127) >> 7) << 4);
                BgSum bs{0.0, {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0}, 0, 0, Cz};
                if (fast)
                    bs = bg_walk_fast(wl, x0, nb, W, pw0, rt, bs);
                else
                    bs = bg_walk(seqw, x0, nb, W, fw, lut, bs);
                const double Bl = bs.B;
                double Btot = Bl, Bpre = 0.0;
                bool bgbadg = bgbad;
                if constexpr (G > 1) {
#pragma unroll
                    for (int q = 0; q < G - 1; ++q) {
                        const double v = __shfl(Bl, gbase + q, 64);
                        if (q < part) Bpre = Bpre + v;
                    }
                    Btot = __shfl(Bpre + Bl, gbase + G - 1, 64);
#pragma unroll
                    for (int d = 1; d < G; d <<= 1) bgbadg |= __shfl_xor((int)bgbadg, d, 64) != 0;
                }
                const double scale = exp2((double)W * lref);
                const double Br = Btot * scale, Mr = ldexp(Mt, -m);
                const double T = Br + Mr;
                // every weight's error: the backgrounds' relative bound, the motifs' eps,
                // the scale's rounding
                const double rel = fast ? bg_fast_rel_err(W, K) : bg_rel_err(W, fw);
                const double eb = Br * rel + (double)npass * eps + T * 0x1.0p-50;
                const bool ok2 = bgl && !bgbadg && T > 4.0 * eb && T < INFINITY;
                const double d2 = (8.0 * ncat + 64.0) * 0x1.0p-53 + eb / T * (1.0 + (T + eb) / (T - eb));
                const double Ur = u * T, Dr = d2 * T;
                if (ok2 && Ur - Dr > Br) {
                    // past every background boundary: a motif category
                    ok = true;
                    U = ldexp(Ur - Br, m);
                    D = ldexp(Dr, m);
                }
                // else the first background whose upper boundary reaches Ur - Dr: in
                // the last chunk that starts below it
                const double Ub = Ur / scale, Db = Dr / scale, Tb = Ub - Db;
                const bool mine_bg = ok2 && !ok && Bpre + Bl >= Tb && (part == 0 || Bpre < Tb);
                int cst = 0;
                double P = Bpre;
#pragma unroll
                for (int i = 1; i < 8; ++i) {
                    const bool in = i * Cz < nb && Bpre + bs.pre[i] < Tb;
                    cst = in ? i : cst;
                    P = in ? Bpre + bs.pre[i] : P;
                }
                BgFind bf{P, Tb, Ub, Db, -1, false, false};
                if (fast) {
                    wl.w0 = cst * Cz / 16;
                    bf = bg_walk_fast(wl, x0 + cst * Cz, mine_bg ? nb - cst * Cz : 0, W, pw0, rt, bf);
                } else
                    bf = bg_walk(seqw, x0 + cst * Cz, mine_bg ? nb - cst * Cz : 0, W, fw, lut, bf);
                bg_found = bf.found;
                bg_cert = bf.cert;
                bg_staged = fast;
                bg_pk = bf.pk;
                nbgp += __popcll(__ballot(bgl && lead));
            }
            const double Tg = U - D;
            const bool mine = ok && (double)Opre < Tg && (double)(Opre + s.M) >= Tg;
            // the 16-window block that holds the target: chunk prefixes from registers,
            // then at most 4 block sums from memory (loaded together)
            int bb = -1;
            int64_t Pb = 0;
            if (mine) {
                int b0;
                int64_t run;
                int32_t v[4] = {0, 0, 0, 0};
                if (short_lanes) {
                    int qf = -1;
                    int64_t before = 0, last = 0;
#pragma unroll
                    for (int i = kChunkCk - 1; i >= 0; --i) {  // oldest chunk first
                        const int q = nch_max - 1 - i;
                        const int64_t P = Opre + ck[i];
                        const bool hit = q >= 0 && qf < 0 && (double)P >= Tg;
                        before = (q >= 0 && qf < 0 && !hit) ? P : before;
                        qf = hit ? q : qf;
                        last = q >= 0 ? P : last;
                    }
                    if (qf >= 0) {
                        // chunk qf's blocks 4qf - 1 .. 4qf + 2 (block -1 of chunk 0 is empty)
                        b0 = 4 * qf - 1;
                        run = qf > 0 ? before : Opre;
                    } else {  // past the last chunk end: the trailing block
                        b0 = 4 * nch_max - 1;
                        run = last;
                    }
#pragma unroll
                    for (int t = 0; t < 4; ++t) {
                        const int b = b0 + t;
                        v[t] = b >= 0 && b < 4 * nch_max ? ckp[(int64_t)b * 64] : 0;
                    }
                } else {
                    // long lanes: walk the block sums in memory, 8 loads in flight at a time
                    b0 = -1;
                    run = Opre;
                    const int nb = (nwin + 15) >> 4;
                    for (int c0 = 0; c0 < nb && b0 < 0; c0 += 8) {
                        int32_t x[8];
#pragma unroll
                        for (int t = 0; t < 8; ++t) x[t] = c0 + t < nb ? ckp[(int64_t)(c0 + t) * 64] : 0;
#pragma unroll
                        for (int t = 0; t < 8; ++t) {
                            if (b0 < 0 && c0 + t < nb) {
                                if ((double)(run + x[t]) >= Tg)
                                    b0 = c0 + t;
                                else
                                    run += x[t];
                            }
                        }
                    }
                    if (b0 < 0) b0 = 0;
                    v[0] = ckp[(int64_t)b0 * 64];
                }
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    if (bb < 0 && b0 + t >= 0) {
                        if ((double)(run + v[t]) >= Tg) {
                            bb = b0 + t;
                            Pb = run;
                        }
                        run += v[t];
                    }
                }
            }
            STAMP(5);
            bool found = false, cert = false;
            int pk = -1;
            uint32_t win = 0;
            const bool rer = mine && bb >= 0;
#ifdef GS_NO_RERUN
            if (false) {
#else
            if (__builtin_amdgcn_readfirstlane(__ballot(rer) != 0)) {
#endif
                // re-run the ring over block bb: same tables, same scores
                const int xb = x0 + 16 * max(bb, 0);
                const uint32_t *bp = a.pk + wo + (xb >> 4);
                Words7 bw7;
                uint32_t *bw = bw7.w;
                bw[0] = xb > 0 ? bp[-1] : 0u;
                bw[1] = bp[0];
                bw[2] = bp[1];
                bw[3] = bp[2];
                bw[4] = bw[5] = bw[6] = 0u;
                const BlockScores bs = rerun_scores(bw7, (uint32_t)(fine_lane - lds), sh);
                const int *scs = bs.v;
                // the block's windows in order: the first passing one whose upper
                // boundary reaches U - D holds the pick (branch-free selects)
                int64_t P = Pb;
                const int kb = 16 * max(bb, 0);
#ifdef GS_NO_DEC
                for (int t = 0; t < 0; ++t) {
#else
#pragma unroll
                for (int t = 0; t < 16; ++t) {
#endif
                    const int sc = scs[t];
                    const bool pass = kb + t < nwin && sc > thr_hi;
                    const double lo = (double)P;
                    P += pass ? sc : 0;
                    const double hi = (double)P;
                    const bool hit = rer && !found && pass && U <= hi + D;
                    cert = hit ? (U >= lo + D && U <= hi - D) : cert;
                    pk = hit ? xb + t : pk;
                    found = found || hit;
                }
                if (found) {
                    const int t = pk - xb;
                    win = funnel(bw[2], bw[1], 2 * t);
                }
            }
            STAMP(6);
            // the picked window's weight: the reference's binary64 left fold of
            // PPM'/PCV (.fs:283-292), then log2 (.fs:737)
            bool win_ok = false;
#ifdef GS_NO_FOLD
            if (false) {
#else
            if (found && cert) {
#endif
                pw = picked_weight(win, gw, p >= 0, W, sPPM, pcv[0], pcv[1], pcv[2], pcv[3]);
                win_ok = pw > a.cutoff;
            }
            if (bg_found && bg_cert) {
                // a background category: the reference's binary64 fold of PCV (.fs:123-124)
                uint32_t wv;
                if (bg_staged) {
                    const int r = (bg_pk >> 4) - (x0 >> 4);  // staged word index
                    const uint32_t *b0 = (const uint32_t *)(wslice + kBgWordsOff + 16 * lane);
                    wv = funnel(b0[((r + 1) >> 2) * 256 + ((r + 1) & 3)], b0[(r >> 2) * 256 + (r & 3)],
                                2 * (bg_pk & 15));
                } else {
                    const uint32_t *q = seqw + (bg_pk >> 4);
                    wv = funnel(q[1], q[0], 2 * (bg_pk & 15));
                }
                double Gx = 1.0;
                for (int j = 0; j < W; ++j) {
                    const uint32_t e = (wv >> (2 * j)) & 3u;
                    Gx = Gx * (e == 0 ? pcv[0] : e == 1 ? pcv[1] : e == 2 ? pcv[2] : pcv[3]);
                }
                pw = Gx;
                pk = -1;
                win = 0;
                win_ok = true;
            }
            nbgk += __popcll(__ballot(bg_found && bg_cert));
            // the group's result: from the part that held the pick
            if constexpr (G > 1) {
                const unsigned long long b = __ballot(win_ok);
                const unsigned long long gm = (b >> gbase) & ((1ull << G) - 1ull);
                const int src = gm ? gbase + __ffsll((long long)gm) - 1 : gbase;
                const int pk_s = __shfl(pk, src, 64);
                const double pw_s = __shfl(pw, src, 64);
                const uint32_t win_s = (uint32_t)__shfl((int)win, src, 64);
                win_ok = gm != 0;
                pk = pk_s;
                pw = pw_s;
                win = win_s;
            }
            need_fb = keep && !win_ok;
            // why (gs_stats [2..6]): out of range / in the cut-off band, the exact weight
            // disagreed, the background path could not separate the total or found no
            // lane, no candidate block, u within the bound of a CDF boundary
            {
                const bool lf = need_fb && lead;
                const int why = (badg || uns) ? 0 : (found && cert) ? 1
                              : (bgl && !ok) ? 2 : (!found && !bg_found) ? 3 : 4;
#pragma unroll
                for (int r = 0; r < 5; ++r) nwhy[r] += __popcll(__ballot(lf && why == r));
            }
            newp = pk;
            nsw = win & wmask;
            if (keep && !need_fb && lead) {
                a.pos_out[sq] = newp;
                a.pwms_out[sq] = pw;
            }
            // sequences the bound cannot settle are marked and rescanned after the
            // tile loop (their registers would otherwise be live across the scan)
            if (need_fb && lead) a.pos_out[sq] = kFbMark;
            nfall += __popcll(__ballot(need_fb && lead));
            if (need_fb) keep = false;  // their aggregates come with the rescan
        }

        STAMP(7);
        // ---- aggregates of the new snapshot: C[a][j] += segment, T[a] += comp - segment ----
        {
#ifdef GS_NO_AGG
            const bool km = false;
#else
            const bool km = lead && keep && newp >= 0;
#endif
            // C: two bit-plane ballots per column give the four symbols' counts
            const unsigned long long K = __ballot(km);
            if (K != 0) {
                int cv = 0, segtot[4] = {0, 0, 0, 0};
                for (int j = 0; j < W; ++j) {
                    const unsigned long long b0 = __ballot(km && ((nsw >> (2 * j)) & 1u));
                    const unsigned long long b1 = __ballot(km && ((nsw >> (2 * j + 1)) & 1u));
                    const int c3 = __popcll(b0 & b1), c2 = __popcll(b1 & ~b0), c1 = __popcll(b0 & ~b1);
                    const int c0 = __popcll(K) - c1 - c2 - c3;
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
                // T: composition minus segment of every kept motif
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    if (e < A) {
                        const int t = wave_sum_i32(km ? cmp[e] : 0) - segtot[e];
                        if (lane == 0 && t) waggT[e] += t;
                    }
                }
            }  // K != 0 (the all-background state: no segment to add)
        }
        wave_sync();
        STAMP(8);
    }
    // ---- exact binary64 rescans of the marked sequences, one at a time on the wavefront ----
    // (a device-wide queue shared by all wavefronts was tried: the claims of ~2000
    // wavefronts finishing together serialise on one address and cost milliseconds)
#ifdef GS_NO_RESCAN
    if (false) {
#else
    if (mode == 0 && __builtin_amdgcn_readfirstlane(nfall) > 0) {
#endif
        for (int ti = 0; ti < tcnt; ++ti) {
            const int seq = (t0 + ti) * SPT + lane / G;
            const bool m = part == 0 && seq < a.n_local &&
                           __hip_atomic_load(&a.pos_out[seq], __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT) == kFbMark;
            unsigned long long todo = __ballot(m);
            while (todo) {
                const int src = __ffsll((long long)todo) - 1;
                todo &= todo - 1;
                rescan_seq<WM>(a, __builtin_amdgcn_readlane(seq, src), rng_stream, wslice, sPPM, sT,
                               sumT, lane, waggC, waggT STAMP_ARGS);
            }
        }
    }
    // gs_stats: the wavefronts' counts summed in LDS, one device atomic per nonzero
    // counter and workgroup (after the barrier below)
    uint32_t *sStat = (uint32_t *)(lds + O_STAT);
    if (lane == 0) {
        if (nfall) atomicAdd(&sStat[0], (uint32_t)nfall);
#pragma unroll
        for (int r = 0; r < 5; ++r)
            if (nwhy[r]) atomicAdd(&sStat[1 + r], (uint32_t)nwhy[r]);
        if (nbgp) atomicAdd(&sStat[6], (uint32_t)nbgp);
        if (nbgk) atomicAdd(&sStat[7], (uint32_t)nbgk);
    }

    STAMP(9);
    // ---- flush: the workgroup's sums into replica blockIdx % 8, one atomic a cell ----
    __syncthreads();
    STAMP(10);
    STAMP_FLUSH(tcnt);
    if (tid < 8) {
        const uint32_t v = sStat[tid];
        if (v) atomicAdd(&GS_STAT(a)[tid == 0 ? 0 : tid <= 5 ? tid + 1 : tid + 2], (unsigned long long)v);
    }
    int64_t *dst = a.rep + (int64_t)(blockIdx.x % kRepl) * a.stride;
    for (int c = tid; c < cells; c += blockDim.x) {
        int64_t v = 0;
#pragma unroll
        for (int w2 = 0; w2 < kDnaWaves; ++w2) {
            const unsigned char *wa = lds + O_WAGG + w2 * WAGG_BYTES;
            v += c < AW ? (int64_t)((const int32_t *)wa)[c] : ((const int64_t *)(wa + 256))[c - AW];
        }
        if (v != 0) atomicAdd((unsigned long long *)&dst[c], (unsigned long long)v);
    }
    // ---- the last workgroup reduces the replicas into agg_out and re-zeroes them ----
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    // (no static __shared__ in this kernel: it would move the dynamic carve's base and
    // cost an address add per LDS access)
    int &s_last = *(int *)(lds + O_MISC + 32);
    if (tid == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned int prev = atomicAdd(a.done, 1u);
        s_last = prev == gridDim.x - 1;
    }
    __syncthreads();
    if (!s_last) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    for (int c = tid; c < cells; c += blockDim.x) {
        int64_t v = 0;
#pragma unroll
        for (int r = 0; r < kRepl; ++r)
            v += (int64_t)atomicExch((unsigned long long *)&a.rep[(int64_t)r * a.stride + c], 0ull);
        a.agg_out[c] = v;
    }
    if (tid == 0) {
        atomicExch(a.done, 0u);
        if (a.sweep_ctr && mode == 0) atomicAdd(a.sweep_ctr, 1ull);
    }
}

// Reduce the 8 replicas of the general sweep kernel's aggregates into one vector
// (to = 0) or spread a vector into replica 0 with the others zeroed (to = 1).
__global__ void __launch_bounds__(256) gs_agg_convert_kernel(int64_t *rep, int64_t *vec,
                                                             int32_t cells, int32_t stride,
                                                             int32_t to) {
    for (int c = threadIdx.x; c < kRepl * stride; c += blockDim.x) {
        const int r = c / stride, k = c - r * stride;
        if (to == 0) {
            if (r == 0 && k < cells) {
                int64_t v = 0;
                for (int q = 0; q < kRepl; ++q) v += rep[(int64_t)q * stride + k];
                vec[k] = v;
            }
        } else {
            rep[c] = (r == 0 && k < cells) ? vec[k] : 0;
        }
    }
}

#ifdef GS_DNA_ONLY
#define GS_DNA_FOR_EACH(X) X(16, 1)
#else
// WM is the exact rescan's unroll width: 8 for W <= 8, else 16
#define GS_DNA_FOR_EACH(X) X(8, 1) X(8, 2) X(8, 4) X(16, 1) X(16, 2) X(16, 4)
#endif

static const void *dna_kernel_ptr(int wm, int g) {
#define GS_CASE(W_, G_) \
    if (wm == W_ && g == G_) return (const void *)&gs_sweep_dna_kernel<W_, G_>;
    GS_DNA_FOR_EACH(GS_CASE)
#undef GS_CASE
    return nullptr;
}

int gs_dna_lds_bytes() { return kSmemBytes; }

hipError_t gs_dna_occupancy(int *blocks_per_cu, int W, int G) {
    const void *k = dna_kernel_ptr(W <= 8 ? 8 : 16, G);
    if (!k) return hipErrorInvalidValue;
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, k, 64 * kDnaWaves,
                                                        (size_t)kSmemBytes);
}

hipError_t gs_dna_launch(const DnaArgs &a, int G, int grid, hipStream_t stream, hipEvent_t start,
                         hipEvent_t stop) {
    const void *k = dna_kernel_ptr(a.W <= 8 ? 8 : 16, G);
    if (!k) return hipErrorInvalidValue;
    DnaArgs args = a;
    void *params[] = {&args};
    if (!start && !stop)
        return hipLaunchKernel(k, dim3(grid), dim3(64 * kDnaWaves), params, (size_t)kSmemBytes,
                               stream);
    return hipExtLaunchKernel(k, dim3(grid), dim3(64 * kDnaWaves), params, (size_t)kSmemBytes,
                              stream, start, stop, 0);
}

hipError_t gs_agg_convert_launch(int64_t *rep, int64_t *vec, int32_t cells, int32_t stride,
                                 int32_t to, hipStream_t stream) {
    hipLaunchKernelGGL(gs_agg_convert_kernel, dim3(1), dim3(256), 0, stream, rep, vec, cells,
                       stride, to);
    return hipGetLastError();
}
