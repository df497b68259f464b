// gs_sweep_bg.hip — the synchronous sweep of a snapshot in the all-background state.
//
// MotifSampler.findBestMotifIndicesByWithStartPositions (.fs:935-970), motifAmount
// = 1, when no window of any sequence can pass the cut-off (gs_bgregime.h): every
// target's categories are its K background products G_k = prod_j PCV[s_{k+j}]
// (.fs:123-124, .fs:759-784), the pick is the roulette over them (.fs:746-754) and
// the result is Positions [] with the picked product as PWMS.  A chain started
// from uniform random positions is in this state from its second sweep on (no
// motif category survives the first), so this kernel carries it.  Packed 2-bit
// sequences (gs_sweep_dna.hip layout), alphabets of at most 4 symbols.
//
// G lanes per target (1 .. 64), lane `part` owns windows [part Rn, part Rn + Rn):
//   - the hold-one-out PCV (.fs:945-954) from the snapshot's aggregates;
//   - g_k by incremental binary64 products, g_k = g_{k-1} R[s_{k-1+W}][s_{k-1}]
//     from a per-lane ratio table R[i][o] = PCV[i] (1 / PCV[o]) in LDS, the lane's
//     first window pcv[0]^W times its rows (s_j, 0); each g_k within
//     (5W + 3K + 20) 2^-53 relative of the reference's fold;
//   - the group's total and each lane's prefix, the target u T located in the
//     lane that holds it (a second walk from the last of 8 chunk starts below it),
//     certified against every rounding of the path, the picked window's weight
//     then folded exactly as the reference does;
//   - a pick the bound cannot certify is replayed by one lane with the
//     reference's sequential List.sum and running acc over exact folds (an
//     overrun raises GS_E_ROULETTE_OVERRUN like .fs:752).
// Compiled with -ffp-contract=off.
#include <hip/hip_runtime.h>

#include "gs_bgregime.h"
#include "gs_common.h"
#include "gs_stamps.h"
#include "gs_wave.h"

using namespace gs;

namespace {

constexpr int kBgWaves = 4;
constexpr int O_C = 0;       // int32 [A*W]
constexpr int O_T = 256;     // int64 [4], [4] = sum
                             // 304..640: double [2 W + 3] bg_regime scratch
constexpr int O_WAVE = 640;  // per wavefront: ratio tables [16 rows][64 lanes] binary64
constexpr int kWaveBytes = 16 * 64 * 8;
constexpr int kSmem = O_WAVE + kBgWaves * kWaveBytes;

__device__ __forceinline__ uint32_t funnel(uint32_t hi, uint32_t lo, int sh) {
    return __builtin_amdgcn_alignbit(hi, lo, (uint32_t)sh);
}

__device__ __forceinline__ void raise_error(const BgArgs &a, int code, int64_t gidx) {
    atomicCAS(a.err_code, 0, code);
    atomicMin(a.err_index, (unsigned long long)gidx);
}

// Pass 1 visitor: the lane's sum and its value at the starts of 8 chunks of Cz
// windows (whole 16-window blocks).
struct Sum {
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
    __device__ __forceinline__ void blkw(uint32_t, uint32_t) {}
    __device__ __forceinline__ bool win(int, double g) {
        B = B + g;
        return false;
    }
};
// Pass 2 visitor: from the running sum P, the first window whose upper boundary
// reaches Tb; certified when Ub lies inside [lo + Db, hi - Db].
struct Find {
    double P, Tb, Ub, Db;
    int pk;
    bool found, cert;
    uint32_t w1, w2, wbits;  // the block's words; the picked window's symbols
    static constexpr bool kStops = true;
    __device__ __forceinline__ void blk(int) {}
    __device__ __forceinline__ void blkw(uint32_t a1, uint32_t a2) {
        w1 = a1;
        w2 = a2;
    }
    __device__ __forceinline__ bool win(int k, double g) {
        const double lo = P;
        P = P + g;
        const bool hit = P >= Tb;
        cert = hit && Ub >= lo + Db && Ub <= P - Db;
        pk = hit ? k : pk;
        // window k starts at symbol k % 16 of the block's first word (x0 % 16 == 0)
        wbits = hit ? __builtin_amdgcn_alignbit(w2, w1, (uint32_t)(2 * (k & 15))) : wbits;
        found = hit;
        return hit;
    }
};

template <bool FULL, class V>
__device__ __forceinline__ void walk_block(double &g, bool &done, uint32_t nw, uint32_t ow, int b, int nwin,
                                           int x0, const double *rt, V &v) {
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

__device__ __forceinline__ uint4 load_words(const uint32_t *p) {
    uint4 v;
    __builtin_memcpy(&v, p, 16);  // 4-byte aligned 16-byte load
    return v;
}

// Windows [x0, x0 + nwin) of the sequence at seqw, x0 % 16 == 0, W <= 16, by
// 64-window super-blocks: super-block s reads words 4s - 1 .. 4s + 4 of the range
// (prev, cur, the next super-block's first word); the 16 bytes of the super-block
// after next are requested as one starts, so the register copy that retires them
// (which waits for the load) comes 64 windows later.
template <class V>
__device__ __forceinline__ V walk(const uint32_t *seqw, int x0, int nwin, int W, double pw0, const double *rt,
                                  V v) {
    if (nwin <= 0) return v;
    const uint32_t *wq = seqw + (x0 >> 4);
    uint32_t prev = x0 > 0 ? wq[-1] : 0u;
    uint4 cur = load_words(wq), nxt = load_words(wq + 4);
    double f[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) f[j] = rt[__builtin_amdgcn_ubfe(cur.x, 2 * j, 2) * 64];
    double g = pw0;
#pragma unroll
    for (int j = 0; j < 16; ++j)
        if (j < W) g = g * f[j];
    const int shn = 2 * (W - 1);
    bool done = false;
    for (int b = 0; b < nwin && !done; b += 64) {
        const uint4 nn = load_words(wq + (b >> 4) + 8);
        const uint32_t w[6] = {prev, cur.x, cur.y, cur.z, cur.w, nxt.x};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int bb = b + 16 * k;
            if (bb < nwin && !done) {
                // in-symbols of windows bb..bb+15 start at x0 + bb + W - 1, out-symbols at x0 + bb - 1
                const uint32_t nw = funnel(w[k + 2], w[k + 1], shn), ow = funnel(w[k + 1], w[k], 30);
                v.blk(bb);
                v.blkw(w[k + 1], w[k + 2]);
                if (bb + 16 <= nwin)
                    walk_block<true>(g, done, nw, ow, bb, nwin, x0, rt, v);
                else
                    walk_block<false>(g, done, nw, ow, bb, nwin, x0, rt, v);
            }
        }
        prev = cur.w;
        cur = nxt;
        nxt = nn;
    }
    return v;
}

// The second walk (a visitor that stops: the find pass, at most a chunk of windows
// past its start): one 16-window block per iteration, the next block's word loaded
// as a block starts (compact code; a one-window loop and the 4-block super-block
// walk measured no faster: tools/stamps_bg.py).
template <class V>
__device__ __forceinline__ V walk_short(const uint32_t *seqw, int x0, int nwin, int W, double pw0,
                                        const double *rt, V v) {
    if (nwin <= 0) return v;
    const uint32_t *wq = seqw + (x0 >> 4);
    uint32_t wa = x0 > 0 ? wq[-1] : 0u, wb = wq[0], wc = wq[1];
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
        const uint32_t wd = wq[(b >> 4) + 2];
        const uint32_t nw = funnel(wc, wb, shn), ow = funnel(wb, wa, 30);
        v.blk(b);
        v.blkw(wb, wc);
        walk_block<false>(g, done, nw, ow, b, nwin, x0, rt, v);
        wa = wb;
        wb = wc;
        wc = wd;
    }
    return v;
}

// The reference's binary64 fold of a window's PCV factors (.fs:123-124), its W
// symbols at the low bits of wv.
__device__ __forceinline__ double fold_bits(uint32_t wv, int W, const double (&pcv)[4]) {
    double g = 1.0;
    for (int j = 0; j < W; ++j) {
        const uint32_t e = (wv >> (2 * j)) & 3u;
        g = g * (e == 0 ? pcv[0] : e == 1 ? pcv[1] : e == 2 ? pcv[2] : pcv[3]);
    }
    return g;
}

// The same for window k of the sequence at seqw.
__device__ __forceinline__ double fold_window(const uint32_t *seqw, int k, int W, const double (&pcv)[4]) {
    const uint32_t *q = seqw + (k >> 4);
    const uint32_t wv = funnel(q[1], q[0], 2 * (k & 15));
    double g = 1.0;
    for (int j = 0; j < W; ++j) {
        const uint32_t e = (wv >> (2 * j)) & 3u;
        g = g * (e == 0 ? pcv[0] : e == 1 ? pcv[1] : e == 2 ? pcv[2] : pcv[3]);
    }
    return g;
}

}  // namespace

// The tiles of one wavefront (all of gs_sweep_bg_kernel's work past the snapshot).
template <int G>
__device__ __forceinline__ void bg_tiles(const BgArgs &a, unsigned char *lds, uint64_t rng_stream) {
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int A = a.A, W = a.W;
    const int64_t *sT = (const int64_t *)(lds + O_T);
    double *rt = (double *)(lds + O_WAVE + wid * kWaveBytes) + lane;
    STAMP_DECL
    STAMP(0);
    int64_t sumT = 0;
    for (int e = 0; e < A; ++e) sumT += sT[e];
    const uint32_t wmask = W >= 16 ? 0xffffffffu : ((1u << (2 * W)) - 1u);

    constexpr int SPT = 64 / G;  // targets per wavefront pass
    const int part = lane % G, gbase = lane - part;
    const bool lead = part == 0;
    const int ntiles = (a.n_local + SPT - 1) / SPT;
    int nbgdrop = 0, nser = 0;
    // the next tile's descriptors are requested while this one is swept
    struct Desc {
        int L, p;
        int64_t wo;
        int cmp[4];
    };
    auto load_desc = [&](int tile) {
        const int seq = min(tile * SPT + lane / G, a.n_local - 1);
        Desc d;
        d.L = a.len[seq];
        d.p = a.pos_in[seq];
        d.wo = a.pkoff[seq];
#pragma unroll
        for (int e = 0; e < 4; ++e) d.cmp[e] = e < A ? a.comp[(int64_t)seq * (A + 1) + e] : 0;
        return d;
    };
    const int tstride = gridDim.x * kBgWaves;
    int tile = blockIdx.x * kBgWaves + wid;
    Desc nd = load_desc(min(tile, ntiles - 1));
    for (; tile < ntiles; tile += tstride) {
        STAMP(7);
        const Desc dd = nd;
        if (tile + tstride < ntiles) nd = load_desc(tile + tstride);
        const int seq = tile * SPT + lane / G;
        const bool act = seq < a.n_local;
        const int sq = act ? seq : a.n_local - 1;
        const int64_t gidx = a.global_offset + sq;
        const int L = dd.L, p = dd.p;
        const int64_t wo = dd.wo;
        const uint32_t *seqw = a.pk + wo;
        int cmp[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) cmp[e] = dd.cmp[e];
        uint32_t gw = 0;
        if (p >= 0) gw = funnel(seqw[(p >> 4) + 1], seqw[p >> 4], 2 * (p & 15)) & wmask;
        const double u = a.u_in ? a.u_in[sq] : uniform(a.seed, rng_stream, (uint64_t)gidx);
        // hold-one-out background (.fs:945-954) and PCV (.fs:109-120)
        const int64_t tot = sumT + (p >= 0 ? W : L);
        bool keep = act;
        if (act && tot > 2147483647LL) {  // Checked Array.sum (.fs:117)
            if (lead) raise_error(a, 3, gidx);
            keep = false;
        }
        double pcv[4] = {1.0, 1.0, 1.0, 1.0};
        bool bad = false;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            if (e < A) {
                int x = cmp[e];
                if (p >= 0) {
                    const uint32_t y = ~(gw ^ (0x55555555u * (uint32_t)e));
                    x = __popc(y & (y >> 1) & 0x55555555u & wmask);
                }
                pcv[e] = ((double)(sT[e] + x) + a.pc) / ((double)tot + a.apc);
                bad |= !(pcv[e] > 0.0) || !(pcv[e] < INFINITY);
            }
        }
        // ratio table and the first window's scale
        {
            double inv[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) inv[e] = 1.0 / pcv[e];
#pragma unroll
            for (int c = 0; c < 16; ++c) rt[c * 64] = pcv[c & 3] * inv[c >> 2];
        }
        double pw0 = 1.0;
        for (int j = 0; j < W; ++j) pw0 = pw0 * pcv[0];
        STAMP(1);
        const int K = L - W + 1;
        const int Rn = G == 1 ? K : ((((K + G - 1) / G) + 15) & ~15);
        const int x0 = min(part * Rn, K), nwin = min(K, x0 + Rn) - x0;
        const bool walkable = keep && !bad;
        const int nb = walkable ? nwin : 0;
        const int Cz = max(16, ((nb + 127) >> 7) << 4);
        Sum s1{0.0, {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0}, 0, 0, Cz};
        s1 = walk(seqw, x0, nb, W, pw0, rt, s1);
        STAMP(2);
        // the group's total and this lane's exclusive prefix
        const double Bl = s1.B;
        double incl = Bl;
        bool badg = !walkable;
        if constexpr (G > 1) {
#pragma unroll
            for (int d = 1; d < G; d <<= 1) {
                const double v = __shfl_up(incl, d, 64);
                if (part >= d) incl = incl + v;
            }
#pragma unroll
            for (int d = 1; d < G; d <<= 1) badg |= __shfl_xor((int)badg, d, 64) != 0;
        }
        const double Bpre = incl - Bl;  // within the bound below (rounding of the scan)
        const double T = G > 1 ? __shfl(incl, gbase + G - 1, 64) : Bl;
        // every weight's relative bound, the scans' roundings, the roulette's own
        const double rel = (double)(5 * W + 3 * K + 20) * 0x1.0p-53 * (1.0 + 0x1.0p-10);
        const double eb = T * rel + T * (double)(4 * G + 64) * 0x1.0p-53;
        const double ncat = (double)(K + 2);
        const bool ok = keep && !badg && T > 4.0 * eb && T < INFINITY && !a.force_replay;
        const double d2 = (8.0 * ncat + 64.0) * 0x1.0p-53 + eb / T * (1.0 + (T + eb) / (T - eb));
        const double Ub = u * T, Db = d2 * T, Tb = Ub - Db;
        const bool mine = ok && Bpre + Bl >= Tb && (part == 0 || Bpre < Tb);
        int cst = 0;
        double P = Bpre;
#pragma unroll
        for (int i = 1; i < 8; ++i) {
            const bool in = i * Cz < nb && Bpre + s1.pre[i] < Tb;
            cst = in ? i : cst;
            P = in ? Bpre + s1.pre[i] : P;
        }
        STAMP(3);
        Find f2{P, Tb, Ub, Db, -1, false, false, 0u, 0u, 0u};
        const int xs = x0 + cst * Cz;
        double pws = pw0;
        f2 = walk_short(seqw, xs, mine ? nb - cst * Cz : 0, W, pws, rt, f2);
#if defined(GS_STAMPS) && !defined(GS_TLINE_ONLY) && !defined(GS_TL_FINE) && !defined(GS_TL_PRO)
        // diagnostics: windows left after the chunk start, the hit's offset in it,
        // targets that walk (slots 8..10), the wavefront's maxima
        {
            const int r1 = mine ? nb - cst * Cz : 0, r2 = mine && f2.found ? f2.pk - xs + 1 : 0;
            int m1 = r1, m2 = r2;
            for (int o = 32; o >= 1; o >>= 1) {
                m1 = max(m1, __shfl_xor(m1, o, 64));
                m2 = max(m2, __shfl_xor(m2, o, 64));
            }
            const int nm = __popcll(__ballot(mine));
            if (lane == 0) {
                st_acc[8] += (unsigned long long)m1;
                st_acc[9] += (unsigned long long)m2;
                st_acc[10] += (unsigned long long)nm;
            }
        }
#endif
        STAMP(4);
        const bool got = f2.found && f2.cert;
        double pw = 0.0;
        bool res = got;
        if (got) {
            pw = fold_bits(f2.wbits, W, pcv);  // the words the walk held, no reload
        }
        if constexpr (G > 1) {
            const unsigned long long b = __ballot(got);
            const unsigned long long gm = (b >> gbase) & ((G == 64) ? ~0ull : ((1ull << G) - 1ull));
            const int src = gm ? gbase + __ffsll((long long)gm) - 1 : gbase;
            pw = __shfl(pw, src, 64);
            res = gm != 0;
        }
        STAMP(5);
        nbgdrop += __popcll(__ballot(act && lead && !keep));  // overflow errors: no pick
        nser += __popcll(__ballot(keep && lead && !res));
        if (keep && lead) {
            if (res) {
                a.pos_out[sq] = -1;
                a.pwms_out[sq] = pw;
            } else {
                // the reference's sequential sums (.fs:747-754) over exact folds
                double sacc = 0.0, acc = 0.0;
                for (int k = 0; k < K; ++k) sacc = sacc + fold_window(seqw, k, W, pcv);
                int rk = -1;
                double rw = 0.0;
                for (int k = 0; k < K && rk < 0; ++k) {
                    const double x = fold_window(seqw, k, W, pcv);
                    const double wgt = x / sacc;
                    if (acc <= u && u <= acc + wgt) {
                        rk = k;
                        rw = x;
                    }
                    acc = acc + wgt;
                }
                a.pos_out[sq] = -1;
                if (rk >= 0)
                    a.pwms_out[sq] = rw;
                else
                    raise_error(a, 2, gidx);  // every category missed (.fs:752)
            }
        }
    }
    // statistics without one atomic per wavefront on the same counters (they
    // serialise at the L2: ~100 us for 4096 wavefronts): every target of the rank
    // takes the background path once, counted by workgroup 0; the rare exceptions
    // (overflow errors, sequential replays) adjust the counts where they occur
    if (blockIdx.x == 0 && tid == 0) {
        atomicAdd(&GS_STAT(a)[8], (unsigned long long)a.n_local);
        atomicAdd(&GS_STAT(a)[9], (unsigned long long)a.n_local);
    }
    STAMP(6);
    STAMP_FLUSH(1);
    const int nout = nbgdrop + nser;  // not certified: out of bg_picks
    if (lane == 0 && nout) {
        atomicAdd(&GS_STAT(a)[9], (unsigned long long)(-(long long)nout));
        if (nbgdrop) atomicAdd(&GS_STAT(a)[8], (unsigned long long)(-(long long)nbgdrop));
        if (nser) atomicAdd(&GS_STAT(a)[1], (unsigned long long)nser);
    }
}

template <int G>
__global__ void __launch_bounds__(64 * kBgWaves) gs_sweep_bg_kernel(BgArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int tid = threadIdx.x;
    const int A = a.A, W = a.W, AW = A * W;
    int32_t *sC = (int32_t *)(lds + O_C);
    int64_t *sT = (int64_t *)(lds + O_T);
    const int err0 = __hip_atomic_load(a.err_code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int c = tid; c < AW + A; c += blockDim.x) {
        int64_t v = 0;
        for (int r = 0; r < a.nrep; ++r) v += a.agg_in[(int64_t)r * a.stride + c];
        if (c < AW)
            sC[c] = (int32_t)v;
        else
            sT[c - AW] = v;
    }
    __syncthreads();
    if (a.n_local <= 0) return;  // (the engine's empty launch that loads the code)
    // the counter is read by every workgroup before the last one advances it
    const uint64_t rng_stream = a.sweep_ctr ? stream_sweep(*a.sweep_ctr) : a.stream;
    // a void snapshot (an error raised earlier): no tiles, the counter still advances
    if (__builtin_amdgcn_readfirstlane(err0) == 0) bg_tiles<G>(a, lds, rng_stream);
    if (a.done) {
        // the last workgroup advances the sweep counter (a captured chain's next sweep)
        __syncthreads();
        int *s_last = (int *)(lds + O_C);
        if (tid == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            const unsigned int prev = atomicAdd(a.done, 1u);
            *s_last = prev == gridDim.x - 1;
        }
        __syncthreads();
        if (*s_last && tid == 0) {
            atomicExch(a.done, 0u);
            atomicAdd(a.sweep_ctr, 1ull);
        }
    }
}

static const void *bg_kernel_ptr(int g) {
    switch (g) {
        case 1: return (const void *)&gs_sweep_bg_kernel<1>;
        case 2: return (const void *)&gs_sweep_bg_kernel<2>;
        case 4: return (const void *)&gs_sweep_bg_kernel<4>;
        case 8: return (const void *)&gs_sweep_bg_kernel<8>;
        case 16: return (const void *)&gs_sweep_bg_kernel<16>;
        case 32: return (const void *)&gs_sweep_bg_kernel<32>;
        case 64: return (const void *)&gs_sweep_bg_kernel<64>;
        default: return nullptr;
    }
}

hipError_t gs_bg_occupancy(int *blocks_per_cu, int G) {
    const void *k = bg_kernel_ptr(G);
    if (!k) return hipErrorInvalidValue;
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, k, 64 * kBgWaves, (size_t)kSmem);
}

hipError_t gs_bg_launch(const BgArgs &a, int G, int grid, hipStream_t stream, hipEvent_t start,
                        hipEvent_t stop) {
    const void *k = bg_kernel_ptr(G);
    if (!k) return hipErrorInvalidValue;
    BgArgs args = a;
    void *params[] = {&args};
    if (!start && !stop)
        return hipLaunchKernel(k, dim3(grid), dim3(64 * kBgWaves), params, (size_t)kSmem, stream);
    return hipExtLaunchKernel(k, dim3(grid), dim3(64 * kBgWaves), params, (size_t)kSmem, stream, start,
                              stop, 0);
}

int gs_bg_waves() { return kBgWaves; }
