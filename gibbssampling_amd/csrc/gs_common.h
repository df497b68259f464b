// gs_common.h — definitions shared by host code and gfx950 kernels.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#define GS_HD __host__ __device__ __forceinline__
#else
#define GS_HD static inline
#endif

// The done counters' ordering (the last workgroup of a sweep reduces what every other
// one flushed).  Every value a done counter orders is exchanged through device-scope
// atomics -- the flushes into the aggregate replicas, the counters, the replicas'
// reduction -- and atomics to one address are performed at one point whichever XCD
// issues them, so a workgroup's returning flush atomics, waited for (vmcnt 0) before
// its done-counter atomic, are ordered before it without an agent-scope release: on
// gfx950 that release writes the XCD's L2 back (buffer_wbl2), and the acquire
// invalidates it, in every workgroup of every sweep (config 2, the handed-over tables:
// 22.9 us a sweep with them, 18.5 without).  -DGS_L2_FENCE restores them (A/B builds).
#if defined(__HIPCC__) || defined(__HIP__)
#ifdef GS_L2_FENCE
#define GS_DONE_FENCE(order) __builtin_amdgcn_fence(order, "agent")
#define GS_FLUSH_ADD(p, v) atomicAdd((p), (v))
#else
#define GS_DONE_FENCE(order) ((void)0)
#define GS_FLUSH_ADD(p, v)                                  \
    do {                                                    \
        const unsigned long long gs_r_ = atomicAdd((p), (v)); \
        asm volatile("" ::"v"(gs_r_));                      \
    } while (0)
#endif
#endif

namespace gs {

constexpr int kSlots = 49;      // CompositeVector rows: code - 42 (.fs:17)
constexpr int kSlot0 = 42;
constexpr int kNonAlpha = 64;   // encoded byte of a non-alphabet symbol = 64 + slot
constexpr int kEncSpace = 128;  // size of per-sequence tables indexed by encoded byte
constexpr int kRepl = 8;        // replicas of the aggregate accumulators (one per XCD group)
constexpr int kWave = 64;
constexpr int kStampSlots = 16;  // diagnostic phase stamps: 15 phases + sequence count
// diagnostic timeline (stamps build): kTlMarks s_memrealtime marks per wavefront of
// the last launch, for up to kTlWaves wavefronts, after the phase slots
constexpr int kTlMarks = 8;
constexpr int kTlWaves = 16384;
constexpr long long kStampBytes = 8ll * (kStampSlots + (long long)kTlWaves * kTlMarks);
// The gs_stats counters are kept in kRepl replicas of kStatStride (one 128-byte line
// each), a workgroup adding into replica blockIdx % kRepl: one device-scope atomic
// per counter and wavefront on a single address serialised at the L2 (~10 ns each;
// 4096 wavefronts cost ~80 us).  gs_stats sums the replicas.
constexpr int kStatStride = 16;
// The DNA sweeps' done counters: [0] and [1..kRepl] (gs_sweep_live.hip), then the
// long sweep's kWorkPools work counters, one 128-byte line each at uint 32 (1 + pool)
constexpr int kWorkPools = 16;
constexpr int kDoneBytes = 128 * (1 + kWorkPools);
#if defined(__HIPCC__) || defined(__HIP__)
#define GS_STAT(a) ((a).fallbacks + (blockIdx.x % kRepl) * kStatStride)
#endif

// Counter RNG (splitmix64 finaliser), bit-identical to oracle/gibbs_oracle.c.
GS_HD uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
GS_HD double uniform(uint64_t seed, uint64_t stream, uint64_t index) {
    uint64_t h = mix64(seed ^ mix64(stream ^ mix64(index)));
    return (double)(h >> 11) * 0x1.0p-53;
}
GS_HD int32_t uniform_int(uint64_t seed, uint64_t stream, uint64_t index, int32_t k) {
    int32_t r = (int32_t)(uniform(seed, stream, index) * (double)k);
    return r >= k ? k - 1 : r;
}
GS_HD uint64_t stream_sweep(uint64_t t) { return (1ULL << 40) | t; }
GS_HD uint64_t stream_init(uint64_t target) { return (2ULL << 40) | target; }
GS_HD uint64_t stream_init_shared() { return 3ULL << 40; }

// ln(2.0) correctly rounded: FSharpAux log2 x = Math.Log(x)/Math.Log(2.0).
constexpr double kLn2 = 0x1.62e42fefa39efp-1;

// Error budget of the binary32 transcendentals the certified scan uses
// (gs_wave.h flog2 / fexp2).  gs_fastmath_check measures them on every binary32
// mantissa: 1.51 ulp (log2, incl. rounding the binary64 mantissa) and 1.39 ulp
// (exp2) on MI355X; the budget is 2.6x / 2.9x those and the GPU tests assert
// the measurement stays within half of it.
constexpr double kLog2AbsErr = 0x1.0p-22;  // |log2 error| on mantissas in [0.5, 1)
constexpr double kExp2RelErr = 0x1.0p-22;  // relative error of 2^f, f in [0, 1)

// Scan modes of the sweep kernel.
constexpr int kScanCertified = 0;  // binary32 log-domain scan + certified decisions
constexpr int kScanExact = 1;      // binary64 folds for every window (diagnostics)

// Wavefronts per workgroup of the sweep kernel, by scan group H (measured:
// profiles/r1/s2/ab_waves_per_block.json): 4 for |symbols| <= 16 (DNA: 2 and 4 alike,
// 8 slower), 12 above (protein cfg5: 237 / 195 / 177 us at 4 / 2 / 8; 12 = one
// workgroup of 3 wavefronts a SIMD once the rescans' exact table shares the groups'
// log tables, round 5).  The launch halves it while the workgroup's LDS does not fit.
GS_HD constexpr int sweep_waves(int H) { return H == 1 ? 12 : 4; }

// Kernel arguments of the fused sweep kernel (gs_sweep.hip).
struct SweepArgs {
    const uint8_t *seq;   // encoded symbols; sequence n at seq + doff[n] (16-byte aligned)
    const uint8_t *pseq;  // the same layout in pair codes s[i] + E*s[i+1] (E <= 16; s[L] = 0)
    const int64_t *doff;
    const int32_t *len;
    const int32_t *comp;  // [n_local][E+1]: symbol counts by encoded symbol, then the
                          // count of symbols outside the alphabet (static per sequence)
    int32_t n_local;
    int32_t scan;         // kScanCertified / kScanExact
    int32_t mode;         // 0 = sweep, 1 = aggregates of pos_in only
    int64_t global_offset;
    int32_t A, W;
    int32_t E;            // encoded symbol space: alphabet 0..A-1, other symbols A..E-1
    int32_t cells;        // A*W count cells followed by A composition cells
    int32_t stride;       // int64 elements per replica (padded)
    double pc, cutoff, thr_lo, den, apc;
    double thr_hi;        // S > thr_hi => log2 S > cutOff certainly (the log can wait)
    const double *pcv_fixed;  // [E] by encoded symbol: the caller's PCV (ByPCV twins), or null
    const int32_t *pos_in;
    int32_t *pos_out;
    double *pwms_out;
    const double *u_in;   // explicit uniforms (nullable -> counter RNG)
    uint64_t seed, stream;
    // 16 bytes that keep the fields below at the kernarg offsets measured fastest
    // (cfg2: 20.0 vs 21.9 us per sweep with them 16 bytes lower; 8 or 32 bytes do
    // as well, the same 16 bytes in front of `seq` do not; profiles/r1/s2/ab_*.json)
    uint64_t layout_pad[2];
    const int64_t *agg_in;   // kRepl * stride, aggregates of the snapshot
    int64_t *agg_out;        // kRepl * stride, accumulates aggregates of the new snapshot
    int64_t *agg_zero;       // kRepl * stride, zeroed for the next sweep (nullable)
    int32_t *err_code;
    unsigned long long *err_index;
    unsigned long long *fallbacks;  // GS_N_STATS counters (gs_stats)
    unsigned long long *stamps;  // diagnostic build only (GS_STAMPS): per-phase cycles
    // dynamic LDS carve (bytes): workgroup-shared part, then 4 wavefront slices
    // workgroup-shared part, 4 wavefront slices, each ending in 64/gl group slices
    int32_t gl;           // lanes per sequence (16, 32 or 64)
    int32_t waves;        // wavefronts per workgroup (sweep_waves(H), or fewer for LDS)
    int32_t o_cg, o_T, o_ppmG, o_ppmM, o_lppmG, o_bmax, o_lT, o_wave, wave_bytes;
    int32_t w_aggC, w_aggT, w_tab, w_res, w_misc, w_group, group_bytes;
    int32_t g_lt, g_gt, g_seq, g_pcv, g_lpcv, g_cmax, g_cnt, g_wfac;
    // workgroup 0 writes whether this sweep's snapshot is in the all-background
    // state (gs_bgregime.h) to *bg_note (nullable); the host then sweeps the rest
    // of the chain with gs_sweep_bg_kernel (the state is absorbing)
    int32_t *bg_note;
    int32_t Lmax, cmin;
    unsigned int *done;   // nullable: finished workgroups; the last one folds agg_out's
                          // replicas into replica 0 and resets it (the multi-GPU exchange)
    int64_t seq_stride;   // > 0: every sequence is Lmax long and sequence n starts at
                          // n * seq_stride (no descriptor round trip); 0: descriptors
    int32_t wq, wr;       // n_local / (wavefronts of the launch) and the remainder (set by
                          // gs_sweep_launch)
    int32_t ek;           // 4: the four-symbol kernel and its layout (host carve), else 0
    // EK = 0: the groups' log tables, contiguous in the wavefront slice (group gi's at
    // w_lt + gi * lt_bytes); the rescans' exact table w_tab aliases them when they are
    // at least its size (they are dead while a rescan runs: restored after it)
    int32_t w_lt, lt_bytes;
    // EK = 4: the workgroup tables of the snapshot (ek4_layout [0, o_wave): C, T, PPM,
    // PPM', their log2, the PCV log table), built once a sweep and copied by every
    // workgroup's prologue: ftab_in (never null on that path) is this sweep's, and with
    // ftab_out set the last workgroup (two-level done counter, `done`) builds the next
    // sweep's from the replicas it accumulated
    const unsigned char *ftab_in;
    unsigned char *ftab_out;
    int32_t fold;         // with `done`: the last workgroup folds the replicas into replica 0
    // H = 1 (more than 16 symbols): group gi's motif table at w_lt + gi * lt_bytes
    // (binary32 log2 PPM', code-major rows of mt_stride(WM) entries), its fixed-point
    // prefix sums of the positions' log2 PCV at w_pfx + gi * pfx_bytes (= lt_bytes)
    int32_t w_pfx, pfx_bytes;
};
// bytes of one workgroup-table image (ek4_layout o_wave at WM = 32, rounded up)
constexpr int kFtabBytes = 8192;

// The DNA sweep kernel (gs_sweep_dna.hip): alphabets of at most 4 symbols with no
// other symbol in the data, motifs of at most 16 columns.  One lane scores one
// sequence (or 1/G of it) as a sliding ring over 2-bit packed pair codes.
constexpr int kDnaMaxW = 16;
constexpr int kDnaMaxL = 8192;      // longest sequence (the fallback stages it in LDS)
constexpr int kDnaWaves = 4;        // wavefronts per workgroup
// per wavefront: the fine table [16 codes][64 lanes][8 x int16] (16 KB), or, in a
// wavefront of background walks, the ratio tables (8 KB) and the lanes' staged
// words (10 KB); two 4-wavefront workgroups still fit a CU's 160 KB
constexpr int kDnaFineBytes = 18 * 1024;

struct DnaArgs {
    const uint32_t *pk;       // 2-bit symbols, 16 per word (symbol i at bits 2(i % 16))
    const int64_t *pkoff;     // [n_local] first word of sequence n (a multiple of 4)
    const int32_t *len;
    const int32_t *comp;      // [n_local][E+1] static symbol histograms (E == A)
    int32_t n_local, A, W, mode;   // mode 0: sweep, 1: aggregates of pos_in only
    int64_t global_offset;
    int32_t cells, stride;    // A*W + A aggregate cells; replica stride (int64 elements)
    double pc, cutoff, den, apc;
    double thr_lo;            // products below it certainly fail the cut-off (exact rescans)
    const int64_t *agg_in;    // [cells] C then T of the snapshot (all ranks)
    int64_t *rep;             // kRepl * stride, zero on entry; the last workgroup zeroes it again
    int64_t *agg_out;         // [cells] this rank's C then T of the new snapshot
    unsigned int *done;       // finished workgroups (0 on entry; the last one resets it; the live
                              // sweep counts per replica group in [1..8], then in [0])
    const int32_t *pos_in;
    int32_t *pos_out;
    double *pwms_out;
    const double *u_in;       // explicit uniforms, or null: counter RNG
    uint64_t seed;
    unsigned long long *sweep_ctr;  // RNG stream of this sweep; the last workgroup adds 1
    int32_t *ckp;             // per wavefront [maxblk][64] block sums of the passing scores
    int32_t maxblk;
    int32_t *err_code;
    unsigned long long *err_index;
    unsigned long long *fallbacks;
    unsigned long long *stamps;  // diagnostic build only (GS_STAMPS): per-phase cycles
    // workgroup 0 writes whether this sweep's snapshot is in the all-background
    // state (gs_bgregime.h) to *bg_note (nullable), as in SweepArgs
    int32_t *bg_note;
    int32_t Lmax, cmin;
    int32_t live_slice;       // gs_sweep_live_kernel: LDS bytes per wavefront (set by its launcher)
    int32_t live_force;       // tests: every target through the exact rescan
    const int64_t *compsum;   // [A] the rank's symbol totals: T starts from them (the live sweep)
    int32_t pk_stride;        // > 0: every sequence is Lmax long and pkoff[n] = n * pk_stride
                              // (gs_sweep_long_kernel: the words need no descriptor); 0: ragged
    // the in-kernel exchange of the aggregate vector (gs_exchange_open; live and long
    // sweeps): the last workgroup writes this rank's partial into every rank's exchange
    // buffer, waits for every rank's and sums them into agg_out -- the sweep's all-reduce
    // without a collective launch.  Null: off (the communicator's or the caller's)
    int64_t *const *xpeer;    // [xranks] every rank's exchange buffer, mapped here (kXchBytes)
    unsigned long long *xseq; // this context's exchange count (the sweeps' sequence numbers)
    int32_t xranks, xrank;
};
// An exchange buffer: [2 parities][kXchRanks][2 kXchStride] uint64 words, cell c of a
// rank's partial in words 2c (low half) and 2c + 1 (high half), each word = (flag << 32)
// | half, the flag the sweep's sequence number (never 0): a word carries its own
// arrival, so neither side needs a fence (each 8-byte store is single-copy atomic)
constexpr int kXchRanks = 64;
constexpr int kXchStride = 80;  // >= A W + A cells of the packed-layout sweeps (A <= 4, W <= 16)
constexpr long long kXchBytes = 8LL * 2 * kXchRanks * 2 * kXchStride;

// The live-chain sweep (gs_sweep_live.hip): the DnaArgs layout and protocol, a
// filter scan over an upper-bound table, refinement of the windows that can pass.
constexpr int kLiveWaves = 8;   // wavefronts per workgroup (they share the workgroup's tables)
// windows a lane owns at most (G lanes per target): 16-aligned ranges of K / G
GS_HD int live_rn_max(int Lmax, int W, int G) {
    const int K = Lmax - W + 1 > 1 ? Lmax - W + 1 : 1;
    return G == 1 ? K : ((((K + G - 1) / G) + 15) & ~15);
}
// per wavefront, [entry][64 lanes]: the lanes' candidate masks (one bit a window,
// 4 B), their sequence words (4 B: window k reads words k/16 and k/16 + 1), their
// 32-window chunk sums of passing weights (8 B)
GS_HD int live_nmw(int rn) { return (rn + 31) / 32; }
GS_HD int live_nw(int rn) { return (rn + 15) / 16 + 1; }
GS_HD int live_nb(int rn) { return (rn + 31) / 32; }
// the exact rescan of one target (in the same slice): the unpacked sequence, then the
// (PWM, PCV) table [4][wm + 1] x 16 B and scratch
GS_HD int live_tab_off(int Lmax, int wm) { return (Lmax + wm + 112 + 15) & ~15; }
GS_HD int live_rescan_slice(int Lmax, int wm) { return live_tab_off(Lmax, wm) + 4 * (wm + 1) * 16 + 64; }
// the slice: the larger of the two uses, a multiple of 256 bytes
GS_HD int live_slice_bytes(int Lmax, int W, int G, int wm) {
    const int rn = live_rn_max(Lmax, W, G);
    const int lanes = 256 * (live_nmw(rn) + live_nw(rn)) + 512 * live_nb(rn);
    const int rs = (live_rescan_slice(Lmax, wm) + 255) & ~255;
    return lanes > rs ? lanes : rs;
}

// The sweep of a snapshot in the all-background state (gs_sweep_bg.hip): packed
// 2-bit sequences as for the DNA kernel.  The host launches it only for a snapshot
// known to be in the state with no target keeping a motif (C = 0, T = 0: nrep = 0,
// the aggregates are not read), which every later snapshot of the chain is too.
struct BgArgs {
    const uint32_t *pk;
    const int64_t *pkoff;
    const int32_t *len;
    const int32_t *comp;      // [n_local][A+1]
    int32_t n_local, A, W, Lmax, cmin;
    int64_t global_offset;
    int32_t nrep, stride;     // agg_in: nrep replicas of stride int64 (1: the DNA vector)
    double pc, cutoff, den, apc;
    const int64_t *agg_in;
    const int32_t *pos_in;
    int32_t *pos_out;
    double *pwms_out;
    const double *u_in;       // explicit uniforms, or null: counter RNG
    uint64_t seed, stream;    // stream: the RNG stream when sweep_ctr is null
    unsigned long long *sweep_ctr;  // the RNG stream's sweep index (nullable)
    unsigned int *done;       // nullable: finished workgroups; the last one advances
                              // *sweep_ctr and resets it (a captured chain's next sweep)
    int32_t *err_code;
    unsigned long long *err_index;
    unsigned long long *fallbacks;
    int32_t force_replay;     // tests: every pick by the exact sequential replay
    unsigned long long *stamps;  // diagnostic build only (GS_STAMPS): per-phase cycles
};

// Group size of the certified scan's log tables: pairs of positions when the
// pair code s[i] + E*s[i+1] fits a byte, single positions otherwise.
GS_HD int scan_group(int E) { return E <= 16 ? 2 : 1; }

// Row strides (in entries) of the sweep kernel's symbol-major LDS tables for the
// unroll width WM (a multiple of 4): odd, so that rows of different symbols or
// codes start in different LDS banks.
constexpr int tab_stride(int wm) { return wm + 1; }     // exact (PWM, PCV), 16 B entries
constexpr int lt_stride(int wm) { return wm + 1; }      // (log2 PWM, log2 PCV), 8 B entries
constexpr int gt_stride(int wm) { return wm / 2 + 1; }  // pair sums, 8 B entries
constexpr int mt_stride(int wm) { return wm + 1; }      // H = 1 motif terms log2 PPM', 4 B entries (odd)

// LDS layout of the four-symbol sweep kernel (gs_sweep_kernel<WM, 2, GL, 4>): every
// offset is a compile-time constant of (WM, GL) — ds_read immediates instead of one
// SGPR or VGPR per base — sized by WM >= W; the group slice ends in the sequence,
// whose length sets the group and wavefront strides (SweepArgs group_bytes /
// wave_bytes).  The host carve (gs_engine.cpp sweep_carve) uses the same function.
struct Ek4Layout {
    int o_cg, o_T, o_ppmG, o_ppmM, o_lppmG, o_bmax, o_lT, o_wave;
    int w_aggC, w_aggT, w_tab, w_res, w_misc, w_group;
    int g_lt, g_gt, g_pcv, g_lpcv, g_cmax, g_seq;
};
constexpr int ek4_a16(int x) { return (x + 15) & ~15; }
constexpr Ek4Layout ek4_layout(int WM, int GL) {
    Ek4Layout l{};
    int o = 0;
    l.o_cg = o;    o = ek4_a16(o + 4 * 4 * WM);
    l.o_T = o;     o = ek4_a16(o + 8 * 5);
    l.o_ppmG = o;  o = ek4_a16(o + 8 * 4 * WM);
    l.o_ppmM = o;  o = ek4_a16(o + 8 * 4 * WM);
    l.o_lppmG = o; o = ek4_a16(o + 16 * 4 * WM);
    l.o_bmax = o;  o = ek4_a16(o + 4 * 8);
    l.o_lT = o;    o = ek4_a16(o + 8 * (4 * (WM + 1) + 1));
    l.o_wave = o;
    o = 0;
    l.w_aggC = o;  o = ek4_a16(o + 4 * 4 * WM);
    l.w_aggT = o;  o = ek4_a16(o + 8 * 4);
    l.w_tab = o;   o = ek4_a16(o + 16 * tab_stride(WM) * 4);
    l.w_res = o;   o = ek4_a16(o + 16 * 64);
    l.w_misc = o;  o = ek4_a16(o + 32);
    l.w_group = o;
    o = 0;
    l.g_lt = o;    // (none: the pair table is built directly)
    l.g_gt = o;    o = ek4_a16(o + 128 * (WM / 2));  // group-major [WM/2][16 codes]
    l.g_pcv = o;   o = ek4_a16(o + 8 * 4);
    l.g_lpcv = o;  o = ek4_a16(o + 8 * 4);
    l.g_cmax = o;  o = ek4_a16(o + 16 * WM); // the picked window's factors alias it
    // the sequence (Lmax + WM + 96 bytes, + 64: the odd group's is 64 B further), then
    // the scan's copy of its codes x 8 (as long)
    l.g_seq = o;
    return l;
}

static_assert(ek4_layout(32, 16).o_wave <= kFtabBytes, "workgroup-table image");

// findBestMotifIndicesWithStartPositions (.fs:885-929) and its site-sampler twin
// getBestPWMSsWithStartPositions (.fs:554-585): Gauss–Seidel passes, one
// persistent workgroup scoring consecutive targets speculatively (gs_greedy.hip).
struct GreedyArgs {
    const uint8_t *seq;
    const int64_t *doff;
    const int32_t *len;
    const int32_t *comp;     // [n][E+1] static symbol histograms
    int32_t n;               // every sequence of the sampler (single device)
    int32_t A, W, E;
    int32_t cells, stride;
    double pc, cutoff, thr_lo, den, apc;
    int32_t max_passes;
    int64_t *agg;            // kRepl * stride: read at start, final aggregates written back
    int32_t *pos;            // [n] in/out (acc of .fs:886)
    double *pwms;            // [n] in/out
    int32_t *passes_out;
    int32_t *err_code;
    unsigned long long *err_index;
    // LDS carve (bytes): workgroup part, then the visit ring (2 * waves slots), then
    // one slice per wavefront
    int32_t o_C, o_T, o_ppmG, o_ppmM, o_ctl;
    int32_t o_ring, ring_seq_bytes;          // slot s: sequence bytes at o_ring + s * ring_seq_bytes
    int32_t o_rt, o_rL, o_rp, o_rpw, o_rcomp;  // slot metadata: target, length, position, PWMS, comp[64]
    int32_t o_wave, wave_bytes;
    int32_t w_tab, w_pcv;                    // motif: (PWM, PCV) table, PCV
    int32_t w_dt, w_bg, w_comp;              // site: D_k table [K][A], background, composition
    int32_t site;                            // 0: motif sampler greedy, 1: site sampler
    int32_t site_coop;                       // site: all wavefronts on a lone visit
    int32_t motif_coop;                      // motif sampler: the same for visits with K*W >= it (0: off)
    float coop_rate;                         // site: keep lone-visit steps while moves/visit > it (0: off)
    int32_t dt16;                            // site: D table as uint16 (K * W < 2^16)
    // mid-pass exit (hand-over to the speculative steps): after every exit_chunk
    // visits, stop when fewer than exit_chunk / exit_ratio of them moved; exit_out =
    // {visits of the pass done (0: no exit), the pass moved}.  exit_chunk 0: off.
    int32_t exit_chunk, exit_ratio;
    int32_t *exit_out;
    int32_t o_red;                           // [4 * waves] u64: workgroup argmax scratch
    const double *pcv_fixed;                 // [E]: the caller's PCV (ByPCV / WithBPV), or null
    unsigned long long *stamps;  // diagnostic build only (GS_STAMPS)
};

struct SpecCtl;
// Speculative Gauss–Seidel step result of the site sampler: getBestPWMSs of one visit.
struct SiteRes {
    double score;
    int32_t pos, pad;
};

// getPWMOfRandomStarts, per-target argmax scan (gs_starts.hip).
struct StartsArgs {
    const uint8_t *seq;
    const int64_t *doff;
    const int32_t *len;
    int32_t n_local;
    int32_t mode;            // 0 exact per-target draws, 1 one shared start vector,
                             // 2 the explicit start vector `starts`
    int64_t global_offset;
    int32_t A, W;
    int32_t cells, stride;
    double pc, den, apc;
    uint64_t seed;
    const int32_t *starts;   // mode 2: [n_local] start of every sequence
    const double *pcv_fixed; // [E]: the caller's PCV (…WithBPV: no background, no drift), or null
    const double *ppm_fixed; // [A][W]: the caller's PPM (getMotifsWithBestPWMSOfPPM), or null
    // modes 1/2: aggregates of the start vector; mode 0: aggregates of an
    // all-sequences snapshot (only the composition cells are used there).
    const int64_t *agg;      // kRepl * stride
    const int32_t *cpart;    // mode 0: [n_global][A*W] counts of the others' random segments
    double *score_out;
    int32_t *pos_out;
    int32_t *err_code;
    unsigned long long *err_index;
    int32_t o_ppm, o_Dt, o_cg, o_compall, o_bg, o_comp, o_seq;
    // speculative Gauss–Seidel (mode 2 on the live positions): visits
    // [spec_ctl->base, + gridDim.x) scored into spec_res instead of score_out/pos_out
    const SpecCtl *spec_ctl;
    SiteRes *spec_res;
    // getBestPWMSs of ONE target against the caller's FCV (gs_best_pwms): single =
    // target + 1 (0: every local target), bg_fixed = [A] background counts by
    // alphabet symbol then the sum over all 49 slots (nullable)
    int32_t single;
    const int64_t *bg_fixed;
    // the D table [(Lmax+1)][A] in HBM (one slice of dt_stride int32 per workgroup)
    // when it does not fit the LDS with the rest (long sequences); null: in LDS
    int32_t *dt_global;
    int64_t dt_stride;
};

// Commit step of the site sampler's speculative Gauss–Seidel passes (gs_starts.hip).
struct SiteCommitArgs {
    SpecCtl *ctl;
    const SiteRes *res;
    int32_t slots, n, A, W, max_passes;
    const uint8_t *seq;
    const int64_t *doff;
    double *score;           // acc scores, in/out
    int32_t *pos;            // acc positions, in/out
    int64_t *agg;            // replica 0 of the live aggregates (C then T cells)
};

// motifAmount >= 1 with Positions lists (gs_multi.hip): the sweep
// findBestMotifIndicesByWithStartPositions (.fs:935-970) and the greedy passes
// findBestMotifIndicesWithStartPositions (.fs:885-929) over the categories of
// calculateNormalizedSegmentScores (.fs:759-784) including every combination of
// calculatePWMsForSegmentCombinations (.fs:727-742).
// A MotifIndex list of sequence n is (cnt[n], pos[n*cap + 0 .. cnt[n])), in F#
// list order (the most recently consed position first).
constexpr int kMultiMaxAmount = 16;   // motifAmount bound (positions per list)
constexpr int kMultiErrArena = 15;    // device status: a target's categories overflowed its arena
// Speculative greedy passes of the list path: visits [base, base + slots) are scored
// in parallel against the live aggregates, then committed in order up to the first
// one that moves its Positions list.
struct SpecCtl {
    int32_t base, pass, changed, done;
};
struct SpecRes {
    int32_t cnt, accept, moved, status;
    int32_t pos[kMultiMaxAmount];
    double pw;
};
struct MultiArgs {
    const uint8_t *seq;
    const int64_t *doff;
    const int32_t *len;
    const int32_t *comp;       // [n_local][E+1]
    int32_t n_local;
    int64_t global_offset;
    int32_t A, W, E, M;        // M = motifAmount
    int32_t cap_in, cap_out;   // list capacities of the snapshot / of the results
    double pc, cutoff, den, apc;
    double thr_lo, thr_hi;     // products below / above: log2 certainly fails / passes cutOff
    const double *pcv_fixed;   // [E] the caller's PCV (…ByPCV twins), or null
    const int32_t *cnt_in, *pos_in;   // snapshot (sweep); unused by the greedy
    int32_t *cnt_out, *pos_out;       // sweep: results; greedy: the live acc, in/out
    double *pwms_out;
    const int64_t *agg;        // [A*W + A]: C then T of the snapshot (sweep / greedy start)
    const double *u;           // explicit uniforms (nullable -> counter RNG)
    uint64_t seed, stream;
    const int32_t *targets;    // nullable: all local targets
    int32_t n_targets;
    double *scratch;           // per workgroup slot: S[kmax], G[kmax], then the arena
    int64_t slot_doubles;
    int32_t kmax, arena_cap;   // windows per sequence (max), categories per slot
    int32_t *ovf_list, *ovf_count;   // targets whose categories overflowed the arena
    int32_t max_passes;        // greedy
    int32_t *passes_out;       // greedy
    unsigned long long *err;   // packed (global index << 4) | status, atomicMin
    unsigned long long *fallbacks;   // [1]: picks taken by the serial replay
    // speculative greedy (gs_multi_spec_*): control block, one result per slot,
    // the live aggregates (read by the scoring kernel, updated by the commit kernel)
    struct SpecCtl *spec_ctl;
    struct SpecRes *spec_res;
    int32_t spec_slots;
    int64_t *agg_rw;
    int32_t o_tab, o_pcv, o_seq, o_agg;   // LDS carve (bytes)
    int32_t o_S;               // greedy: LDS window scores S[kmax], G[kmax] (-1: in scratch)
};

// Exact-mode initialiser: per-target count matrices over this rank's sequences.
struct PartialArgs {
    const uint8_t *seq;
    const int64_t *doff;
    const int32_t *len;
    int32_t n_local;
    int64_t global_offset;
    int64_t n_global;
    int32_t A, W;
    uint64_t seed;
    int32_t *cpart;          // [n_global][A*W]
};

}  // namespace gs
