// gs_ctx.h — host-side state of one context (struct gs_ctx), the engine's internal
// interface (gs_engine.cpp) and the kernel launchers (*.hip).  Internal: the public
// C ABI is include/gibbs_hip.h, implemented in gs_api.cpp.
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/gibbs_hip.h"
#include "gs_common.h"

using namespace gs;

// Engine tuning: fixed defaults (the measured choices), changed only
// through gs_set_tuning (diagnostics, A/B runs, tests of every engine path);
// the library never reads the environment.  Set before gs_set_sequences.
struct gs_tuning {
    int32_t blocks_per_cu_cap = 8;  // cap on resident sweep workgroups per CU (grid sizing)
    int32_t group_lanes = 0;  // general sweep: lanes per sequence (16, 32, 64); 0 = automatic
    int32_t sweep_waves = 0;  // general sweep: wavefronts per workgroup (1, 2, 3, 4, 6, 8, 12); 0 = automatic
    int32_t dna_mode = -1;  // DNA sweep kernel: -1 automatic (sizes where it is the faster kernel), 0 never, 1 whenever admissible
    int32_t dna_G = 0;  // DNA sweep: lanes per sequence (1, 2, 4); 0 = automatic
    int32_t live_mode = -1;  // DNA-path sweeps by the live-chain kernel (gs_sweep_live.hip): -1 / 1 yes (1: at every size), 0 the older DNA kernel
    int32_t live_G = 0;      // its lanes per target (1, 2, 4, 8); 0 = automatic
    int32_t live_force = 0;  // tests: every live-kernel target through its exact rescan
    int32_t live_waves_per_simd = 2;  // automatic lane count: the fewest giving this many wavefronts per SIMD ...
    int32_t live_max_win = 192;       // ... and at most this many windows a lane (LDS slice)
    int32_t live_waves = 0;           // wavefronts per workgroup (2..8: the prologue's tables take 128 threads); 0: 8, halved (to 2) while the grid leaves CUs idle
    int32_t long_mode = -1;  // long-sequence sweep (gs_sweep_long.hip) on DNA-path sweeps: -1 automatic (long sequences), 0 never, 1 whenever it fits
    int32_t long_waves = 4;  // its wavefronts per workgroup (2, 4, 8)
    int32_t bg_mode = -1;  // all-background sweep kernel: -1 from 64 targets per CU, 1 whenever admissible, 0 never
    int32_t bg_G = 0;      // its lanes per target (1 .. 64); 0 = automatic
    int32_t bg_force_replay = 0;  // tests: its picks by the exact sequential replay
    int32_t graph_mode = -1;  // hipGraph replay of sweep chains: -1 with a communicator, 0 off, 1 on
    int32_t site_coop = 1;  // site greedy: every wavefront on a lone visit (0 off)
    double coop_rate = 0.35;  // site greedy: lone-visit steps while moves per visit exceed it (0 off)
    int32_t motif_coop = 4096;  // motif greedy: whole-workgroup scoring of visits with K*W >= it (0 off)
    int32_t site_dt16 = 1;  // site greedy: two-byte D table when it fits
    int32_t site_exit_chunk = 1024;  // site greedy: mid-pass hand-over check every chunk visits (0 off)
    int32_t site_exit_ratio = 16;  // ... when a chunk moves fewer than chunk / ratio starts
    int32_t greedy_exit_chunk = 1024;  // motif greedy: the same check
    int32_t greedy_exit_ratio = 16;  // motif greedy: the same ratio
    int32_t greedy_waves = 8;  // speculation width of the greedy kernel (targets scored per step)
    int32_t multi_greedy_threads = 512;  // list-path greedy: threads per workgroup (64 .. 1024, multiple of 64)
    int32_t multi_spec_slots = 256;  // list-path greedy: visits scored per speculative step
    int32_t greedy_switch = 16;  // star greedy -> speculative passes once a pass moves < N / it targets (0 never)
    int32_t ftab_mode = 0;  // four-symbol sweep's workgroup tables: 0 built by every workgroup, 1 by a table kernel before the sweep, 2 handed over by the previous sweep's last workgroup (one GPU; else 1); 1 and 2 need the -DGS_FTAB build
    int32_t site_switch = 4;  // the same for the site sampler (cfg2: 4 / 16 / 2 -> 231 / 245 / 252 ms)
};

// name -> field, for gs_set_tuning / gs_get_tuning
struct gs_tuning_field {
    const char *name;
    bool (*set)(gs_tuning &, double);
    double (*get)(const gs_tuning &);
};
extern const gs_tuning_field kTuningFields[];
extern const int kTuningFieldCount;

int gs_sweep_wm(int W);
int gs_sweep_group_lanes(int E, int Lmax);
int gs_sweep_ek(const SweepArgs &a);  // 4: the four-symbol kernel takes this launch
hipError_t gs_sweep_occupancy(int *blocks_per_cu, const SweepArgs &a, int waves,
                              size_t lds_bytes);
hipError_t gs_sweep_tables_launch(int W, const int64_t *rep, int32_t stride, double pc, double den,
                                  double apc, unsigned char *out, hipStream_t stream);
hipError_t gs_sweep_launch(const SweepArgs &a, int grid, size_t lds_bytes, hipStream_t stream,
                           hipEvent_t start, hipEvent_t stop);
hipError_t gs_composition_launch(const uint8_t *seq, const int64_t *doff, const int32_t *len,
                                 int32_t n_local, int32_t A, int32_t E, int32_t *comp, int n_cu,
                                 hipStream_t stream);
hipError_t gs_fastmath_launch(unsigned int *out, hipStream_t stream);
hipError_t gs_set_counter_launch(unsigned long long *p, unsigned long long v, unsigned int *z,
                                 hipStream_t stream);
hipError_t gs_uniforms_launch(double *u, int32_t n_local, int64_t global_offset, uint64_t seed,
                              int32_t sweeps, unsigned long long *ctr, unsigned int *done,
                              int n_cu, hipStream_t stream);
int gs_dna_lds_bytes();
hipError_t gs_dna_occupancy(int *blocks_per_cu, int W, int G);
hipError_t gs_dna_launch(const DnaArgs &a, int G, int grid, hipStream_t stream, hipEvent_t start,
                         hipEvent_t stop);
int gs_live_lds_bytes(int Lmax, int W, int G, int waves);
int gs_live_wm(int W);
hipError_t gs_live_occupancy(int *blocks_per_cu, int W, int G, int Lmax, int waves);
hipError_t gs_live_launch(const DnaArgs &a, int G, int grid, int waves, hipStream_t stream,
                          hipEvent_t start, hipEvent_t stop);
bool gs_long_fits(int Lmax, int W);
int gs_long_lds_bytes(int Lmax, int W, int waves);
hipError_t gs_long_occupancy(int *blocks_per_cu, int W, int Lmax, int waves);
hipError_t gs_long_launch(const DnaArgs &a, int grid, int waves, hipStream_t stream, hipEvent_t start,
                          hipEvent_t stop);
hipError_t gs_bg_occupancy(int *blocks_per_cu, int G);
hipError_t gs_bg_launch(const BgArgs &a, int G, int grid, hipStream_t stream, hipEvent_t start,
                        hipEvent_t stop);
int gs_bg_waves();
hipError_t gs_agg_convert_launch(int64_t *rep, int64_t *vec, int32_t cells, int32_t stride,
                                 int32_t to, hipStream_t stream);
hipError_t gs_starts_launch(const StartsArgs &a, int grid, size_t lds_bytes, hipStream_t s);
hipError_t gs_greedy_launch(const GreedyArgs &a, int waves, size_t lds_bytes, hipStream_t stream,
                            hipEvent_t start, hipEvent_t stop);
hipError_t gs_starts_partial_launch(const PartialArgs &a, int grid, hipStream_t s);
hipError_t gs_site_shift_launch(const int32_t *pos, const int32_t *len, int32_t n, int32_t W,
                                int32_t dir, int32_t *out, hipStream_t s);
hipError_t gs_multi_agg_launch(const MultiArgs &a, int64_t *out, int n_cu, hipStream_t s);
hipError_t gs_multi_sweep_launch(const MultiArgs &a, int grid, size_t lds, hipStream_t s);
hipError_t gs_multi_spec_launch(const MultiArgs &a, int threads, size_t lds, int steps,
                                hipStream_t s);
hipError_t gs_single_lists_launch(const int32_t *pos, int32_t n, int32_t *cnt, int32_t *lst,
                                  int to_lists, hipStream_t s);
hipError_t gs_count_diff_launch(const int32_t *a, const int32_t *b, int32_t n, int32_t *out,
                                hipStream_t s);
hipError_t gs_site_accept_launch(const double *tmp_score, const int32_t *tmp_pos, double *score,
                                 int32_t *pos, int32_t n, int32_t *moved, hipStream_t s);
hipError_t gs_site_spec_launch(const StartsArgs &a, const SiteCommitArgs &ca, size_t lds_bytes,
                               int steps, hipStream_t s);

struct gs_ctx {
    int device = 0;
    gs_tuning tune;
    hipStream_t stream = nullptr;
    std::string err;
    int64_t err_index = -1;
    // sequences
    int32_t n_local = 0;
    int64_t n_global = 0, global_offset = 0;
    int32_t A = 0;
    uint8_t alphabet[kSlots] = {};
    uint8_t enc[kSlots] = {};
    int32_t Lmin = 0, Lmax = 0;
    int64_t seq_stride = 0;  // > 0: equal lengths, sequence n at n * seq_stride (SweepArgs)
    int32_t pk_stride = 0;  // packed words between sequences when every length is Lmax (DnaArgs)
    int32_t cmin = 0;  // fewest occurrences of an alphabet symbol in one sequence (packed data)
    std::vector<int32_t> h_len;
    uint8_t *d_seq = nullptr;
    uint8_t *d_pseq = nullptr;  // pair codes s[i] + E*s[i+1] (E <= 16), the d_seq layout
    int64_t *d_doff = nullptr;
    int32_t *d_len = nullptr;
    int32_t *d_comp = nullptr;      // [n_local][E+1] static symbol histograms
    int32_t scan = kScanCertified;  // gs_set_scan_mode
    // DNA sweep (gs_sweep_dna.hip): alphabets of <= 4 symbols with no other symbol in
    // the data.  2-bit packed sequences, the snapshot's aggregates as one vector
    // (C then T, int64) that the last workgroup of each sweep reduces in-kernel.
    bool dna_ok = false;
    bool dna_agree = true;          // every rank's data admits the DNA sweep (set_snapshot)
    bool bg_agree = true;           // every rank's tuning admits the all-background takeover
    uint32_t *d_pk = nullptr;
    int64_t *d_pkoff = nullptr;
    int64_t *d_aggv[2] = {nullptr, nullptr};
    int cur_aggv = 0;
    bool vec_valid = false, rep_valid = false;  // which form of the aggregates is current
    int64_t *d_rep = nullptr;       // kRepl * stride, zero between sweeps
    unsigned int *d_dna_done = nullptr;
    unsigned int *d_gen_done = nullptr;  // the general sweep kernel's two-level done counter (kDoneBytes)
    // the four-symbol sweep's workgroup tables (gs_sweep.hip ek4_build_tables), one image
    // of kFtabBytes per aggregate buffer d_agg[k]; ftab_agg: the buffer whose image is
    // current (for pc ftab_pc), -1 none.  Only the chain of sweeps keeps it: every
    // other entry point that can touch the aggregates drops it (gs_api.cpp)
    unsigned char *d_ftab = nullptr;
    // the in-kernel exchange (gs_exchange_open): this context's buffer (kXchBytes), the
    // ranks' buffers as mapped here (device array), the peers' IPC mappings to close,
    // the exchange count; xranks = 0: off
    int64_t *d_xbuf = nullptr;
    int64_t **d_xpeer = nullptr;
    unsigned long long *d_xseq = nullptr;
    std::vector<void *> xmapped;
    int32_t xranks = 0, xrank = 0;
    bool xch_used = false;  // the last packed-layout sweep exchanged in-kernel
    int ftab_agg = -1;
    double ftab_pc = 0.0;
    int64_t *d_compsum = nullptr;   // [4] this rank's symbol totals (packed data)
    int32_t *d_ckp = nullptr;
    int64_t ckp_elems = 0;
    int32_t *d_dt = nullptr;        // site scans: D tables in HBM for long sequences
    int64_t dt_elems = 0;
    // snapshot state
    int32_t W = 0;
    bool have_state = false;
    int32_t *d_pos[2] = {nullptr, nullptr};
    int cur_pos = 0;
    double *d_pwms = nullptr;
    double *d_u = nullptr;
    int32_t *d_aux = nullptr;       // [n_local + 4]: per-target scratch, then counters
    int64_t *d_agg[3] = {nullptr, nullptr, nullptr};
    int cur_agg = 0;
    int32_t cells = 0, stride = 0;
    int32_t *d_err_code = nullptr;
    unsigned long long *d_err_index = nullptr;
    unsigned long long *d_fallbacks = nullptr;
    int32_t *d_bg_note = nullptr;  // the sweep kernels' note: snapshot in the all-background state
    // the chain is in the all-background state (for these pc / cutOff): swept by
    // gs_sweep_bg_kernel alone; snap_all_none: the snapshot set had every position []
    bool bg_absorbed = false, bg_zeroed = false, snap_all_none = false, capturing = false;
    double bg_pc = 0.0, bg_cutoff = 0.0;
    // the note of a chain's last sweep, copied to pinned host memory behind the chain
    // (no synchronisation inside a chain call) and read at the next decision point
    bool note_pending = false;
    int32_t *h_note = nullptr;
    hipEvent_t note_ev = nullptr;
    double note_pc = 0.0, note_cutoff = 0.0;
    int bg_occ[7] = {0, 0, 0, 0, 0, 0, 0};  // gs_sweep_bg_kernel blocks per CU by log2 G
    int bg_warmed = 0;                      // lane counts whose code is loaded (bit log2 G)
    int live_occ[12][4] = {};
    int long_occ[3][3] = {};  // gs_sweep_long_kernel blocks per CU by WM (8, 12, 16) x waves (2, 4, 8)
    // gs_sweep_kernel blocks per CU for the last (W, E, lanes, waves, LDS) asked: a host
    // API call per sweep costs about as much as a short sweep
    int sweep_occ = 0;
    int32_t last_sweep[4] = {0, 0, 0, 0};  // gs_last_sweep_launch: ek, lanes, waves, grid
    int dna_occ[3] = {0, 0, 0}, dna_occ_W = 0;  // gs_sweep_dna_kernel by G (1, 2, 4), for W
    int64_t sweep_occ_key[6] = {-1, -1, -1, -1, -1, -1};  // gs_sweep_live_kernel blocks per CU by G (1, 2, 4, 8) x WM, waves (8, 4, 2, 1)
    int32_t max_lds = 0, n_cu = 0;
    int32_t E = 0;                  // encoded symbol space (alphabet first)
    // the caller's background / profile (…ByPCV, …WithBPV, …OfPPM twins)
    bool use_pcv = false, use_ppm = false;
    double *d_pcv_fixed = nullptr;  // [64] by encoded symbol
    double *d_ppm_fixed = nullptr;  // [A][ppm_W]
    int32_t ppm_W = 0;
    int32_t last_greedy_waves = 0;
    unsigned long long *d_stamps = nullptr;  // diagnostic build only
    // hipGraph replay of sweep chains: one graph = a uniforms kernel (the counter-RNG
    // draws of kGraphSweeps sweeps from a device sweep counter, d_u6) + kGraphSweeps x
    // (sweep kernel reading d_u6, all-reduce), so the launch arguments repeat with
    // the period of the buffer rotations (2 x 3)
    double *d_u6 = nullptr;
    unsigned long long *d_sweep_ctr = nullptr;
    unsigned int *d_done_ctr = nullptr;
    bool graph_broken = false;      // capture failed once: direct launches from then on
    uint64_t graph_gen = 1;         // bumped whenever captured arguments may change
    struct GraphEntry {
        hipGraphExec_t exec = nullptr;
        uint64_t gen = 0, seed = 0;
        int pos = 0, agg = 0;
        bool dna = false, bg = false;
        double pc = 0.0, cutoff = 0.0;
    };
    std::vector<GraphEntry> graphs;
    // motifAmount >= 2 path (gs_multi.hip): category arenas, packed device status
    double *d_mscratch = nullptr;
    int64_t mscratch_bytes = 0;
    unsigned long long *d_merr = nullptr;
    // rccl
    ncclComm_t comm = nullptr;
    int32_t nranks = 1, rank = 0;
    // profiling
    bool prof = false;
    int32_t prof_stride = 1;       // time every prof_stride-th launch (gs_profile_enable)
    int64_t prof_sweep_calls = 0, prof_ar_calls = 0, prof_bg_calls = 0;
    hipEvent_t region_start = nullptr, region_stop = nullptr;
    bool region_stopped = false;  // gs_profile_region_stop recorded the stop event
    std::vector<hipEvent_t> ev_pool;
    // ev_bg: all-background sweep dispatches, added to the sweep time (not counted as sweeps)
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_sweep, ev_ar, ev_bg;
    double prof_sweep_ms = 0.0, prof_ar_ms = 0.0;
    int64_t prof_sweeps = 0, prof_ars = 0;
};

namespace gs_host {

inline int fail(gs_ctx *c, int code, const std::string &msg, int64_t idx = -1) {
    if (c) {
        c->err = msg;
        c->err_index = idx;
    }
    return code;
}


#define HIP_TRY(ctx, x)                                                               \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess)                                                         \
            return fail(ctx, GS_E_HIP, std::string(#x ": ") + hipGetErrorString(e_)); \
    } while (0)

#define RCCL_TRY(ctx, x)                                                                 \
    do {                                                                                 \
        ncclResult_t r_ = (x);                                                           \
        if (r_ != ncclSuccess)                                                           \
            return fail(ctx, GS_E_RCCL, std::string(#x ": ") + ncclGetErrorString(r_)); \
    } while (0)

template <class T>
void dfree(T *&p) {
    if (p) (void)hipFree((void *)p);
    p = nullptr;
}


inline int64_t align16(int64_t x) { return (x + 15) & ~int64_t(15); }

constexpr int kGraphSweeps = 6;  // lcm of the position (2) and aggregate (3) rotations
constexpr int kSpecBatch = 32;   // speculative greedy steps enqueued between host checks

// Device buffers of one list-path call, freed on scope exit.
struct MultiBufs {
    int32_t *cnt = nullptr, *pos = nullptr, *cnt2 = nullptr, *pos2 = nullptr;
    int32_t *ovf = nullptr, *targets = nullptr;
    double *pwms = nullptr, *u = nullptr;
    int64_t *agg = nullptr;
    ~MultiBufs() {
        dfree(cnt);
        dfree(pos);
        dfree(cnt2);
        dfree(pos2);
        dfree(ovf);
        dfree(targets);
        dfree(pwms);
        dfree(u);
        dfree(agg);
    }
};


constexpr int64_t kArenaBudget = 4ll << 30;     // bytes of category arenas per launch
constexpr int64_t kArenaMax = 1ll << 28;        // categories per target

void drop_graphs(gs_ctx *c);
void free_state(gs_ctx *c);
int64_t sweep_carve(SweepArgs &a, int A, int E, int W, int Lmax, int gl, int waves, bool ek4);
double cutoff_threshold(double cutoff);
double cutoff_threshold_hi(double cutoff);
int check_dev(gs_ctx *c);
int alloc_state(gs_ctx *c, int32_t W);
int validate_W(gs_ctx *c, int32_t W);
int validate_pos(gs_ctx *c, int32_t W, const int32_t *pos);
hipEvent_t get_event(gs_ctx *c);
int allreduce_agg(gs_ctx *c, int idx);
int launch_sweep(gs_ctx *c, int mode, double pc, double cutoff, const double *u_dev, uint64_t seed,
                 uint64_t stream, int agg_in, int agg_out, int agg_zero);
bool use_dna(const gs_ctx *c);
bool bg_wanted(const gs_ctx *c);
bool bg_ready(gs_ctx *c, double pc, double cutoff);
int bg_check_note(gs_ctx *c, double pc, double cutoff);
int bg_resolve(gs_ctx *c);
int bg_warm(gs_ctx *c);
int32_t *bg_note_ptr(gs_ctx *c);
int launch_bg(gs_ctx *c, double pc, double cutoff, const double *u_dev, uint64_t seed,
              uint64_t stream, bool device_ctr);
int dna_lanes(const gs_ctx *c);
bool use_live(const gs_ctx *c);
bool use_long(const gs_ctx *c);
int live_fit_waves(const gs_ctx *c, int G, int want);
int live_lanes(const gs_ctx *c);
int need_rep(gs_ctx *c);
int need_vec(gs_ctx *c);
int allreduce_vec(gs_ctx *c, int idx);
int launch_dna(gs_ctx *c, double pc, double cutoff, const double *u_dev, uint64_t seed);
int set_snapshot(gs_ctx *c, int32_t W, const int32_t *pos);
int one_sweep(gs_ctx *c, double pc, double cutoff, const double *u_dev, uint64_t seed,
              uint64_t stream);
bool graphs_wanted(gs_ctx *c);
int graph_buffers(gs_ctx *c);
hipGraphExec_t sweep_graph(gs_ctx *c, double pc, double cutoff, uint64_t seed);
int starts_pass(gs_ctx *c, int mode, int32_t W, double pc, uint64_t seed, const int32_t *d_starts,
                const int32_t *d_cpart, const int64_t *agg, double *d_score, int32_t *d_pos_out,
                const double *d_ppm = nullptr, StartsArgs *build_only = nullptr,
                int64_t *lds_out = nullptr);
int check_device_error(gs_ctx *c);
int greedy_run(gs_ctx *c, int site, double pc, double cutoff, int32_t max_passes,
                      int32_t *passes_out, double *kernel_ms_out, int32_t exit_chunk = 0,
                      int32_t exit_ratio = 0, int32_t *exit_info = nullptr);
int validate_site_pos(gs_ctx *c, int32_t W, const int32_t *pos);
int site_greedy(gs_ctx *c, double pc, int32_t max_passes, int32_t *passes_out);
int site_shift(gs_ctx *c, double pc, int32_t dir, int32_t max_passes, int32_t *passes);
int site_upload(gs_ctx *c, int32_t W, const int32_t *pos, const double *score);
int site_download(gs_ctx *c, int32_t *pos, double *score);
int site_refine(gs_ctx *c, double pc, int32_t shift, int32_t max_passes, int32_t *passes);
int validate_lists(gs_ctx *c, int32_t M, int32_t W, int32_t cap, const int32_t *cnt,
                   const int32_t *pos);
int64_t multi_args(gs_ctx *c, MultiArgs &a, int32_t M, int32_t W, int32_t cap, double pc,
                   double cutoff, bool greedy);
int multi_scratch(gs_ctx *c, MultiArgs &a, int64_t slots, int64_t arena_cap);
int multi_status(gs_ctx *c, unsigned long long *status_out = nullptr);
int multi_upload(gs_ctx *c, MultiBufs &b, MultiArgs &a, int32_t cap, const int32_t *cnt,
                 const int32_t *pos);
int multi_sweep_dev(gs_ctx *c, MultiBufs &b, MultiArgs &a, int64_t lds);
int multi_download(gs_ctx *c, const MultiBufs &b, int32_t cap, const int32_t *dcnt,
                   const int32_t *dpos, const double *dpw, int32_t *cnt, int32_t *pos,
                   double *pwms);
int multi_greedy_dev(gs_ctx *c, MultiArgs &a, int64_t lds, int32_t cap, int32_t max_passes,
                     int32_t *dcnt, int32_t *dpos, double *dpw, int64_t *agg,
                     const int32_t *cnt0, const int32_t *pos0, const double *pw0,
                     int32_t *passes_out, int32_t base0 = 0, int32_t changed0 = 0);
int multi_lds_check(gs_ctx *c, int64_t lds);
int greedy_hybrid(gs_ctx *c, double pc, double cutoff, int32_t max_passes, int32_t *passes_out,
                  double *kernel_ms_out);

}  // namespace gs_host
