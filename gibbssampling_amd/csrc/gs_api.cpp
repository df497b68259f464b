// gs_api.cpp — C ABI (include/gibbs_hip.h) over the gfx950 kernels.
//
// Host responsibilities: input validation with the reference's error behaviour,
// the HBM layout (encoded symbols, 16-byte aligned per sequence), the device
// snapshot state (positions double buffer, triple-buffered XCD-replicated
// aggregate accumulators), one in-place RCCL all-reduce of the aggregates per
// sweep when several processes form one sampler, and hipEvent timing.
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

int gs_sweep_wm(int W);
int gs_sweep_group_lanes(int E, int Lmax);
hipError_t gs_sweep_occupancy(int *blocks_per_cu, int W, int E, int gl, int waves,
                              size_t lds_bytes);
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
    std::vector<int32_t> h_len;
    uint8_t *d_seq = nullptr;
    int64_t *d_doff = nullptr;
    int32_t *d_len = nullptr;
    int32_t *d_comp = nullptr;      // [n_local][E+1] static symbol histograms
    int32_t scan = kScanCertified;  // gs_set_scan_mode
    // DNA sweep (gs_sweep_dna.hip): alphabets of <= 4 symbols with no other symbol in
    // the data.  2-bit packed sequences, the snapshot's aggregates as one vector
    // (C then T, int64) that the last workgroup of each sweep reduces in-kernel.
    bool dna_ok = false;
    bool dna_agree = true;          // every rank's data admits the DNA sweep (set_snapshot)
    bool dna_enable = true;         // GS_DNA=0 forces the general kernel (A/B, tests)
    int32_t dna_G = 0;              // lanes per sequence, 0 = automatic (GS_DNA_G)
    uint32_t *d_pk = nullptr;
    int64_t *d_pkoff = nullptr;
    int64_t *d_aggv[2] = {nullptr, nullptr};
    int cur_aggv = 0;
    bool vec_valid = false, rep_valid = false;  // which form of the aggregates is current
    int64_t *d_rep = nullptr;       // kRepl * stride, zero between sweeps
    unsigned int *d_dna_done = nullptr;
    int32_t *d_ckp = nullptr;
    int64_t ckp_elems = 0;
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
    int32_t max_lds = 0, n_cu = 0;
    int32_t E = 0;                  // encoded symbol space (alphabet first)
    int32_t blocks_per_cu_cap = 8;  // tuning knob (GS_BLOCKS_PER_CU)
    int32_t group_lanes = 0;        // lanes per sequence; 0 = automatic (GS_GROUP_LANES)
    int32_t sweep_waves = 0;        // wavefronts per sweep workgroup; 0 = automatic
    bool site_coop = true;          // site greedy: all wavefronts on a lone visit (GS_SITE_COOP)
    int32_t motif_coop = 4096;      // motif greedy: the same for visits with K*W >= it (GS_GREEDY_COOP, 0 off)
    float coop_rate = 0.35f;        // site greedy: lone-visit steps while moves/visit exceed it (GS_COOP_RATE, 0 off)
    bool site_dt16 = true;          // site greedy: two-byte D table when it fits (GS_SITE_DT16)
    int32_t site_exit_chunk = 1024; // site greedy: mid-pass hand-over check (GS_SITE_EXIT_CHUNK)
    int32_t site_exit_ratio = 16;   // ... when a chunk moves < chunk / ratio (GS_SITE_EXIT_RATIO)
    int32_t greedy_exit_chunk = 1024;  // the same for the motif greedy (GS_GREEDY_EXIT_CHUNK)
    int32_t greedy_exit_ratio = 16;    // (GS_GREEDY_EXIT_RATIO)
    int32_t greedy_waves = 8;       // speculation width of the greedy kernel (GS_GREEDY_WAVES)
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
    int32_t graph_mode = -1;        // GS_GRAPH: -1 auto (with a communicator), 0 off, 1 on
    bool graph_broken = false;      // capture failed once: direct launches from then on
    uint64_t graph_gen = 1;         // bumped whenever captured arguments may change
    struct GraphEntry {
        hipGraphExec_t exec = nullptr;
        uint64_t gen = 0, seed = 0;
        int pos = 0, agg = 0;
        bool dna = false;
        double pc = 0.0, cutoff = 0.0;
    };
    std::vector<GraphEntry> graphs;
    // motifAmount >= 2 path (gs_multi.hip): category arenas, packed device status
    double *d_mscratch = nullptr;
    int64_t mscratch_bytes = 0;
    int32_t multi_greedy_threads = 512;  // workgroup of the list-path greedy (GS_MULTI_GREEDY_THREADS)
    int32_t multi_spec_slots = 256;      // visits scored per speculative step (GS_MULTI_SPEC_SLOTS)
    int32_t greedy_switch = 16;          // star greedy -> speculative passes once a pass moves
                                         // fewer than N / greedy_switch targets (0: never)
    int32_t site_switch = 4;             // the same for the site sampler (GS_SITE_SWITCH);
                                         // cfg2: 4 / 16 / 2 -> 231 / 245 / 252 ms
    unsigned long long *d_merr = nullptr;
    // rccl
    ncclComm_t comm = nullptr;
    int32_t nranks = 1, rank = 0;
    // profiling
    bool prof = false;
    int32_t prof_stride = 1;       // time every prof_stride-th launch (gs_profile_enable)
    int64_t prof_sweep_calls = 0, prof_ar_calls = 0;
    hipEvent_t region_start = nullptr, region_stop = nullptr;
    std::vector<hipEvent_t> ev_pool;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_sweep, ev_ar;
    double prof_sweep_ms = 0.0, prof_ar_ms = 0.0;
    int64_t prof_sweeps = 0, prof_ars = 0;
};

namespace {

const char *kVersion = "gibbs_hip 0.1.0 (gfx950)";

int fail(gs_ctx *c, int code, const std::string &msg, int64_t idx = -1) {
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

void drop_graphs(gs_ctx *c) {
    for (auto &g : c->graphs)
        if (g.exec) (void)hipGraphExecDestroy(g.exec);
    c->graphs.clear();
    ++c->graph_gen;
}

void free_state(gs_ctx *c) {
    drop_graphs(c);
    dfree(c->d_u6);
    dfree(c->d_pos[0]);
    dfree(c->d_pos[1]);
    dfree(c->d_pwms);
    dfree(c->d_u);
    dfree(c->d_aux);
    for (auto &b : c->d_agg) dfree(b);
    for (auto &b : c->d_aggv) dfree(b);
    dfree(c->d_rep);
    dfree(c->d_dna_done);
    dfree(c->d_ckp);
    c->ckp_elems = 0;
    c->vec_valid = c->rep_valid = false;
    c->have_state = false;
    c->W = 0;
}

int64_t align16(int64_t x) { return (x + 15) & ~int64_t(15); }

// Dynamic LDS of the sweep kernel: workgroup-shared aggregates + PPM tables,
// then one slice per wavefront (4 per workgroup), each holding the wavefront's
// aggregates, the shared binary64 table of rescans and the batch results, then
// one slice per lane group (64/gl per wavefront).  Returns total bytes.
int64_t sweep_carve(SweepArgs &a, int A, int E, int W, int Lmax, int gl, int waves) {
    const int WM = gs_sweep_wm(W);
    int64_t o = 0;
    auto take = [&](int64_t b) {
        int64_t r = o;
        o = align16(o + b);
        return (int32_t)r;
    };
    a.gl = gl;
    a.o_cg = take(4 * (int64_t)A * W);
    a.o_T = take(8 * (int64_t)(A + 1));  // T[a] and their sum
    a.o_ppmG = take(8 * (int64_t)A * W);
    a.o_ppmM = take(8 * (int64_t)A * W);
    a.o_lppmG = take(4 * (int64_t)A * W);
    a.o_lppmM = take(4 * (int64_t)A * W);
    a.o_bmax = take(4);
    a.o_wave = (int32_t)o;
    const int64_t base = o;
    o = 0;
    a.w_aggC = take(4 * (int64_t)A * W);
    a.w_aggT = take(8 * (int64_t)A);
    a.w_tab = take(16 * (int64_t)tab_stride(WM) * E);
    a.w_res = take(16 * 64);
    a.w_misc = take(32);
    a.w_group = (int32_t)o;
    const int64_t wave_fixed = o;
    o = 0;
    a.g_lt = take(8 * (int64_t)lt_stride(WM) * E);
    if (scan_group(E) == 2) {
        a.g_gt = take(8 * (int64_t)gt_stride(WM) * E * E);
        a.g_code = take((int64_t)Lmax + WM + 80);
    } else {
        a.g_gt = a.g_code = 0;
    }
    a.g_seq = take((int64_t)Lmax + WM + 96);  // + the 16-byte zero tail
    a.g_pcv = take(8 * (int64_t)gl);
    a.g_lpcv = take(4 * (int64_t)gl);
    a.g_cnt = take(4 * (int64_t)gl);
    a.g_wfac = take(16 * (int64_t)WM);
    a.group_bytes = (int32_t)o;
    a.wave_bytes = (int32_t)(wave_fixed + (64 / gl) * o);
    a.waves = waves;
    return base + waves * (int64_t)a.wave_bytes;
}

// Host-side roulette pre-filter threshold: any S below thr_lo has
// log2(S) < cutOff - 1e-6 and cannot pass the cut-off (.fs:735).
double cutoff_threshold(double cutoff) {
    if (std::isnan(cutoff)) return INFINITY;
    if (cutoff > 1000.0) return INFINITY;  // only +inf scores can pass; they bypass below
    if (cutoff < -1000.0) return 0.0;
    return std::exp2(cutoff) * (1.0 - 0x1.0p-20);
}

// Any S above thr_hi has log(S)/log(2) > cutOff after rounding: the margin 2^-40
// dwarfs the exp2 / log / division roundings (< 2^-50 relative here).
double cutoff_threshold_hi(double cutoff) {
    if (!(cutoff >= -1000.0 && cutoff <= 1000.0)) return INFINITY;  // also NaN
    return std::exp2(cutoff) * (1.0 + 0x1.0p-40);
}

int check_dev(gs_ctx *c) {
    HIP_TRY(c, hipSetDevice(c->device));
    return GS_OK;
}

int alloc_state(gs_ctx *c, int32_t W) {
    if (c->have_state && c->W == W) return GS_OK;
    free_state(c);
    const int64_t n = std::max<int32_t>(1, c->n_local);
    HIP_TRY(c, hipMalloc(&c->d_pos[0], n * 4));
    HIP_TRY(c, hipMalloc(&c->d_pos[1], n * 4));
    HIP_TRY(c, hipMalloc(&c->d_pwms, n * 8));
    HIP_TRY(c, hipMalloc(&c->d_u, n * 8));
    HIP_TRY(c, hipMalloc(&c->d_aux, (n + 4) * 4));
    c->cells = c->A * W + c->A;
    c->stride = (int32_t)((c->cells + 15) / 16 * 16);  // 128-byte multiple per replica
    for (auto &b : c->d_agg) HIP_TRY(c, hipMalloc(&b, (size_t)kRepl * c->stride * 8));
    if (c->dna_ok) {
        for (auto &b : c->d_aggv) HIP_TRY(c, hipMalloc(&b, (size_t)std::max(1, c->cells) * 8));
        HIP_TRY(c, hipMalloc(&c->d_rep, (size_t)kRepl * c->stride * 8));
        HIP_TRY(c, hipMalloc(&c->d_dna_done, 4));
        HIP_TRY(c, hipMemset(c->d_rep, 0, (size_t)kRepl * c->stride * 8));
        HIP_TRY(c, hipMemset(c->d_dna_done, 0, 4));
        if (!c->d_sweep_ctr) {
            HIP_TRY(c, hipMalloc(&c->d_sweep_ctr, 8));
            HIP_TRY(c, hipMalloc(&c->d_done_ctr, 4));
        }
    }
    c->W = W;
    return GS_OK;
}

int validate_W(gs_ctx *c, int32_t W) {
    if (!c->d_seq) return fail(c, GS_E_STATE, "gs_set_sequences has not been called");
    if (W < 1 || W > 64) return fail(c, GS_E_ARG, "motifLength must be in [1, 64]");
    if (c->n_local > 0 && c->Lmin < W)
        return fail(c, GS_E_ARG, "a sequence is shorter than motifLength (Array.take, .fs:152)");
    return GS_OK;
}

int validate_pos(gs_ctx *c, int32_t W, const int32_t *pos) {
    for (int32_t n = 0; n < c->n_local; ++n) {
        int32_t p = pos[n];
        if (p == -1) continue;
        if (p < 0 || p + W > c->h_len[n])
            return fail(c, GS_E_ARG, "motif position outside its sequence (getSegment, .fs:149-153)",
                        c->global_offset + n);
    }
    return GS_OK;
}

hipEvent_t get_event(gs_ctx *c) {
    if (!c->ev_pool.empty()) {
        hipEvent_t e = c->ev_pool.back();
        c->ev_pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    (void)hipEventCreate(&e);
    return e;
}

int allreduce_agg(gs_ctx *c, int idx) {
    if (!c->comm) return GS_OK;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    const bool timed = c->prof && (c->prof_ar_calls++ % c->prof_stride) == 0;
    if (timed) {
        e0 = get_event(c);
        e1 = get_event(c);
        HIP_TRY(c, hipEventRecord(e0, c->stream));
    }
    RCCL_TRY(c, ncclAllReduce(c->d_agg[idx], c->d_agg[idx], (size_t)kRepl * c->stride, ncclInt64,
                              ncclSum, c->comm, c->stream));
    if (timed) {
        HIP_TRY(c, hipEventRecord(e1, c->stream));
        c->ev_ar.emplace_back(e0, e1);
    }
    return GS_OK;
}

int launch_sweep(gs_ctx *c, int mode, double pc, double cutoff, const double *u_dev, uint64_t seed,
                 uint64_t stream, int agg_in, int agg_out, int agg_zero) {
    SweepArgs a{};
    int gl = gs_sweep_group_lanes(c->E, c->Lmax);
    if (c->group_lanes > 0 && c->E + 1 <= c->group_lanes &&
        !(scan_group(c->E) == 1 && c->group_lanes < 32))
        gl = c->group_lanes;
    int waves = sweep_waves(scan_group(c->E));
    if (c->sweep_waves > 0 && c->sweep_waves <= sweep_waves(scan_group(c->E))) waves = c->sweep_waves;
    int64_t lds_bytes = sweep_carve(a, c->A, c->E, c->W, c->Lmax, gl, waves);
    while (waves > 1 && lds_bytes > c->max_lds)
        lds_bytes = sweep_carve(a, c->A, c->E, c->W, c->Lmax, gl, waves /= 2);
    if (lds_bytes > c->max_lds)
        return fail(c, GS_E_UNSUPPORTED,
                    "longest sequence needs " + std::to_string(lds_bytes) +
                        " B of LDS per workgroup; this build supports up to " +
                        std::to_string(c->max_lds));
    a.seq = c->d_seq;
    a.doff = c->d_doff;
    a.len = c->d_len;
    a.comp = c->d_comp;
    a.n_local = c->n_local;
    a.scan = c->scan;
    a.mode = mode;
    a.global_offset = c->global_offset;
    a.A = c->A;
    a.W = c->W;
    a.E = c->E;
    a.cells = c->cells;
    a.stride = c->stride;
    a.pc = pc;
    a.cutoff = cutoff;
    a.thr_lo = cutoff_threshold(cutoff);
    a.thr_hi = cutoff_threshold_hi(cutoff);
    a.pcv_fixed = c->use_pcv ? c->d_pcv_fixed : nullptr;
    // normalizePPM: (float sourceCount) + ((float alphabet.Length) * pseudoCount), .fs:257
    a.apc = (double)c->A * pc;
    a.den = (double)(c->n_global - 1) + a.apc;
    a.pos_in = c->d_pos[c->cur_pos];
    a.pos_out = c->d_pos[1 - c->cur_pos];
    a.pwms_out = c->d_pwms;
    a.u_in = u_dev;
    a.seed = seed;
    a.stream = stream;
    a.agg_in = agg_in >= 0 ? c->d_agg[agg_in] : nullptr;
    a.agg_out = c->d_agg[agg_out];
    a.agg_zero = agg_zero >= 0 ? c->d_agg[agg_zero] : nullptr;
    a.err_code = c->d_err_code;
    a.err_index = c->d_err_index;
    a.fallbacks = c->d_fallbacks;
#ifdef GS_STAMPS
    if (!c->d_stamps) {
        HIP_TRY(c, hipMalloc(&c->d_stamps, 8 * kStampSlots));
        HIP_TRY(c, hipMemset(c->d_stamps, 0, 8 * kStampSlots));
    }
    a.stamps = mode == 0 ? c->d_stamps : nullptr;
#endif
    int per_cu = 0;
    HIP_TRY(c, gs_sweep_occupancy(&per_cu, c->W, c->E, gl, waves, (size_t)lds_bytes));
    per_cu = std::max(1, std::min(per_cu, c->blocks_per_cu_cap));
    // one wavefront scores 64/gl sequences at a time; sweep_waves(H) per workgroup
    const int64_t waves_needed = (c->n_local + 64 / gl - 1) / (64 / gl);
    const int64_t blocks_needed = (waves_needed + waves - 1) / waves;
    int grid = (int)std::max<int64_t>(1, std::min<int64_t>(blocks_needed, (int64_t)c->n_cu * per_cu));
    hipEvent_t e0 = nullptr, e1 = nullptr;
    const bool timed = c->prof && mode == 0 && (c->prof_sweep_calls++ % c->prof_stride) == 0;
    if (timed) {  // kernel-attached events: the dispatch's own start / stop times
        e0 = get_event(c);
        e1 = get_event(c);
    }
    HIP_TRY(c, gs_sweep_launch(a, grid, (size_t)lds_bytes, c->stream, e0, e1));
    if (timed) c->ev_sweep.emplace_back(e0, e1);
    return GS_OK;
}

bool use_dna(const gs_ctx *c) {
    return c->dna_ok && c->dna_agree && c->dna_enable && c->W <= kDnaMaxW && !c->use_pcv &&
           c->scan == kScanCertified;
}

// Lanes per sequence of the DNA sweep: one while that fills a wavefront per SIMD,
// else 2 or 4 (shorter lanes, more wavefronts).
int dna_lanes(const gs_ctx *c) {
    if (c->dna_G == 1 || c->dna_G == 2 || c->dna_G == 4) return c->dna_G;
    for (int g = 1; g < 4; g *= 2)
        if ((int64_t)(c->n_local + 64 / g - 1) / (64 / g) >= (int64_t)c->n_cu * 4) return g;
    return 4;
}

// The aggregates in the other form, when the current one is the only valid one:
// the vector (DNA sweeps) <-> the replicas (every other kernel).
int need_rep(gs_ctx *c) {
    if (c->rep_valid || !c->vec_valid) return GS_OK;
    HIP_TRY(c, gs_agg_convert_launch(c->d_agg[c->cur_agg], c->d_aggv[c->cur_aggv], c->cells,
                                     c->stride, 1, c->stream));
    c->rep_valid = true;
    return GS_OK;
}
int need_vec(gs_ctx *c) {
    if (c->vec_valid || !c->rep_valid) return GS_OK;
    HIP_TRY(c, gs_agg_convert_launch(c->d_agg[c->cur_agg], c->d_aggv[c->cur_aggv], c->cells,
                                     c->stride, 0, c->stream));
    c->vec_valid = true;
    return GS_OK;
}

int allreduce_vec(gs_ctx *c, int idx) {
    if (!c->comm) return GS_OK;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    const bool timed = c->prof && (c->prof_ar_calls++ % c->prof_stride) == 0;
    if (timed) {
        e0 = get_event(c);
        e1 = get_event(c);
        HIP_TRY(c, hipEventRecord(e0, c->stream));
    }
    RCCL_TRY(c, ncclAllReduce(c->d_aggv[idx], c->d_aggv[idx], (size_t)c->cells, ncclInt64, ncclSum,
                              c->comm, c->stream));
    if (timed) {
        HIP_TRY(c, hipEventRecord(e1, c->stream));
        c->ev_ar.emplace_back(e0, e1);
    }
    return GS_OK;
}

// One DNA sweep (gs_sweep_dna.hip): snapshot d_pos[cur_pos] with aggregates
// d_aggv[cur_aggv] -> d_pos[1 - cur_pos], d_pwms, this rank's aggregates in
// d_aggv[1 - cur_aggv].  u_dev: explicit uniforms, else the counter RNG at the
// device sweep counter.
int launch_dna(gs_ctx *c, double pc, double cutoff, const double *u_dev, uint64_t seed) {
    DnaArgs a{};
    const int G = dna_lanes(c);
    a.pk = c->d_pk;
    a.pkoff = c->d_pkoff;
    a.len = c->d_len;
    a.comp = c->d_comp;
    a.n_local = c->n_local;
    a.A = c->A;
    a.W = c->W;
    a.mode = 0;
    a.global_offset = c->global_offset;
    a.cells = c->cells;
    a.stride = c->stride;
    a.pc = pc;
    a.cutoff = cutoff;
    a.apc = (double)c->A * pc;
    a.den = (double)(c->n_global - 1) + a.apc;
    a.thr_lo = cutoff_threshold(cutoff);
    a.agg_in = c->d_aggv[c->cur_aggv];
    a.rep = c->d_rep;
    a.agg_out = c->d_aggv[1 - c->cur_aggv];
    a.done = c->d_dna_done;
    a.pos_in = c->d_pos[c->cur_pos];
    a.pos_out = c->d_pos[1 - c->cur_pos];
    a.pwms_out = c->d_pwms;
    a.u_in = u_dev;
    a.seed = seed;
    a.sweep_ctr = u_dev ? nullptr : c->d_sweep_ctr;
    a.err_code = c->d_err_code;
    a.err_index = c->d_err_index;
    a.fallbacks = c->d_fallbacks;
#ifdef GS_STAMPS
    if (!c->d_stamps) {
        HIP_TRY(c, hipMalloc(&c->d_stamps, 8 * kStampSlots));
        HIP_TRY(c, hipMemset(c->d_stamps, 0, 8 * kStampSlots));
    }
    a.stamps = c->d_stamps;
#endif
    int per_cu = 0;
    HIP_TRY(c, gs_dna_occupancy(&per_cu, c->W, G));
    per_cu = std::max(1, std::min(per_cu, 2));
    const int64_t tiles = (c->n_local + 64 / G - 1) / (64 / G);
    const int64_t blocks = (tiles + kDnaWaves - 1) / kDnaWaves;
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(blocks, (int64_t)c->n_cu * per_cu));
    // checkpoint scratch: per wavefront [maxblk][64] block sums
    const int K = c->Lmax - c->W + 1;
    const int R = G == 1 ? K : ((((K + G - 1) / G) + 15) & ~15);
    a.maxblk = 4 * ((R + 14 + 63) / 64) + 4;
    const int64_t need = (int64_t)grid * kDnaWaves * a.maxblk * 64;
    if (need > c->ckp_elems) {
        dfree(c->d_ckp);
        HIP_TRY(c, hipMalloc(&c->d_ckp, (size_t)need * 4));
        c->ckp_elems = need;
    }
    a.ckp = c->d_ckp;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    const bool timed = c->prof && (c->prof_sweep_calls++ % c->prof_stride) == 0;
    if (timed) {
        e0 = get_event(c);
        e1 = get_event(c);
    }
    HIP_TRY(c, gs_dna_launch(a, G, grid, c->stream, e0, e1));
    if (timed) c->ev_sweep.emplace_back(e0, e1);
    return GS_OK;
}

// Upload positions and compute the aggregates of that snapshot into d_agg[0].
int set_snapshot(gs_ctx *c, int32_t W, const int32_t *pos) {
    int rc;
    if ((rc = validate_W(c, W))) return rc;
    if ((rc = validate_pos(c, W, pos))) return rc;
    if ((rc = alloc_state(c, W))) return rc;
    HIP_TRY(c, hipMemcpyAsync(c->d_pos[0], pos, (size_t)c->n_local * 4, hipMemcpyHostToDevice,
                              c->stream));
    c->cur_pos = 0;
    for (auto &b : c->d_agg)
        HIP_TRY(c, hipMemsetAsync(b, 0, (size_t)kRepl * c->stride * 8, c->stream));
    HIP_TRY(c, hipMemsetAsync(c->d_err_code, 0, 4, c->stream));
    HIP_TRY(c, hipMemsetAsync(c->d_err_index, 0xff, 8, c->stream));
    if (c->n_local > 0)
        if ((rc = launch_sweep(c, 1, 0.0, 0.0, nullptr, 0, 0, -1, 0, -1))) return rc;
    if ((rc = allreduce_agg(c, 0))) return rc;
    c->cur_agg = 0;
    c->rep_valid = true;
    c->vec_valid = false;
    if (c->comm) {
        // the sweep kernel must be the same on every rank (their collectives differ)
        int32_t *d_flag = c->d_aux + c->n_local;
        const int32_t mine = c->dna_ok ? 1 : 0;
        HIP_TRY(c, hipMemcpyAsync(d_flag, &mine, 4, hipMemcpyHostToDevice, c->stream));
        RCCL_TRY(c, ncclAllReduce(d_flag, d_flag, 1, ncclInt32, ncclMin, c->comm, c->stream));
        int32_t all = 0;
        HIP_TRY(c, hipMemcpyAsync(&all, d_flag, 4, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(c, hipStreamSynchronize(c->stream));
        c->dna_agree = all != 0;
    } else {
        c->dna_agree = true;
    }
    if (c->dna_ok) {
        c->cur_aggv = 0;
        HIP_TRY(c, hipMemsetAsync(c->d_rep, 0, (size_t)kRepl * c->stride * 8, c->stream));
        HIP_TRY(c, hipMemsetAsync(c->d_dna_done, 0, 4, c->stream));
        if (use_dna(c) && (rc = need_vec(c))) return rc;
    }
    c->have_state = true;
    return GS_OK;
}

int one_sweep(gs_ctx *c, double pc, double cutoff, const double *u_dev, uint64_t seed,
              uint64_t stream) {
    int rc;
    if (use_dna(c)) {
        if ((rc = need_vec(c))) return rc;
        if ((rc = launch_dna(c, pc, cutoff, u_dev, seed))) return rc;
        const int o = 1 - c->cur_aggv;
        if ((rc = allreduce_vec(c, o))) return rc;
        c->cur_aggv = o;
        c->cur_pos = 1 - c->cur_pos;
        c->rep_valid = false;
        return GS_OK;
    }
    if ((rc = need_rep(c))) return rc;
    c->vec_valid = false;
    const int i = c->cur_agg, o = (i + 1) % 3, z = (i + 2) % 3;
    if (c->n_local > 0) {
        if ((rc = launch_sweep(c, 0, pc, cutoff, u_dev, seed, stream, i, o, z))) return rc;
    } else {
        HIP_TRY(c, hipMemsetAsync(c->d_agg[o], 0, (size_t)kRepl * c->stride * 8, c->stream));
    }
    if ((rc = allreduce_agg(c, o))) return rc;
    c->cur_agg = o;
    c->cur_pos = 1 - c->cur_pos;
    return GS_OK;
}

constexpr int kGraphSweeps = 6;  // lcm of the position (2) and aggregate (3) rotations
constexpr int kSpecBatch = 32;   // speculative greedy steps enqueued between host checks

bool graphs_wanted(gs_ctx *c) {
    if (c->graph_broken || c->prof) return false;
    return c->graph_mode == 1 || (c->graph_mode < 0 && c->comm != nullptr);
}

int graph_buffers(gs_ctx *c) {
    if (!c->d_sweep_ctr) {
        HIP_TRY(c, hipMalloc(&c->d_sweep_ctr, 8));
        HIP_TRY(c, hipMalloc(&c->d_done_ctr, 4));
    }
    if (!c->d_u6)
        HIP_TRY(c, hipMalloc(&c->d_u6, (size_t)std::max<int32_t>(1, c->n_local) * kGraphSweeps * 8));
    return GS_OK;
}

// The captured chain of kGraphSweeps sweeps (kernel + all-reduce each) for the
// current buffer phase and parameters, or nullptr when capture is unavailable.
hipGraphExec_t sweep_graph(gs_ctx *c, double pc, double cutoff, uint64_t seed) {
    // the DNA sweep draws its uniforms from the device sweep counter itself: its
    // graph is the sweeps alone; the general kernel's starts with a uniforms kernel
    const bool dna = use_dna(c);
    const int aggp = dna ? c->cur_aggv : c->cur_agg;
    for (auto &g : c->graphs)
        if (g.gen == c->graph_gen && g.pos == c->cur_pos && g.agg == aggp && g.dna == dna &&
            g.seed == seed && g.pc == pc && g.cutoff == cutoff)
            return g.exec;
    const int pos0 = c->cur_pos, agg0 = c->cur_agg, aggv0 = c->cur_aggv;
    const bool vv = c->vec_valid, rv = c->rep_valid;
    hipGraph_t graph = nullptr;
    hipGraphExec_t exec = nullptr;
    bool ok = hipStreamBeginCapture(c->stream, hipStreamCaptureModeRelaxed) == hipSuccess;
    if (!dna)
        ok = ok && gs_uniforms_launch(c->d_u6, c->n_local, c->global_offset, seed, kGraphSweeps,
                                      c->d_sweep_ctr, c->d_done_ctr, c->n_cu, c->stream) == hipSuccess;
    for (int k = 0; ok && k < kGraphSweeps; ++k)
        ok = one_sweep(c, pc, cutoff, dna ? nullptr : c->d_u6 + (size_t)k * c->n_local, seed, 0) ==
             GS_OK;
    const bool ended = hipStreamEndCapture(c->stream, &graph) == hipSuccess;
    ok = ok && ended && graph != nullptr &&
         hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0) == hipSuccess;
    if (graph) (void)hipGraphDestroy(graph);
    c->cur_pos = pos0;  // a full period: the phase is unchanged
    c->cur_agg = agg0;
    c->cur_aggv = aggv0;
    c->vec_valid = vv;
    c->rep_valid = rv;
    (void)hipGetLastError();
    if (!ok) {
        if (exec) (void)hipGraphExecDestroy(exec);
        c->graph_broken = true;
        c->err.clear();
        return nullptr;
    }
    gs_ctx::GraphEntry e;
    e.exec = exec;
    e.gen = c->graph_gen;
    e.seed = seed;
    e.pos = pos0;
    e.agg = aggp;
    e.dna = dna;
    e.pc = pc;
    e.cutoff = cutoff;
    c->graphs.push_back(e);
    return exec;
}

// One Jacobi pass of getBestPWMSs over the local targets (gs_starts_kernel),
// enqueued on the context stream: the others at the start vector of `mode`
// (0 per-target draws in d_cpart, 1 shared draws, 2 d_starts) whose aggregates
// are in agg; results to d_score / d_pos_out.  d_ppm (nullable): the caller's PPM
// instead of the others' (getMotifsWithBestPWMSOfPPM); a fixed PCV applies to all.
int starts_pass(gs_ctx *c, int mode, int32_t W, double pc, uint64_t seed, const int32_t *d_starts,
                const int32_t *d_cpart, const int64_t *agg, double *d_score, int32_t *d_pos_out,
                const double *d_ppm = nullptr, StartsArgs *build_only = nullptr,
                int64_t *lds_out = nullptr) {
    const int A = c->A, AW = A * W;
    int64_t o = 0;
    auto take = [&](int64_t b) {
        int64_t q = o;
        o = align16(o + b);
        return (int32_t)q;
    };
    StartsArgs a{};
    a.o_ppm = take(8 * (int64_t)AW);
    a.o_Dt = take(4 * (int64_t)(c->Lmax + 1) * A);
    a.o_cg = take(4 * 2 * (int64_t)AW);
    a.o_compall = take(8 * (int64_t)A);
    a.o_bg = take(8 * (int64_t)A);
    a.o_comp = take(4 * kEncSpace);
    a.o_seq = take(align16(c->Lmax) + 64);
    if (o > c->max_lds)
        return fail(c, GS_E_UNSUPPORTED, "longest sequence exceeds the site scan's LDS budget");
    a.seq = c->d_seq;
    a.doff = c->d_doff;
    a.len = c->d_len;
    a.n_local = c->n_local;
    a.mode = mode;
    a.global_offset = c->global_offset;
    a.A = A;
    a.W = W;
    a.cells = c->cells;
    a.stride = c->stride;
    a.pc = pc;
    a.apc = (double)A * pc;
    a.den = (double)(c->n_global - 1) + a.apc;
    a.seed = seed;
    a.starts = d_starts;
    a.pcv_fixed = c->use_pcv ? c->d_pcv_fixed : nullptr;
    a.ppm_fixed = d_ppm;
    a.agg = agg;
    a.cpart = d_cpart;
    a.score_out = d_score;
    a.pos_out = d_pos_out;
    a.err_code = c->d_err_code;
    a.err_index = c->d_err_index;
    if (build_only) {
        *build_only = a;
        if (lds_out) *lds_out = o;
        return GS_OK;
    }
    if (c->n_local > 0) {
        int grid = std::max(1, std::min<int>(c->n_local, c->n_cu * 8));
        HIP_TRY(c, gs_starts_launch(a, grid, (size_t)o, c->stream));
    }
    return GS_OK;
}

int check_device_error(gs_ctx *c) {
    int32_t code = 0;
    unsigned long long idx = 0;
    HIP_TRY(c, hipMemcpy(&code, c->d_err_code, 4, hipMemcpyDeviceToHost));
    HIP_TRY(c, hipMemcpy(&idx, c->d_err_index, 8, hipMemcpyDeviceToHost));
    if (code == 0) return GS_OK;
    c->have_state = false;  // snapshot is no longer meaningful
    const char *m = code == 2   ? "roulette wheel ran past the last category (.fs:752)"
                    : code == 3 ? "background count sum overflows int32 (.fs:117)"
                                : "device error";
    return fail(c, code, m, (int64_t)idx);
}

}  // namespace

extern "C" {

const char *gs_version(void) { return kVersion; }

int gs_create(int32_t device_id, gs_ctx **out) {
    if (!out) return GS_E_ARG;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return GS_E_HIP;
    if (device_id < 0 || device_id >= ndev) return GS_E_ARG;
    gs_ctx *c = new gs_ctx();
    c->device = device_id;
    if (hipSetDevice(device_id) != hipSuccess ||
        hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc(&c->d_err_code, 4) != hipSuccess || hipMalloc(&c->d_err_index, 8) != hipSuccess ||
        hipMalloc(&c->d_fallbacks, 8 * GS_N_STATS) != hipSuccess) {
        delete c;
        return GS_E_HIP;
    }
    (void)hipMemset(c->d_err_code, 0, 4);
    (void)hipMemset(c->d_err_index, 0xff, 8);
    (void)hipMemset(c->d_fallbacks, 0, 8 * GS_N_STATS);
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device_id) == hipSuccess) {
        c->max_lds = (int32_t)prop.sharedMemPerBlock;
        c->n_cu = prop.multiProcessorCount;
    }
    if (c->max_lds <= 0) c->max_lds = 65536;
    if (c->n_cu <= 0) c->n_cu = 256;
    // diagnostic knob: cap on resident sweep workgroups per CU (grid sizing)
    if (const char *s = std::getenv("GS_BLOCKS_PER_CU")) {
        const int v = std::atoi(s);
        if (v >= 1 && v <= 32) c->blocks_per_cu_cap = v;
    }
    // diagnostic knob: force the lanes per sequence (16, 32, 64) where admissible
    if (const char *s = std::getenv("GS_GROUP_LANES")) {
        const int v = std::atoi(s);
        if (v == 16 || v == 32 || v == 64) c->group_lanes = v;
    }
    // diagnostic knob: wavefronts per sweep workgroup (1 .. sweep_waves(H))
    if (const char *s = std::getenv("GS_SWEEP_WAVES")) {
        const int v = std::atoi(s);
        if (v == 1 || v == 2 || v == 4 || v == 8) c->sweep_waves = v;
    }
    // A/B knob: the site greedy's whole-workgroup scoring of lone visits (GS_SITE_COOP=0 off)
    if (const char *s = std::getenv("GS_SITE_COOP")) c->site_coop = std::atoi(s) != 0;
    if (const char *s = std::getenv("GS_COOP_RATE")) {
        const double v = std::atof(s);
        if (v >= 0.0 && v <= 1.0) c->coop_rate = (float)v;
    }
    if (const char *s = std::getenv("GS_GREEDY_COOP")) {
        const int v = std::atoi(s);
        if (v >= 0) c->motif_coop = v;
    }
    if (const char *s = std::getenv("GS_SITE_DT16")) c->site_dt16 = std::atoi(s) != 0;
    if (const char *s = std::getenv("GS_GREEDY_EXIT_CHUNK")) {
        const int v = std::atoi(s);
        if (v >= 0) c->greedy_exit_chunk = v;
    }
    if (const char *s = std::getenv("GS_GREEDY_EXIT_RATIO")) {
        const int v = std::atoi(s);
        if (v >= 1) c->greedy_exit_ratio = v;
    }
    if (const char *s = std::getenv("GS_SITE_EXIT_RATIO")) {
        const int v = std::atoi(s);
        if (v >= 1) c->site_exit_ratio = v;
    }
    if (const char *s = std::getenv("GS_SITE_EXIT_CHUNK")) {
        const int v = std::atoi(s);
        if (v >= 0) c->site_exit_chunk = v;
    }
    // A/B knobs of the DNA sweep: GS_DNA=0 forces the general kernel, GS_DNA_G lanes per sequence
    if (const char *s = std::getenv("GS_DNA")) c->dna_enable = std::atoi(s) != 0;
    if (const char *s = std::getenv("GS_DNA_G")) {
        const int v = std::atoi(s);
        if (v == 1 || v == 2 || v == 4) c->dna_G = v;
    }
    // hipGraph replay of sweep chains: GS_GRAPH=0 off, 1 on, unset = with a communicator
    if (const char *s = std::getenv("GS_GRAPH")) c->graph_mode = std::atoi(s) ? 1 : 0;
    // tuning knob: threads of the list-path greedy workgroup (64..1024, multiple of 64)
    if (const char *s = std::getenv("GS_MULTI_GREEDY_THREADS")) {
        const int v = std::atoi(s);
        if (v >= 64 && v <= 1024 && v % 64 == 0) c->multi_greedy_threads = v;
    }
    // the star greedy's hand-over to speculative passes (GS_GREEDY_SWITCH, 0 = off)
    if (const char *s = std::getenv("GS_GREEDY_SWITCH")) {
        const int v = std::atoi(s);
        if (v >= 0) c->greedy_switch = v;
    }
    if (const char *s = std::getenv("GS_SITE_SWITCH")) {
        const int v = std::atoi(s);
        if (v >= 0) c->site_switch = v;
    }
    // tuning knob: visits scored per speculative step of the list-path greedy
    if (const char *s = std::getenv("GS_MULTI_SPEC_SLOTS")) {
        const int v = std::atoi(s);
        if (v >= 1 && v <= 4096) c->multi_spec_slots = v;
    }
    // tuning knob: wavefronts (= targets scored per step) of the greedy kernel
    if (const char *s = std::getenv("GS_GREEDY_WAVES")) {
        const int v = std::atoi(s);
        if (v >= 1 && v <= 8) c->greedy_waves = v;
    }
    *out = c;
    return GS_OK;
}

int gs_destroy(gs_ctx *c) {
    if (!c) return GS_OK;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->comm) ncclCommDestroy(c->comm);
    free_state(c);
    dfree(c->d_seq);
    dfree(c->d_doff);
    dfree(c->d_len);
    dfree(c->d_comp);
    dfree(c->d_pk);
    dfree(c->d_pkoff);
    dfree(c->d_err_code);
    dfree(c->d_err_index);
    dfree(c->d_fallbacks);
    for (auto &p : c->ev_sweep) {
        (void)hipEventDestroy(p.first);
        (void)hipEventDestroy(p.second);
    }
    for (auto &p : c->ev_ar) {
        (void)hipEventDestroy(p.first);
        (void)hipEventDestroy(p.second);
    }
    for (auto e : c->ev_pool) (void)hipEventDestroy(e);
    dfree(c->d_pcv_fixed);
    dfree(c->d_ppm_fixed);
    dfree(c->d_mscratch);
    dfree(c->d_merr);
    dfree(c->d_sweep_ctr);
    dfree(c->d_done_ctr);
    if (c->region_start) (void)hipEventDestroy(c->region_start);
    if (c->region_stop) (void)hipEventDestroy(c->region_stop);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
    return GS_OK;
}

const char *gs_last_error(const gs_ctx *c) { return c ? c->err.c_str() : "null context"; }
int64_t gs_error_index(const gs_ctx *c) { return c ? c->err_index : -1; }

int gs_set_sequences(gs_ctx *c, const uint8_t *codes, const int64_t *offsets, int32_t n_local,
                     const uint8_t *alphabet, int32_t alphabet_len, int64_t n_global,
                     int64_t global_offset) {
    if (!c) return GS_E_ARG;
    int rc;
    if ((rc = check_dev(c))) return rc;
    if (n_local < 0 || !offsets || (n_local > 0 && !codes) || !alphabet)
        return fail(c, GS_E_ARG, "null or negative argument");
    if (alphabet_len < 1 || alphabet_len > kSlots)
        return fail(c, GS_E_ARG, "alphabet length must be in [1, 49]");
    if (n_global < (int64_t)n_local || global_offset < 0 || global_offset + n_local > n_global)
        return fail(c, GS_E_ARG, "inconsistent shard geometry");
    // Encoded symbols: alphabet[a] -> a; every other slot present in the data -> A, A+1, ...
    // (the CompositeVector slot order of .fs:17 is only an index; the sampler's
    // arithmetic depends on membership and counts).
    uint8_t enc[kSlots];
    bool seen[kSlots] = {};
    for (int s = 0; s < kSlots; ++s) enc[s] = 0xff;
    for (int a = 0; a < alphabet_len; ++a) {
        int code = alphabet[a];
        if (code < kSlot0 || code >= kSlot0 + kSlots)
            return fail(c, GS_E_ARG, "alphabet symbol outside the 49 CompositeVector slots");
        if (seen[code - kSlot0])
            return fail(c, GS_E_ARG, "duplicate alphabet symbol (unsupported: it double-counts)");
        seen[code - kSlot0] = true;
        enc[code - kSlot0] = (uint8_t)a;
    }
    int E = alphabet_len;
    if (n_local > 0) {
        bool present[256] = {};
        const int64_t nbytes = offsets[n_local] - offsets[0];
        for (int64_t i = 0; i < nbytes; ++i) present[codes[offsets[0] + i]] = true;
        for (int code = 0; code < 256; ++code) {
            if (!present[code]) continue;
            if (code < kSlot0 || code >= kSlot0 + kSlots)
                return fail(c, GS_E_ARG, "symbol code outside [42, 90]");
            if (enc[code - kSlot0] == 0xff) enc[code - kSlot0] = (uint8_t)E++;
        }
    }
    if (offsets[0] != 0) return fail(c, GS_E_ARG, "offsets[0] must be 0");
    std::vector<int32_t> len(n_local);
    std::vector<int64_t> doff(n_local);
    int64_t dpos = 0;
    int32_t lmin = INT32_MAX, lmax = 0;
    for (int32_t n = 0; n < n_local; ++n) {
        int64_t L = offsets[n + 1] - offsets[n];
        if (L < 0 || L > INT32_MAX / 2) return fail(c, GS_E_ARG, "bad sequence length", n);
        len[n] = (int32_t)L;
        lmin = std::min(lmin, (int32_t)L);
        lmax = std::max(lmax, (int32_t)L);
        doff[n] = dpos;
        dpos += align16(L);
    }
    const int64_t total = dpos + 64;
    std::vector<uint8_t> h(total, 0);
    for (int32_t n = 0; n < n_local; ++n) {
        const uint8_t *src = codes + offsets[n];
        uint8_t *dst = h.data() + doff[n];
        for (int32_t i = 0; i < len[n]; ++i) {
            dst[i] = enc[src[i] - kSlot0];
        }
    }
    // the DNA sweep's layout: 2-bit symbols, 16 a word, each sequence on a 16-byte
    // boundary, a tail of zero words for the scan's read-ahead past the last one
    const bool dna = E == alphabet_len && alphabet_len <= 4 && lmax <= kDnaMaxL;
    std::vector<int64_t> pkoff;
    std::vector<uint32_t> pk;
    if (dna) {
        pkoff.resize(n_local);
        int64_t w = 0;
        for (int32_t n = 0; n < n_local; ++n) {
            pkoff[n] = w;
            w += ((len[n] + 15) / 16 + 3) / 4 * 4;
        }
        pk.assign((size_t)(w + kDnaMaxL / 16 + 64), 0u);
        for (int32_t n = 0; n < n_local; ++n) {
            const uint8_t *e = h.data() + doff[n];
            uint32_t *dst = pk.data() + pkoff[n];
            for (int32_t i = 0; i < len[n]; ++i) dst[i >> 4] |= (uint32_t)e[i] << (2 * (i & 15));
        }
    }
    free_state(c);
    dfree(c->d_seq);
    dfree(c->d_doff);
    dfree(c->d_len);
    dfree(c->d_comp);
    dfree(c->d_pk);
    dfree(c->d_pkoff);
    c->dna_ok = false;
    if (dna) {
        HIP_TRY(c, hipMalloc(&c->d_pk, pk.size() * 4));
        HIP_TRY(c, hipMalloc(&c->d_pkoff, (size_t)std::max<int32_t>(1, n_local) * 8));
        HIP_TRY(c, hipMemcpy(c->d_pk, pk.data(), pk.size() * 4, hipMemcpyHostToDevice));
        if (n_local > 0)
            HIP_TRY(c, hipMemcpy(c->d_pkoff, pkoff.data(), (size_t)n_local * 8, hipMemcpyHostToDevice));
        c->dna_ok = true;
    }
    HIP_TRY(c, hipMalloc(&c->d_seq, (size_t)total));
    HIP_TRY(c, hipMalloc(&c->d_doff, (size_t)std::max<int32_t>(1, n_local) * 8));
    HIP_TRY(c, hipMalloc(&c->d_len, (size_t)std::max<int32_t>(1, n_local) * 4));
    HIP_TRY(c, hipMalloc(&c->d_comp, (size_t)std::max<int32_t>(1, n_local) * (E + 1) * 4));
    HIP_TRY(c, hipMemcpy(c->d_seq, h.data(), (size_t)total, hipMemcpyHostToDevice));
    if (n_local > 0) {
        HIP_TRY(c, hipMemcpy(c->d_doff, doff.data(), (size_t)n_local * 8, hipMemcpyHostToDevice));
        HIP_TRY(c, hipMemcpy(c->d_len, len.data(), (size_t)n_local * 4, hipMemcpyHostToDevice));
        // symbol histograms are static: computed once here, read by every sweep
        HIP_TRY(c, gs_composition_launch(c->d_seq, c->d_doff, c->d_len, n_local, alphabet_len, E,
                                         c->d_comp, c->n_cu, c->stream));
        HIP_TRY(c, hipStreamSynchronize(c->stream));
    }
    c->n_local = n_local;
    c->n_global = n_global;
    c->global_offset = global_offset;
    c->A = alphabet_len;
    c->E = E;
    std::memcpy(c->alphabet, alphabet, (size_t)alphabet_len);
    std::memcpy(c->enc, enc, sizeof(enc));
    c->Lmin = n_local ? lmin : 0;
    c->Lmax = lmax;
    c->h_len = std::move(len);
    c->use_pcv = c->use_ppm = false;  // their encoding belonged to the old sequences
    drop_graphs(c);
    return GS_OK;
}

int gs_set_fixed_pcv(gs_ctx *c, const double *pcv49) {
    if (!c) return GS_E_ARG;
    int rc;
    if ((rc = check_dev(c))) return rc;
    if (!c->d_seq) return fail(c, GS_E_STATE, "gs_set_sequences has not been called");
    if (!pcv49) {
        c->use_pcv = false;
        drop_graphs(c);
        return GS_OK;
    }
    // by encoded symbol: the caller's value at each symbol's CompositeVector slot
    std::vector<double> h(64, 0.0);
    for (int s = 0; s < kSlots; ++s)
        if (c->enc[s] != 0xff) h[c->enc[s]] = pcv49[s];
    if (!c->d_pcv_fixed) HIP_TRY(c, hipMalloc(&c->d_pcv_fixed, 64 * sizeof(double)));
    HIP_TRY(c, hipMemcpy(c->d_pcv_fixed, h.data(), 64 * sizeof(double), hipMemcpyHostToDevice));
    c->use_pcv = true;
    drop_graphs(c);
    return GS_OK;
}

int gs_set_fixed_ppm(gs_ctx *c, const double *ppm49, int32_t W) {
    if (!c) return GS_E_ARG;
    int rc;
    if ((rc = check_dev(c))) return rc;
    if (!c->d_seq) return fail(c, GS_E_STATE, "gs_set_sequences has not been called");
    if (!ppm49) {
        c->use_ppm = false;
        return GS_OK;
    }
    if (W < 1 || W > 64) return fail(c, GS_E_ARG, "motifLength must be in [1, 64]");
    // alphabet order, as the initialiser's PPM table
    std::vector<double> h((size_t)c->A * W);
    for (int a = 0; a < c->A; ++a)
        for (int j = 0; j < W; ++j) h[(size_t)a * W + j] = ppm49[(c->alphabet[a] - kSlot0) * W + j];
    dfree(c->d_ppm_fixed);
    HIP_TRY(c, hipMalloc(&c->d_ppm_fixed, h.size() * sizeof(double)));
    HIP_TRY(c, hipMemcpy(c->d_ppm_fixed, h.data(), h.size() * sizeof(double),
                         hipMemcpyHostToDevice));
    c->ppm_W = W;
    c->use_ppm = true;
    return GS_OK;
}

int gs_comm_unique_id(uint8_t out[GS_UNIQUE_ID_BYTES]) {
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return GS_E_RCCL;
    static_assert(sizeof(id) == GS_UNIQUE_ID_BYTES, "unique id size");
    std::memcpy(out, &id, sizeof(id));
    return GS_OK;
}

int gs_comm_init(gs_ctx *c, const uint8_t id_bytes[GS_UNIQUE_ID_BYTES], int32_t nranks,
                 int32_t rank) {
    if (!c || nranks < 1 || rank < 0 || rank >= nranks) return GS_E_ARG;
    int rc;
    if ((rc = check_dev(c))) return rc;
    if (c->comm) {
        ncclCommDestroy(c->comm);
        c->comm = nullptr;
    }
    c->nranks = nranks;
    c->rank = rank;
    drop_graphs(c);  // captured all-reduces name the old communicator
    // a one-rank communicator is real too: it runs the same in-stream all-reduce path
    ncclUniqueId id;
    std::memcpy(&id, id_bytes, sizeof(id));
    RCCL_TRY(c, ncclCommInitRank(&c->comm, nranks, id, rank));
    return GS_OK;
}

int gs_state_set_positions(gs_ctx *c, int32_t W, const int32_t *pos) {
    if (!c || (!pos && c->n_local > 0)) return GS_E_ARG;
    int rc;
    if ((rc = check_dev(c))) return rc;
    return set_snapshot(c, W, pos);
}

int gs_run_sweeps(gs_ctx *c, double pc, double cutoff, int32_t n_sweeps, uint64_t seed,
                  int64_t first_sweep) {
    if (!c || n_sweeps < 0) return GS_E_ARG;
    int rc;
    if ((rc = check_dev(c))) return rc;
    if (!c->have_state) return fail(c, GS_E_STATE, "no snapshot: call gs_state_set_positions");
    int32_t t = 0;
    if (use_dna(c)) {
        // the DNA sweep reads its sweep index from the device counter and the last
        // workgroup of each sweep advances it
        if ((rc = need_vec(c))) return rc;
        HIP_TRY(c, gs_set_counter_launch(c->d_sweep_ctr, (unsigned long long)first_sweep,
                                         c->d_done_ctr, c->stream));
    }
    if (graphs_wanted(c) && n_sweeps >= kGraphSweeps) {
        if ((rc = graph_buffers(c))) return rc;
        if (hipGraphExec_t g = sweep_graph(c, pc, cutoff, seed)) {
            HIP_TRY(c, gs_set_counter_launch(c->d_sweep_ctr, (unsigned long long)first_sweep,
                                             c->d_done_ctr, c->stream));
            for (; t + kGraphSweeps <= n_sweeps; t += kGraphSweeps)
                HIP_TRY(c, hipGraphLaunch(g, c->stream));
        }
    }
    for (; t < n_sweeps; ++t)
        if ((rc = one_sweep(c, pc, cutoff, nullptr, seed,
                            stream_sweep((uint64_t)(first_sweep + t)))))
            return rc;
    return GS_OK;
}

int gs_prepare_sweeps(gs_ctx *c, double pc, double cutoff, uint64_t seed) {
    if (!c) return GS_E_ARG;
    int rc;
    if ((rc = check_dev(c))) return rc;
    if (!c->have_state) return fail(c, GS_E_STATE, "no snapshot: call gs_state_set_positions");
    if (!graphs_wanted(c)) return GS_OK;
    if ((rc = graph_buffers(c))) return rc;
    if (use_dna(c) && (rc = need_vec(c))) return rc;
    (void)sweep_graph(c, pc, cutoff, seed);  // nullptr: direct launches later, not an error
    return GS_OK;
}

int gs_synchronize(gs_ctx *c) {
    if (!c) return GS_E_ARG;
    int rc;
    if ((rc = check_dev(c))) return rc;
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    if (c->d_err_code) return check_device_error(c);
    return GS_OK;
}

int gs_state_get(gs_ctx *c, int32_t *pos_out, double *pwms_out) {
    if (!c) return GS_E_ARG;
    int rc;
    if ((rc = gs_synchronize(c))) return rc;
    if (!c->have_state) return fail(c, GS_E_STATE, "no snapshot");
    if (c->n_local == 0) return GS_OK;
    if (pos_out)
        HIP_TRY(c, hipMemcpy(pos_out, c->d_pos[c->cur_pos], (size_t)c->n_local * 4,
                             hipMemcpyDeviceToHost));
    if (pwms_out)
        HIP_TRY(c, hipMemcpy(pwms_out, c->d_pwms, (size_t)c->n_local * 8, hipMemcpyDeviceToHost));
    return GS_OK;
}

int gs_motif_sweep(gs_ctx *c, int32_t W, double pc, double cutoff, const int32_t *pos_in,
                   const double *u, int32_t *pos_out, double *pwms_out) {
    if (!c || (c->n_local > 0 && (!pos_in || !u || !pos_out || !pwms_out))) return GS_E_ARG;
    int rc;
    if ((rc = check_dev(c))) return rc;
    if ((rc = set_snapshot(c, W, pos_in))) return rc;
    if (c->n_local > 0)
        HIP_TRY(c, hipMemcpyAsync(c->d_u, u, (size_t)c->n_local * 8, hipMemcpyHostToDevice,
                                  c->stream));
    if ((rc = one_sweep(c, pc, cutoff, c->d_u, 0, 0))) return rc;
    return gs_state_get(c, pos_out, pwms_out);
}

int gs_motif_run(gs_ctx *c, int32_t W, double pc, double cutoff, int32_t n_sweeps, uint64_t seed,
                 int64_t first_sweep, int32_t *pos_inout, double *pwms_out) {
    if (!c || (c->n_local > 0 && !pos_inout)) return GS_E_ARG;
    int rc;
    if ((rc = gs_state_set_positions(c, W, pos_inout))) return rc;
    if ((rc = gs_run_sweeps(c, pc, cutoff, n_sweeps, seed, first_sweep))) return rc;
    return gs_state_get(c, pos_inout, pwms_out);
}

// The speculative Gauss–Seidel kernel (gs_greedy.hip) on the resident snapshot
// (d_pos[cur_pos], d_pwms, d_agg[cur_agg]); site = 1: the site sampler's twin.
// exit_info (nullable): {visits of the pass done before a mid-pass exit (0: none),
// the pass moved}, with the exit rule of GreedyArgs::exit_chunk (exit_chunk > 0).
static int greedy_run(gs_ctx *c, int site, double pc, double cutoff, int32_t max_passes,
                      int32_t *passes_out, double *kernel_ms_out, int32_t exit_chunk = 0,
                      int32_t exit_ratio = 0, int32_t *exit_info = nullptr) {
    int rc;
    int32_t passes = 0;
    float ms = 0.0f;
    if (c->n_local > 0) {
        GreedyArgs a{};
        const int A = c->A, E = c->E, W = c->W, WM = gs_sweep_wm(W);
        // workgroup part, then per wavefront: a tab slice and two ring slots
        int64_t o = 0;
        auto take = [&](int64_t b) {
            int64_t q = o;
            o = align16(o + b);
            return (int32_t)q;
        };
        a.o_C = take(4 * (int64_t)A * W);
        a.o_T = take(8 * (int64_t)A);
        a.o_ppmG = take(8 * (int64_t)A * W);
        a.o_ppmM = take(8 * (int64_t)A * W);
        a.o_ctl = take(4 * 64);
        const int64_t fixed = o;
        a.ring_seq_bytes = (int32_t)(align16(c->Lmax) + align16(WM) + 32);
        int64_t wb = 0;
        if (site) {  // D_k table [K][A], the others' background, the composition
            a.w_dt = 0;
            // D_k[b] <= (k + 1) W <= Lmax W: two bytes an entry when that fits
            a.dt16 = (int64_t)c->Lmax * W < 65536 && c->site_dt16 ? 1 : 0;
            wb = align16((a.dt16 ? 2 : 4) * (int64_t)c->Lmax * A);
            a.w_bg = (int32_t)wb;
            wb += 8 * 64;
            a.w_comp = (int32_t)wb;
            wb += 4 * 64;
        } else {     // (PWM, PCV) table, PCV
            a.w_tab = 0;
            wb = align16(16 * (int64_t)E * tab_stride(WM));
            a.w_pcv = (int32_t)wb;
            wb += 8 * 64;
        }
        a.wave_bytes = (int32_t)wb;
        a.site = site;
        a.pcv_fixed = c->use_pcv ? c->d_pcv_fixed : nullptr;
        const int64_t per_wave = wb + 2 * (a.ring_seq_bytes + 4 * 3 + 8 + 4 * 64) + 64 + 32;
        int waves = c->greedy_waves;
        while (waves > 1 && fixed + per_wave * waves > c->max_lds) --waves;
        if ((int64_t)waves > c->n_local) waves = (int)std::max<int64_t>(1, c->n_local);
        while (waves & (waves - 1)) waves &= waves - 1;  // a power of two (ring indexing)
        const int R = 2 * waves;
        a.o_ring = take((int64_t)R * a.ring_seq_bytes);
        a.o_rt = take(4 * (int64_t)R);
        a.o_rL = take(4 * (int64_t)R);
        a.o_rp = take(4 * (int64_t)R);
        a.o_rpw = take(8 * (int64_t)R);
        a.o_rcomp = take(4 * 64 * (int64_t)R);
        a.o_red = take(8 * 4 * (int64_t)waves);
        a.o_wave = take((int64_t)waves * a.wave_bytes);
        a.site_coop = site && c->site_coop ? 1 : 0;
        a.motif_coop = site ? 0 : c->motif_coop;
        a.coop_rate = site ? c->coop_rate : 0.0f;  // motif (cfg5): 217 -> 234 ms with it
        if (o > c->max_lds)
            return fail(c, GS_E_UNSUPPORTED,
                        "longest sequence exceeds the greedy kernel's LDS budget (" +
                            std::to_string(o) + " > " + std::to_string(c->max_lds) + " B)");
        c->last_greedy_waves = waves;
        a.seq = c->d_seq;
        a.doff = c->d_doff;
        a.len = c->d_len;
        a.comp = c->d_comp;
        a.n = c->n_local;
        a.A = A;
        a.W = W;
        a.E = E;
        a.cells = c->cells;
        a.stride = c->stride;
        a.pc = pc;
        a.cutoff = cutoff;
        a.thr_lo = cutoff_threshold(cutoff);
        a.apc = (double)A * pc;
        a.den = (double)(c->n_global - 1) + a.apc;
        a.max_passes = max_passes;
        if ((rc = need_rep(c))) return rc;
        c->vec_valid = false;  // the passes rewrite the replicas
        a.agg = c->d_agg[c->cur_agg];
        a.pos = c->d_pos[c->cur_pos];
        a.pwms = c->d_pwms;
        a.passes_out = c->d_aux + c->n_local;
        a.exit_chunk = exit_info ? exit_chunk : 0;
        a.exit_ratio = exit_ratio;
        a.exit_out = exit_info ? c->d_aux + c->n_local + 1 : nullptr;
        a.err_code = c->d_err_code;
        a.err_index = c->d_err_index;
#ifdef GS_STAMPS
        if (!c->d_stamps) {
            HIP_TRY(c, hipMalloc(&c->d_stamps, 8 * kStampSlots));
            HIP_TRY(c, hipMemset(c->d_stamps, 0, 8 * kStampSlots));
        }
        a.stamps = c->d_stamps;
#endif
        hipEvent_t e0 = get_event(c), e1 = get_event(c);
        HIP_TRY(c, gs_greedy_launch(a, waves, (size_t)o, c->stream, e0, e1));
        HIP_TRY(c, hipStreamSynchronize(c->stream));
        HIP_TRY(c, hipEventElapsedTime(&ms, e0, e1));
        c->ev_pool.push_back(e0);
        c->ev_pool.push_back(e1);
        if ((rc = check_device_error(c))) return rc;
        HIP_TRY(c, hipMemcpy(&passes, a.passes_out, 4, hipMemcpyDeviceToHost));
        if (exit_info) HIP_TRY(c, hipMemcpy(exit_info, a.exit_out, 8, hipMemcpyDeviceToHost));
    }
    if (passes_out) *passes_out = passes;
    if (kernel_ms_out) *kernel_ms_out = (double)ms;
    return GS_OK;
}

int greedy_hybrid(gs_ctx *c, double pc, double cutoff, int32_t max_passes, int32_t *passes_out,
                  double *kernel_ms_out);

int gs_run_greedy(gs_ctx *c, double pc, double cutoff, int32_t max_passes, int32_t *passes_out,
                  double *kernel_ms_out) {
    if (!c || max_passes < 1) return GS_E_ARG;
    int rc;
    if ((rc = check_dev(c))) return rc;
    if (!c->have_state) return fail(c, GS_E_STATE, "no snapshot: call gs_state_set_positions");
    if ((int64_t)c->n_local != c->n_global)
        return fail(c, GS_E_UNSUPPORTED,
                    "the greedy refinement walks every target in order (.fs:885-929): it needs "
                    "all sequences on one device");
    if (c->greedy_switch > 0 && !c->use_pcv)
        return greedy_hybrid(c, pc, cutoff, max_passes, passes_out, kernel_ms_out);
    return greedy_run(c, 0, pc, cutoff, max_passes, passes_out, kernel_ms_out);
}

int gs_motif_greedy(gs_ctx *c, int32_t W, double pc, double cutoff, int32_t max_passes,
                    int32_t *pos_inout, double *pwms_inout, int32_t *passes_out) {
    if (!c || (c->n_local > 0 && (!pos_inout || !pwms_inout))) return GS_E_ARG;
    int rc;
    if ((rc = check_dev(c))) return rc;
    if ((rc = set_snapshot(c, W, pos_inout))) return rc;
    if (c->n_local > 0)
        HIP_TRY(c, hipMemcpyAsync(c->d_pwms, pwms_inout, (size_t)c->n_local * 8,
                                  hipMemcpyHostToDevice, c->stream));
    if ((rc = gs_run_greedy(c, pc, cutoff, max_passes, passes_out, nullptr))) return rc;
    return gs_state_get(c, pos_inout, pwms_inout);
}

int gs_motif_sampling(gs_ctx *c, int32_t W, double pc, double cutoff, uint64_t seed,
                      int32_t init_mode, int32_t max_passes, int32_t *pos_out, double *pwms_out,
                      int32_t *passes_out) {
    if (!c || max_passes < 1 || (c->n_local > 0 && (!pos_out || !pwms_out))) return GS_E_ARG;
    int rc;
    // getPWMOfRandomStarts |> createMotifIndex prob [position] (.fs:1035-1036); the
    // sweep reads positions only, so the start scores stay on the host
    if ((rc = gs_random_starts(c, W, pc, seed, init_mode, pwms_out, pos_out))) return rc;
    if ((rc = gs_state_set_positions(c, W, pos_out))) return rc;
    // |> findBestMotifIndicesByWithStartPositions (.fs:1037): sweep 0 of `seed`
    if ((rc = gs_run_sweeps(c, pc, cutoff, 1, seed, 0))) return rc;
    // |> findBestMotifIndicesWithStartPositions (.fs:1038)
    if ((rc = gs_run_greedy(c, pc, cutoff, max_passes, passes_out, nullptr))) return rc;
    return gs_state_get(c, pos_out, pwms_out);
}

int gs_counts(gs_ctx *c, int32_t W, const int32_t *pos, int64_t *C_out, int64_t *T_out) {
    if (!c || !C_out || !T_out || (c->n_local > 0 && !pos)) return GS_E_ARG;
    int rc;
    if ((rc = check_dev(c))) return rc;
    if ((rc = set_snapshot(c, W, pos))) return rc;
    if ((rc = gs_synchronize(c))) return rc;
    std::vector<int64_t> h((size_t)kRepl * c->stride);
    HIP_TRY(c, hipMemcpy(h.data(), c->d_agg[c->cur_agg], h.size() * 8, hipMemcpyDeviceToHost));
    const int A = c->A, AW = A * W;
    for (int x = 0; x < c->cells; ++x) {
        int64_t s = 0;
        for (int r = 0; r < kRepl; ++r) s += h[(size_t)r * c->stride + x];
        if (x < AW)
            C_out[x] = s;
        else
            T_out[x - AW] = s;  // the kernel accumulates composition - segment directly
    }
    return GS_OK;
}

int64_t gs_agg_size(const gs_ctx *c) {
    return (c && c->have_state) ? (int64_t)kRepl * c->stride : 0;
}

int gs_agg_download(gs_ctx *c, int64_t *out) {
    if (!c || !out) return GS_E_ARG;
    int rc;
    if ((rc = gs_synchronize(c))) return rc;
    if (!c->have_state) return fail(c, GS_E_STATE, "no snapshot");
    if ((rc = need_rep(c))) return rc;
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    HIP_TRY(c, hipMemcpy(out, c->d_agg[c->cur_agg], (size_t)kRepl * c->stride * 8,
                         hipMemcpyDeviceToHost));
    return GS_OK;
}

int gs_agg_upload(gs_ctx *c, const int64_t *in) {
    if (!c || !in) return GS_E_ARG;
    int rc;
    if ((rc = check_dev(c))) return rc;
    if (!c->have_state) return fail(c, GS_E_STATE, "no snapshot");
    HIP_TRY(c, hipMemcpyAsync(c->d_agg[c->cur_agg], in, (size_t)kRepl * c->stride * 8,
                              hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    c->rep_valid = true;
    c->vec_valid = false;
    return GS_OK;
}

int gs_random_starts(gs_ctx *c, int32_t W, double pc, uint64_t seed, int32_t mode,
                     double *score_out, int32_t *pos_out) {
    if (!c || (mode != 0 && mode != 1) || (c->n_local > 0 && (!score_out || !pos_out)))
        return GS_E_ARG;
    int rc;
    if ((rc = check_dev(c))) return rc;
    if ((rc = validate_W(c, W))) return rc;
    if (c->use_ppm && c->ppm_W != W)
        return fail(c, GS_E_ARG, "the fixed PPM was set for another motifLength");
    // start vector for the aggregate pass: the shared draws (mode 1), or any valid
    // snapshot (mode 0 only needs the all-sequence composition totals from it)
    std::vector<int32_t> r((size_t)c->n_local, 0);
    if (mode == 1)
        for (int32_t n = 0; n < c->n_local; ++n)
            r[n] = uniform_int(seed, stream_init_shared(), (uint64_t)(c->global_offset + n),
                               c->h_len[n] - W + 1);
    if ((rc = set_snapshot(c, W, r.data()))) return rc;
    const int A = c->A, AW = A * W;
    int32_t *d_cpart = nullptr;
    if (mode == 0) {
        const size_t bytes = (size_t)c->n_global * AW * 4;
        HIP_TRY(c, hipMalloc(&d_cpart, std::max<size_t>(bytes, 4)));
        HIP_TRY(c, hipMemsetAsync(d_cpart, 0, bytes, c->stream));
        PartialArgs p{};
        p.seq = c->d_seq;
        p.doff = c->d_doff;
        p.len = c->d_len;
        p.n_local = c->n_local;
        p.global_offset = c->global_offset;
        p.n_global = c->n_global;
        p.A = A;
        p.W = W;
        p.seed = seed;
        p.cpart = d_cpart;
        if (c->n_local > 0) {
            int grid = (int)std::max<int64_t>(1, std::min<int64_t>(c->n_global, c->n_cu * 8));
            HIP_TRY(c, gs_starts_partial_launch(p, grid, c->stream));
        }
        if (c->comm)
            RCCL_TRY(c, ncclAllReduce(d_cpart, d_cpart, (size_t)c->n_global * AW, ncclInt32,
                                      ncclSum, c->comm, c->stream));
    }
    rc = starts_pass(c, mode, W, pc, seed, nullptr, d_cpart, c->d_agg[c->cur_agg], c->d_pwms,
                     c->d_pos[1], c->use_ppm ? c->d_ppm_fixed : nullptr);
    if (rc == GS_OK) HIP_TRY(c, hipStreamSynchronize(c->stream));
    dfree(d_cpart);
    if (rc) return rc;
    c->have_state = false;  // the snapshot buffers were used as scratch
    if ((rc = check_device_error(c))) return rc;
    if (c->n_local > 0) {
        HIP_TRY(c, hipMemcpy(score_out, c->d_pwms, (size_t)c->n_local * 8, hipMemcpyDeviceToHost));
        HIP_TRY(c, hipMemcpy(pos_out, c->d_pos[1], (size_t)c->n_local * 4, hipMemcpyDeviceToHost));
    }
    return GS_OK;
}

double gs_uniform(uint64_t seed, uint64_t stream, uint64_t index) {
    return uniform(seed, stream, index);
}
uint64_t gs_stream_sweep(uint64_t sweep) { return stream_sweep(sweep); }

namespace {

// Site-sampler positions are plain starts: every entry in [0, L_n - W].
int validate_site_pos(gs_ctx *c, int32_t W, const int32_t *pos) {
    for (int32_t n = 0; n < c->n_local; ++n)
        if (pos[n] < 0 || pos[n] + W > c->h_len[n])
            return fail(c, GS_E_ARG, "start position outside its sequence (getSegment, .fs:149-153)",
                        c->global_offset + n);
    return GS_OK;
}

// getBestPWMSsWithStartPositions on the snapshot just set (d_pos[0], d_agg[0])
// with the scores in d_pwms: the speculative Gauss–Seidel kernel, synchronous.
// getBestPWMSsWithStartPositions (.fs:554-585) on the uploaded acc (d_pos[0] starts,
// d_pwms scores, d_agg[cur_agg] their aggregates): the star site engine one pass per
// launch while passes move many starts; once a pass moves fewer than N / greedy_switch,
// speculative steps (every visit of [base, base + slots) scanned in parallel against
// the live starts by gs_starts_kernel, committed in order up to the first move).
int site_greedy(gs_ctx *c, double pc, int32_t max_passes, int32_t *passes_out) {
    if (c->site_switch <= 0) return greedy_run(c, 1, pc, 0.0, max_passes, passes_out, nullptr);
    const int32_t n = c->n_local;
    const int64_t nn = std::max<int32_t>(1, n);
    int rc;
    int32_t *d_prev = nullptr, *d_moves = nullptr;
    SpecCtl *ctl = nullptr;
    SiteRes *res = nullptr;
    auto cleanup = [&]() {
        dfree(d_prev);
        dfree(d_moves);
        dfree(ctl);
        dfree(res);
    };
    if (hipMalloc(&d_prev, nn * 4) != hipSuccess || hipMalloc(&d_moves, 4) != hipSuccess) {
        cleanup();
        return fail(c, GS_E_HIP, "hipMalloc(site hand-over)");
    }
    int32_t passes = 0, spec_base = 0, spec_changed = 0;
    bool spec = false;
    while (passes < max_passes && n > 0) {
        int32_t *pos = c->d_pos[c->cur_pos];
        hipError_t e = hipMemcpyAsync(d_prev, pos, (size_t)n * 4, hipMemcpyDeviceToDevice, c->stream);
        int32_t p1 = 0;
        if (e != hipSuccess) {
            cleanup();
            return fail(c, GS_E_HIP, "site hand-over copy");
        }
        // the star engine stops inside the pass once a chunk of visits moves fewer
        // than chunk / site_switch starts; the speculative steps take the rest
        int32_t ex[2] = {0, 0};
        if ((rc = greedy_run(c, 1, pc, 0.0, 1, &p1, nullptr, c->site_exit_chunk, c->site_exit_ratio,
                             c->site_exit_chunk > 0 ? ex : nullptr))) {
            cleanup();
            return rc;
        }
        if (ex[0] > 0) {  // mid-pass: the speculative steps resume at visit ex[0]
            spec_base = ex[0];
            spec_changed = ex[1];
            spec = true;
            break;
        }
        ++passes;
        int32_t moves = 0;
        e = hipMemsetAsync(d_moves, 0, 4, c->stream);
        if (e == hipSuccess) e = gs_count_diff_launch(d_prev, pos, n, d_moves, c->stream);
        if (e == hipSuccess) e = hipMemcpyAsync(&moves, d_moves, 4, hipMemcpyDeviceToHost, c->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
        if (e != hipSuccess) {
            cleanup();
            return fail(c, GS_E_HIP, "site move count");
        }
        if (moves == 0) break;
        if ((int64_t)moves * c->site_switch < n && passes < max_passes) {
            spec = true;
            break;
        }
    }
    if (spec) {
        const int32_t slots =
            (int32_t)std::max<int64_t>(1, std::min<int64_t>(n, c->multi_spec_slots));
        StartsArgs a{};
        int64_t lds = 0;
        int32_t *pos = c->d_pos[c->cur_pos];
        if ((rc = starts_pass(c, 2, c->W, pc, 0, pos, nullptr, c->d_agg[c->cur_agg], nullptr,
                              nullptr, nullptr, &a, &lds))) {
            cleanup();
            return rc;
        }
        if (hipMalloc(&ctl, sizeof(SpecCtl)) != hipSuccess ||
            hipMalloc(&res, sizeof(SiteRes) * (size_t)slots) != hipSuccess) {
            cleanup();
            return fail(c, GS_E_HIP, "hipMalloc(site speculation)");
        }
        a.spec_ctl = ctl;
        a.spec_res = res;
        SiteCommitArgs ca{};
        ca.ctl = ctl;
        ca.res = res;
        ca.slots = slots;
        ca.n = n;
        ca.A = c->A;
        ca.W = c->W;
        ca.max_passes = max_passes - passes;
        ca.seq = c->d_seq;
        ca.doff = c->d_doff;
        ca.score = c->d_pwms;
        ca.pos = pos;
        ca.agg = c->d_agg[c->cur_agg];  // replica 0: the sums over replicas are what count
        SpecCtl h{};
        h.base = spec_base;  // 0, or where the star engine left the pass
        h.changed = spec_changed;
        hipError_t e = hipStreamSynchronize(c->stream);
        if (e == hipSuccess) e = hipMemcpy(ctl, &h, sizeof(SpecCtl), hipMemcpyHostToDevice);
        const int64_t step_limit = ((int64_t)n + 1) * ca.max_passes + kSpecBatch;
        int64_t steps = 0;
        while (e == hipSuccess) {
            e = gs_site_spec_launch(a, ca, (size_t)lds, kSpecBatch, c->stream);
            if (e == hipSuccess) e = hipMemcpyAsync(&h, ctl, sizeof(h), hipMemcpyDeviceToHost, c->stream);
            if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
            steps += kSpecBatch;
            if (h.done || steps > step_limit) break;
        }
        if (e != hipSuccess || !h.done) {
            cleanup();
            return fail(c, GS_E_HIP, e != hipSuccess ? std::string("site speculation: ") + hipGetErrorString(e)
                                                     : std::string("site speculation made no progress"));
        }
        passes += h.pass;
    }
    cleanup();
    if ((rc = check_device_error(c))) return rc;
    if (passes_out) *passes_out = passes;
    return GS_OK;
}

// The ±1 shifted passes (Jacobi): acc positions in d_pos[0], acc scores in d_pwms.
// Per pass: shifted start vector -> d_pos[1], its aggregates -> d_agg[0] (all-reduced
// over the ranks), one getBestPWMSs pass -> (d_u, d_aux), accept; the pass-end
// comparison with bestMotif counts the moved targets over all ranks.
int site_shift(gs_ctx *c, double pc, int32_t dir, int32_t max_passes, int32_t *passes) {
    const int32_t n = c->n_local;
    int32_t *moved = c->d_aux + n;
    int rc;
    for (int32_t pass = 1;; ++pass) {
        *passes = pass;
        HIP_TRY(c, gs_site_shift_launch(c->d_pos[0], c->d_len, n, c->W, dir, c->d_pos[1], c->stream));
        HIP_TRY(c, hipMemsetAsync(c->d_agg[0], 0, (size_t)kRepl * c->stride * 8, c->stream));
        c->cur_pos = 1;
        if (n > 0)
            if ((rc = launch_sweep(c, 1, 0.0, 0.0, nullptr, 0, 0, -1, 0, -1))) return rc;
        c->cur_pos = 0;
        if ((rc = allreduce_agg(c, 0))) return rc;
        if ((rc = starts_pass(c, 2, c->W, pc, 0, c->d_pos[1], nullptr, c->d_agg[0], c->d_u,
                              c->d_aux)))
            return rc;
        HIP_TRY(c, hipMemsetAsync(moved, 0, 4, c->stream));
        HIP_TRY(c, gs_site_accept_launch(c->d_u, c->d_aux, c->d_pwms, c->d_pos[0], n, moved,
                                         c->stream));
        if (c->comm)
            RCCL_TRY(c, ncclAllReduce(moved, moved, 1, ncclInt32, ncclSum, c->comm, c->stream));
        int32_t h = 0;
        HIP_TRY(c, hipMemcpyAsync(&h, moved, 4, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(c, hipStreamSynchronize(c->stream));
        if ((rc = check_device_error(c))) return rc;
        if (h == 0 || pass >= max_passes) return GS_OK;
    }
}

// Upload (pos, score) as the acc of a site-sampler refinement.
int site_upload(gs_ctx *c, int32_t W, const int32_t *pos, const double *score) {
    int rc;
    if ((rc = validate_W(c, W))) return rc;
    if ((rc = validate_site_pos(c, W, pos))) return rc;
    if ((rc = set_snapshot(c, W, pos))) return rc;
    if (c->n_local > 0)
        HIP_TRY(c, hipMemcpyAsync(c->d_pwms, score, (size_t)c->n_local * 8, hipMemcpyHostToDevice,
                                  c->stream));
    return GS_OK;
}

int site_download(gs_ctx *c, int32_t *pos, double *score) {
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    if (c->n_local > 0) {
        HIP_TRY(c, hipMemcpy(pos, c->d_pos[0], (size_t)c->n_local * 4, hipMemcpyDeviceToHost));
        HIP_TRY(c, hipMemcpy(score, c->d_pwms, (size_t)c->n_local * 8, hipMemcpyDeviceToHost));
    }
    c->have_state = false;  // the snapshot buffers held site-sampler state
    return GS_OK;
}

int site_refine(gs_ctx *c, double pc, int32_t shift, int32_t max_passes, int32_t *passes) {
    if (shift == 0) {
        if ((int64_t)c->n_local != c->n_global)
            return fail(c, GS_E_UNSUPPORTED,
                        "getBestPWMSsWithStartPositions walks every target in order (.fs:554-585): "
                        "it needs all sequences on one device");
        return site_greedy(c, pc, max_passes, passes);
    }
    return site_shift(c, pc, shift, max_passes, passes);
}

}  // namespace

int gs_site_scan(gs_ctx *c, int32_t W, double pc, const int32_t *pos, double *score_out,
                 int32_t *pos_out) {
    if (!c || (c->n_local > 0 && (!pos || !score_out || !pos_out))) return GS_E_ARG;
    int rc;
    if ((rc = check_dev(c))) return rc;
    if ((rc = validate_W(c, W))) return rc;
    if ((rc = validate_site_pos(c, W, pos))) return rc;
    if ((rc = set_snapshot(c, W, pos))) return rc;
    if ((rc = starts_pass(c, 2, W, pc, 0, c->d_pos[0], nullptr, c->d_agg[0], c->d_pwms,
                          c->d_pos[1])))
        return rc;
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    c->have_state = false;
    if ((rc = check_device_error(c))) return rc;
    if (c->n_local > 0) {
        HIP_TRY(c, hipMemcpy(score_out, c->d_pwms, (size_t)c->n_local * 8, hipMemcpyDeviceToHost));
        HIP_TRY(c, hipMemcpy(pos_out, c->d_pos[1], (size_t)c->n_local * 4, hipMemcpyDeviceToHost));
    }
    return GS_OK;
}

int gs_site_refine(gs_ctx *c, int32_t W, double pc, int32_t shift, int32_t max_passes,
                   int32_t *pos_inout, double *score_inout, int32_t *passes_out) {
    if (!c || shift < -1 || shift > 1 || max_passes < 1 ||
        (c->n_local > 0 && (!pos_inout || !score_inout)))
        return GS_E_ARG;
    int rc;
    if ((rc = check_dev(c))) return rc;
    if ((rc = site_upload(c, W, pos_inout, score_inout))) return rc;
    int32_t passes = 0;
    if ((rc = site_refine(c, pc, shift, max_passes, &passes))) return rc;
    if (passes_out) *passes_out = passes;
    return site_download(c, pos_inout, score_inout);
}

int gs_site_sampling(gs_ctx *c, int32_t W, double pc, uint64_t seed, int32_t init_mode,
                     int32_t max_passes, int32_t *pos_out, double *score_out,
                     int32_t *passes_out) {
    if (!c || max_passes < 1 || (c->n_local > 0 && (!pos_out || !score_out))) return GS_E_ARG;
    int rc;
    if ((rc = gs_random_starts(c, W, pc, seed, init_mode, score_out, pos_out))) return rc;
    if ((rc = site_upload(c, W, pos_out, score_out))) return rc;
    // getBestPWMSsWithStartPositions |> getLeftShifted.. |> getRightShifted.. (.fs:697-701)
    const int32_t shifts[3] = {0, -1, 1};
    for (int i = 0; i < 3; ++i) {
        int32_t passes = 0;
        if ((rc = site_refine(c, pc, shifts[i], max_passes, &passes))) return rc;
        if (passes_out) passes_out[i] = passes;
        if (shifts[i] == 0) {
            // the shifted passes start from the refined acc in d_pos[0] / d_pwms
            c->cur_pos = 0;
        }
    }
    return site_download(c, pos_out, score_out);
}

int gs_profile_enable(gs_ctx *c, int32_t enable) {
    if (!c || enable < 0) return GS_E_ARG;
    c->prof = enable != 0;
    c->prof_stride = enable > 0 ? enable : 1;
    c->prof_sweep_calls = c->prof_ar_calls = 0;
    return GS_OK;
}

int gs_profile_region_begin(gs_ctx *c) {
    if (!c) return GS_E_ARG;
    int rc;
    if ((rc = check_dev(c))) return rc;
    if (!c->region_start) HIP_TRY(c, hipEventCreate(&c->region_start));
    if (!c->region_stop) HIP_TRY(c, hipEventCreate(&c->region_stop));
    HIP_TRY(c, hipEventRecord(c->region_start, c->stream));
    return GS_OK;
}

int gs_profile_region_end(gs_ctx *c, double *ms) {
    if (!c || !ms) return GS_E_ARG;
    if (!c->region_start) return fail(c, GS_E_STATE, "gs_profile_region_begin was not called");
    HIP_TRY(c, hipEventRecord(c->region_stop, c->stream));
    HIP_TRY(c, hipEventSynchronize(c->region_stop));
    float f = 0.0f;
    HIP_TRY(c, hipEventElapsedTime(&f, c->region_start, c->region_stop));
    *ms = (double)f;
    return GS_OK;
}

int gs_profile_read(gs_ctx *c, double *sweep_ms, int64_t *sweeps, double *ar_ms, int64_t *ars) {
    if (!c) return GS_E_ARG;
    int rc;
    if ((rc = check_dev(c))) return rc;
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    for (auto &p : c->ev_sweep) {
        float ms = 0.f;
        HIP_TRY(c, hipEventElapsedTime(&ms, p.first, p.second));
        c->prof_sweep_ms += ms;
        c->prof_sweeps += 1;
        c->ev_pool.push_back(p.first);
        c->ev_pool.push_back(p.second);
    }
    c->ev_sweep.clear();
    for (auto &p : c->ev_ar) {
        float ms = 0.f;
        HIP_TRY(c, hipEventElapsedTime(&ms, p.first, p.second));
        c->prof_ar_ms += ms;
        c->prof_ars += 1;
        c->ev_pool.push_back(p.first);
        c->ev_pool.push_back(p.second);
    }
    c->ev_ar.clear();
    if (sweep_ms) *sweep_ms = c->prof_sweep_ms;
    if (sweeps) *sweeps = c->prof_sweeps;
    if (ar_ms) *ar_ms = c->prof_ar_ms;
    if (ars) *ars = c->prof_ars;
    c->prof_sweep_ms = c->prof_ar_ms = 0.0;
    c->prof_sweeps = c->prof_ars = 0;
    return GS_OK;
}

#ifdef GS_STAMPS
// Diagnostic build only (not in the public header): summed per-phase s_memtime
// cycles of the sweep kernel's wavefronts, [7] = sequences processed.
int gs_debug_stamps(gs_ctx *c, unsigned long long *out, int32_t reset) {
    if (!c || !out) return GS_E_ARG;
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    if (!c->d_stamps) {
        std::memset(out, 0, 8 * kStampSlots);
        return GS_OK;
    }
    HIP_TRY(c, hipMemcpy(out, c->d_stamps, 8 * kStampSlots, hipMemcpyDeviceToHost));
    if (reset) HIP_TRY(c, hipMemset(c->d_stamps, 0, 8 * kStampSlots));
    return GS_OK;
}
#endif

int gs_stats(gs_ctx *c, int64_t *out, int32_t n) {
    if (!c || !out || n < 0) return GS_E_ARG;
    int rc;
    if ((rc = check_dev(c))) return rc;
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    unsigned long long v[GS_N_STATS] = {};
    HIP_TRY(c, hipMemcpy(v, c->d_fallbacks, sizeof(v), hipMemcpyDeviceToHost));
    for (int i = 0; i < n && i < GS_N_STATS; ++i) out[i] = (int64_t)v[i];
    return GS_OK;
}

int gs_set_scan_mode(gs_ctx *c, int32_t mode) {
    if (!c || (mode != GS_SCAN_CERTIFIED && mode != GS_SCAN_EXACT)) return GS_E_ARG;
    c->scan = mode;
    drop_graphs(c);
    return GS_OK;
}

int gs_fastmath_check(gs_ctx *c, double *log2_abs_err, double *exp2_rel_err) {
    if (!c || !log2_abs_err || !exp2_rel_err) return GS_E_ARG;
    int rc;
    if ((rc = check_dev(c))) return rc;
    unsigned int *d = nullptr;
    HIP_TRY(c, hipMalloc(&d, 8));
    unsigned int h[2] = {0, 0};
    hipError_t e = hipMemsetAsync(d, 0, 8, c->stream);
    if (e == hipSuccess) e = gs_fastmath_launch(d, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e == hipSuccess) e = hipMemcpy(h, d, 8, hipMemcpyDeviceToHost);
    (void)hipFree(d);
    if (e != hipSuccess) return fail(c, GS_E_HIP, std::string("gs_fastmath_check: ") + hipGetErrorString(e));
    float fl, fe;
    std::memcpy(&fl, &h[0], 4);
    std::memcpy(&fe, &h[1], 4);
    *log2_abs_err = fl;
    *exp2_rel_err = fe;
    return GS_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// motifAmount >= 1 with Positions lists (gs_multi.hip).
namespace {

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

int validate_lists(gs_ctx *c, int32_t M, int32_t W, int32_t cap, const int32_t *cnt,
                   const int32_t *pos) {
    int rc;
    if ((rc = validate_W(c, W))) return rc;
    if (M < 1 || M > kMultiMaxAmount)
        return fail(c, GS_E_ARG, "motifAmount must be in [1, " + std::to_string(kMultiMaxAmount) + "]");
    if (cap < M || cap > kMultiMaxAmount)
        return fail(c, GS_E_ARG, "list capacity must be in [motifAmount, 16]");
    for (int32_t n = 0; n < c->n_local; ++n) {
        if (cnt[n] < 0 || cnt[n] > cap)
            return fail(c, GS_E_ARG, "Positions list longer than its capacity", c->global_offset + n);
        for (int32_t i = 0; i < cnt[n]; ++i) {
            const int32_t p = pos[(int64_t)n * cap + i];
            if (p < 0 || p + W > c->h_len[n])
                return fail(c, GS_E_ARG,
                            "motif position outside its sequence (getSegment, .fs:149-153)",
                            c->global_offset + n);
        }
    }
    return GS_OK;
}

// Common kernel arguments; LDS carve for the sweep (greedy adds the aggregates).
int64_t multi_args(gs_ctx *c, MultiArgs &a, int32_t M, int32_t W, int32_t cap, double pc,
                   double cutoff, bool greedy) {
    a.seq = c->d_seq;
    a.doff = c->d_doff;
    a.len = c->d_len;
    a.comp = c->d_comp;
    a.n_local = c->n_local;
    a.global_offset = c->global_offset;
    a.A = c->A;
    a.W = W;
    a.E = c->E;
    a.M = M;
    a.cap_in = a.cap_out = cap;
    a.pc = pc;
    a.cutoff = cutoff;
    a.thr_lo = cutoff_threshold(cutoff);
    a.thr_hi = cutoff_threshold_hi(cutoff);
    a.apc = (double)c->A * pc;
    a.den = (double)(c->n_global - 1) + a.apc;  // normalizePPM (sources.Length - 1), .fs:964
    a.pcv_fixed = c->use_pcv ? c->d_pcv_fixed : nullptr;
    a.err = c->d_merr;
    a.fallbacks = c->d_fallbacks;
    a.kmax = std::max(1, c->Lmax - W + 1);
    int64_t o = 0;
    auto take = [&](int64_t b) {
        int64_t q = o;
        o = align16(o + b);
        return (int32_t)q;
    };
    a.o_tab = take(8 * (int64_t)c->E * W);
    a.o_pcv = take(8 * 64);
    a.o_seq = take(align16(c->Lmax) + 16);
    a.o_agg = greedy ? take(8 * (int64_t)(c->A * W + c->A)) : 0;
    a.o_S = -1;
    // window scores in LDS when they fit (read once per child product)
    if (o + 16 * (int64_t)a.kmax + 1024 <= c->max_lds) a.o_S = take(16 * (int64_t)a.kmax);
    return o;
}

// Scratch: `slots` arenas of `arena_cap` categories each (+ the S, G windows).
int multi_scratch(gs_ctx *c, MultiArgs &a, int64_t slots, int64_t arena_cap) {
    a.arena_cap = (int32_t)arena_cap;
    a.slot_doubles = 2 * (int64_t)a.kmax + 3 * arena_cap;
    const int64_t need = slots * a.slot_doubles * 8;
    if (need > c->mscratch_bytes) {
        dfree(c->d_mscratch);
        c->mscratch_bytes = 0;
        HIP_TRY(c, hipMalloc(&c->d_mscratch, (size_t)need));
        c->mscratch_bytes = need;
    }
    a.scratch = c->d_mscratch;
    return GS_OK;
}

constexpr int64_t kArenaBudget = 4ll << 30;     // bytes of category arenas per launch
constexpr int64_t kArenaMax = 1ll << 28;        // categories per target

int multi_status(gs_ctx *c, unsigned long long *status_out = nullptr) {
    unsigned long long e = ~0ull;
    HIP_TRY(c, hipMemcpy(&e, c->d_merr, 8, hipMemcpyDeviceToHost));
    if (status_out) *status_out = e;
    if (e == ~0ull) return GS_OK;
    const int st = (int)(e & 15ull);
    const int64_t idx = (int64_t)(e >> 4);
    if (st == kMultiErrArena) return GS_OK;  // handled by the caller
    const char *m = st == 2   ? "roulette wheel ran past the last category (.fs:752)"
                    : st == 3 ? "background count sum overflows int32 (.fs:117)"
                              : "device error";
    return fail(c, st == 2 ? GS_E_ROULETTE_OVERRUN : st == 3 ? GS_E_OVERFLOW : GS_E_HIP, m, idx);
}

// Upload a list snapshot and build its aggregates (all-reduced over the ranks).
int multi_upload(gs_ctx *c, MultiBufs &b, MultiArgs &a, int32_t cap, const int32_t *cnt,
                 const int32_t *pos) {
    const int64_t n = std::max<int32_t>(1, c->n_local);
    const int cells = c->A * a.W + c->A;
    HIP_TRY(c, hipMalloc(&b.cnt, n * 4));
    HIP_TRY(c, hipMalloc(&b.pos, n * cap * 4));
    HIP_TRY(c, hipMalloc(&b.agg, (size_t)cells * 8));
    if (!c->d_merr) HIP_TRY(c, hipMalloc(&c->d_merr, 8));
    HIP_TRY(c, hipMemsetAsync(c->d_merr, 0xff, 8, c->stream));
    HIP_TRY(c, hipMemsetAsync(b.agg, 0, (size_t)cells * 8, c->stream));
    if (c->n_local > 0) {
        HIP_TRY(c, hipMemcpyAsync(b.cnt, cnt, (size_t)c->n_local * 4, hipMemcpyHostToDevice,
                                  c->stream));
        HIP_TRY(c, hipMemcpyAsync(b.pos, pos, (size_t)c->n_local * cap * 4, hipMemcpyHostToDevice,
                                  c->stream));
    }
    a.cnt_in = b.cnt;
    a.pos_in = b.pos;
    HIP_TRY(c, gs_multi_agg_launch(a, b.agg, c->n_cu, c->stream));
    if (c->comm)
        RCCL_TRY(c, ncclAllReduce(b.agg, b.agg, (size_t)cells, ncclInt64, ncclSum, c->comm,
                                  c->stream));
    a.agg = b.agg;
    return GS_OK;
}

// One sweep of the list path from (cnt_in, pos_in) on the device; results in
// b.cnt2 / b.pos2 / b.pwms.  Targets whose categories overflow their arena are
// scored again with a larger arena.
int multi_sweep_dev(gs_ctx *c, MultiBufs &b, MultiArgs &a, int64_t lds) {
    const int64_t n = std::max<int32_t>(1, c->n_local);
    HIP_TRY(c, hipMalloc(&b.cnt2, n * 4));
    HIP_TRY(c, hipMalloc(&b.pos2, n * a.cap_out * 4));
    HIP_TRY(c, hipMalloc(&b.pwms, n * 8));
    HIP_TRY(c, hipMalloc(&b.ovf, (n + 1) * 4));
    HIP_TRY(c, hipMalloc(&b.targets, n * 4));
    HIP_TRY(c, hipMemsetAsync(b.pos2, 0xff, (size_t)n * a.cap_out * 4, c->stream));
    a.cnt_out = b.cnt2;
    a.pos_out = b.pos2;
    a.pwms_out = b.pwms;
    a.ovf_list = b.ovf + 1;
    a.ovf_count = b.ovf;
    a.targets = nullptr;
    a.n_targets = c->n_local;
    int64_t arena = std::max<int64_t>(2048, 4 * (int64_t)a.kmax);
    while (a.n_targets > 0) {
        const int64_t slot_bytes = (2 * (int64_t)a.kmax + 3 * arena) * 8;
        int64_t grid = std::min<int64_t>(a.n_targets, (int64_t)c->n_cu * 8);
        grid = std::max<int64_t>(1, std::min<int64_t>(grid, kArenaBudget / slot_bytes));
        int rc;
        if ((rc = multi_scratch(c, a, grid, arena))) return rc;
        HIP_TRY(c, hipMemsetAsync(b.ovf, 0, 4, c->stream));
        HIP_TRY(c, gs_multi_sweep_launch(a, (int)grid, (size_t)lds, c->stream));
        int32_t novf = 0;
        HIP_TRY(c, hipMemcpyAsync(&novf, b.ovf, 4, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(c, hipStreamSynchronize(c->stream));
        if (novf == 0) break;
        if (arena * 16 > kArenaMax)
            return fail(c, GS_E_UNSUPPORTED,
                        "a sequence has more than 2^28 motif combinations (calculatePWMsFor"
                        "SegmentCombinations, .fs:727-742)");
        arena *= 16;
        HIP_TRY(c, hipMemcpyAsync(b.targets, b.ovf + 1, (size_t)novf * 4, hipMemcpyDeviceToDevice,
                                  c->stream));
        a.targets = b.targets;
        a.n_targets = novf;
    }
    return multi_status(c);
}

int multi_download(gs_ctx *c, const MultiBufs &b, int32_t cap, const int32_t *dcnt,
                   const int32_t *dpos, const double *dpw, int32_t *cnt, int32_t *pos,
                   double *pwms) {
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    (void)b;
    if (c->n_local == 0) return GS_OK;
    HIP_TRY(c, hipMemcpy(cnt, dcnt, (size_t)c->n_local * 4, hipMemcpyDeviceToHost));
    HIP_TRY(c, hipMemcpy(pos, dpos, (size_t)c->n_local * cap * 4, hipMemcpyDeviceToHost));
    HIP_TRY(c, hipMemcpy(pwms, dpw, (size_t)c->n_local * 8, hipMemcpyDeviceToHost));
    return GS_OK;
}

// Greedy passes on the device lists (cnt, pos, pwms: in/out) with the live
// aggregates in agg (those of the lists): speculative steps (gs_multi.hip), enqueued
// kSpecBatch at a time between host checks of the control block.  A pass whose
// categories overflow an arena restarts from the uploaded lists with a larger one.

int multi_greedy_dev(gs_ctx *c, MultiArgs &a, int64_t lds, int32_t cap, int32_t max_passes,
                     int32_t *dcnt, int32_t *dpos, double *dpw, int64_t *agg,
                     const int32_t *cnt0, const int32_t *pos0, const double *pw0,
                     int32_t *passes_out, int32_t base0 = 0, int32_t changed0 = 0) {
    a.cnt_out = dcnt;
    a.pos_out = dpos;
    a.pwms_out = dpw;
    a.max_passes = max_passes;
    a.agg_rw = agg;
    a.spec_slots = (int32_t)std::max<int64_t>(1, std::min<int64_t>(c->n_local, c->multi_spec_slots));
    SpecCtl *ctl = nullptr;
    SpecRes *res = nullptr;
    HIP_TRY(c, hipMalloc(&ctl, sizeof(SpecCtl)));
    if (hipMalloc(&res, sizeof(SpecRes) * (size_t)a.spec_slots) != hipSuccess) {
        dfree(ctl);
        return fail(c, GS_E_HIP, "hipMalloc(speculation results)");
    }
    a.spec_ctl = ctl;
    a.spec_res = res;
    int64_t arena = std::max<int64_t>(4096, 8 * (int64_t)a.kmax);
    const int64_t step_limit = ((int64_t)c->n_local + 1) * max_passes + kSpecBatch;
    int rc = GS_OK;
    for (;;) {
        if ((rc = multi_scratch(c, a, a.spec_slots, arena))) break;
        SpecCtl h{};
        h.base = base0;  // 0, or where the star engine left the pass (greedy_hybrid)
        h.changed = changed0;
        int64_t steps = 0;
        hipError_t e = hipStreamSynchronize(c->stream);
        if (e == hipSuccess) e = hipMemcpy(ctl, &h, sizeof(SpecCtl), hipMemcpyHostToDevice);
        while (e == hipSuccess && c->n_local > 0) {
            e = gs_multi_spec_launch(a, c->multi_greedy_threads, (size_t)lds, kSpecBatch, c->stream);
            if (e == hipSuccess) e = hipMemcpyAsync(&h, ctl, sizeof(h), hipMemcpyDeviceToHost, c->stream);
            if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
            steps += kSpecBatch;
            if (h.done || steps > step_limit) break;
        }
        if (e != hipSuccess) {
            rc = fail(c, GS_E_HIP, std::string("list-path greedy: ") + hipGetErrorString(e));
            break;
        }
        if (c->n_local > 0 && !h.done) {
            rc = fail(c, GS_E_HIP, "list-path greedy made no progress");
            break;
        }
        unsigned long long st = ~0ull;
        if ((rc = multi_status(c, &st))) break;
        if (st == ~0ull) {
            if (passes_out) *passes_out = h.pass;
            break;
        }
        // arena overflow: restart from the caller's lists with a larger arena
        if (arena * 16 > kArenaMax) {
            rc = fail(c, GS_E_UNSUPPORTED,
                      "a sequence has more than 2^28 motif combinations (.fs:727-742)");
            break;
        }
        arena *= 16;
        const int cells = c->A * a.W + c->A;
        e = hipMemcpy(dcnt, cnt0, (size_t)c->n_local * 4, hipMemcpyHostToDevice);
        if (e == hipSuccess)
            e = hipMemcpy(dpos, pos0, (size_t)c->n_local * cap * 4, hipMemcpyHostToDevice);
        if (e == hipSuccess) e = hipMemcpy(dpw, pw0, (size_t)c->n_local * 8, hipMemcpyHostToDevice);
        if (e == hipSuccess) e = hipMemset(agg, 0, (size_t)cells * 8);
        a.cnt_in = dcnt;
        a.pos_in = dpos;
        if (e == hipSuccess) e = gs_multi_agg_launch(a, agg, c->n_cu, c->stream);
        if (e == hipSuccess) e = hipMemsetAsync(c->d_merr, 0xff, 8, c->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
        if (e != hipSuccess) {
            rc = fail(c, GS_E_HIP, std::string("greedy restart: ") + hipGetErrorString(e));
            break;
        }
    }
    dfree(ctl);
    dfree(res);
    return rc;
}

int multi_lds_check(gs_ctx *c, int64_t lds) {
    if (lds > c->max_lds)
        return fail(c, GS_E_UNSUPPORTED,
                    "longest sequence exceeds the list path's LDS budget (" + std::to_string(lds) +
                        " > " + std::to_string(c->max_lds) + " B)");
    return GS_OK;
}

}  // namespace

// findBestMotifIndicesWithStartPositions (.fs:885-929) on the resident snapshot: the
// star engine (gs_greedy.hip), one pass per launch while passes move many targets;
// once a pass moves fewer than N / greedy_switch, the remaining passes run on the
// speculative list path (motifAmount = 1), whose steps commit up to 256 visits when
// moves are rare (cfg2: passes 4-6 take 3 ms there against 19 ms in the star engine).
// Every pass is the reference's either way; the snapshot (positions, PWMS, aggregates)
// is left in the star layout.
int greedy_hybrid(gs_ctx *c, double pc, double cutoff, int32_t max_passes, int32_t *passes_out,
                  double *kernel_ms_out) {
    const int32_t n = c->n_local;
    int rc;
    int32_t *d_prev = nullptr, *d_cnt = nullptr, *d_lst = nullptr, *d_moves = nullptr;
    int64_t *d_lagg = nullptr;
    auto cleanup = [&]() {
        dfree(d_prev);
        dfree(d_cnt);
        dfree(d_lst);
        dfree(d_moves);
        dfree(d_lagg);
    };
    const int64_t nn = std::max<int32_t>(1, n);
    if (hipMalloc(&d_prev, nn * 4) != hipSuccess || hipMalloc(&d_moves, 4) != hipSuccess) {
        cleanup();
        return fail(c, GS_E_HIP, "hipMalloc(greedy hand-over)");
    }
    hipEvent_t e0 = get_event(c), e1 = get_event(c);
    HIP_TRY(c, hipEventRecord(e0, c->stream));
    int32_t passes = 0, spec_base = 0, spec_changed = 0;
    bool spec = false;
    while (passes < max_passes && n > 0) {
        int32_t *pos = c->d_pos[c->cur_pos];
        hipError_t e = hipMemcpyAsync(d_prev, pos, (size_t)n * 4, hipMemcpyDeviceToDevice, c->stream);
        if (e != hipSuccess) {
            cleanup();
            return fail(c, GS_E_HIP, "greedy hand-over copy");
        }
        int32_t p1 = 0;
        int32_t ex[2] = {0, 0};  // mid-pass exit, as in site_greedy
        if ((rc = greedy_run(c, 0, pc, cutoff, 1, &p1, nullptr, c->greedy_exit_chunk,
                             c->greedy_exit_ratio, c->greedy_exit_chunk > 0 ? ex : nullptr))) {
            cleanup();
            return rc;
        }
        if (ex[0] > 0) {
            spec_base = ex[0];
            spec_changed = ex[1];
            spec = true;
            break;
        }
        ++passes;
        int32_t moves = 0;
        e = hipMemsetAsync(d_moves, 0, 4, c->stream);
        if (e == hipSuccess) e = gs_count_diff_launch(d_prev, pos, n, d_moves, c->stream);
        if (e == hipSuccess) e = hipMemcpyAsync(&moves, d_moves, 4, hipMemcpyDeviceToHost, c->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
        if (e != hipSuccess) {
            cleanup();
            return fail(c, GS_E_HIP, "greedy move count");
        }
        if (moves == 0) break;  // the pass left every position: converged (.fs:888)
        if ((int64_t)moves * c->greedy_switch < n && passes < max_passes) {
            spec = true;
            break;
        }
    }
    if (spec) {
        // the star snapshot as Positions lists (motifAmount = 1, capacity 1)
        MultiArgs a{};
        const int64_t lds = multi_args(c, a, 1, c->W, 1, pc, cutoff, true);
        const int cells = c->A * c->W + c->A;
        hipError_t e = lds > c->max_lds ? hipErrorInvalidValue : hipSuccess;
        if (e == hipSuccess) e = hipMalloc(&d_cnt, nn * 4);
        if (e == hipSuccess) e = hipMalloc(&d_lst, nn * 4);
        if (e == hipSuccess) e = hipMalloc(&d_lagg, (size_t)cells * 8);
        if (e == hipSuccess) {
            if (!c->d_merr) e = hipMalloc(&c->d_merr, 8);
        }
        if (e == hipSuccess) e = hipMemsetAsync(c->d_merr, 0xff, 8, c->stream);
        if (e == hipSuccess)
            e = gs_single_lists_launch(c->d_pos[c->cur_pos], n, d_cnt, d_lst, 1, c->stream);
        if (e == hipSuccess) e = hipMemsetAsync(d_lagg, 0, (size_t)cells * 8, c->stream);
        a.cnt_in = d_cnt;
        a.pos_in = d_lst;
        if (e == hipSuccess) e = gs_multi_agg_launch(a, d_lagg, c->n_cu, c->stream);
        std::vector<int32_t> hc((size_t)n), hp((size_t)n);
        std::vector<double> hw((size_t)n);
        if (e == hipSuccess) e = hipMemcpyAsync(hc.data(), d_cnt, (size_t)n * 4, hipMemcpyDeviceToHost, c->stream);
        if (e == hipSuccess) e = hipMemcpyAsync(hp.data(), d_lst, (size_t)n * 4, hipMemcpyDeviceToHost, c->stream);
        if (e == hipSuccess) e = hipMemcpyAsync(hw.data(), c->d_pwms, (size_t)n * 8, hipMemcpyDeviceToHost, c->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
        if (e != hipSuccess) {
            cleanup();
            return fail(c, GS_E_HIP, "greedy hand-over to the list path");
        }
        int32_t more = 0;
        if ((rc = multi_greedy_dev(c, a, lds, 1, max_passes - passes, d_cnt, d_lst, c->d_pwms,
                                   d_lagg, hc.data(), hp.data(), hw.data(), &more, spec_base,
                                   spec_changed))) {
            cleanup();
            return rc;
        }
        passes += more;
        // back to the star layout: positions, then the snapshot's aggregates
        e = gs_single_lists_launch(c->d_pos[c->cur_pos], n, d_cnt, d_lst, 0, c->stream);
        for (auto &b : c->d_agg)
            if (e == hipSuccess) e = hipMemsetAsync(b, 0, (size_t)kRepl * c->stride * 8, c->stream);
        if (e != hipSuccess) {
            cleanup();
            return fail(c, GS_E_HIP, "greedy hand-back");
        }
        if ((rc = launch_sweep(c, 1, 0.0, 0.0, nullptr, 0, 0, -1, 0, -1))) {
            cleanup();
            return rc;
        }
        c->cur_agg = 0;
        c->rep_valid = true;
        c->vec_valid = false;
    }
    HIP_TRY(c, hipEventRecord(e1, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    float ms = 0.0f;
    HIP_TRY(c, hipEventElapsedTime(&ms, e0, e1));
    c->ev_pool.push_back(e0);
    c->ev_pool.push_back(e1);
    cleanup();
    if ((rc = check_device_error(c))) return rc;
    if (passes_out) *passes_out = passes;
    if (kernel_ms_out) *kernel_ms_out = (double)ms;
    return GS_OK;
}

namespace {

}  // namespace

extern "C" {

int gs_motif_sweep_multi(gs_ctx *c, int32_t motif_amount, int32_t W, double pc, double cutoff,
                         int32_t cap, const int32_t *cnt_in, const int32_t *pos_in,
                         const double *u, int32_t *cnt_out, int32_t *pos_out, double *pwms_out) {
    if (!c || (c->n_local > 0 && (!cnt_in || !pos_in || !u || !cnt_out || !pos_out || !pwms_out)))
        return GS_E_ARG;
    int rc;
    if ((rc = check_dev(c))) return rc;
    if ((rc = validate_lists(c, motif_amount, W, cap, cnt_in, pos_in))) return rc;
    MultiArgs a{};
    const int64_t lds = multi_args(c, a, motif_amount, W, cap, pc, cutoff, false);
    if ((rc = multi_lds_check(c, lds))) return rc;
    MultiBufs b;
    if ((rc = multi_upload(c, b, a, cap, cnt_in, pos_in))) return rc;
    HIP_TRY(c, hipMalloc(&b.u, (size_t)std::max<int32_t>(1, c->n_local) * 8));
    if (c->n_local > 0)
        HIP_TRY(c, hipMemcpyAsync(b.u, u, (size_t)c->n_local * 8, hipMemcpyHostToDevice, c->stream));
    a.u = b.u;
    if ((rc = multi_sweep_dev(c, b, a, lds))) return rc;
    return multi_download(c, b, cap, b.cnt2, b.pos2, b.pwms, cnt_out, pos_out, pwms_out);
}

int gs_motif_greedy_multi(gs_ctx *c, int32_t motif_amount, int32_t W, double pc, double cutoff,
                          int32_t max_passes, int32_t cap, int32_t *cnt_inout, int32_t *pos_inout,
                          double *pwms_inout, int32_t *passes_out) {
    if (!c || max_passes < 1 || (c->n_local > 0 && (!cnt_inout || !pos_inout || !pwms_inout)))
        return GS_E_ARG;
    int rc;
    if ((rc = check_dev(c))) return rc;
    if ((int64_t)c->n_local != c->n_global)
        return fail(c, GS_E_UNSUPPORTED,
                    "the greedy refinement walks every target in order (.fs:885-929): it needs "
                    "all sequences on one device");
    if ((rc = validate_lists(c, motif_amount, W, cap, cnt_inout, pos_inout))) return rc;
    MultiArgs a{};
    const int64_t lds = multi_args(c, a, motif_amount, W, cap, pc, cutoff, true);
    if ((rc = multi_lds_check(c, lds))) return rc;
    MultiBufs b;
    if ((rc = multi_upload(c, b, a, cap, cnt_inout, pos_inout))) return rc;
    HIP_TRY(c, hipMalloc(&b.pwms, (size_t)std::max<int32_t>(1, c->n_local) * 8));
    if (c->n_local > 0)
        HIP_TRY(c, hipMemcpyAsync(b.pwms, pwms_inout, (size_t)c->n_local * 8, hipMemcpyHostToDevice,
                                  c->stream));
    if ((rc = multi_greedy_dev(c, a, lds, cap, max_passes, b.cnt, b.pos, b.pwms, b.agg, cnt_inout,
                               pos_inout, pwms_inout, passes_out)))
        return rc;
    return multi_download(c, b, cap, b.cnt, b.pos, b.pwms, cnt_inout, pos_inout, pwms_inout);
}

int gs_motif_sampling_multi(gs_ctx *c, int32_t motif_amount, int32_t W, double pc, double cutoff,
                            uint64_t seed, int32_t init_mode, int32_t max_passes, int32_t cap,
                            int32_t *cnt_out, int32_t *pos_out, double *pwms_out,
                            int32_t *passes_out) {
    if (!c || max_passes < 1 || (c->n_local > 0 && (!cnt_out || !pos_out || !pwms_out)))
        return GS_E_ARG;
    int rc;
    if ((rc = check_dev(c))) return rc;
    if (motif_amount < 1 || motif_amount > kMultiMaxAmount || cap < motif_amount ||
        cap > kMultiMaxAmount)
        return fail(c, GS_E_ARG, "motifAmount / list capacity out of range");
    if ((int64_t)c->n_local != c->n_global)
        return fail(c, GS_E_UNSUPPORTED, "doMotifSampling's greedy tail needs all sequences on one device");
    // getPWMOfRandomStarts |> createMotifIndex prob [position] (.fs:1035-1036)
    std::vector<int32_t> start((size_t)c->n_local);
    std::vector<double> score((size_t)c->n_local);
    if ((rc = gs_random_starts(c, W, pc, seed, init_mode, score.data(), start.data()))) return rc;
    std::vector<int32_t> cnt0((size_t)c->n_local, 1), pos0((size_t)c->n_local * cap, -1);
    for (int32_t n = 0; n < c->n_local; ++n) pos0[(size_t)n * cap] = start[n];
    MultiArgs a{};
    const int64_t lds = multi_args(c, a, motif_amount, W, cap, pc, cutoff, true);
    if ((rc = multi_lds_check(c, lds))) return rc;
    MultiBufs b;
    if ((rc = multi_upload(c, b, a, cap, cnt0.data(), pos0.data()))) return rc;
    // |> findBestMotifIndicesByWithStartPositions (.fs:1037): uniforms of sweep 0 of `seed`
    a.u = nullptr;
    a.seed = seed;
    a.stream = stream_sweep(0);
    if ((rc = multi_sweep_dev(c, b, a, lds))) return rc;
    // |> findBestMotifIndicesWithStartPositions (.fs:1038), from the sweep's lists
    std::vector<int32_t> cnt1((size_t)c->n_local), pos1((size_t)c->n_local * cap);
    std::vector<double> pw1((size_t)c->n_local);
    if ((rc = multi_download(c, b, cap, b.cnt2, b.pos2, b.pwms, cnt1.data(), pos1.data(),
                             pw1.data())))
        return rc;
    MultiArgs g{};
    (void)multi_args(c, g, motif_amount, W, cap, pc, cutoff, true);
    MultiBufs gb;
    if ((rc = multi_upload(c, gb, g, cap, cnt1.data(), pos1.data()))) return rc;
    HIP_TRY(c, hipMalloc(&gb.pwms, (size_t)std::max<int32_t>(1, c->n_local) * 8));
    if (c->n_local > 0)
        HIP_TRY(c, hipMemcpyAsync(gb.pwms, pw1.data(), (size_t)c->n_local * 8,
                                  hipMemcpyHostToDevice, c->stream));
    if ((rc = multi_greedy_dev(c, g, lds, cap, max_passes, gb.cnt, gb.pos, gb.pwms, gb.agg,
                               cnt1.data(), pos1.data(), pw1.data(), passes_out)))
        return rc;
    return multi_download(c, gb, cap, gb.cnt, gb.pos, gb.pwms, cnt_out, pos_out, pwms_out);
}

}  // extern "C"
