// gs_engine.cpp — the engine behind the C ABI: device state and buffer rotations,
// the choice of sweep kernel (general / DNA) and its launch geometry, RCCL
// all-reduces, hipGraph capture of sweep chains, the greedy / site / list-path
// drivers.  gs_api.cpp validates arguments and calls in here.
#include "gs_ctx.h"

namespace gs_host {





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
    dfree(c->d_gen_done);
    dfree(c->d_ftab);
    c->ftab_agg = -1;
    dfree(c->d_ckp);
    c->ckp_elems = 0;
    dfree(c->d_dt);
    c->dt_elems = 0;
    c->vec_valid = c->rep_valid = false;
    c->have_state = false;
    c->bg_absorbed = c->bg_zeroed = c->snap_all_none = false;
    c->note_pending = false;
    c->W = 0;
}


// Dynamic LDS of the sweep kernel: workgroup-shared aggregates + PPM tables,
// then one slice per wavefront (4 per workgroup), each holding the wavefront's
// aggregates, the shared binary64 table of rescans and the batch results, then
// one slice per lane group (64/gl per wavefront).  Returns total bytes.
int64_t sweep_carve(SweepArgs &a, int A, int E, int W, int Lmax, int gl, int waves, bool ek4) {
    const int WM = gs_sweep_wm(W);
    a.gl = gl;
    a.waves = waves;
    a.ek = ek4 ? 4 : 0;
    if (ek4) {  // gs_sweep_kernel<WM, 2, gl, 4>: its own compile-time layout
        const Ek4Layout l = ek4_layout(WM, gl);
        a.o_cg = l.o_cg, a.o_T = l.o_T, a.o_ppmG = l.o_ppmG, a.o_ppmM = l.o_ppmM;
        a.o_lppmG = l.o_lppmG, a.o_bmax = l.o_bmax, a.o_lT = l.o_lT, a.o_wave = l.o_wave;
        a.w_aggC = l.w_aggC, a.w_aggT = l.w_aggT, a.w_tab = l.w_tab, a.w_res = l.w_res;
        a.w_misc = l.w_misc, a.w_group = l.w_group;
        a.g_lt = l.g_lt, a.g_gt = l.g_gt, a.g_pcv = l.g_pcv, a.g_lpcv = a.g_cnt = l.g_lpcv;
        a.g_cmax = a.g_wfac = l.g_cmax, a.g_seq = l.g_seq;
        // group stride = 128 mod 256: each 32-lane half's two groups read their pair
        // tables from opposite bank halves (gs_sweep.hip pair_entry)
        // the sequence and its codes x 8 (the scan's copy), each with the odd group's 64 B
        const int64_t gb = l.g_seq + 2 * (align16((int64_t)Lmax + WM + 96) + 64);
        a.group_bytes = (int32_t)((gb + 127) / 256 * 256 + 128);
        a.wave_bytes = (int32_t)(l.w_group + (64 / gl) * (int64_t)a.group_bytes);
        return l.o_wave + waves * (int64_t)a.wave_bytes;
    }
    int64_t o = 0;
    auto take = [&](int64_t b) {
        int64_t r = o;
        o = align16(o + b);
        return (int32_t)r;
    };
    a.o_cg = take(4 * (int64_t)A * W);
    a.o_T = take(8 * (int64_t)(A + 1));  // T[a] and their sum
    a.o_ppmG = take(8 * (int64_t)A * W);
    a.o_ppmM = take(8 * (int64_t)A * W);
    // binary64 log2 PPM and log2 PPM' (count-minus-one cells), or for more than 16
    // symbols the same in binary32 and their largest finite magnitude
    a.o_lppmG = take((scan_group(E) == 2 ? 16 : 8) * (int64_t)A * W);
    a.o_bmax = take(4 * 16);  // one slot per wavefront
    a.o_lT = take(8 * (4 * (int64_t)(W + 1) + 1));  // the four-symbol path's PCV log table
    a.o_wave = (int32_t)o;
    const int64_t base = o;
    o = 0;
    a.w_aggC = take(4 * (int64_t)A * W);
    a.w_aggT = take(8 * (int64_t)A);
    a.w_misc = take(32);
    const int64_t tab_bytes = 16 * (int64_t)tab_stride(WM) * E;
    if (scan_group(E) == 2) {
        a.w_res = take(16 * 64);
        // the groups' log tables side by side; the rescans' exact table in them when they
        // are as large (two groups or more: lt_stride = tab_stride, 8- vs 16-byte entries)
        a.lt_bytes = (int32_t)align16(8 * (int64_t)lt_stride(WM) * E);
        a.w_lt = take((64 / gl) * (int64_t)a.lt_bytes);
        a.w_tab = (64 / gl) * (int64_t)a.lt_bytes >= tab_bytes ? a.w_lt : take(tab_bytes);
        a.w_pfx = a.pfx_bytes = 0;
    } else {
        // H = 1: per group its motif table (binary32 log2 PPM', code-major, E rows of
        // mt_stride(WM) entries), then its prefix sums of the positions' log2 PCV (int32,
        // Lmax + 1 entries: a lane's reads past its group's last window land in the next
        // group's area or past the allocation, and are not used); the group stride is
        // 128 mod 256 B, so two groups' table rows sit in disjoint bank sets.  The
        // rescans' exact table over the groups' area (as large as it, at least); no
        // batch results on this path (stored as each pick is made)
        const int ng = 64 / gl;
        const int64_t mt = align16(4 * (int64_t)mt_stride(WM) * E);
        int64_t gs = mt + align16(4 * ((int64_t)Lmax + 1));
        if (ng > 1) gs = (gs + 127) / 256 * 256 + 128;
        a.lt_bytes = a.pfx_bytes = (int32_t)gs;  // (the group stride of both)
        const int64_t region = std::max<int64_t>(ng * gs, tab_bytes);
        a.w_lt = take(region);
        a.w_pfx = a.w_lt + (int32_t)mt;
        a.w_res = a.w_lt;  // (unused)
        a.w_tab = a.w_lt;
    }
    a.w_group = (int32_t)o;
    const int64_t wave_fixed = o;
    o = 0;
    a.g_lt = 0;  // (unused: w_lt)
    a.g_gt = scan_group(E) == 2 ? take(8 * (int64_t)gt_stride(WM) * E * E) : 0;
    a.g_seq = take((int64_t)Lmax + WM + 96);  // + the 16-byte zero tail
    a.g_pcv = take(8 * (int64_t)gl);
    // the own-segment counts are read before the binary64 log2 PCV is written
    a.g_lpcv = a.g_cnt = take(8 * (int64_t)gl);
    // the picked window's factors; before them, during the table build, the column
    // maxima and the own segment's log2 PPM' per column
    a.g_wfac = a.g_cmax = take(16 * (int64_t)WM);
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
    HIP_TRY(c, hipMalloc(&c->d_gen_done, kDoneBytes));
    HIP_TRY(c, hipMemset(c->d_gen_done, 0, kDoneBytes));
    HIP_TRY(c, hipMalloc(&c->d_ftab, 3 * (size_t)kFtabBytes));
    if (c->dna_ok) {
        for (auto &b : c->d_aggv) HIP_TRY(c, hipMalloc(&b, (size_t)std::max(1, c->cells) * 8));
        HIP_TRY(c, hipMalloc(&c->d_rep, (size_t)kRepl * c->stride * 8));
        HIP_TRY(c, hipMalloc(&c->d_dna_done, kDoneBytes));  // gs_common.h kDoneBytes
        HIP_TRY(c, hipMemset(c->d_rep, 0, (size_t)kRepl * c->stride * 8));
        HIP_TRY(c, hipMemset(c->d_dna_done, 0, kDoneBytes));
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
    // replica 0 only: the sweep kernel's last workgroup folded the others into it
    RCCL_TRY(c, ncclAllReduce(c->d_agg[idx], c->d_agg[idx], (size_t)c->cells, ncclInt64, ncclSum, c->comm,
                              c->stream));
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
    if (c->tune.group_lanes > 0 && c->E + 1 <= c->tune.group_lanes &&
        !(scan_group(c->E) == 1 && c->tune.group_lanes < 32))
        gl = c->tune.group_lanes;
    int waves = sweep_waves(scan_group(c->E));
    // the tuning's ceiling is the alphabet's default: 4 wavefronts a workgroup for the
    // pair tables (E <= 16), 12 for H = 1; a larger value is an error, not the default
    if (c->tune.sweep_waves > waves)
        return fail(c, GS_E_ARG,
                    "sweep_waves " + std::to_string(c->tune.sweep_waves) + " exceeds " +
                        std::to_string(waves) + " for this alphabet (gs_set_tuning)");
    if (c->tune.sweep_waves > 0) waves = c->tune.sweep_waves;
    // the four-symbol kernel (gs_sweep.hip gs_sweep_ek: DNA without other symbols, the
    // certified sweep without a caller's PCV, W a multiple of 4 up to 32, 4 wavefronts
    // a workgroup) has a layout of its own; the other cases the general carve
    const bool ek4 = c->A == 4 && c->E == 4 && mode == 0 && c->scan == kScanCertified &&
                     !c->use_pcv && gs_sweep_wm(c->W) == c->W && c->W <= 32;
    int64_t lds_bytes = sweep_carve(a, c->A, c->E, c->W, c->Lmax, gl, waves, ek4 && waves == 4);
    while (waves > 1 && lds_bytes > c->max_lds) {
        waves /= 2;  // (its own statement: the carve's two uses of waves see the halved value)
        lds_bytes = sweep_carve(a, c->A, c->E, c->W, c->Lmax, gl, waves, ek4 && waves == 4);
    }
    if (lds_bytes > c->max_lds)
        return fail(c, GS_E_UNSUPPORTED,
                    "longest sequence needs " + std::to_string(lds_bytes) +
                        " B of LDS per workgroup; this build supports up to " +
                        std::to_string(c->max_lds));
    a.seq = c->d_seq;
    a.pseq = c->d_pseq;
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
    // with a communicator the last workgroup folds the replicas into one vector: the
    // all-reduce then carries A W + A cells, not kRepl times that
    a.done = c->comm ? c->d_gen_done : nullptr;
    a.fold = c->comm ? 1 : 0;
    a.err_code = c->d_err_code;
    a.err_index = c->d_err_index;
    a.fallbacks = c->d_fallbacks;
    a.bg_note = (mode == 0 && !c->bg_absorbed) ? bg_note_ptr(c) : nullptr;
    a.Lmax = c->Lmax;
    a.cmin = c->cmin;
    a.seq_stride = c->seq_stride;
#ifdef GS_STAMPS
    if (!c->d_stamps) {
        HIP_TRY(c, hipMalloc(&c->d_stamps, kStampBytes));
        HIP_TRY(c, hipMemset(c->d_stamps, 0, kStampBytes));
    }
    a.stamps = mode == 0 ? c->d_stamps : nullptr;
#endif
    const int64_t key[6] = {c->W, c->E, gl, waves, lds_bytes, c->A * 2 + (gs_sweep_ek(a) == 4)};
    if (!std::equal(key, key + 6, c->sweep_occ_key)) {
        HIP_TRY(c, gs_sweep_occupancy(&c->sweep_occ, a, waves, (size_t)lds_bytes));
        std::copy(key, key + 6, c->sweep_occ_key);
    }
    int per_cu = std::max(1, std::min(c->sweep_occ, c->tune.blocks_per_cu_cap));
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
    // the four-symbol kernel's workgroup tables (gs_sweep.hip ek4_build_tables): built by
    // every workgroup (ftab_mode 0), or finished -- by a one-workgroup kernel before the
    // sweep (1), or handed over by the previous sweep's last workgroup when that sweep
    // built them from these aggregates (2: one GPU, no all-reduce in between; the sweep
    // then hands over the next ones)
    const bool ek_f = mode == 0 && gs_sweep_ek(a) == 4 && c->tune.ftab_mode > 0;
#ifndef GS_FTAB
    if (ek_f)
        return fail(c, GS_E_UNSUPPORTED, "ftab_mode > 0 needs the -DGS_FTAB build (libgibbs_hip_ftab.so)");
#endif
    const bool ftab_next = ek_f && c->tune.ftab_mode == 2 && !c->comm && !c->capturing;
    if (ek_f) {
        unsigned char *const fin = c->d_ftab + (size_t)agg_in * kFtabBytes;
        if (!(c->ftab_agg == agg_in && c->ftab_pc == pc && ftab_next))
            HIP_TRY(c, gs_sweep_tables_launch(c->W, a.agg_in, c->stride, pc, a.den, a.apc, fin, c->stream));
        a.ftab_in = fin;
        if (ftab_next) {
            a.ftab_out = c->d_ftab + (size_t)agg_out * kFtabBytes;
            a.done = c->d_gen_done;
        }
    }
    c->ftab_agg = -1;
    HIP_TRY(c, gs_sweep_launch(a, grid, (size_t)lds_bytes, c->stream, e0, e1));
    if (ftab_next) {
        c->ftab_agg = agg_out;
        c->ftab_pc = pc;
    }
    c->last_sweep[0] = gs_sweep_ek(a);
    c->last_sweep[1] = gl;
    c->last_sweep[2] = waves;
    c->last_sweep[3] = grid;
    if (timed) c->ev_sweep.emplace_back(e0, e1);
    return GS_OK;
}

bool use_dna(const gs_ctx *c) {
    if (!(c->dna_ok && c->dna_agree && c->W <= kDnaMaxW && !c->use_pcv && c->scan == kScanCertified))
        return false;
    if (c->tune.dna_mode >= 0) return c->tune.dna_mode == 1;
    if (c->tune.live_mode == 1) return true;
    // automatic: the packed-layout kernels once there is a wavefront of whole
    // sequences per CU (measured, init-regime chains: cfg2 10k x 200 general 22.6 us
    // vs live 41 us; cfg3 100k x 500 general 285 us vs live 126 us; cfg4 1M x 200
    // 836 vs 273 us).  The rank's agreement uses n_global so every rank of a sampler
    // picks the same kernel.
    return c->n_global >= (int64_t)64 * c->n_cu;
}

// The all-background sweep (gs_sweep_bg.hip) takes over a chain once its snapshot is
// in the all-background state, which is absorbing (every pick a background: C = 0,
// T = 0 again, the bound only tighter).  Admissible for packed data, the certified
// scan and the hold-one-out background.  The host learns the state from the sweep
// kernels' note (workgroup 0 evaluates gs_bgregime.h on each sweep's snapshot; read
// at the end of a chain call) or, for a snapshot it sets with every position [] and
// no communicator, from the same bound evaluated here (C = 0, T = 0).
bool bg_wanted(const gs_ctx *c) {
    // (A W >= 2 W + 3: the general kernel evaluates the bound in its PPM table's space)
    return c->tune.bg_mode != 0 && c->dna_ok && c->W <= kDnaMaxW && !c->use_pcv &&
           c->scan == kScanCertified && c->n_local > 0 && c->A * c->W >= 2 * c->W + 3;
}

// gs_bgregime.h with C = 0, T = 0 (every position []), on the host.
static bool host_bg_regime(const gs_ctx *c, double pc, double cutoff) {
    const double apc = (double)c->A * pc, den = (double)(c->n_global - 1) + apc;
    const double ub = (double)c->W * std::log2(pc / den);
    const double lo = ((double)std::max(c->cmin, 0) + pc) / ((double)std::max(c->Lmax, c->W) + apc);
    if (!(lo > 0.0)) return false;
    const double b = ub - (double)c->W * std::log2(lo);
    return b < cutoff - 1e-6 && std::fabs(cutoff) < 1000.0;
}

// Is the current snapshot (with these parameters) known to be in the state?
bool bg_ready(gs_ctx *c, double pc, double cutoff) {
    if (!bg_wanted(c)) return false;
    if (c->bg_absorbed && c->bg_pc == pc && c->bg_cutoff == cutoff) return true;
    // (the host knows every position of the sampler only when it holds them all)
    if (c->snap_all_none && !c->comm && c->n_global == c->n_local && host_bg_regime(c, pc, cutoff)) {
        c->bg_absorbed = true;
        c->bg_pc = pc;
        c->bg_cutoff = cutoff;
        (void)bg_warm(c);
        return true;
    }
    return false;
}

// The first dispatch of a kernel loads its code object (~0.6 ms measured for
// gs_sweep_bg_kernel, tools/warm_probe.py): done once per lane count, with an empty
// launch (no targets: nothing read or written), when a chain is taken over, so that
// it does not land inside a timed chain.
static int launch_bg_empty(gs_ctx *c, int G);
int bg_warm(gs_ctx *c) {
    if (!bg_wanted(c)) return GS_OK;
    return launch_bg_empty(c, -1);
}

// After a chain call: queue the read of the last sweep kernel's note (bg_resolve
// adopts the state from it at the next decision point).
int bg_check_note(gs_ctx *c, double pc, double cutoff) {
    if (!c->d_bg_note || c->bg_absorbed) return GS_OK;
    // every rank's targets must be in the state for the chain to stay there: the
    // notes are combined over the ranks.  The combine is a collective, so whether a
    // rank takes part depends on the sampler's parameters only (bg_wanted without
    // its per-rank terms); a rank whose own targets cannot be taken over (none, or
    // not DNA) votes no.  A sharded sampler without a communicator, whose aggregates
    // are exchanged by the caller, is never taken over.
    if (c->comm) {
        // (agreed or sampler-wide terms only: a rank whose own tuning has since turned
        // the takeover off still joins, and votes no through bg_wanted below)
        if (!c->bg_agree || c->W > kDnaMaxW || c->use_pcv || c->scan != kScanCertified ||
            c->A * c->W < 2 * c->W + 3)
            return GS_OK;
        if (!bg_wanted(c)) HIP_TRY(c, hipMemsetAsync(c->d_bg_note, 0, 4, c->stream));
        RCCL_TRY(c, ncclAllReduce(c->d_bg_note, c->d_bg_note, 1, ncclInt32, ncclMin, c->comm, c->stream));
    } else if (!bg_wanted(c) || c->n_global != c->n_local) {
        return GS_OK;
    }
    // the note travels to pinned host memory behind the chain: the chain call itself
    // never waits for the device
    if (!c->h_note) HIP_TRY(c, hipHostMalloc((void **)&c->h_note, 4, hipHostMallocDefault));
    if (!c->note_ev) HIP_TRY(c, hipEventCreateWithFlags(&c->note_ev, hipEventDisableTiming));
    HIP_TRY(c, hipMemcpyAsync(c->h_note, c->d_bg_note, 4, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, hipEventRecord(c->note_ev, c->stream));
    c->note_pending = true;
    c->note_pc = pc;
    c->note_cutoff = cutoff;
    return GS_OK;
}

// Adopt the all-background state if the queued note says the last chain ended in it.
// Called before anything decides which kernel sweeps next (chain calls, sweeps,
// synchronisation), never inside a stream capture.  Every rank of a sampler passes
// the same decision points, and the note was min-combined over the ranks.
int bg_resolve(gs_ctx *c) {
    if (!c->note_pending || c->capturing) return GS_OK;
    c->note_pending = false;
    HIP_TRY(c, hipEventSynchronize(c->note_ev));
    if (*c->h_note == 1 && bg_wanted(c)) {
        c->bg_absorbed = true;
        c->bg_pc = c->note_pc;
        c->bg_cutoff = c->note_cutoff;
        return bg_warm(c);
    }
    return GS_OK;
}

int32_t *bg_note_ptr(gs_ctx *c) { return bg_wanted(c) ? c->d_bg_note : nullptr; }

// Lanes per target of the all-background sweep: one, unless that leaves fewer than
// a wavefront of targets per SIMD (each extra lane repeats the target's fixed work:
// PCV, ratio table, certification).  Measured (profiles/r2/s4/ab_bg_lanes*.jsonl,
// profiles/r2/s6): cfg2 10k x 200 G = 8 / 16 / 32 18.0 / 19.4 / 23.7 us; cfg3 100k
// x 500 G = 1 / 2 38.3 / 39.8, its 50k and 25k shards G = 2 best; cfg4 1M x 200 and
// every shard down to 125k G = 1.
static int bg_lanes(const gs_ctx *c) {
    if (c->tune.bg_G > 0) return c->tune.bg_G;
    for (int g = 1; g < 64; g *= 2)
        if ((c->n_local * (int64_t)g + 63) / 64 >= (int64_t)c->n_cu * 4) return g;
    return 64;
}

int launch_bg(gs_ctx *c, double pc, double cutoff, const double *u_dev, uint64_t seed, uint64_t stream,
              bool device_ctr) {
    BgArgs a{};
    const int G = bg_lanes(c);
    a.pk = c->d_pk;
    a.pkoff = c->d_pkoff;
    a.len = c->d_len;
    a.comp = c->d_comp;
    a.n_local = c->n_local;
    a.A = c->A;
    a.W = c->W;
    a.Lmax = c->Lmax;
    a.cmin = c->cmin;
    a.global_offset = c->global_offset;
    a.nrep = 0;  // C = 0, T = 0: the aggregates are not read
    a.stride = c->stride;
    a.pc = pc;
    a.cutoff = cutoff;
    a.apc = (double)c->A * pc;
    a.den = (double)(c->n_global - 1) + a.apc;
    a.agg_in = nullptr;
    a.pos_in = c->d_pos[c->cur_pos];
    a.pos_out = c->d_pos[1 - c->cur_pos];
    a.pwms_out = c->d_pwms;
    a.u_in = u_dev;
    a.seed = seed;
    a.stream = stream;
    a.sweep_ctr = (!u_dev && device_ctr) ? c->d_sweep_ctr : nullptr;
    // with the device counter the kernel's last workgroup advances it
    a.done = a.sweep_ctr ? c->d_dna_done : nullptr;
    a.err_code = c->d_err_code;
    a.err_index = c->d_err_index;
    a.fallbacks = c->d_fallbacks;
    a.force_replay = c->tune.bg_force_replay;
#ifdef GS_STAMPS
    if (!c->d_stamps) {
        HIP_TRY(c, hipMalloc(&c->d_stamps, kStampBytes));
        HIP_TRY(c, hipMemset(c->d_stamps, 0, kStampBytes));
    }
    a.stamps = c->d_stamps;
#endif
    // occupancy per lane count, queried once (a host API call per sweep costs as much
    // as a short sweep)
    int gi = 0;
    while ((1 << gi) < G) ++gi;
    if (c->bg_occ[gi] <= 0) HIP_TRY(c, gs_bg_occupancy(&c->bg_occ[gi], G));
    const int per_cu = c->bg_occ[gi];
    const int64_t tiles = (c->n_local + 64 / G - 1) / (64 / G);
    const int64_t blocks = (tiles + gs_bg_waves() - 1) / gs_bg_waves();
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(blocks, (int64_t)c->n_cu * std::max(1, per_cu)));
    hipEvent_t e0 = nullptr, e1 = nullptr;
    const bool timed = c->prof && (c->prof_bg_calls++ % c->prof_stride) == 0;
    if (timed) {
        e0 = get_event(c);
        e1 = get_event(c);
    }
    HIP_TRY(c, gs_bg_launch(a, G, grid, c->stream, e0, e1));
    if (timed) c->ev_bg.emplace_back(e0, e1);
    return GS_OK;
}

static int launch_bg_empty(gs_ctx *c, int) {
    const int G = bg_lanes(c);
    int gi = 0;
    while ((1 << gi) < G) ++gi;
    if (c->bg_warmed & (1 << gi)) return GS_OK;
    if (c->bg_occ[gi] <= 0) HIP_TRY(c, gs_bg_occupancy(&c->bg_occ[gi], G));
    BgArgs a{};
    a.n_local = 0;  // no targets
    a.A = c->A;
    a.W = c->W;
    a.err_code = c->d_err_code;
    a.err_index = c->d_err_index;
    a.fallbacks = c->d_fallbacks;
    HIP_TRY(c, gs_bg_launch(a, G, 1, c->stream, nullptr, nullptr));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    c->bg_warmed |= 1 << gi;
    return GS_OK;
}

// Lanes per sequence of the DNA sweep: one while that fills a wavefront per SIMD,
// else 2 or 4 (shorter lanes, more wavefronts).
int dna_lanes(const gs_ctx *c) {
    if (c->tune.dna_G == 1 || c->tune.dna_G == 2 || c->tune.dna_G == 4) return c->tune.dna_G;
    for (int g = 1; g < 4; g *= 2)
        if ((int64_t)(c->n_local + 64 / g - 1) / (64 / g) >= (int64_t)c->n_cu * 4) return g;
    return 4;
}

// DNA-path sweeps by the live-chain kernel (gs_sweep_live.hip): always with
// live_mode 1; automatically while one lane holds a sequence's windows (K <=
// live_max_win), else the round-2 packed kernel (gs_sweep_dna.hip), measured faster on
// long sequences (init-regime chains: cfg4 1M x 200 live 259 vs 380 us; cfg3 100k x 500
// live 123 (G = 4) / 121 (G = 2) vs 111 us).
bool use_live(const gs_ctx *c) {
    if (c->tune.live_mode == 0) return false;
    // a shape whose workgroup does not fit the LDS at any lane count (long sequences:
    // the lanes' masks and words grow with the windows a lane owns) takes the older
    // packed kernel, whose LDS does not depend on the length
    if (live_fit_waves(c, live_lanes(c), kLiveWaves) == 0) return false;
    if (c->tune.live_mode == 1) return true;
    return live_rn_max(c->Lmax, c->W, 1) <= c->tune.live_max_win;
}

// DNA-path sweeps by the long-sequence kernel (gs_sweep_long.hip): one 16-lane row a
// target, exact fixed-point window scores.  Its time hardly depends on the length (the
// per-target work dominates), the packed kernels' grows with it: automatically from
// 320 windows, within its 16 x 32 (measured, init regime, 100k targets: 88 vs 108 us
// at 400 bp W = 15, 82 vs 98 us at 350 bp W = 12, 83 vs 89 us at 300 bp; 200k x 300 bp
// W = 15 154 vs 147 us); long_mode 1 whenever it fits.
bool use_long(const gs_ctx *c) {
    if (c->tune.long_mode == 0 || !gs_long_fits(c->Lmax, c->W)) return false;
    if (c->tune.long_mode == 1) return true;
    return c->Lmax - c->W + 1 >= 320;
}

// Wavefronts per live-kernel workgroup at G lanes a target: `want`, halved while the
// workgroup's LDS exceeds the device's; 0 when not even 2 fit (the prologue's
// tables take 128 threads).  The per-wavefront slice shrinks as G grows, so G = 8 is
// the last lane count to try.
int live_fit_waves(const gs_ctx *c, int G, int want) {
    for (int w = want; w >= 2; w /= 2)
        if ((int64_t)gs_live_lds_bytes(c->Lmax, c->W, G, w) <= (int64_t)c->max_lds) return w;
    return 0;
}

// Lanes per target of the live-chain kernel: the fewest that give at most
// live_max_win windows a lane (the lane's masks, words and block sums in LDS) and
// live_waves_per_simd wavefronts of targets per SIMD (each extra lane repeats the
// target's fixed work), within the LDS a workgroup may take.
int live_lanes(const gs_ctx *c) {
    auto fits = [&](int g) {
        return (int64_t)gs_live_lds_bytes(c->Lmax, c->W, g, kLiveWaves) <= (int64_t)c->max_lds;
    };
    int gmin = 1;
    while (gmin < 8 && (live_rn_max(c->Lmax, c->W, gmin) > c->tune.live_max_win || !fits(gmin))) gmin *= 2;
    if (c->tune.live_G > 0) return std::max(c->tune.live_G, gmin);
    const int64_t want = (int64_t)c->n_cu * 4 * c->tune.live_waves_per_simd;
    for (int g = gmin; g < 8; g *= 2)
        if ((c->n_local * (int64_t)g + 63) / 64 >= want) return g;
    return 8;
}

// The aggregates in the other form, when the current one is the only valid one:
// the vector (DNA sweeps) <-> the replicas (every other kernel).
int need_rep(gs_ctx *c) {
    if (c->rep_valid || !c->vec_valid) return GS_OK;
    c->ftab_agg = -1;
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
    a.bg_note = c->bg_absorbed ? nullptr : bg_note_ptr(c);
    a.Lmax = c->Lmax;
    a.cmin = c->cmin;
    a.live_force = c->tune.live_force;
    a.pk_stride = c->pk_stride;
    // the in-kernel exchange of the aggregate vector (gs_exchange_open): the live and
    // long sweeps' last workgroup sums every rank's partial (no all-reduce after them)
    c->xch_used = c->xranks > 0 && (use_long(c) || use_live(c));
    if (c->xch_used) {
        a.xpeer = c->d_xpeer;
        a.xseq = c->d_xseq;
        a.xranks = c->xranks;
        a.xrank = c->xrank;
    }
#ifdef GS_STAMPS
    if (!c->d_stamps) {
        HIP_TRY(c, hipMalloc(&c->d_stamps, kStampBytes));
        HIP_TRY(c, hipMemset(c->d_stamps, 0, kStampBytes));
    }
    a.stamps = c->d_stamps;
#endif
    if (use_long(c)) {
        const int waves = c->tune.long_waves;
        const int wi = waves == 2 ? 0 : waves == 4 ? 1 : 2;
        const int mi = c->W <= 8 ? 0 : c->W <= 12 ? 1 : 2;
        int &occ = c->long_occ[mi][wi];
        if (occ <= 0) HIP_TRY(c, gs_long_occupancy(&occ, c->W, c->Lmax, waves));
        if (occ <= 0) return fail(c, GS_E_UNSUPPORTED, "the long sweep's workgroup does not fit a CU");
        const int per_cu = std::max(1, std::min(occ, c->tune.blocks_per_cu_cap));
        // four targets a wavefront iteration
        const int64_t iters = (c->n_local + 3) / 4;
        const int64_t blocks = (iters + waves - 1) / waves;
        const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(blocks, (int64_t)c->n_cu * per_cu));
        hipEvent_t e0 = nullptr, e1 = nullptr;
        const bool timed = c->prof && (c->prof_sweep_calls++ % c->prof_stride) == 0;
        if (timed) {
            e0 = get_event(c);
            e1 = get_event(c);
        }
        a.compsum = c->d_compsum;
        HIP_TRY(c, gs_long_launch(a, grid, waves, c->stream, e0, e1));
        if (timed) c->ev_sweep.emplace_back(e0, e1);
        return GS_OK;
    }
    if (use_live(c)) {
        const int GL = live_lanes(c);
        const int oi = (GL == 1 ? 0 : GL == 2 ? 1 : GL == 4 ? 2 : 3) + 4 * (gs_live_wm(c->W) / 4 - 2);
        const int64_t tiles = (c->n_local + 64 / GL - 1) / (64 / GL);
        // wavefronts per workgroup: 8 (they share the workgroup's tables), fewer
        // while 8 would leave CUs without a workgroup (small sweeps)
        int waves = c->tune.live_waves;
        if (waves <= 0) {
            waves = kLiveWaves;
            while (waves > 2 && (tiles + waves - 1) / waves < (int64_t)c->n_cu) waves /= 2;
        }
        waves = live_fit_waves(c, GL, waves);
        if (waves == 0)
            return fail(c, GS_E_UNSUPPORTED, "the live sweep's workgroup does not fit the LDS at Lmax = " +
                                                 std::to_string(c->Lmax));
        const int wi = waves >= 8 ? 0 : waves >= 4 ? 1 : waves >= 2 ? 2 : 3;
        int &occ = c->live_occ[oi][wi];
        if (occ <= 0) HIP_TRY(c, gs_live_occupancy(&occ, c->W, GL, c->Lmax, waves));
        const int per_cu = std::max(1, std::min(occ, c->tune.blocks_per_cu_cap * kLiveWaves / waves));
        const int64_t blocks = (tiles + waves - 1) / waves;
        const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(blocks, (int64_t)c->n_cu * per_cu));
        hipEvent_t e0 = nullptr, e1 = nullptr;
        const bool timed = c->prof && (c->prof_sweep_calls++ % c->prof_stride) == 0;
        if (timed) {
            e0 = get_event(c);
            e1 = get_event(c);
        }
        a.compsum = c->d_compsum;
        HIP_TRY(c, gs_live_launch(a, GL, grid, waves, c->stream, e0, e1));
        if (timed) c->ev_sweep.emplace_back(e0, e1);
        return GS_OK;
    }
    const int gi = G == 1 ? 0 : G == 2 ? 1 : 2;
    if (c->dna_occ_W != c->W) {
        c->dna_occ[0] = c->dna_occ[1] = c->dna_occ[2] = 0;
        c->dna_occ_W = c->W;
    }
    if (c->dna_occ[gi] <= 0) HIP_TRY(c, gs_dna_occupancy(&c->dna_occ[gi], c->W, G));
    const int per_cu = std::max(1, std::min(c->dna_occ[gi], 2));
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
    c->bg_absorbed = c->bg_zeroed = false;
    c->note_pending = false;  // a note of the previous snapshot's chain
    if (!c->d_bg_note) HIP_TRY(c, hipMalloc(&c->d_bg_note, 4));  // (not inside a capture)
    c->snap_all_none = true;
    for (int32_t n = 0; n < c->n_local && c->snap_all_none; ++n) c->snap_all_none = pos[n] < 0;
    if (c->d_bg_note) HIP_TRY(c, hipMemsetAsync(c->d_bg_note, 0, 4, c->stream));
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
        // ... and so must the all-background note's combine (bg_check_note): every
        // rank joins it only if every rank's tuning allows the takeover
        const int32_t mine[2] = {c->dna_ok ? 1 : 0, c->tune.bg_mode != 0 ? 1 : 0};
        HIP_TRY(c, hipMemcpyAsync(d_flag, mine, 8, hipMemcpyHostToDevice, c->stream));
        RCCL_TRY(c, ncclAllReduce(d_flag, d_flag, 2, ncclInt32, ncclMin, c->comm, c->stream));
        int32_t all[2] = {0, 0};
        HIP_TRY(c, hipMemcpyAsync(all, d_flag, 8, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(c, hipStreamSynchronize(c->stream));
        c->dna_agree = all[0] != 0;
        c->bg_agree = all[1] != 0;
    } else {
        c->dna_agree = true;
        c->bg_agree = true;
    }
    HIP_TRY(c, hipMemsetAsync(c->d_gen_done, 0, kDoneBytes, c->stream));
    c->ftab_agg = -1;
    if (c->dna_ok) {
        c->cur_aggv = 0;
        HIP_TRY(c, hipMemsetAsync(c->d_rep, 0, (size_t)kRepl * c->stride * 8, c->stream));
        HIP_TRY(c, hipMemsetAsync(c->d_dna_done, 0, kDoneBytes, c->stream));
        if (use_dna(c) && (rc = need_vec(c))) return rc;
    }
    c->have_state = true;
    return GS_OK;
}

int one_sweep(gs_ctx *c, double pc, double cutoff, const double *u_dev, uint64_t seed,
              uint64_t stream) {
    int rc;
    if ((rc = bg_resolve(c))) return rc;
    if (bg_ready(c, pc, cutoff)) {
        // the all-background state: every aggregate buffer is zero and stays zero on
        // every rank (all ranks adopted it together, bg_check_note), so the sum over
        // the ranks is zero too and the all-reduce is skipped: the ranks sweep
        // independently from here on
        c->ftab_agg = -1;
        if (!c->bg_zeroed) {
            for (auto &b : c->d_agg)
                if (b) HIP_TRY(c, hipMemsetAsync(b, 0, (size_t)kRepl * c->stride * 8, c->stream));
            for (auto &b : c->d_aggv)
                if (b) HIP_TRY(c, hipMemsetAsync(b, 0, (size_t)std::max(1, c->cells) * 8, c->stream));
            c->bg_zeroed = true;
        }
        // inside a captured chain the sweep index comes from the device counter,
        // which the kernel's last workgroup advances; direct launches pass it
        const bool dev = use_dna(c) && !u_dev && c->capturing;
        if ((rc = launch_bg(c, pc, cutoff, u_dev, seed, stream, dev))) return rc;
        if (use_dna(c))
            c->cur_aggv = 1 - c->cur_aggv;
        else
            c->cur_agg = (c->cur_agg + 1) % 3;
        c->rep_valid = true;
        c->vec_valid = true;
        c->cur_pos = 1 - c->cur_pos;
        return GS_OK;
    }
    // a sweep kernel may place motifs: whatever was known of the state (for other
    // pc / cutOff, or of the snapshot as set) no longer holds
    c->bg_absorbed = c->bg_zeroed = c->snap_all_none = false;
    if (use_dna(c)) {
        if ((rc = need_vec(c))) return rc;
        if ((rc = launch_dna(c, pc, cutoff, u_dev, seed))) return rc;
        const int o = 1 - c->cur_aggv;
        if (!c->xch_used && (rc = allreduce_vec(c, o))) return rc;  // (else summed in-kernel)
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


bool graphs_wanted(gs_ctx *c) {
    if (c->graph_broken || c->prof) return false;
    return c->tune.graph_mode == 1 || (c->tune.graph_mode < 0 && c->comm != nullptr);
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
    const bool bgnow = bg_ready(c, pc, cutoff);
    const int aggp = dna ? c->cur_aggv : c->cur_agg;
    for (auto &g : c->graphs)
        if (g.gen == c->graph_gen && g.pos == c->cur_pos && g.agg == aggp && g.dna == dna &&
            g.bg == bgnow && g.seed == seed && g.pc == pc && g.cutoff == cutoff)
            return g.exec;
    const int pos0 = c->cur_pos, agg0 = c->cur_agg, aggv0 = c->cur_aggv;
    const bool vv = c->vec_valid, rv = c->rep_valid;
    hipGraph_t graph = nullptr;
    hipGraphExec_t exec = nullptr;
    bool ok = hipStreamBeginCapture(c->stream, hipStreamCaptureModeRelaxed) == hipSuccess;
    c->capturing = true;
    if (!dna)
        ok = ok && gs_uniforms_launch(c->d_u6, c->n_local, c->global_offset, seed, kGraphSweeps,
                                      c->d_sweep_ctr, c->d_done_ctr, c->n_cu, c->stream) == hipSuccess;
    for (int k = 0; ok && k < kGraphSweeps; ++k)
        ok = one_sweep(c, pc, cutoff, dna ? nullptr : c->d_u6 + (size_t)k * c->n_local, seed, 0) ==
             GS_OK;
    const bool ended = hipStreamEndCapture(c->stream, &graph) == hipSuccess;
    c->capturing = false;
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
    e.bg = bgnow;
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
                const double *d_ppm, StartsArgs *build_only,
                int64_t *lds_out) {
    const int A = c->A, AW = A * W;
    int64_t o = 0;
    auto take = [&](int64_t b) {
        int64_t q = o;
        o = align16(o + b);
        return (int32_t)q;
    };
    StartsArgs a{};
    const int64_t dt_elems = (int64_t)(c->Lmax + 1) * A;
    // the D table goes to HBM when it does not fit the LDS with the rest
    int64_t rest = 0;
    for (int64_t b : {8 * (int64_t)AW, 4 * 2 * (int64_t)AW, 8 * (int64_t)A, 8 * (int64_t)A,
                      4 * (int64_t)kEncSpace, align16(c->Lmax) + 64})
        rest += align16(b);
    const bool gd = rest + align16(4 * dt_elems) > c->max_lds;
    if (rest > c->max_lds)
        return fail(c, GS_E_UNSUPPORTED, "longest sequence exceeds the site scan's LDS budget");
    a.o_ppm = take(8 * (int64_t)AW);
    a.o_Dt = gd ? 0 : take(4 * dt_elems);
    a.o_cg = take(4 * 2 * (int64_t)AW);
    a.o_compall = take(8 * (int64_t)A);
    a.o_bg = take(8 * (int64_t)A);
    a.o_comp = take(4 * kEncSpace);
    a.o_seq = take(align16(c->Lmax) + 64);
    // workgroups that may run this pass at once: the direct grid, or the site sampler's
    // speculative slots
    const int gd_blocks = std::max<int>(c->n_cu * 2, c->tune.multi_spec_slots);
    if (gd) {
        const int64_t need = (int64_t)gd_blocks * dt_elems;
        if (need > c->dt_elems) {
            dfree(c->d_dt);
            HIP_TRY(c, hipMalloc(&c->d_dt, (size_t)need * 4));
            c->dt_elems = need;
        }
        a.dt_global = c->d_dt;
        a.dt_stride = dt_elems;
    }
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
        int grid = std::max(1, std::min<int>(c->n_local, gd ? gd_blocks : c->n_cu * 8));
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
                    : code == 5 ? "in-kernel aggregate exchange: a rank did not reach the sweep within 0.5 s"
                                : "device error";
    return fail(c, code, m, (int64_t)idx);
}

// The speculative Gauss–Seidel kernel (gs_greedy.hip) on the resident snapshot
// (d_pos[cur_pos], d_pwms, d_agg[cur_agg]); site = 1: the site sampler's twin.
// exit_info (nullable): {visits of the pass done before a mid-pass exit (0: none),
// the pass moved}, with the exit rule of GreedyArgs::exit_chunk (exit_chunk > 0).
int greedy_run(gs_ctx *c, int site, double pc, double cutoff, int32_t max_passes,
                      int32_t *passes_out, double *kernel_ms_out, int32_t exit_chunk,
                      int32_t exit_ratio, int32_t *exit_info) {
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
            a.dt16 = (int64_t)c->Lmax * W < 65536 && c->tune.site_dt16 ? 1 : 0;
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
        int waves = c->tune.greedy_waves;
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
        a.site_coop = site && c->tune.site_coop ? 1 : 0;
        a.motif_coop = site ? 0 : c->tune.motif_coop;
        a.coop_rate = site ? c->tune.coop_rate : 0.0f;  // motif (cfg5): 217 -> 234 ms with it
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
            HIP_TRY(c, hipMalloc(&c->d_stamps, kStampBytes));
            HIP_TRY(c, hipMemset(c->d_stamps, 0, kStampBytes));
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
    if (c->tune.site_switch <= 0) return greedy_run(c, 1, pc, 0.0, max_passes, passes_out, nullptr);
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
        if ((rc = greedy_run(c, 1, pc, 0.0, 1, &p1, nullptr, c->tune.site_exit_chunk, c->tune.site_exit_ratio,
                             c->tune.site_exit_chunk > 0 ? ex : nullptr))) {
            if (rc == GS_E_UNSUPPORTED && passes == 0) {
                // the star engine's LDS carve cannot hold these sequences: every pass
                // runs as speculative steps (the scan's D table goes to HBM)
                c->err.clear();
                spec_base = 0;
                spec_changed = 0;
                spec = true;
                break;
            }
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
        if ((int64_t)moves * c->tune.site_switch < n && passes < max_passes) {
            spec = true;
            break;
        }
    }
    if (spec) {
        const int32_t slots =
            (int32_t)std::max<int64_t>(1, std::min<int64_t>(n, c->tune.multi_spec_slots));
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


// ---------------------------------------------------------------------------
// motifAmount >= 1 with Positions lists (gs_multi.hip).


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


int multi_status(gs_ctx *c, unsigned long long *status_out) {
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
                     int32_t *passes_out, int32_t base0, int32_t changed0) {
    a.cnt_out = dcnt;
    a.pos_out = dpos;
    a.pwms_out = dpw;
    a.max_passes = max_passes;
    a.agg_rw = agg;
    a.spec_slots = (int32_t)std::max<int64_t>(1, std::min<int64_t>(c->n_local, c->tune.multi_spec_slots));
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
            e = gs_multi_spec_launch(a, c->tune.multi_greedy_threads, (size_t)lds, kSpecBatch, c->stream);
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
        if ((rc = greedy_run(c, 0, pc, cutoff, 1, &p1, nullptr, c->tune.greedy_exit_chunk,
                             c->tune.greedy_exit_ratio, c->tune.greedy_exit_chunk > 0 ? ex : nullptr))) {
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
        if ((int64_t)moves * c->tune.greedy_switch < n && passes < max_passes) {
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
}  // namespace gs_host
