/*
 * gibbs_hip.h — C ABI of libgibbs_hip.so, the MI355X-native hot path of the
 * Gibbs motif sampler (drop-in for Etschbeijer/GibbsSampling, GibbsSampling.fs).
 *
 * The reference has no FFI; its "API" is the curried F# module functions.  Each
 * entry point below names the F# function it replaces (".fs" = GibbsSampling/
 * GibbsSampling.fs in the reference).  The P/Invoke shim that binds these from
 * .NET is in INTEGRATION.md.
 *
 * Conventions
 *  - C linkage, no exceptions cross the ABI; every call returns a gs_status.
 *  - Host buffers are caller-owned; device state lives inside the opaque gs_ctx.
 *  - One context drives ONE GPU (one process per GPU).  Several processes form one
 *    sampler through gs_comm_init (RCCL over xGMI); each then holds a contiguous
 *    shard of the sequences and all per-sequence arrays below are shard-local.
 *  - Sequences are ASCII symbol codes (BioItem.symbol, .fs:17) in [42, 90],
 *    already parsed by BioArray.ofNucleotideString / ofAminoAcidSymbolString
 *    (see gibbssampling_amd/bioarray.py for that parsing contract).
 *  - MotifIndex (.fs:712-716) with motifAmount = 1 is passed as
 *    (int32 position, double PWMS); position -1 encodes Positions = [].
 *  - A context is not thread-safe.
 */
#ifndef GIBBS_HIP_H
#define GIBBS_HIP_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct gs_ctx gs_ctx;

typedef enum {
    GS_OK = 0,
    GS_E_ARG = 1,              /* .NET ArgumentOutOfRangeException / ArgumentException   */
    GS_E_ROULETTE_OVERRUN = 2, /* list index past the end in rouletteWheelSelection .fs:752 */
    GS_E_OVERFLOW = 3,         /* Checked int32 Array.sum overflow (.fs:117)              */
    GS_E_HIP = 4,              /* HIP runtime failure -> InvalidOperationException        */
    GS_E_RCCL = 5,             /* RCCL failure -> InvalidOperationException               */
    GS_E_STATE = 6,            /* call order violated (no sequences / no snapshot)        */
    GS_E_UNSUPPORTED = 7       /* shape outside what this build handles   */
} gs_status;

#define GS_UNIQUE_ID_BYTES 128

/* --- lifetime ---------------------------------------------------------- */
int gs_create(int32_t device_id, gs_ctx **out);
int gs_destroy(gs_ctx *ctx);
const char *gs_last_error(const gs_ctx *ctx);
/* Global index of the sequence that raised the last per-sequence error (-1 if none). */
int64_t gs_error_index(const gs_ctx *ctx);
const char *gs_version(void);

/* --- data -------------------------------------------------------------- */
/* Replaces the `sources` / `alphabet` arguments shared by every entry point.
 * codes: concatenated ASCII codes of this rank's n_local sequences, offsets[n_local+1].
 * n_global: sequences over all ranks (the N in N-1 of normalizePPM, .fs:964);
 * global_offset: global index of this rank's first sequence.  Single process:
 * n_global = n_local, global_offset = 0. */
int gs_set_sequences(gs_ctx *ctx, const uint8_t *codes, const int64_t *offsets, int32_t n_local,
                     const uint8_t *alphabet, int32_t alphabet_len, int64_t n_global,
                     int64_t global_offset);

/* --- multi-GPU (one process per GPU) ----------------------------------- */
int gs_comm_unique_id(uint8_t out[GS_UNIQUE_ID_BYTES]);
int gs_comm_init(gs_ctx *ctx, const uint8_t id[GS_UNIQUE_ID_BYTES], int32_t nranks, int32_t rank);

/* In-kernel exchange of the per-sweep aggregate vector (round 6; no reference
 * counterpart: it replaces the all-reduce of .fs:940-942's shared snapshot between
 * ranks).  Every rank's context exports an exchange buffer (gs_exchange_handle: a
 * HIP IPC handle, GS_IPC_HANDLE_BYTES), the caller all-gathers the handles over any
 * transport and every rank opens them (gs_exchange_open, then a barrier of the
 * caller's before the next sweep).  From then on the packed-layout sweeps (live and
 * long kernels) end with their last workgroup writing the rank's partial into every
 * rank's buffer and summing every rank's: no all-reduce after the sweep (neither the
 * communicator's nor the caller's host-staged one below).  Positions set from outside
 * still need the caller's (or the communicator's) exchange of their aggregates; other
 * kernels keep theirs.  A peer that does not arrive within 0.5 s fails the sweep with
 * GS_E_RCCL.  gs_exchange_close returns to the all-reduce. */
#define GS_IPC_HANDLE_BYTES 64
int gs_exchange_handle(gs_ctx *ctx, uint8_t out[GS_IPC_HANDLE_BYTES]);
int gs_exchange_open(gs_ctx *ctx, const uint8_t *handles, int32_t nranks, int32_t rank);
int gs_exchange_close(gs_ctx *ctx);

/* Host-staged exchange of the per-sweep aggregates, for callers that combine
 * shards without RCCL (e.g. over their own transport, or several contexts on one
 * device): after gs_state_set_positions / each gs_run_sweeps(.., 1, ..) call,
 * download this rank's partial aggregates, sum them over the shards on the host
 * and upload the sum before the next sweep.  Size in int64 elements. */
int64_t gs_agg_size(const gs_ctx *ctx);
int gs_agg_download(gs_ctx *ctx, int64_t *out);
int gs_agg_upload(gs_ctx *ctx, const int64_t *in);

/* --- ★ the hot path ---------------------------------------------------- */
/* One synchronous sweep == MotifSampler.findBestMotifIndicesByWithStartPositions
 * (.fs:935-970) with motifAmount = 1: for every sequence, hold-one-out count
 * matrix / background rebuild from the snapshot pos_in, PWM, every W-mer window
 * scored, roulette-wheel pick with uniform u[n] (the n-th rnd.NextDouble(), .fs:968).
 * pos_in/u/pos_out/pwms_out are shard-local arrays of n_local entries. */
int gs_motif_sweep(gs_ctx *ctx, int32_t W, double pseudo_count, double cut_off,
                   const int32_t *pos_in, const double *u, int32_t *pos_out, double *pwms_out);

/* Device-resident chain of sweeps (the Gibbs iteration).  gs_state_set_positions
 * uploads a snapshot; gs_run_sweeps enqueues n_sweeps sweeps asynchronously, the
 * uniform of sequence n in sweep t being gs_uniform(seed, stream_sweep(t), n);
 * gs_state_get synchronises and downloads the latest snapshot. */
int gs_state_set_positions(gs_ctx *ctx, int32_t W, const int32_t *pos);
int gs_run_sweeps(gs_ctx *ctx, double pseudo_count, double cut_off, int32_t n_sweeps,
                  uint64_t seed, int64_t first_sweep);
int gs_state_get(gs_ctx *ctx, int32_t *pos_out, double *pwms_out);
/* With a communicator gs_run_sweeps replays chains of 6 sweeps as hipGraphs
 * (captured once per buffer phase and (pseudo_count, cut_off, seed)).  This builds the
 * graph for the current phase ahead of time (no sweep runs); optional. */
int gs_prepare_sweeps(gs_ctx *ctx, double pseudo_count, double cut_off, uint64_t seed);
int gs_synchronize(gs_ctx *ctx);
/* set + run + get in one call. */
int gs_motif_run(gs_ctx *ctx, int32_t W, double pseudo_count, double cut_off, int32_t n_sweeps,
                 uint64_t seed, int64_t first_sweep, int32_t *pos_inout, double *pwms_out);

/* --- greedy refinement ------------------------------ */
/* MotifSampler.findBestMotifIndicesWithStartPositions (.fs:885-929), motifAmount
 * = 1: Gauss–Seidel passes over the targets in order, each rebuilt from the live
 * positions, scored like the sweep, the head of the descending category sort kept
 * when its weight beats the target's current one (.fs:923); passes repeat until
 * one moves no position, at most max_passes (>= 1).  Needs every sequence on one
 * device (n_local == n_global), else GS_E_UNSUPPORTED.
 * gs_run_greedy refines the device-resident snapshot in place (after
 * gs_run_sweeps: the doMotifSampling pipeline, .fs:1034-1038) and synchronises;
 * kernel_ms_out (nullable) is the dispatch's own duration.
 * gs_motif_greedy uploads pos/pwms (the motifMem argument), refines, downloads. */
int gs_run_greedy(gs_ctx *ctx, double pseudo_count, double cut_off, int32_t max_passes,
                  int32_t *passes_out, double *kernel_ms_out);
int gs_motif_greedy(gs_ctx *ctx, int32_t W, double pseudo_count, double cut_off,
                    int32_t max_passes, int32_t *pos_inout, double *pwms_inout,
                    int32_t *passes_out);
/* doMotifSampling (.fs:1034-1038), motifAmount = 1, device-resident: gs_random_starts
 * (init_mode) -> one sweep (uniforms of sweep 0 of `seed`) -> gs_run_greedy.
 * Single device (the greedy passes). */
int gs_motif_sampling(gs_ctx *ctx, int32_t W, double pseudo_count, double cut_off,
                      uint64_t seed, int32_t init_mode, int32_t max_passes, int32_t *pos_out,
                      double *pwms_out, int32_t *passes_out);

/* --- motifAmount >= 1 with Positions lists ---------- */
/* MotifIndex (.fs:712-716) with Positions lists: entry n is (cnt[n], pos[n*cap ..
 * n*cap + cnt[n])) in F# list order (the most recently consed position first, as
 * calculatePWMsForSegmentCombinations builds them, .fs:735) and pwms[n];
 * motif_amount <= cap <= 16.  The categories are those of
 * calculateNormalizedSegmentScores (.fs:759-784): every window's background
 * score, then combos(1) ++ ... ++ combos(motifAmount) (.fs:727-742: windows
 * pairwise more than W apart, every prefix product over the cut-off).
 * gs_motif_sweep_multi: findBestMotifIndicesByWithStartPositions (.fs:935-970),
 *   explicit uniforms; shards over ranks like gs_motif_sweep.
 * gs_motif_greedy_multi: findBestMotifIndicesWithStartPositions (.fs:885-929) in
 *   place (single device).
 * gs_motif_sampling_multi: doMotifSampling (.fs:1034-1038): gs_random_starts
 *   (init_mode) -> one sweep (uniforms of sweep 0 of `seed`) -> greedy passes.
 * Both also follow gs_set_fixed_pcv (the …ByPCV twins, .fs:788-853). */
int gs_motif_sweep_multi(gs_ctx *ctx, int32_t motif_amount, int32_t W, double pseudo_count,
                         double cut_off, int32_t cap, const int32_t *cnt_in, const int32_t *pos_in,
                         const double *u, int32_t *cnt_out, int32_t *pos_out, double *pwms_out);
int gs_motif_greedy_multi(gs_ctx *ctx, int32_t motif_amount, int32_t W, double pseudo_count,
                          double cut_off, int32_t max_passes, int32_t cap, int32_t *cnt_inout,
                          int32_t *pos_inout, double *pwms_inout, int32_t *passes_out);
int gs_motif_sampling_multi(gs_ctx *ctx, int32_t motif_amount, int32_t W, double pseudo_count,
                            double cut_off, uint64_t seed, int32_t init_mode, int32_t max_passes,
                            int32_t cap, int32_t *cnt_out, int32_t *pos_out, double *pwms_out,
                            int32_t *passes_out);

/* Global aggregates of a snapshot (parity hook): C[a*W+j] = number of motif
 * segments with alphabet[a] at column j (the PFM of .fs:955-962 over ALL
 * sequences), T[a] = sum over sequences with a motif of the alphabet[a] count
 * outside the segment (createFCVWithout + fuseFrequencyVectors, .fs:945-952). */
int gs_counts(gs_ctx *ctx, int32_t W, const int32_t *pos, int64_t *C_out, int64_t *T_out);

/* --- initialiser ------------------------------------------------------- */
/* SiteSampler.getPWMOfRandomStarts (.fs:589-611): per target, start positions for
 * all other sequences, hold-one-out PWM, getBestPWMSs argmax scan with the
 * reference's in-place background drift (.fs:462-479).
 * mode 0 (exact): every target draws its own N-1 starts,
 *   r_{n,m} = gs_uniform_int(seed, stream_init(n), m, L_m-W+1)   (O(N^2) like .fs);
 * mode 1 (shared): one start vector r_m = gs_uniform_int(seed, stream_init_shared, m, ..).
 * score_out = log2 of the best window score, pos_out = its start (shard-local). */
int gs_random_starts(gs_ctx *ctx, int32_t W, double pseudo_count, uint64_t seed, int32_t mode,
                     double *score_out, int32_t *pos_out);

/* SiteSampler.getBestPWMSs (.fs:462-479) of local sequence `target` against the
 * caller's background counts fcv49 (FrequencyCompositeVector, 49 slots by
 * code - 42) and position probability matrix ppm49 (49 slot rows x W, row-major),
 * with the reference's in-place background drift (quirk Q1): every window k scores
 * against fcv + (k+1) comp(source) - (the window counts of windows 0..k).
 * score_out = log2 of the first maximal window score (-inf when none is > 0 or
 * L < W), pos_out = its start (0 then).  The reference also leaves fcVector
 * mutated; the library does not write the caller's array (the F# shim in
 * INTEGRATION.md replays that bookkeeping with the reference's own helpers). */
int gs_best_pwms(gs_ctx *ctx, int32_t W, double pseudo_count, int32_t target,
                 const int32_t *fcv49, const double *ppm49, double *score_out, int32_t *pos_out);

/* --- fixed background / fixed profile --------------- */
/* The reference's …ByPCV / …WithBPV twins take the caller's
 * ProbabilityCompositeVector pcv (49 slots, .fs:103-112) instead of the
 * hold-one-out background: PWM = PPM / pcv and background categories Π pcv
 * (.fs:788-853), no background drift in the site scans (getBestPWMSsWithBPV,
 * .fs:301-313), no Checked-sum overflow.  While set (non-null; reset by
 * gs_set_sequences), EVERY entry point computes its twin: gs_motif_sweep /
 * gs_run_sweeps = findBestMotifPositionsWithStartPositionsByPCV, gs_run_greedy =
 * findBestMotifPositionsWithStartPositionByPCV, gs_random_starts =
 * getPWMOfRandomStartsWithBPV, gs_site_refine 0/-1/+1 = findBestMotifWithStartPosition
 * / getLeft / getRightShiftedBestPWMSsWithBPV.
 * gs_set_fixed_ppm: the caller's PositionProbabilityMatrix (49 slot rows x W) for the
 * initialiser only: gs_random_starts = getMotifsWithBestPWMSOfPPM (.fs:644-662), so
 * gs_motif_sampling / gs_site_sampling become doMotifSamplingWithPPM (.fs:1028-1032)
 * / doSiteSamplingWithPPM (.fs:703-707). */
int gs_set_fixed_pcv(gs_ctx *ctx, const double *pcv49);
int gs_set_fixed_ppm(gs_ctx *ctx, const double *ppm49, int32_t W);

/* --- site sampler --------------------------------- */
/* Site-sampler positions are (float*int)[] (.fs:589): a start in [0, L-W] and
 * the log2 score of getBestPWMSs; every array is shard-local.
 * gs_site_scan: getBestPWMSs (.fs:462-479, with the in-place background drift Q1)
 *   of every target with all other sequences at pos (one Jacobi pass; the body
 *   the refinements below share, .fs:489-507 / .fs:525-542 / .fs:560-577). */
int gs_site_scan(gs_ctx *ctx, int32_t W, double pseudo_count, const int32_t *pos,
                 double *score_out, int32_t *pos_out);
/* Refinement passes on (pos, score) = startPositions, in place:
 *   shift  0: getBestPWMSsWithStartPositions (.fs:554-585), Gauss–Seidel over the
 *             live positions (all sequences on one device, else GS_E_UNSUPPORTED);
 *   shift -1: getLeftShiftedBestPWMSs (.fs:519-550), the others at the pass-start
 *             snapshot moved one left (Jacobi: shards over ranks);
 *   shift +1: getRightShiftedBestPWMSs (.fs:483-517), moved one right.
 * A target takes the scan's result when its score is strictly larger; passes
 * repeat until a pass moves no position, at most max_passes (>= 1). */
int gs_site_refine(gs_ctx *ctx, int32_t W, double pseudo_count, int32_t shift,
                   int32_t max_passes, int32_t *pos_inout, double *score_inout,
                   int32_t *passes_out);
/* doSiteSampling (.fs:697-701): gs_random_starts(init_mode) |> refine 0 |> -1 |> +1.
 * passes_out (nullable) receives the three stages' pass counts. */
int gs_site_sampling(gs_ctx *ctx, int32_t W, double pseudo_count, uint64_t seed,
                     int32_t init_mode, int32_t max_passes, int32_t *pos_out,
                     double *score_out, int32_t *passes_out);

/* --- counter RNG (identical on host, device and in the oracle) -------- */
double gs_uniform(uint64_t seed, uint64_t stream, uint64_t index);
uint64_t gs_stream_sweep(uint64_t sweep);

/* --- measurement ------------------------------------------------------- */
/* enable = k > 0: every k-th sweep launch (and all-reduce) is timed by hipEvents
 * attached to the dispatch on the library's stream (each timed launch widens the
 * dispatch gap by a few microseconds, so a timed run samples: k = 16 costs ~0.3 us
 * per sweep); enable = 0 switches timing off.  gs_profile_read returns the summed
 * milliseconds and the number of timed launches since the last read. */
int gs_profile_enable(gs_ctx *ctx, int32_t enable);
int gs_profile_read(gs_ctx *ctx, double *sweep_kernel_ms, int64_t *sweep_launches,
                    double *allreduce_ms, int64_t *allreduce_calls);
/* Device time of everything enqueued between the two calls (events on the
 * library's stream; no per-launch events, so no dispatch gap is widened).
 * region_end synchronises; region_stop (optional) records the stop event without
 * waiting, so that a caller's own device synchronisation ends the region and
 * region_end then only reads the time. */
int gs_profile_region_begin(gs_ctx *ctx);
int gs_profile_region_stop(gs_ctx *ctx);
int gs_profile_region_end(gs_ctx *ctx, double *ms);
/* Diagnostics, cumulative per context; fills out[0 .. min(n, GS_N_STATS)-1]:
 *  [0] sequences the certified binary32 scan could not decide (rescanned in binary64),
 *  [1] picks the binary64 scan could not certify either (one lane then redid the
 *      reference's sequential sums, .fs:747-754),
 *  [2..7] reasons for [0]: [2] a score out of range or negative, [3] the exactly
 *      recomputed weight disagreed, [4] total not separated from its error bound,
 *      [5] no candidate lane, [6] u within the bound of a CDF boundary, [7] u
 *      between two lanes' blocks,
 *  [8] sequences whose pick went through a background-weight path (the DNA
 *      sweep's, or the all-background sweep's: no motif category, or u near the
 *      background block), [9] of them, picks certified among the background
 *      categories,
 *  [10..12] the live-chain sweep's reasons for [0] besides [2..6]: [10] a window
 *      within the error bound of the cut-off, [11] more passing windows than a
 *      lane's list holds, [12] no passing window (every pick a background),
 *  [13] descriptor reads at an index outside [0, n_local) (the sweep kernels audit
 *      their descriptor loads; any nonzero value is a defect). */
#define GS_N_STATS 14
int gs_stats(gs_ctx *ctx, int64_t *out, int32_t n);
/* Name of the sweep kernel the next synchronous sweep of the current state runs
 * (for alphabets of <= 4 symbols with no other symbol, W <= 16: "gs_sweep_long_kernel"
 * from 320 windows, "gs_sweep_live_kernel" / "gs_sweep_dna_kernel" at the other sizes
 * where the packed layout is the faster one; else "gs_sweep_kernel"); for
 * measurement records.  A snapshot in the
 * all-background state (no window can pass the cut-off) is swept instead by
 * gs_sweep_bg_kernel, launched ahead of it (gs_stats [8] counts its targets). */
const char *gs_sweep_kernel_name(const gs_ctx *ctx);
/* The last gs_sweep_kernel launch of this context: out[0] its instantiation's EK
 * (4: the four-symbol kernel, 0: the general one), out[1] lanes per sequence, out[2]
 * wavefronts per workgroup, out[3] workgroups; all 0 before the first (diagnostics,
 * for tests that must know which instantiation ran). */
int gs_last_sweep_launch(const gs_ctx *ctx, int32_t *out);

/* --- scan mode ---------------------------------------------------------- */
/* GS_SCAN_CERTIFIED (default): windows are scored in the log2 domain in binary32
 * under a rigorous per-sequence error bound; cut-off tests and the roulette pick
 * are decided only when the bound settles them, else in binary64.  Results are
 * identical to GS_SCAN_EXACT, which folds every window in binary64 (.fs:759-777)
 * and exists for diagnostics and parity tests. */
#define GS_SCAN_CERTIFIED 0
#define GS_SCAN_EXACT 1
int gs_set_scan_mode(gs_ctx *ctx, int32_t mode);
/* Engine tuning (no reference counterpart; results never depend on it).  Every
 * field has a fixed default -- the measured choice -- and the library
 * reads no environment variables.  Fields: blocks_per_cu_cap, group_lanes,
 * sweep_waves (1, 2, 3, 4, 6, 8, 12; at most 4 when the data hold <= 16 symbols, the pair
 * tables' kernel, else 12: a larger value fails the sweep with GS_E_ARG), dna_mode (-1 automatic, 0 general sweep kernel, 1 DNA kernel
 * whenever admissible), dna_G, live_mode (-1 automatic: the live-chain packed
 * kernel while one lane holds a sequence's windows, 0 never, 1 always when the
 * packed layout is taken), live_G, live_waves, live_max_win, live_waves_per_simd,
 * live_force (tests: every live-kernel target by the exact rescan), long_mode (-1
 * automatic: the long-sequence kernel from 320 windows, 0 never, 1 whenever it fits:
 * DNA, W <= 16, at most 512 windows), long_waves (2, 4, 8 wavefronts a workgroup), bg_mode (-1
 * automatic, 0 never, 1 whenever
 * admissible: the all-background sweep kernel), bg_G, bg_force_replay (tests:
 * its picks by the exact sequential replay), graph_mode, site_coop, coop_rate, motif_coop,
 * site_dt16, site_exit_chunk, site_exit_ratio, greedy_exit_chunk,
 * greedy_exit_ratio, greedy_waves, multi_greedy_threads, multi_spec_slots,
 * greedy_switch, site_switch.  GS_E_ARG for an unknown name or a value out of
 * range.  Set before gs_set_sequences (launch geometry is fixed there). */
int gs_set_tuning(gs_ctx *ctx, const char *name, double value);
int gs_get_tuning(const gs_ctx *ctx, const char *name, double *value);
/* Measured worst-case errors of the device's binary32 log2 / exp2 (the
 * certified scan's error model budgets 2^-20 for each). */
int gs_fastmath_check(gs_ctx *ctx, double *log2_abs_err, double *exp2_rel_err);

#ifdef __cplusplus
}
#endif
#endif
