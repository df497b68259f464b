// gs_api.cpp — C ABI (include/gibbs_hip.h) over the gfx950 kernels.
//
// Entry points only: argument validation with the reference's error behaviour and
// the calls into the engine (gs_engine.cpp).  The HBM layout (encoded symbols, 16-byte
// aligned per sequence), the device snapshot state and the RCCL all-reduces live
// there.
#include "gs_ctx.h"

using namespace gs_host;

// gs_tuning fields by name; integral fields take integral values only
#define GS_TUNING_FIELD(f, ok)                                                  \
    {#f,                                                                       \
     [](gs_tuning &t, double v) {                                              \
         using T = decltype(t.f);                                              \
         if (!(ok) || (T)v != v) return false;                                 \
         t.f = (T)v;                                                           \
         return true;                                                          \
     },                                                                        \
     [](const gs_tuning &t) { return (double)t.f; }}
const gs_tuning_field kTuningFields[] = {
    GS_TUNING_FIELD(blocks_per_cu_cap, v >= 1 && v <= 32),
    GS_TUNING_FIELD(group_lanes, v == 0 || v == 16 || v == 32 || v == 64),
    GS_TUNING_FIELD(sweep_waves, v == 0 || v == 1 || v == 2 || v == 3 || v == 4 || v == 6 || v == 8 || v == 12),
    GS_TUNING_FIELD(dna_mode, v == -1 || v == 0 || v == 1),
    GS_TUNING_FIELD(dna_G, v == 0 || v == 1 || v == 2 || v == 4),
    GS_TUNING_FIELD(live_mode, v == -1 || v == 0 || v == 1),
    GS_TUNING_FIELD(live_G, v == 0 || v == 1 || v == 2 || v == 4 || v == 8),
    GS_TUNING_FIELD(live_waves_per_simd, v >= 1 && v <= 8),
    GS_TUNING_FIELD(live_force, v == 0 || v == 1),
    GS_TUNING_FIELD(live_max_win, v >= 16 && v <= 8192),
    GS_TUNING_FIELD(live_waves, v == 0 || (v >= 2 && v <= 8)),
    GS_TUNING_FIELD(long_mode, v == -1 || v == 0 || v == 1),
    GS_TUNING_FIELD(long_waves, v == 2 || v == 4 || v == 8),
    GS_TUNING_FIELD(bg_mode, v == -1 || v == 0 || v == 1),
    GS_TUNING_FIELD(bg_G, v == 0 || v == 1 || v == 2 || v == 4 || v == 8 || v == 16 || v == 32 || v == 64),
    GS_TUNING_FIELD(bg_force_replay, v == 0 || v == 1),
    GS_TUNING_FIELD(graph_mode, v == -1 || v == 0 || v == 1),
    GS_TUNING_FIELD(site_coop, v == 0 || v == 1),
    GS_TUNING_FIELD(coop_rate, v >= 0.0 && v <= 1.0),
    GS_TUNING_FIELD(motif_coop, v >= 0 && v <= 1e9),
    GS_TUNING_FIELD(site_dt16, v == 0 || v == 1),
    GS_TUNING_FIELD(site_exit_chunk, v >= 0 && v <= 1e9),
    GS_TUNING_FIELD(site_exit_ratio, v >= 1 && v <= 1e9),
    GS_TUNING_FIELD(greedy_exit_chunk, v >= 0 && v <= 1e9),
    GS_TUNING_FIELD(greedy_exit_ratio, v >= 1 && v <= 1e9),
    GS_TUNING_FIELD(greedy_waves, v >= 1 && v <= 8),
    GS_TUNING_FIELD(multi_greedy_threads, v >= 64 && v <= 1024 && (int)v % 64 == 0),
    GS_TUNING_FIELD(multi_spec_slots, v >= 1 && v <= 4096),
    GS_TUNING_FIELD(greedy_switch, v >= 0 && v <= 1e9),
    GS_TUNING_FIELD(site_switch, v >= 0 && v <= 1e9),
    GS_TUNING_FIELD(ftab_mode, v == 0 || v == 1 || v == 2),
};
#undef GS_TUNING_FIELD
const int kTuningFieldCount = (int)(sizeof(kTuningFields) / sizeof(kTuningFields[0]));

// Every entry point that can touch the aggregates outside the sweep chain drops the
// four-symbol sweep's handed-over workgroup tables (the next sweep rebuilds them).
static inline void drop_ftab(gs_ctx *c) {
    if (c) c->ftab_agg = -1;
}

namespace {
const char *kVersion = "gibbs_hip 0.1.0 (gfx950)";

}  // namespace

// The all-background takeover (gs_engine.cpp bg_ready) is dropped by every call
// that changes what the next sweep computes: the sampler's parameters (fixed PCV,
// scan mode, communicator) or its positions outside set_snapshot (which drops it
// itself).  Called only once a call's arguments are validated, so that a rejected
// call on one rank leaves every rank's state alike.
static void exchange_unmap(gs_ctx *c);

static void takeover_reset(gs_ctx *c) {
    c->bg_absorbed = c->bg_zeroed = c->snap_all_none = false;
    c->note_pending = false;
}

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
        hipMalloc(&c->d_fallbacks, 8 * kRepl * kStatStride) != hipSuccess) {
        delete c;
        return GS_E_HIP;
    }
    (void)hipMemset(c->d_err_code, 0, 4);
    (void)hipMemset(c->d_err_index, 0xff, 8);
    (void)hipMemset(c->d_fallbacks, 0, 8 * kRepl * kStatStride);
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device_id) == hipSuccess) {
        c->max_lds = (int32_t)prop.sharedMemPerBlock;
        c->n_cu = prop.multiProcessorCount;
    }
    if (c->max_lds <= 0) c->max_lds = 65536;
    if (c->n_cu <= 0) c->n_cu = 256;
    *out = c;
    return GS_OK;
}

int gs_set_tuning(gs_ctx *c, const char *name, double value) {
    if (!c || !name) return GS_E_ARG;
    drop_ftab(c);  // (the sweep chain's handed-over tables: gs_ctx.h d_ftab)
    for (int i = 0; i < kTuningFieldCount; ++i) {
        if (std::strcmp(kTuningFields[i].name, name) != 0) continue;
        if (!kTuningFields[i].set(c->tune, value))
            return fail(c, GS_E_ARG, std::string("gs_set_tuning: value out of range for ") + name);
        drop_graphs(c);  // captured launch geometry may change
        return GS_OK;
    }
    return fail(c, GS_E_ARG, std::string("gs_set_tuning: unknown field ") + name);
}

const char *gs_sweep_kernel_name(const gs_ctx *c) {
    if (!c) return "";
    if (!use_dna(c)) return "gs_sweep_kernel";
    return use_long(c) ? "gs_sweep_long_kernel" : use_live(c) ? "gs_sweep_live_kernel" : "gs_sweep_dna_kernel";
}

int gs_get_tuning(const gs_ctx *c, const char *name, double *value) {
    if (!c || !name || !value) return GS_E_ARG;
    for (int i = 0; i < kTuningFieldCount; ++i) {
        if (std::strcmp(kTuningFields[i].name, name) == 0) {
            *value = kTuningFields[i].get(c->tune);
            return GS_OK;
        }
    }
    return GS_E_ARG;
}

int gs_destroy(gs_ctx *c) {
    if (!c) return GS_OK;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->comm) ncclCommDestroy(c->comm);
    free_state(c);
    dfree(c->d_seq);
    dfree(c->d_pseq);
    dfree(c->d_doff);
    dfree(c->d_len);
    dfree(c->d_compsum);
    dfree(c->d_comp);
    dfree(c->d_pk);
    dfree(c->d_pkoff);
    exchange_unmap(c);
    dfree(c->d_xbuf);
    dfree(c->d_xpeer);
    dfree(c->d_xseq);
    dfree(c->d_err_code);
    dfree(c->d_err_index);
    dfree(c->d_fallbacks);
    dfree(c->d_bg_note);
    for (auto &p : c->ev_sweep) {
        (void)hipEventDestroy(p.first);
        (void)hipEventDestroy(p.second);
    }
    for (auto &p : c->ev_ar) {
        (void)hipEventDestroy(p.first);
        (void)hipEventDestroy(p.second);
    }
    for (auto &p : c->ev_bg) {
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
    if (c->note_ev) (void)hipEventDestroy(c->note_ev);
    if (c->h_note) (void)hipHostFree(c->h_note);
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
    drop_ftab(c);  // (the sweep chain's handed-over tables: gs_ctx.h d_ftab)
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
    int32_t pk_stride = 0;
    int32_t cmin = INT32_MAX;  // fewest occurrences of an alphabet symbol in a sequence
    int64_t compsum[4] = {0, 0, 0, 0};  // this rank's symbol totals (the live sweep's T)
    if (dna) {
        pkoff.resize(n_local);
        int64_t w = 0;
        bool same = true;
        for (int32_t n = 0; n < n_local; ++n) {
            pkoff[n] = w;
            w += ((len[n] + 15) / 16 + 3) / 4 * 4;
            same = same && len[n] == len[0];
        }
        pk_stride = (same && n_local > 0) ? ((len[0] + 15) / 16 + 3) / 4 * 4 : 0;
        pk.assign((size_t)(w + kDnaMaxL / 16 + 64), 0u);
        for (int32_t n = 0; n < n_local; ++n) {
            const uint8_t *e = h.data() + doff[n];
            uint32_t *dst = pk.data() + pkoff[n];
            int32_t cnt[4] = {0, 0, 0, 0};
            for (int32_t i = 0; i < len[n]; ++i) {
                dst[i >> 4] |= (uint32_t)e[i] << (2 * (i & 15));
                ++cnt[e[i] & 3];
            }
            for (int e2 = 0; e2 < alphabet_len; ++e2) {
                cmin = std::min(cmin, cnt[e2]);
                compsum[e2] += cnt[e2];
            }
        }
    }
    free_state(c);
    dfree(c->d_seq);
    dfree(c->d_pseq);
    dfree(c->d_doff);
    dfree(c->d_len);
    dfree(c->d_comp);
    dfree(c->d_pk);
    dfree(c->d_pkoff);
    c->dna_ok = false;
    c->pk_stride = 0;
    if (dna) {
        HIP_TRY(c, hipMalloc(&c->d_pk, pk.size() * 4));
        HIP_TRY(c, hipMalloc(&c->d_pkoff, (size_t)std::max<int32_t>(1, n_local) * 8));
        HIP_TRY(c, hipMemcpy(c->d_pk, pk.data(), pk.size() * 4, hipMemcpyHostToDevice));
        if (n_local > 0)
            HIP_TRY(c, hipMemcpy(c->d_pkoff, pkoff.data(), (size_t)n_local * 8, hipMemcpyHostToDevice));
        c->dna_ok = true;
        c->pk_stride = pk_stride;
        if (!c->d_compsum) HIP_TRY(c, hipMalloc(&c->d_compsum, 4 * 8));
        HIP_TRY(c, hipMemcpy(c->d_compsum, compsum, 4 * 8, hipMemcpyHostToDevice));
    }
    HIP_TRY(c, hipMalloc(&c->d_seq, (size_t)total));
    HIP_TRY(c, hipMalloc(&c->d_doff, (size_t)std::max<int32_t>(1, n_local) * 8));
    HIP_TRY(c, hipMalloc(&c->d_len, (size_t)std::max<int32_t>(1, n_local) * 4));
    HIP_TRY(c, hipMalloc(&c->d_comp, (size_t)std::max<int32_t>(1, n_local) * (E + 1) * 4));
    HIP_TRY(c, hipMemcpy(c->d_seq, h.data(), (size_t)total, hipMemcpyHostToDevice));
    if (scan_group(E) == 2) {
        // the sweep kernel's pair codes (gs_sweep.hip): byte i = s[i] + E s[i+1] < 256,
        // with s[L] = 0 (the padding)
        for (int32_t n = 0; n < n_local; ++n) {
            uint8_t *e = h.data() + doff[n];
            for (int32_t i = 0; i < len[n]; ++i) e[i] = (uint8_t)(e[i] + E * (i + 1 < len[n] ? e[i + 1] : 0));
        }
        HIP_TRY(c, hipMalloc(&c->d_pseq, (size_t)total));
        HIP_TRY(c, hipMemcpy(c->d_pseq, h.data(), (size_t)total, hipMemcpyHostToDevice));
    }
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
    // equal lengths laid out at a fixed stride (the sweep kernel then computes the
    // offsets of its first sequences instead of loading them)
    c->seq_stride = 0;
    if (n_local > 1 && lmin == lmax && doff[0] == 0 && doff[1] > 0) {
        bool fixed = true;
        for (int32_t n = 0; n < n_local && fixed; ++n) fixed = doff[n] == (int64_t)n * doff[1];
        if (fixed) c->seq_stride = doff[1];
    }
    // cached occupancies depend on the longest sequence (LDS carve)
    for (auto &row : c->live_occ)
        for (int &v : row) v = 0;
    for (auto &row : c->long_occ)  // (its LDS carve takes Lmax too: the rescan staging)
        for (int &v : row) v = 0;
    c->sweep_occ_key[0] = -1;
    c->cmin = (dna && n_local > 0) ? cmin : 0;
    c->h_len = std::move(len);
    c->use_pcv = c->use_ppm = false;  // their encoding belonged to the old sequences
    drop_graphs(c);
    return GS_OK;
}

int gs_set_fixed_pcv(gs_ctx *c, const double *pcv49) {
    if (!c) return GS_E_ARG;
    drop_ftab(c);  // (the sweep chain's handed-over tables: gs_ctx.h d_ftab)
    int rc;
    if ((rc = check_dev(c))) return rc;
    if (!c->d_seq) return fail(c, GS_E_STATE, "gs_set_sequences has not been called");
    takeover_reset(c);
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
    drop_ftab(c);  // (the sweep chain's handed-over tables: gs_ctx.h d_ftab)
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
    drop_ftab(c);  // (the sweep chain's handed-over tables: gs_ctx.h d_ftab)
    int rc;
    if ((rc = check_dev(c))) return rc;
    takeover_reset(c);
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

static void exchange_unmap(gs_ctx *c) {
    for (void *p : c->xmapped) (void)hipIpcCloseMemHandle(p);
    c->xmapped.clear();
    c->xranks = c->xrank = 0;
}

int gs_exchange_handle(gs_ctx *c, uint8_t out[GS_IPC_HANDLE_BYTES]) {
    if (!c || !out) return GS_E_ARG;
    static_assert(sizeof(hipIpcMemHandle_t) == GS_IPC_HANDLE_BYTES, "IPC handle size");
    int rc;
    if ((rc = check_dev(c))) return rc;
    if (!c->d_xbuf) {
        // uncached: the partials and flags are written by the peers' GPUs over xGMI and
        // polled here while the sweep runs, so no L2 (of any XCD, of any GPU) may hold
        // a stale line of them
        HIP_TRY(c, hipExtMallocWithFlags((void **)&c->d_xbuf, (size_t)kXchBytes, hipDeviceMallocUncached));
        HIP_TRY(c, hipMalloc(&c->d_xpeer, sizeof(int64_t *) * kXchRanks));
        HIP_TRY(c, hipMalloc(&c->d_xseq, 8));
    }
    hipIpcMemHandle_t h;
    HIP_TRY(c, hipIpcGetMemHandle(&h, c->d_xbuf));
    std::memcpy(out, &h, GS_IPC_HANDLE_BYTES);
    return GS_OK;
}

int gs_exchange_open(gs_ctx *c, const uint8_t *handles, int32_t nranks, int32_t rank) {
    if (!c || !handles || nranks < 1 || nranks > kXchRanks || rank < 0 || rank >= nranks) return GS_E_ARG;
    if (!c->d_xbuf) return fail(c, GS_E_STATE, "gs_exchange_handle has not been called");
    int rc;
    if ((rc = check_dev(c))) return rc;
    HIP_TRY(c, hipStreamSynchronize(c->stream));  // (no sweep in flight on the old mappings)
    exchange_unmap(c);
    drop_graphs(c);  // captured sweeps name the exchange arguments
    std::vector<int64_t *> ptrs((size_t)nranks);
    for (int q = 0; q < nranks; ++q) {
        if (q == rank) {
            ptrs[q] = c->d_xbuf;
            continue;
        }
        hipIpcMemHandle_t h;
        std::memcpy(&h, handles + (size_t)q * GS_IPC_HANDLE_BYTES, GS_IPC_HANDLE_BYTES);
        void *p = nullptr;
        const hipError_t e = hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess);
        if (e != hipSuccess) {
            exchange_unmap(c);
            return fail(c, GS_E_HIP, std::string("hipIpcOpenMemHandle: ") + hipGetErrorString(e));
        }
        c->xmapped.push_back(p);
        ptrs[q] = (int64_t *)p;
    }
    // a fresh buffer and count: flags 0, no sweep exchanged yet (every rank opens before
    // any rank sweeps: the caller's barrier)
    HIP_TRY(c, hipMemset(c->d_xbuf, 0, (size_t)kXchBytes));
    HIP_TRY(c, hipMemset(c->d_xseq, 0, 8));
    HIP_TRY(c, hipMemcpy(c->d_xpeer, ptrs.data(), sizeof(int64_t *) * nranks, hipMemcpyHostToDevice));
    c->xranks = nranks;
    c->xrank = rank;
    return GS_OK;
}

int gs_exchange_close(gs_ctx *c) {
    if (!c) return GS_E_ARG;
    int rc;
    if ((rc = check_dev(c))) return rc;
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    drop_graphs(c);
    exchange_unmap(c);
    return GS_OK;
}

int gs_state_set_positions(gs_ctx *c, int32_t W, const int32_t *pos) {
    if (!c || (!pos && c->n_local > 0)) return GS_E_ARG;
    drop_ftab(c);  // (the sweep chain's handed-over tables: gs_ctx.h d_ftab)
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
    if ((rc = bg_resolve(c))) return rc;
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
    // the rest of the chain by the all-background kernel once a sweep saw the state
    return n_sweeps > 0 ? bg_check_note(c, pc, cutoff) : GS_OK;
}

int gs_prepare_sweeps(gs_ctx *c, double pc, double cutoff, uint64_t seed) {
    if (!c) return GS_E_ARG;
    int rc;
    if ((rc = check_dev(c))) return rc;
    if (!c->have_state) return fail(c, GS_E_STATE, "no snapshot: call gs_state_set_positions");
    if ((rc = bg_resolve(c))) return rc;
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
    if ((rc = bg_resolve(c))) return rc;
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
    drop_ftab(c);  // (the sweep chain's handed-over tables: gs_ctx.h d_ftab)
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
    drop_ftab(c);  // (the sweep chain's handed-over tables: gs_ctx.h d_ftab)
    int rc;
    if ((rc = gs_state_set_positions(c, W, pos_inout))) return rc;
    if ((rc = gs_run_sweeps(c, pc, cutoff, n_sweeps, seed, first_sweep))) return rc;
    return gs_state_get(c, pos_inout, pwms_out);
}


int gs_run_greedy(gs_ctx *c, double pc, double cutoff, int32_t max_passes, int32_t *passes_out,
                  double *kernel_ms_out) {
    if (!c || max_passes < 1) return GS_E_ARG;
    drop_ftab(c);  // (the sweep chain's handed-over tables: gs_ctx.h d_ftab)
    int rc;
    if ((rc = check_dev(c))) return rc;
    if (!c->have_state) return fail(c, GS_E_STATE, "no snapshot: call gs_state_set_positions");
    if ((int64_t)c->n_local != c->n_global)
        return fail(c, GS_E_UNSUPPORTED,
                    "the greedy refinement walks every target in order (.fs:885-929): it needs "
                    "all sequences on one device");
    takeover_reset(c);  // the passes move positions in place
    if (c->tune.greedy_switch > 0 && !c->use_pcv)
        return greedy_hybrid(c, pc, cutoff, max_passes, passes_out, kernel_ms_out);
    return greedy_run(c, 0, pc, cutoff, max_passes, passes_out, kernel_ms_out);
}

int gs_motif_greedy(gs_ctx *c, int32_t W, double pc, double cutoff, int32_t max_passes,
                    int32_t *pos_inout, double *pwms_inout, int32_t *passes_out) {
    if (!c || (c->n_local > 0 && (!pos_inout || !pwms_inout))) return GS_E_ARG;
    drop_ftab(c);  // (the sweep chain's handed-over tables: gs_ctx.h d_ftab)
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
    drop_ftab(c);  // (the sweep chain's handed-over tables: gs_ctx.h d_ftab)
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
    drop_ftab(c);  // (the sweep chain's handed-over tables: gs_ctx.h d_ftab)
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
    drop_ftab(c);  // (the sweep chain's handed-over tables: gs_ctx.h d_ftab)
    int rc;
    if ((rc = check_dev(c))) return rc;
    if (!c->have_state) return fail(c, GS_E_STATE, "no snapshot");
    HIP_TRY(c, hipMemcpyAsync(c->d_agg[c->cur_agg], in, (size_t)kRepl * c->stride * 8,
                              hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    c->rep_valid = true;
    c->vec_valid = false;
    c->bg_absorbed = c->bg_zeroed = c->snap_all_none = false;  // aggregates set from outside
    c->note_pending = false;
    return GS_OK;
}

int gs_random_starts(gs_ctx *c, int32_t W, double pc, uint64_t seed, int32_t mode,
                     double *score_out, int32_t *pos_out) {
    drop_ftab(c);  // (the sweep chain's handed-over tables: gs_ctx.h d_ftab)
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

int gs_best_pwms(gs_ctx *c, int32_t W, double pc, int32_t target, const int32_t *fcv49,
                 const double *ppm49, double *score_out, int32_t *pos_out) {
    if (!c || !fcv49 || !ppm49 || !score_out || !pos_out) return GS_E_ARG;
    drop_ftab(c);  // (the sweep chain's handed-over tables: gs_ctx.h d_ftab)
    int rc;
    if ((rc = check_dev(c))) return rc;
    if (!c->d_seq) return fail(c, GS_E_STATE, "gs_set_sequences has not been called");
    if (W < 1 || W > 64) return fail(c, GS_E_ARG, "motifLength must be in [1, 64]");
    if (target < 0 || target >= c->n_local) return fail(c, GS_E_ARG, "target out of range");
    if (c->h_len[target] < W) {  // the loop's first test fails: log2 0.0, index 0 (.fs:464)
        *score_out = -INFINITY;
        *pos_out = 0;
        return GS_OK;
    }
    const int A = c->A, AW = A * W;
    // the caller's PPM and background by alphabet symbol, the background's 49-slot sum
    std::vector<double> ppm((size_t)AW);
    std::vector<int64_t> bg((size_t)A + 1, 0);
    for (int a = 0; a < A; ++a) {
        const int slot = c->alphabet[a] - kSlot0;
        for (int j = 0; j < W; ++j) ppm[(size_t)a * W + j] = ppm49[slot * W + j];
        bg[a] = fcv49[slot];
    }
    for (int s = 0; s < kSlots; ++s) bg[A] += fcv49[s];
    StartsArgs a{};
    int64_t lds = 0;
    if ((rc = starts_pass(c, 1, W, pc, 0, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                          &a, &lds)))
        return rc;
    const int cells = AW + A;
    double *d_ppm = nullptr, *d_score = nullptr;
    int64_t *d_bg = nullptr, *d_agg = nullptr;
    int32_t *d_pos = nullptr;
    auto cleanup = [&]() {
        dfree(d_ppm);
        dfree(d_bg);
        dfree(d_agg);
        dfree(d_score);
        dfree(d_pos);
    };
    bool ok = hipMalloc(&d_ppm, ppm.size() * 8) == hipSuccess &&
              hipMalloc(&d_bg, bg.size() * 8) == hipSuccess &&
              hipMalloc(&d_agg, (size_t)kRepl * cells * 8) == hipSuccess &&
              hipMalloc(&d_score, (size_t)c->n_local * 8) == hipSuccess &&
              hipMalloc(&d_pos, (size_t)c->n_local * 4) == hipSuccess;
    ok = ok && hipMemcpyAsync(d_ppm, ppm.data(), ppm.size() * 8, hipMemcpyHostToDevice, c->stream) == hipSuccess &&
         hipMemcpyAsync(d_bg, bg.data(), bg.size() * 8, hipMemcpyHostToDevice, c->stream) == hipSuccess &&
         hipMemsetAsync(d_agg, 0, (size_t)kRepl * cells * 8, c->stream) == hipSuccess &&
         hipMemsetAsync(c->d_err_code, 0, 4, c->stream) == hipSuccess &&
         hipMemsetAsync(c->d_err_index, 0xff, 8, c->stream) == hipSuccess;
    if (ok) {
        a.cells = cells;
        a.stride = cells;
        a.agg = d_agg;
        a.ppm_fixed = d_ppm;
        a.pcv_fixed = nullptr;  // getBestPWMSs: the drifting background, never the BPV twin
        a.bg_fixed = d_bg;
        a.single = target + 1;
        a.score_out = d_score;
        a.pos_out = d_pos;
        ok = gs_starts_launch(a, 1, (size_t)lds, c->stream) == hipSuccess &&
             hipStreamSynchronize(c->stream) == hipSuccess &&
             hipMemcpy(score_out, d_score + target, 8, hipMemcpyDeviceToHost) == hipSuccess &&
             hipMemcpy(pos_out, d_pos + target, 4, hipMemcpyDeviceToHost) == hipSuccess;
    }
    cleanup();
    if (!ok) return fail(c, GS_E_HIP, "gs_best_pwms: HIP failure");
    return check_device_error(c);
}

double gs_uniform(uint64_t seed, uint64_t stream, uint64_t index) {
    return uniform(seed, stream, index);
}
uint64_t gs_stream_sweep(uint64_t sweep) { return stream_sweep(sweep); }

int gs_site_scan(gs_ctx *c, int32_t W, double pc, const int32_t *pos, double *score_out,
                 int32_t *pos_out) {
    if (!c || (c->n_local > 0 && (!pos || !score_out || !pos_out))) return GS_E_ARG;
    drop_ftab(c);  // (the sweep chain's handed-over tables: gs_ctx.h d_ftab)
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
    drop_ftab(c);  // (the sweep chain's handed-over tables: gs_ctx.h d_ftab)
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
    drop_ftab(c);  // (the sweep chain's handed-over tables: gs_ctx.h d_ftab)
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
    c->prof_sweep_calls = c->prof_ar_calls = c->prof_bg_calls = 0;
    return GS_OK;
}

int gs_profile_region_begin(gs_ctx *c) {
    if (!c) return GS_E_ARG;
    int rc;
    if ((rc = check_dev(c))) return rc;
    if (!c->region_start) HIP_TRY(c, hipEventCreate(&c->region_start));
    if (!c->region_stop) HIP_TRY(c, hipEventCreate(&c->region_stop));
    HIP_TRY(c, hipEventRecord(c->region_start, c->stream));
    c->region_stopped = false;
    return GS_OK;
}

int gs_profile_region_stop(gs_ctx *c) {
    if (!c) return GS_E_ARG;
    if (!c->region_start) return fail(c, GS_E_STATE, "gs_profile_region_begin was not called");
    HIP_TRY(c, hipEventRecord(c->region_stop, c->stream));
    c->region_stopped = true;
    return GS_OK;
}

int gs_profile_region_end(gs_ctx *c, double *ms) {
    if (!c || !ms) return GS_E_ARG;
    if (!c->region_start) return fail(c, GS_E_STATE, "gs_profile_region_begin was not called");
    if (!c->region_stopped) HIP_TRY(c, hipEventRecord(c->region_stop, c->stream));
    c->region_stopped = false;
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
    for (auto &p : c->ev_bg) {
        float ms = 0.f;
        HIP_TRY(c, hipEventElapsedTime(&ms, p.first, p.second));
        c->prof_sweep_ms += ms;
        c->ev_pool.push_back(p.first);
        c->ev_pool.push_back(p.second);
    }
    c->ev_bg.clear();
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
    if (reset) HIP_TRY(c, hipMemset(c->d_stamps, 0, kStampBytes));
    return GS_OK;
}

// The timeline of the last stamped launch: kTlMarks s_memrealtime marks per
// wavefront (0 = not reached), `waves` wavefronts from the first.
int gs_debug_timeline(gs_ctx *c, unsigned long long *out, int32_t waves) {
    if (!c || !out || waves < 0 || waves > kTlWaves) return GS_E_ARG;
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    if (!c->d_stamps) return fail(c, GS_E_STATE, "no stamped launch yet");
    HIP_TRY(c, hipMemcpy(out, c->d_stamps + kStampSlots, 8ull * kTlMarks * waves, hipMemcpyDeviceToHost));
    HIP_TRY(c, hipMemset(c->d_stamps + kStampSlots, 0, 8ull * kTlMarks * kTlWaves));
    return GS_OK;
}
#endif

int gs_last_sweep_launch(const gs_ctx *c, int32_t *out) {
    if (!c || !out) return GS_E_ARG;
    for (int i = 0; i < 4; ++i) out[i] = c->last_sweep[i];
    return GS_OK;
}

int gs_stats(gs_ctx *c, int64_t *out, int32_t n) {
    if (!c || !out || n < 0) return GS_E_ARG;
    int rc;
    if ((rc = check_dev(c))) return rc;
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    unsigned long long v[kRepl * kStatStride] = {};
    HIP_TRY(c, hipMemcpy(v, c->d_fallbacks, sizeof(v), hipMemcpyDeviceToHost));
    for (int i = 0; i < n && i < GS_N_STATS; ++i) {
        unsigned long long t = 0;  // the per-XCD replicas (kStatStride)
        for (int r = 0; r < kRepl; ++r) t += v[r * kStatStride + i];
        out[i] = (int64_t)t;
    }
    return GS_OK;
}

int gs_set_scan_mode(gs_ctx *c, int32_t mode) {
    if (!c || (mode != GS_SCAN_CERTIFIED && mode != GS_SCAN_EXACT)) return GS_E_ARG;
    drop_ftab(c);  // (the sweep chain's handed-over tables: gs_ctx.h d_ftab)
    takeover_reset(c);
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

extern "C" {

int gs_motif_sweep_multi(gs_ctx *c, int32_t motif_amount, int32_t W, double pc, double cutoff,
                         int32_t cap, const int32_t *cnt_in, const int32_t *pos_in,
                         const double *u, int32_t *cnt_out, int32_t *pos_out, double *pwms_out) {
    drop_ftab(c);  // (the sweep chain's handed-over tables: gs_ctx.h d_ftab)
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
    drop_ftab(c);  // (the sweep chain's handed-over tables: gs_ctx.h d_ftab)
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
    drop_ftab(c);  // (the sweep chain's handed-over tables: gs_ctx.h d_ftab)
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
