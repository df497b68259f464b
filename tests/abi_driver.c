/*
 * abi_driver.c -- the F# shim's C call sequence for the
 * reference driver's own calls, through dlopen/dlsym like .NET P/Invoke:
 *
 *   site  : getMotifsWithBestInformationContent numberOfRepetitions W pc dnaBases
 *           sources                                          (GibbsSampling.fsx:384)
 *   motif : getMotifsWithBestInformationContents numberOfRepetitions motifAmount W pc
 *           cutOff dnaBases sources                          (GibbsSampling.fsx:407)
 *
 * The repetition loop is the one of .fs:615-640 / .fs:973-998 as the shim writes
 * it; run n uses seed + n (the shim draws a System.Random seed per run).
 *
 * usage: abi_driver <lib.so> site  <reps> <W> <pc> <seed>              < sequences
 *        abi_driver <lib.so> motif <reps> <M> <W> <pc> <cutoff> <seed> < sequences
 * stdin: the alphabet on the first line, then one sequence (ASCII symbol codes)
 * per line.  stdout: one line per sequence, "pwms pos0 pos1 ..." (site: "score pos").
 * Test driver for tests/test_abi_driver.py (not product code).
 */
#include <dlfcn.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "gibbs_hip.h"

#define MAXN 4096
#define MAXL 1 << 20

typedef int (*create_t)(int32_t, gs_ctx **);
typedef int (*destroy_t)(gs_ctx *);
typedef const char *(*lasterr_t)(const gs_ctx *);
typedef int (*setseq_t)(gs_ctx *, const uint8_t *, const int64_t *, int32_t, const uint8_t *, int32_t,
                        int64_t, int64_t);
typedef int (*site_t)(gs_ctx *, int32_t, double, uint64_t, int32_t, int32_t, int32_t *, double *,
                      int32_t *);
typedef int (*motif_t)(gs_ctx *, int32_t, double, double, uint64_t, int32_t, int32_t, int32_t *,
                       double *, int32_t *);
typedef int (*motif_multi_t)(gs_ctx *, int32_t, int32_t, double, double, uint64_t, int32_t, int32_t,
                             int32_t, int32_t *, int32_t *, double *, int32_t *);

static void *sym(void *h, const char *name) {
    void *p = dlsym(h, name);
    if (!p) {
        fprintf(stderr, "missing symbol %s\n", name);
        exit(3);
    }
    return p;
}

static void check(int st, gs_ctx *c, lasterr_t le, const char *what) {
    if (st != 0) {
        fprintf(stderr, "%s failed: status %d: %s\n", what, st, c ? le(c) : "");
        exit(4);
    }
}

/* one run's result: cnt[n] positions at pos[n*cap ..], weight w[n] */
typedef struct {
    int32_t cnt[MAXN], pos[MAXN * 16];
    double w[MAXN];
    int valid;
} run_t;

static double ic(const run_t *r, int n) {
    double s = 0.0;
    for (int i = 0; i < n; ++i) s += r->w[i];
    return s;
}

static int same(const run_t *a, const run_t *b, int n, int cap) {
    if (a->valid != b->valid) return 0;
    for (int i = 0; i < n; ++i) {
        if (a->w[i] != b->w[i] || a->cnt[i] != b->cnt[i]) return 0;
        for (int j = 0; j < a->cnt[i]; ++j)
            if (a->pos[i * cap + j] != b->pos[i * cap + j]) return 0;
    }
    return 1;
}

int main(int argc, char **argv) {
    if (argc < 3) return 2;
    void *h = dlopen(argv[1], RTLD_NOW | RTLD_LOCAL);
    if (!h) {
        fprintf(stderr, "dlopen: %s\n", dlerror());
        return 3;
    }
    create_t gs_create = (create_t)sym(h, "gs_create");
    destroy_t gs_destroy = (destroy_t)sym(h, "gs_destroy");
    lasterr_t gs_last_error = (lasterr_t)sym(h, "gs_last_error");
    setseq_t gs_set_sequences = (setseq_t)sym(h, "gs_set_sequences");
    site_t gs_site_sampling = (site_t)sym(h, "gs_site_sampling");
    motif_t gs_motif_sampling = (motif_t)sym(h, "gs_motif_sampling");
    motif_multi_t gs_motif_sampling_multi = (motif_multi_t)sym(h, "gs_motif_sampling_multi");

    const int site = strcmp(argv[2], "site") == 0;
    if (site ? argc != 7 : argc != 9) return 2;
    const int reps = atoi(argv[3]);
    const int M = site ? 1 : atoi(argv[4]);
    const int W = atoi(argv[site ? 4 : 5]);
    const double pc = atof(argv[site ? 5 : 6]);
    const double cutoff = site ? 0.0 : atof(argv[7]);
    const uint64_t seed = strtoull(argv[site ? 6 : 8], NULL, 10);

    /* sources (GpuDevice.bind: symbol codes and offsets, once) */
    static char line[MAXL];
    static uint8_t codes[MAXL];
    static int64_t offsets[MAXN + 1];
    uint8_t alpha[64];
    if (!fgets(line, sizeof line, stdin)) return 2;
    int A = (int)strcspn(line, "\r\n");
    memcpy(alpha, line, (size_t)A);
    int n = 0;
    int64_t tot = 0;
    offsets[0] = 0;
    while (n < MAXN && fgets(line, sizeof line, stdin)) {
        const int L = (int)strcspn(line, "\r\n");
        memcpy(codes + tot, line, (size_t)L);
        tot += L;
        offsets[++n] = tot;
    }
    gs_ctx *c = NULL;
    check(gs_create(0, &c), NULL, gs_last_error, "gs_create");
    check(gs_set_sequences(c, codes, offsets, n, alpha, A, n, 0), c, gs_last_error, "gs_set_sequences");

    /* the repetition loop of .fs:615-640 / .fs:973-998: stop after reps + 1 steps or
     * when a run equals the best; a run whose sum beats the best replaces it one step
     * later; the initial best is [| (0., 0) |] / [| createMotifIndex 0. [] |] */
    const int cap = M;
    static run_t acc, best, tmp;
    acc.valid = 0;          /* [||] */
    best.valid = 2;         /* the one-element initial best */
    memset(&best, 0, sizeof best);
    best.valid = 2;
    int32_t passes[3];
    for (int k = 0;; ++k) {
        const int acc_n = acc.valid ? n : 0;
        const int best_n = best.valid == 2 ? 1 : n;
        if (k > reps) break;
        if (acc.valid && best.valid != 2 && same(&acc, &best, n, cap)) break;
        if (ic(&acc, acc_n) > ic(&best, best_n)) {
            if (acc.valid) best = acc;
            acc.valid = 0;
            continue;
        }
        /* one run: doSiteSampling / doMotifSampling on the device */
        if (site) {
            check(gs_site_sampling(c, W, pc, seed + (uint64_t)k, 0, 1000000, tmp.pos, tmp.w, passes), c,
                  gs_last_error, "gs_site_sampling");
            for (int i = 0; i < n; ++i) tmp.cnt[i] = 1;
        } else if (M == 1) {
            int32_t p[MAXN];
            check(gs_motif_sampling(c, W, pc, cutoff, seed + (uint64_t)k, 0, 1000000, p, tmp.w, passes), c,
                  gs_last_error, "gs_motif_sampling");
            for (int i = 0; i < n; ++i) {
                tmp.cnt[i] = p[i] >= 0;
                tmp.pos[i * cap] = p[i];
            }
        } else {
            check(gs_motif_sampling_multi(c, M, W, pc, cutoff, seed + (uint64_t)k, 0, 1000000, cap, tmp.cnt,
                                          tmp.pos, tmp.w, passes),
                  c, gs_last_error, "gs_motif_sampling_multi");
        }
        tmp.valid = 1;
        acc = tmp;
    }
    if (best.valid == 2) {
        printf("initial\n");
    } else {
        for (int i = 0; i < n; ++i) {
            printf("%.17g", best.w[i]);
            for (int j = 0; j < best.cnt[i]; ++j) printf(" %d", best.pos[i * cap + j]);
            printf("\n");
        }
    }
    gs_destroy(c);
    dlclose(h);
    return 0;
}
