/*
 * sanitize_main.c -- runs the CPU oracle (test infrastructure) under host
 * AddressSanitizer + UndefinedBehaviorSanitizer on seeded data sets shaped like the
 * golden fixtures: config-1 DNA, the .fsx dnaBases alphabet with a gap symbol and
 * non-alphabet codes, ragged lengths, a protein set, Positions = [] entries and
 * motifAmount 2 lists.  Cross-checks the faithful and hold-one-out restatements on
 * every case (as tests/test_oracle_crosscheck.py does through ctypes) and exits
 * non-zero on any difference; the sanitizers abort on any memory or UB error.
 * Built and run by tests/test_oracle_sanitize.py (oracle/Makefile target asan).
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "gibbs_oracle.h"

static uint64_t rs = 0x12345678u;
static uint32_t rnd(void) {
    rs = rs * 6364136223846793005ULL + 1442695040888963407ULL;
    return (uint32_t)(rs >> 33);
}

static int fails = 0;
#define CHECK(cond, what)                                   \
    do {                                                    \
        if (!(cond)) {                                      \
            fprintf(stderr, "FAIL %s (%s:%d)\n", what, __FILE__, __LINE__); \
            ++fails;                                        \
        }                                                   \
    } while (0)

static void one_case(int N, int Lmax, int W, const char *alpha, const char *extra, int ragged,
                     int M) {
    const int A = (int)strlen(alpha), X = (int)strlen(extra);
    int64_t *off = calloc((size_t)N + 1, sizeof *off);
    for (int n = 0; n < N; ++n) {
        int L = ragged ? W + (int)(rnd() % (uint32_t)(Lmax - W + 1)) : Lmax;
        off[n + 1] = off[n] + L;
    }
    uint8_t *codes = malloc((size_t)off[N]);
    for (int64_t i = 0; i < off[N]; ++i)
        codes[i] = (X && rnd() % 64 == 0) ? (uint8_t)extra[rnd() % X] : (uint8_t)alpha[rnd() % A];
    go_seqs s = {codes, off, N, (const uint8_t *)alpha, A};
    CHECK(go_validate(&s, W) == GO_OK, "validate");
    const int cap = M;
    int32_t *cnt = calloc((size_t)N, 4), *pos = malloc((size_t)N * cap * 4);
    for (int n = 0; n < N; ++n) {
        const int K = (int)(off[n + 1] - off[n]) - W + 1;
        cnt[n] = (rnd() % 8 == 0) ? 0 : 1;  /* some Positions = [] */
        pos[n * cap] = (int32_t)(rnd() % (uint32_t)K);
        for (int j = 1; j < cap; ++j) pos[n * cap + j] = -1;
    }
    double *u = malloc((size_t)N * 8), *w1 = malloc((size_t)N * 8), *w2 = malloc((size_t)N * 8);
    double *m1 = malloc((size_t)N * 8), *m2 = malloc((size_t)N * 8);
    int32_t *c1 = malloc((size_t)N * 4), *c2 = malloc((size_t)N * 4);
    int32_t *p1 = malloc((size_t)N * cap * 4), *p2 = malloc((size_t)N * cap * 4);
    for (int n = 0; n < N; ++n) u[n] = go_uniform(7, go_stream_sweep(0), (uint64_t)n);
    int32_t e1 = -1, e2 = -1;
    const int r1 = go_sweep_faithful(&s, M, W, 1e-4, 1.0, cnt, pos, cap, u, 0, N, c1, p1, cap, w1, m1, &e1);
    const int r2 = go_sweep_fast(&s, M, W, 1e-4, 1.0, cnt, pos, cap, u, 0, N, c2, p2, cap, w2, m2, &e2, 2);
    CHECK(r1 == r2, "sweep status");
    if (r1 == GO_OK) {
        CHECK(memcmp(c1, c2, (size_t)N * 4) == 0, "sweep counts");
        CHECK(memcmp(p1, p2, (size_t)N * cap * 4) == 0, "sweep positions");
        CHECK(memcmp(w1, w2, (size_t)N * 8) == 0, "sweep PWMS");
    }
    int64_t *C = calloc((size_t)A * W, 8), *T = calloc((size_t)A, 8);
    CHECK(go_counts(&s, W, cnt, pos, cap, C, T) == GO_OK, "counts");
    if (M == 1) {
        /* greedy: the per-target rebuild and the incremental port */
        int32_t pa[4096], pb[4096], ca[4096], cb[4096], pa_n = 0, pb_n = 0;
        double wa[4096], wb[4096];
        int64_t visits = 0;
        for (int n = 0; n < N; ++n) {
            ca[n] = cb[n] = c1[n];
            pa[n] = pb[n] = p1[n];
            wa[n] = wb[n] = w1[n];
        }
        const int g1 = go_greedy(&s, 1, W, 1e-4, 1.0, ca, pa, 1, wa, 50, &pa_n);
        const int g2 = go_greedy_fast(&s, 1, W, 1e-4, 1.0, cb, pb, 1, wb, 50, 0, &pb_n, &visits);
        CHECK(g1 == g2, "greedy status");
        if (g1 == GO_OK) {
            CHECK(pa_n == pb_n && memcmp(pa, pb, (size_t)N * 4) == 0, "greedy positions");
            CHECK(memcmp(wa, wb, (size_t)N * 8) == 0, "greedy PWMS");
        }
        /* the initialiser (both modes), the site scans and refinements */
        double sc[4096];
        int32_t sp[4096], passes = 0;
        CHECK(go_random_starts(&s, W, 1e-4, NULL, 11, 0, 0, N, sc, sp) == GO_OK, "starts mode 0");
        CHECK(go_random_starts(&s, W, 1e-4, NULL, 11, 1, 0, N, sc, sp) == GO_OK, "starts mode 1");
        double sc2[4096];
        int32_t sp2[4096], passes2 = 0;
        int64_t v2 = 0;
        memcpy(sc2, sc, (size_t)N * 8);
        memcpy(sp2, sp, (size_t)N * 4);
        CHECK(go_site_refine(&s, W, 1e-4, 0, sp, sc, 50, &passes) == GO_OK, "site refine");
        CHECK(go_site_refine_fast(&s, W, 1e-4, sp2, sc2, 50, 0, &passes2, &v2) == GO_OK,
              "site refine fast");
        CHECK(passes == passes2 && memcmp(sp, sp2, (size_t)N * 4) == 0, "site refine positions");
        CHECK(go_site_refine(&s, W, 1e-4, -1, sp, sc, 50, &passes) == GO_OK, "left shift");
        CHECK(go_site_refine(&s, W, 1e-4, 1, sp, sc, 50, &passes) == GO_OK, "right shift");
        int64_t fcv[49] = {0};
        double ppm[64 * 16];
        for (int a = 0; a < A; ++a) fcv[alpha[a] - 42] = 100 + rnd() % 1000;
        for (int i = 0; i < A * W; ++i) ppm[i] = 1.0 / A;
        double bs;
        int32_t bp;
        CHECK(go_best_pwms(&s, W, 1e-4, N - 1, fcv, ppm, &bs, &bp) == GO_OK, "best pwms");
    }
    free(off), free(codes), free(cnt), free(pos), free(u), free(w1), free(w2), free(m1), free(m2);
    free(c1), free(c2), free(p1), free(p2), free(C), free(T);
}

int main(void) {
    one_case(100, 50, 8, "ACGT", "", 0, 1);          /* BASELINE config 1 */
    one_case(64, 90, 7, "ATGC-", "*N", 1, 1);        /* dnaBases of the .fsx, non-alphabet codes */
    one_case(40, 200, 12, "ACGT", "", 1, 1);
    one_case(30, 120, 20, "ACDEFGHIKLMNPQRSTVWY", "", 0, 1);  /* protein */
    one_case(25, 80, 6, "ACGT", "*", 1, 2);          /* motifAmount 2 lists */
    one_case(3, 20, 20, "ACGT", "", 0, 1);           /* L == W */
    if (fails) {
        fprintf(stderr, "%d checks failed\n", fails);
        return 1;
    }
    printf("sanitized oracle: all checks passed\n");
    return 0;
}
