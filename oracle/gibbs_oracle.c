/*
 * gibbs_oracle.c — CPU restatement of GibbsSampling.fs (see gibbs_oracle.h).
 *
 * TEST INFRASTRUCTURE ONLY (checker + timed CPU baseline).  Parity is unpinned
 * against reference-produced numbers (the F# reference cannot run here and holds
 * no golden vectors); see the header and DESIGN.md §Oracle.
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off -fopenmp).
 */
#include "gibbs_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define NSLOT 49   /* CompositeVector / BaseMatrix rows: symbol code - 42 (.fs:17, .fs:176) */
#define SLOT0 42
#define GO_MAXM 16 /* max motifAmount supported by the combination enumerator */

/* ------------------------------------------------------------------ RNG */
uint64_t go_mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
double go_uniform(uint64_t seed, uint64_t stream, uint64_t index) {
    uint64_t h = go_mix64(seed ^ go_mix64(stream ^ go_mix64(index)));
    return (double)(h >> 11) * 0x1.0p-53;
}
int32_t go_uniform_int(uint64_t seed, uint64_t stream, uint64_t index, int32_t k) {
    int32_t r = (int32_t)(go_uniform(seed, stream, index) * (double)k);
    return r >= k ? k - 1 : r;
}
uint64_t go_stream_sweep(uint64_t sweep) { return (1ULL << 40) | sweep; }
uint64_t go_stream_init(uint64_t target) { return (2ULL << 40) | target; }
uint64_t go_stream_init_shared(void) { return 3ULL << 40; }

/* FSharpAux.Math.log2 = Math.Log(x, 2.0) = Log(x)/Log(2.0)  (SURVEY App. C). */
double go_log2(double x) { return log(x) / 0x1.62e42fefa39efp-1; }

/* ------------------------------------------------------------------ helpers */
static void alpha_map(const go_seqs *s, int32_t *aidx /*49*/) {
    for (int b = 0; b < NSLOT; ++b) aidx[b] = -1;
    for (int a = 0; a < s->A; ++a) aidx[s->alphabet[a] - SLOT0] = a;
}

int go_validate(const go_seqs *s, int32_t W) {
    if (!s || W < 1 || s->n < 0 || s->A < 1 || s->A > NSLOT) return GO_E_ARG;
    int seen[NSLOT] = {0};
    for (int a = 0; a < s->A; ++a) {
        int c = s->alphabet[a];
        if (c < SLOT0 || c >= SLOT0 + NSLOT || seen[c - SLOT0]) return GO_E_ARG;
        seen[c - SLOT0] = 1;
    }
    if (s->n > 0 && s->off[0] != 0) return GO_E_ARG;
    for (int32_t n = 0; n < s->n; ++n) {
        int64_t L = s->off[n + 1] - s->off[n];
        if (L < W) return GO_E_ARG; /* Array.take / Random.Next throw (.fs:145, .fs:152) */
        for (int64_t i = s->off[n]; i < s->off[n + 1]; ++i)
            if (s->codes[i] < SLOT0 || s->codes[i] >= SLOT0 + NSLOT) return GO_E_ARG;
    }
    return GO_OK;
}

static int check_positions(const go_seqs *s, int32_t W, const int32_t *cnt, const int32_t *pos,
                           int32_t cap) {
    for (int32_t m = 0; m < s->n; ++m) {
        if (cnt[m] < 0 || cnt[m] > cap) return GO_E_ARG;
        int64_t L = s->off[m + 1] - s->off[m];
        for (int i = 0; i < cnt[m]; ++i) {
            int32_t p = pos[(int64_t)m * cap + i];
            if (p < 0 || p + W > L) return GO_E_ARG; /* getSegment .fs:149-153 */
        }
    }
    return GO_OK;
}

/* ---------------------------------------------------------------- categories */
typedef struct {
    double pwms;
    int32_t npos;
    int32_t pos[GO_MAXM];
} cat_t;

typedef struct {
    cat_t *v;
    int64_t n, cap;
} catvec;

static void cat_push(catvec *c, double pwms, const int32_t *pos, int32_t npos) {
    if (c->n == c->cap) {
        c->cap = c->cap ? 2 * c->cap : 256;
        c->v = (cat_t *)realloc(c->v, (size_t)c->cap * sizeof(cat_t));
    }
    cat_t *e = &c->v[c->n++];
    e->pwms = pwms;
    e->npos = npos;
    for (int i = 0; i < npos; ++i) e->pos[i] = pos[i];
}

/* PositionMatrix.ceckForDistance (.fs:129-140): every pair strictly more than width apart. */
static int check_distance(int32_t width, const int32_t *items, int32_t len) {
    if (len <= 1) return 1;
    for (int a = 0; a < len - 1; ++a)
        for (int b = a + 1; b < len; ++b)
            if (!(abs(items[a] - items[b]) > width)) return 0;
    return 1;
}

/* calculatePWMsForSegmentCombinations (.fs:727-742), literal recursion over the list
 * [(S_k, k) for k = kf..K-1]; positions kept most-recent-first like the F# cons list. */
static void combos(double cutoff, int32_t width, int32_t size, double prob, int32_t *positions,
                   int32_t npos, const double *S, int32_t kf, int32_t K, catvec *out) {
    if (kf < K) {
        if (size > 0) {
            int32_t items[GO_MAXM + 1];
            items[0] = kf;
            for (int i = 0; i < npos; ++i) items[i + 1] = positions[i];
            if (check_distance(width, items, npos + 1)) {
                double np = S[kf] * prob;
                if (go_log2(np) > cutoff)
                    combos(cutoff, width, size - 1, np, items, npos + 1, S, kf + 1, K, out);
            }
        }
        if (size >= 0) combos(cutoff, width, size, prob, positions, npos, S, kf + 1, K, out);
    } else if (size == 0) {
        cat_push(out, go_log2(prob), positions, npos);
    }
}

/* rouletteWheelSelection (.fs:746-754). Returns index or -1 on overrun. */
static int64_t roulette(double pick, const catvec *c, double *margin) {
    double sum = 0.0; /* List.sum: left to right from GenericZero */
    for (int64_t i = 0; i < c->n; ++i) sum = sum + c->v[i].pwms;
    double acc = 0.0, mg = INFINITY;
    for (int64_t i = 0; i < c->n; ++i) {
        double w = c->v[i].pwms / sum;
        double hi = acc + w;
        double d0 = fabs(pick - acc), d1 = fabs(pick - hi);
        if (d0 < mg) mg = d0;
        if (d1 < mg) mg = d1;
        if (acc <= pick && pick <= hi) {
            if (margin) *margin = mg;
            return i;
        }
        acc = hi;
    }
    if (margin) *margin = mg;
    return -1;
}

/* ------------------------------------------------------- per-target scoring */
typedef struct {
    double *S, *G;
    catvec cats;
} scratch_t;

/*
 * Everything after the count aggregates for one target of the sweep
 * (.fs:945-968 after the integer rebuilds):
 *   createNormalizedPCVOfFCV (.fs:115-120), normalizePPM (.fs:255-261),
 *   createPositionWeightMatrix (.fs:282-287), calculateNormalizedSegmentScores
 *   (.fs:759-784), rouletteWheelSelection (.fs:746-754).
 * bgc: 49-slot background counts; Cn: A*W (alphabet order) count matrix of the others.
 * mode_greedy: instead of the roulette, List.sortByDescending |> List.head (.fs:917-920).
 */
static int score_target(const go_seqs *s, const int32_t *aidx, int32_t n, int32_t W, double pc,
                        double cutoff, int32_t motif_amount, const int64_t *bgc,
                        const double *pcv_fixed, const int64_t *Cn, double u, int mode_greedy,
                        int literal_combos, scratch_t *sc, cat_t *picked, double *margin) {
    const uint8_t *src = s->codes + s->off[n];
    const int64_t L = s->off[n + 1] - s->off[n];
    const int32_t A = s->A;
    double pcv[NSLOT];
    if (pcv_fixed) {
        /* the ...ByPCV variants (.fs:788-853) take the caller's ProbabilityCompositeVector */
        memcpy(pcv, pcv_fixed, sizeof(pcv));
    } else {
        /* Array.sum of the int32 vector is Checked (overflow throws). */
        int64_t tot = 0;
        for (int b = 0; b < NSLOT; ++b) tot += bgc[b];
        if (tot > INT32_MAX || tot < INT32_MIN) return GO_E_OVERFLOW;
        double sum = (double)tot + (double)A * pc;
        for (int b = 0; b < NSLOT; ++b) pcv[b] = (double)bgc[b];
        for (int a = 0; a < A; ++a) {
            int b = s->alphabet[a] - SLOT0;
            pcv[b] = (pcv[b] + pc) / sum;
        }
    }
    /* PWM rows in slot space (49 x W), zero outside the alphabet. */
    double den = (double)(s->n - 1) + (double)A * pc;
    double *pwm = (double *)calloc((size_t)NSLOT * W, sizeof(double));
    for (int a = 0; a < A; ++a) {
        int b = s->alphabet[a] - SLOT0;
        for (int j = 0; j < W; ++j) {
            double ppm = ((double)Cn[a * W + j] + pc) / den;
            pwm[b * W + j] = ppm / pcv[b];
        }
    }
    const int64_t K = L - W + 1;
    for (int64_t k = 0; k < K; ++k) {
        double sv = 1.0, gv = 1.0;
        for (int j = 0; j < W; ++j) {
            int b = src[k + j] - SLOT0;
            sv = sv * pwm[b * W + j];
            gv = gv * pcv[b];
        }
        sc->S[k] = sv;
        sc->G[k] = gv;
    }
    free(pwm);
    (void)aidx;
    sc->cats.n = 0;
    for (int64_t k = 0; k < K; ++k) cat_push(&sc->cats, sc->G[k], NULL, 0);
    for (int32_t m = 1; m <= motif_amount; ++m) {
        if (m == 1 && !literal_combos) {
            for (int64_t k = 0; k < K; ++k) {
                double lv = go_log2(sc->S[k] * 1.0);
                if (lv > cutoff) {
                    int32_t p = (int32_t)k;
                    cat_push(&sc->cats, go_log2(sc->S[k] * 1.0), &p, 1);
                }
            }
        } else {
            int32_t tmp[GO_MAXM];
            combos(cutoff, W, m, 1.0, tmp, 0, sc->S, 0, (int32_t)K, &sc->cats);
        }
    }
    if (mode_greedy) {
        /* stable sortByDescending |> head: first category holding the maximum; F#
         * generic comparison ranks NaN below every number */
        int64_t best = -1;
        for (int64_t i = 0; i < sc->cats.n; ++i) {
            const double v = sc->cats.v[i].pwms;
            const double b = best < 0 ? NAN : sc->cats.v[best].pwms;
            if (best < 0 || v > b || (b != b && v == v)) best = i;
        }
        if (best < 0) return GO_E_ARG; /* List.head on empty list */
        *picked = sc->cats.v[best];
        return GO_OK;
    }
    int64_t i = roulette(u, &sc->cats, margin);
    if (i < 0) return GO_E_ROULETTE_OVERRUN;
    *picked = sc->cats.v[i];
    return GO_OK;
}

static void comp49(const uint8_t *x, int64_t len, int64_t *c) {
    for (int64_t i = 0; i < len; ++i) c[x[i] - SLOT0]++;
}

static int64_t max_len(const go_seqs *s) {
    int64_t m = 0;
    for (int32_t n = 0; n < s->n; ++n) {
        int64_t L = s->off[n + 1] - s->off[n];
        if (L > m) m = L;
    }
    return m;
}

static void store_pick(const cat_t *p, int32_t n, int32_t *out_cnt, int32_t *out_pos,
                       int32_t out_cap, double *out_pwms) {
    out_pwms[n] = p->pwms;
    int32_t c = p->npos < out_cap ? p->npos : out_cap;
    out_cnt[n] = c;
    for (int i = 0; i < c; ++i) out_pos[(int64_t)n * out_cap + i] = p->pos[i];
}

/* ------------------------------------------------------ faithful O(N^2) sweep */
int go_sweep_faithful(const go_seqs *s, int32_t motif_amount, int32_t W, double pc, double cutoff,
                      const int32_t *in_cnt, const int32_t *in_pos, int32_t in_cap,
                      const double *u, int32_t t0, int32_t t1,
                      int32_t *out_cnt, int32_t *out_pos, int32_t out_cap, double *out_pwms,
                      double *margin, int32_t *err_index) {
    int rc = go_validate(s, W);
    if (rc) return rc;
    if (motif_amount < 1 || motif_amount > GO_MAXM || out_cap < motif_amount) return GO_E_ARG;
    if ((rc = check_positions(s, W, in_cnt, in_pos, in_cap))) return rc;
    int32_t aidx[NSLOT];
    alpha_map(s, aidx);
    const int32_t A = s->A;
    int64_t Lmax = max_len(s);
    scratch_t sc = {(double *)malloc(sizeof(double) * (size_t)Lmax),
                    (double *)malloc(sizeof(double) * (size_t)Lmax), {0}};
    int64_t *pfm = (int64_t *)malloc(sizeof(int64_t) * NSLOT * (size_t)W);
    int64_t *seg = (int64_t *)malloc(sizeof(int64_t) * NSLOT * (size_t)W);
    int64_t *Cn = (int64_t *)malloc(sizeof(int64_t) * (size_t)A * W);
    rc = GO_OK;
    for (int32_t n = t0; n < t1 && rc == GO_OK; ++n) {
        /* background: Array.map2 createFCVWithout over the others' positions, then
         * fuseFrequencyVectors over the alphabet (.fs:945-952, .fs:65-76) */
        int64_t bgc[NSLOT] = {0};
        for (int32_t m = 0; m < s->n; ++m) {
            if (m == n) continue;
            const uint8_t *sm = s->codes + s->off[m];
            int64_t Lm = s->off[m + 1] - s->off[m];
            for (int i = 0; i < in_cnt[m]; ++i) {
                int32_t p = in_pos[(int64_t)m * in_cap + i];
                int64_t fcv[NSLOT] = {0};
                comp49(sm, p, fcv);                      /* resSource.[0..(position-1)] */
                comp49(sm + p + W, Lm - p - W, fcv);     /* resSource.[(position+W)..]  */
                for (int a = 0; a < A; ++a) {
                    int b = s->alphabet[a] - SLOT0;
                    bgc[b] += fcv[b];
                }
            }
        }
        /* increaseInPlaceFCVOf sources.[n] (.fs:953): all 49 slots */
        comp49(s->codes + s->off[n], s->off[n + 1] - s->off[n], bgc);
        /* PFM: createPFMOf per segment, fusePositionFrequencyMatrices (.fs:955-962) */
        memset(pfm, 0, sizeof(int64_t) * NSLOT * (size_t)W);
        for (int32_t m = 0; m < s->n; ++m) {
            if (m == n) continue;
            const uint8_t *sm = s->codes + s->off[m];
            for (int i = 0; i < in_cnt[m]; ++i) {
                int32_t p = in_pos[(int64_t)m * in_cap + i];
                memset(seg, 0, sizeof(int64_t) * NSLOT * (size_t)W);
                for (int j = 0; j < W; ++j) seg[(sm[p + j] - SLOT0) * W + j] += 1;
                for (int c = 0; c < NSLOT * W; ++c) pfm[c] += seg[c];
            }
        }
        for (int a = 0; a < A; ++a)
            for (int j = 0; j < W; ++j) Cn[a * W + j] = pfm[(s->alphabet[a] - SLOT0) * W + j];
        cat_t pick;
        double mg = 0;
        rc = score_target(s, aidx, n, W, pc, cutoff, motif_amount, bgc, NULL, Cn, u[n], 0, 1, &sc,
                          &pick, &mg);
        if (rc) {
            if (err_index) *err_index = n;
            break;
        }
        if (margin) margin[n] = mg;
        store_pick(&pick, n, out_cnt, out_pos, out_cap, out_pwms);
    }
    free(sc.S);
    free(sc.G);
    free(sc.cats.v);
    free(pfm);
    free(seg);
    free(Cn);
    return rc;
}

/* ------------------------------------------------------- aggregates */
int go_counts(const go_seqs *s, int32_t W, const int32_t *in_cnt, const int32_t *in_pos,
              int32_t in_cap, int64_t *C, int64_t *T) {
    int rc = go_validate(s, W);
    if (rc) return rc;
    if ((rc = check_positions(s, W, in_cnt, in_pos, in_cap))) return rc;
    int32_t aidx[NSLOT];
    alpha_map(s, aidx);
    memset(C, 0, sizeof(int64_t) * (size_t)s->A * W);
    memset(T, 0, sizeof(int64_t) * (size_t)s->A);
    for (int32_t m = 0; m < s->n; ++m) {
        const uint8_t *sm = s->codes + s->off[m];
        int64_t Lm = s->off[m + 1] - s->off[m];
        int64_t comp[NSLOT] = {0};
        comp49(sm, Lm, comp);
        for (int i = 0; i < in_cnt[m]; ++i) {
            int32_t p = in_pos[(int64_t)m * in_cap + i];
            int64_t sc[NSLOT] = {0};
            comp49(sm + p, W, sc);
            for (int a = 0; a < s->A; ++a) {
                int b = s->alphabet[a] - SLOT0;
                T[a] += comp[b] - sc[b];
            }
            for (int j = 0; j < W; ++j) {
                int a = aidx[sm[p + j] - SLOT0];
                if (a >= 0) C[a * W + j] += 1;
            }
        }
    }
    return GO_OK;
}

/* hold-one-out aggregates for target n (SURVEY §8(a) identities, generalised to lists) */
static void holdout(const go_seqs *s, const int32_t *aidx, int32_t W, const int64_t *C,
                    const int64_t *T, const int32_t *in_cnt, const int32_t *in_pos,
                    int32_t in_cap, int32_t n, int64_t *bgc, int64_t *Cn) {
    const uint8_t *sn = s->codes + s->off[n];
    int64_t Ln = s->off[n + 1] - s->off[n];
    int64_t comp[NSLOT] = {0};
    comp49(sn, Ln, comp);
    for (int b = 0; b < NSLOT; ++b) bgc[b] = comp[b];
    for (int a = 0; a < s->A; ++a) bgc[s->alphabet[a] - SLOT0] += T[a];
    memcpy(Cn, C, sizeof(int64_t) * (size_t)s->A * W);
    for (int i = 0; i < in_cnt[n]; ++i) {
        int32_t p = in_pos[(int64_t)n * in_cap + i];
        int64_t sc[NSLOT] = {0};
        comp49(sn + p, W, sc);
        for (int a = 0; a < s->A; ++a) {
            int b = s->alphabet[a] - SLOT0;
            bgc[b] -= comp[b] - sc[b];
        }
        for (int j = 0; j < W; ++j) {
            int a = aidx[sn[p + j] - SLOT0];
            if (a >= 0) Cn[a * W + j] -= 1;
        }
    }
}

int go_sweep_fast(const go_seqs *s, int32_t motif_amount, int32_t W, double pc, double cutoff,
                  const int32_t *in_cnt, const int32_t *in_pos, int32_t in_cap,
                  const double *u, int32_t t0, int32_t t1,
                  int32_t *out_cnt, int32_t *out_pos, int32_t out_cap, double *out_pwms,
                  double *margin, int32_t *err_index, int32_t threads) {
    int rc = go_validate(s, W);
    if (rc) return rc;
    if (motif_amount < 1 || motif_amount > GO_MAXM || out_cap < motif_amount) return GO_E_ARG;
    if ((rc = check_positions(s, W, in_cnt, in_pos, in_cap))) return rc;
    int32_t aidx[NSLOT];
    alpha_map(s, aidx);
    const int32_t A = s->A;
    int64_t *C = (int64_t *)malloc(sizeof(int64_t) * (size_t)A * W);
    int64_t *T = (int64_t *)malloc(sizeof(int64_t) * (size_t)A);
    go_counts(s, W, in_cnt, in_pos, in_cap, C, T);
    int64_t Lmax = max_len(s);
    int32_t first_err = INT32_MAX, err_rc = GO_OK;
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel
#endif
    {
        scratch_t sc = {(double *)malloc(sizeof(double) * (size_t)Lmax),
                        (double *)malloc(sizeof(double) * (size_t)Lmax), {0}};
        int64_t *Cn = (int64_t *)malloc(sizeof(int64_t) * (size_t)A * W);
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 16)
#endif
        for (int32_t n = t0; n < t1; ++n) {
            int64_t bgc[NSLOT];
            holdout(s, aidx, W, C, T, in_cnt, in_pos, in_cap, n, bgc, Cn);
            cat_t pick;
            double mg = 0;
            int r = score_target(s, aidx, n, W, pc, cutoff, motif_amount, bgc, NULL, Cn, u[n], 0, 0,
                                 &sc, &pick, &mg);
            if (r) {
#ifdef _OPENMP
#pragma omp critical
#endif
                {
                    if (n < first_err) {
                        first_err = n;
                        err_rc = r;
                    }
                }
                continue;
            }
            if (margin) margin[n] = mg;
            store_pick(&pick, n, out_cnt, out_pos, out_cap, out_pwms);
        }
        free(sc.S);
        free(sc.G);
        free(sc.cats.v);
        free(Cn);
    }
    free(C);
    free(T);
    if (err_rc) {
        if (err_index) *err_index = first_err;
        return err_rc;
    }
    return GO_OK;
}

int go_sweep_shard(const go_seqs *s, int64_t n_global, int32_t W, double pc, double cutoff,
                   const int64_t *C, const int64_t *T, const int32_t *pos, const double *u,
                   int32_t *pos_out, double *pwms_out, int32_t *err_index) {
    int rc = go_validate(s, W);
    if (rc) return rc;
    int32_t *cnt = (int32_t *)malloc(sizeof(int32_t) * (size_t)(s->n ? s->n : 1));
    int32_t *p0 = (int32_t *)malloc(sizeof(int32_t) * (size_t)(s->n ? s->n : 1));
    for (int32_t n = 0; n < s->n; ++n) {
        cnt[n] = pos[n] >= 0;
        p0[n] = pos[n] >= 0 ? pos[n] : 0;
    }
    if ((rc = check_positions(s, W, cnt, p0, 1))) goto out;
    {
        int32_t aidx[NSLOT];
        alpha_map(s, aidx);
        /* the shard sees the global N in normalizePPM (.fs:964) */
        go_seqs g = *s;
        g.n = (int32_t)n_global;
        int64_t Lmax = max_len(s);
        scratch_t sc = {(double *)malloc(sizeof(double) * (size_t)Lmax),
                        (double *)malloc(sizeof(double) * (size_t)Lmax), {0}};
        int64_t *Cn = (int64_t *)malloc(sizeof(int64_t) * (size_t)s->A * W);
        for (int32_t n = 0; n < s->n && rc == GO_OK; ++n) {
            int64_t bgc[NSLOT];
            holdout(s, aidx, W, C, T, cnt, p0, 1, n, bgc, Cn);
            cat_t pick;
            /* score_target reads sequence n through the shard view but N from g */
            g.codes = s->codes;
            g.off = s->off;
            rc = score_target(&g, aidx, n, W, pc, cutoff, 1, bgc, NULL, Cn, u[n], 0, 0, &sc, &pick,
                              NULL);
            if (rc) {
                if (err_index) *err_index = n;
                break;
            }
            pos_out[n] = pick.npos ? pick.pos[0] : -1;
            pwms_out[n] = pick.pwms;
        }
        free(sc.S);
        free(sc.G);
        free(sc.cats.v);
        free(Cn);
    }
out:
    free(cnt);
    free(p0);
    return rc;
}

int go_target_detail(const go_seqs *s, int32_t W, double pc,
                     const int32_t *in_cnt, const int32_t *in_pos, int32_t in_cap, int32_t n,
                     int64_t *bgc_out, double *pcv_out, double *pwm_out, double *S, double *G) {
    int rc = go_validate(s, W);
    if (rc) return rc;
    if ((rc = check_positions(s, W, in_cnt, in_pos, in_cap))) return rc;
    if (n < 0 || n >= s->n) return GO_E_ARG;
    int32_t aidx[NSLOT];
    alpha_map(s, aidx);
    const int32_t A = s->A;
    int64_t *C = (int64_t *)malloc(sizeof(int64_t) * (size_t)A * W);
    int64_t *Cn = (int64_t *)malloc(sizeof(int64_t) * (size_t)A * W);
    int64_t T[NSLOT];
    go_counts(s, W, in_cnt, in_pos, in_cap, C, T);
    int64_t bgc[NSLOT];
    holdout(s, aidx, W, C, T, in_cnt, in_pos, in_cap, n, bgc, Cn);
    int64_t tot = 0;
    for (int b = 0; b < NSLOT; ++b) tot += bgc[b];
    double sum = (double)tot + (double)A * pc;
    double pcv[NSLOT];
    for (int b = 0; b < NSLOT; ++b) pcv[b] = (double)bgc[b];
    for (int a = 0; a < A; ++a) {
        int b = s->alphabet[a] - SLOT0;
        pcv[b] = (pcv[b] + pc) / sum;
    }
    double den = (double)(s->n - 1) + (double)A * pc;
    double pwm49[NSLOT * 64];
    if (W > 64) {
        free(C);
        free(Cn);
        return GO_E_ARG;
    }
    memset(pwm49, 0, sizeof(pwm49));
    for (int a = 0; a < A; ++a) {
        int b = s->alphabet[a] - SLOT0;
        for (int j = 0; j < W; ++j) {
            double ppm = ((double)Cn[a * W + j] + pc) / den;
            pwm49[b * W + j] = ppm / pcv[b];
            if (pwm_out) pwm_out[a * W + j] = pwm49[b * W + j];
        }
    }
    const uint8_t *src = s->codes + s->off[n];
    int64_t K = s->off[n + 1] - s->off[n] - W + 1;
    for (int64_t k = 0; k < K; ++k) {
        double sv = 1.0, gv = 1.0;
        for (int j = 0; j < W; ++j) {
            int b = src[k + j] - SLOT0;
            sv = sv * pwm49[b * W + j];
            gv = gv * pcv[b];
        }
        if (S) S[k] = sv;
        if (G) G[k] = gv;
    }
    if (bgc_out) memcpy(bgc_out, bgc, sizeof(bgc));
    if (pcv_out) memcpy(pcv_out, pcv, sizeof(pcv));
    free(C);
    free(Cn);
    return GO_OK;
}

/* ------------------------------------------------------- site sampler pieces */
int go_best_pwms(const go_seqs *s, int32_t W, double pc, int32_t n, const int64_t *fcv49,
                 const double *ppm, double *score, int32_t *pos) {
    if (n < 0 || n >= s->n) return GO_E_ARG;
    const uint8_t *src = s->codes + s->off[n];
    const int64_t L = s->off[n + 1] - s->off[n];
    const int32_t A = s->A;
    int32_t aidx[NSLOT];
    alpha_map(s, aidx);
    int64_t fcv[NSLOT]; /* the caller's fcVector, mutated in place across windows (Q1) */
    memcpy(fcv, fcv49, sizeof(fcv));
    double high = 0.0;
    int32_t hi = 0;
    for (int64_t k = 0; k + W <= L; ++k) {
        /* increaseInPlaceFCVOf source fcVector (.fs:471, .fs:79-81) */
        for (int64_t i = 0; i < L; ++i) fcv[src[i] - SLOT0] += 1;
        /* substractSegmentCountsFrom segment (.fs:472, .fs:84-88): aliased array */
        for (int j = 0; j < W; ++j) {
            int b = src[k + j] - SLOT0;
            fcv[b] = (fcv[b] - 1 > 0) ? fcv[b] - 1 : 0;
        }
        /* createNormalizedPCVOfFCV (.fs:473, .fs:115-120) */
        int64_t tot = 0;
        for (int b = 0; b < NSLOT; ++b) tot += fcv[b];
        if (tot > INT32_MAX) return GO_E_OVERFLOW;
        double sum = (double)tot + (double)A * pc;
        /* createPositionWeightMatrix + calculateSegmentScoreBy (.fs:474-476) */
        double sv = 1.0;
        for (int j = 0; j < W; ++j) {
            int b = src[k + j] - SLOT0;
            int a = aidx[b];
            double w = 0.0;
            if (a >= 0) {
                double pcv = ((double)fcv[b] + pc) / sum;
                w = ppm[a * W + j] / pcv;
            }
            sv = sv * w;
        }
        if (sv > high) { /* strict '>' (.fs:477) */
            high = sv;
            hi = (int32_t)k;
        }
    }
    *score = go_log2(high);
    *pos = hi;
    return GO_OK;
}

/* SiteSampler.getBestPWMSsWithBPV (.fs:301-313): the caller's pcv (49 slots), no
 * background drift; pwm = ppm / pcv over the alphabet, 0 elsewhere; first maximum. */
int go_best_pwms_bpv(const go_seqs *s, int32_t W, int32_t n, const double *pcv49,
                     const double *ppm, double *score, int32_t *pos) {
    if (n < 0 || n >= s->n) return GO_E_ARG;
    const uint8_t *src = s->codes + s->off[n];
    const int64_t L = s->off[n + 1] - s->off[n];
    int32_t aidx[NSLOT];
    alpha_map(s, aidx);
    double high = 0.0;
    int32_t hi = 0;
    for (int64_t k = 0; k + W <= L; ++k) {
        double sv = 1.0;
        for (int j = 0; j < W; ++j) {
            const int b = src[k + j] - SLOT0, a = aidx[b];
            sv = sv * (a >= 0 ? ppm[a * W + j] / pcv49[b] : 0.0);
        }
        if (sv > high) { /* strict '>' (.fs:312) */
            high = sv;
            hi = (int32_t)k;
        }
    }
    *score = go_log2(high);
    *pos = hi;
    return GO_OK;
}

/* A caller's PositionProbabilityMatrix (49 slot rows x W) in alphabet order. */
static void ppm_from_slots(const go_seqs *s, int32_t W, const double *ppm49, double *ppm) {
    for (int a = 0; a < s->A; ++a)
        for (int j = 0; j < W; ++j) ppm[a * W + j] = ppm49[(s->alphabet[a] - SLOT0) * W + j];
}

int go_random_starts(const go_seqs *s, int32_t W, double pc, const int32_t *draws,
                     uint64_t seed, int32_t mode, int32_t t0, int32_t t1,
                     double *score, int32_t *pos) {
    return go_random_starts_ex(s, W, pc, draws, seed, mode, t0, t1, NULL, NULL, score, pos);
}

int go_random_starts_ex(const go_seqs *s, int32_t W, double pc, const int32_t *draws,
                     uint64_t seed, int32_t mode, int32_t t0, int32_t t1,
                        const double *pcv49, const double *ppm49, double *score, int32_t *pos) {
    int rc = go_validate(s, W);
    if (rc) return rc;
    const int32_t N = s->n, A = s->A;
    int32_t aidx[NSLOT];
    alpha_map(s, aidx);
    double den = (double)(N - 1) + (double)A * pc;
    int64_t *pfm = (int64_t *)malloc(sizeof(int64_t) * (size_t)A * W);
    double *ppm = (double *)malloc(sizeof(double) * (size_t)A * W);
    for (int32_t n = t0; n < t1; ++n) {
        int64_t bg[NSLOT] = {0};
        memset(pfm, 0, sizeof(int64_t) * (size_t)A * W);
        for (int32_t m = 0; m < N; ++m) {
            if (m == n) continue;
            const uint8_t *sm = s->codes + s->off[m];
            int64_t Lm = s->off[m + 1] - s->off[m];
            int32_t r;
            if (draws) {
                r = draws[(int64_t)n * N + m];
                if (r < 0 || r + W > Lm) {
                    rc = GO_E_ARG;
                    goto done;
                }
            } else {
                uint64_t st = mode == 0 ? go_stream_init((uint64_t)n) : go_stream_init_shared();
                r = go_uniform_int(seed, st, (uint64_t)m, (int32_t)(Lm - W + 1));
            }
            int64_t fcv[NSLOT] = {0};
            comp49(sm, r, fcv);
            comp49(sm + r + W, Lm - r - W, fcv);
            for (int a = 0; a < A; ++a) bg[s->alphabet[a] - SLOT0] += fcv[s->alphabet[a] - SLOT0];
            for (int j = 0; j < W; ++j) {
                int a = aidx[sm[r + j] - SLOT0];
                if (a >= 0) pfm[a * W + j] += 1;
            }
        }
        if (ppm49) /* getMotifsWithBestPWMSOfPPM (.fs:644-662): the caller's PPM */
            ppm_from_slots(s, W, ppm49, ppm);
        else
            for (int c = 0; c < A * W; ++c) ppm[c] = ((double)pfm[c] + pc) / den;
        if (pcv49) /* getPWMOfRandomStartsWithBPV (.fs:412-431) */
            rc = go_best_pwms_bpv(s, W, n, pcv49, ppm, &score[n], &pos[n]);
        else
            rc = go_best_pwms(s, W, pc, n, bg, ppm, &score[n], &pos[n]);
        if (rc) goto done;
    }
done:
    free(pfm);
    free(ppm);
    return rc;
}

/* The getBestPWMSs inputs of target n with every other sequence m at start r[m]
 * (.fs:565-577 and twins): createFCVWithout + fuseFrequencyVectors over the
 * alphabet (bg, 49 slots), createPFMOf + fusePositionFrequencyMatrices +
 * createPPMOf + normalizePPM with N-1 (ppm, A*W alphabet order). */
static int site_inputs(const go_seqs *s, int32_t W, double pc, int32_t n, const int32_t *r,
                       const int32_t *aidx, int64_t *bg, int64_t *pfm, double *ppm) {
    const int32_t N = s->n, A = s->A;
    memset(bg, 0, sizeof(int64_t) * NSLOT);
    memset(pfm, 0, sizeof(int64_t) * (size_t)A * W);
    for (int32_t m = 0; m < N; ++m) {
        if (m == n) continue;
        const uint8_t *sm = s->codes + s->off[m];
        const int64_t Lm = s->off[m + 1] - s->off[m];
        const int32_t p = r[m];
        if (p < 0 || p + W > Lm) return GO_E_ARG; /* getSegment / Array.skip (.fs:149-153) */
        int64_t fcv[NSLOT] = {0};
        comp49(sm, p, fcv);
        comp49(sm + p + W, Lm - p - W, fcv);
        for (int a = 0; a < A; ++a) bg[s->alphabet[a] - SLOT0] += fcv[s->alphabet[a] - SLOT0];
        for (int j = 0; j < W; ++j) {
            int a = aidx[sm[p + j] - SLOT0];
            if (a >= 0) pfm[a * W + j] += 1;
        }
    }
    const double den = (double)(N - 1) + (double)A * pc;
    for (int c = 0; c < A * W; ++c) ppm[c] = ((double)pfm[c] + pc) / den;
    return GO_OK;
}

int go_site_scan(const go_seqs *s, int32_t W, double pc, const int32_t *r, int32_t t0, int32_t t1,
                 double *score, int32_t *pos) {
    return go_site_scan_ex(s, W, pc, r, t0, t1, NULL, score, pos);
}

int go_site_refine(const go_seqs *s, int32_t W, double pc, int32_t shift, int32_t *pos,
                   double *score, int32_t max_passes, int32_t *passes_out) {
    return go_site_refine_ex(s, W, pc, shift, NULL, pos, score, max_passes, passes_out);
}

int go_site_scan_ex(const go_seqs *s, int32_t W, double pc, const int32_t *r, int32_t t0,
                    int32_t t1, const double *pcv49, double *score, int32_t *pos) {
    int rc = go_validate(s, W);
    if (rc) return rc;
    if (t0 < 0 || t1 > s->n || t0 > t1) return GO_E_ARG;
    int32_t aidx[NSLOT];
    alpha_map(s, aidx);
    int64_t bg[NSLOT];
    int64_t *pfm = (int64_t *)malloc(sizeof(int64_t) * (size_t)s->A * W);
    double *ppm = (double *)malloc(sizeof(double) * (size_t)s->A * W);
    for (int32_t n = t0; n < t1 && rc == GO_OK; ++n) {
        rc = site_inputs(s, W, pc, n, r, aidx, bg, pfm, ppm);
        if (rc == GO_OK)
            rc = pcv49 ? go_best_pwms_bpv(s, W, n, pcv49, ppm, &score[n], &pos[n])
                       : go_best_pwms(s, W, pc, n, bg, ppm, &score[n], &pos[n]);
    }
    free(pfm);
    free(ppm);
    return rc;
}

int go_site_refine_ex(const go_seqs *s, int32_t W, double pc, int32_t shift,
                      const double *pcv49, int32_t *pos, double *score, int32_t max_passes,
                      int32_t *passes_out) {
    int rc = go_validate(s, W);
    if (rc) return rc;
    if (shift < -1 || shift > 1 || max_passes < 1) return GO_E_ARG;
    const int32_t N = s->n;
    for (int32_t n = 0; n < N; ++n)
        if (pos[n] < 0 || pos[n] + W > s->off[n + 1] - s->off[n]) return GO_E_ARG;
    int32_t aidx[NSLOT];
    alpha_map(s, aidx);
    int64_t bg[NSLOT];
    int64_t *pfm = (int64_t *)malloc(sizeof(int64_t) * (size_t)s->A * W);
    double *ppm = (double *)malloc(sizeof(double) * (size_t)s->A * W);
    int32_t *best = (int32_t *)malloc(sizeof(int32_t) * (size_t)(N ? N : 1));
    int32_t *r = (int32_t *)malloc(sizeof(int32_t) * (size_t)(N ? N : 1));
    int32_t passes = 0;
    for (;;) {
        memcpy(best, pos, sizeof(int32_t) * (size_t)N); /* bestMotif = Array.copy acc */
        ++passes;
        if (shift != 0) {
            /* the others at the pass-start snapshot, shifted (.fs:489-492, .fs:525-527) */
            for (int32_t m = 0; m < N; ++m) {
                const int64_t Lm = s->off[m + 1] - s->off[m];
                if (shift > 0)
                    r[m] = best[m] <= Lm - W - 1 ? best[m] + 1 : best[m];
                else
                    r[m] = best[m] > 0 ? best[m] - 1 : best[m];
            }
        }
        for (int32_t n = 0; n < N; ++n) {
            /* getBestPWMSsWithStartPositions reads the live acc (.fs:560-562) */
            rc = site_inputs(s, W, pc, n, shift == 0 ? pos : r, aidx, bg, pfm, ppm);
            if (rc) goto done;
            double sc;
            int32_t p;
            /* ...WithBPV twins (.fs:318-409): the caller's pcv, no drift */
            rc = pcv49 ? go_best_pwms_bpv(s, W, n, pcv49, ppm, &sc, &p)
                       : go_best_pwms(s, W, pc, n, bg, ppm, &sc, &p);
            if (rc) goto done;
            if (sc > score[n]) { /* fst tmp > fst acc.[n] (.fs:579) */
                score[n] = sc;
                pos[n] = p;
            }
        }
        if (memcmp(best, pos, sizeof(int32_t) * (size_t)N) == 0 || passes >= max_passes) break;
    }
done:
    if (passes_out) *passes_out = passes;
    free(pfm);
    free(ppm);
    free(best);
    free(r);
    return rc;
}

/* go_site_refine (shift 0) with the others' aggregates kept by subtraction instead of
 * rebuilt per target (site_inputs): the same bg / pfm integers, so the same picks; the
 * timed CPU port of getBestPWMSsWithStartPositions (.fs:554-585).  Stops after t_limit
 * visits (t_limit <= 0: no limit). */
static void site_contrib(const go_seqs *s, const int32_t *aidx, int32_t W, int32_t m, int32_t p,
                         int64_t sign, int64_t *bg, int64_t *pfm) {
    const uint8_t *sm = s->codes + s->off[m];
    const int64_t Lm = s->off[m + 1] - s->off[m];
    int64_t fcv[NSLOT] = {0};
    comp49(sm, p, fcv);
    comp49(sm + p + W, Lm - p - W, fcv);
    for (int a = 0; a < s->A; ++a) bg[s->alphabet[a] - SLOT0] += sign * fcv[s->alphabet[a] - SLOT0];
    for (int j = 0; j < W; ++j) {
        const int a = aidx[sm[p + j] - SLOT0];
        if (a >= 0) pfm[a * W + j] += sign;
    }
}

int go_site_refine_fast(const go_seqs *s, int32_t W, double pc, int32_t *pos, double *score,
                        int32_t max_passes, int64_t t_limit, int32_t *passes_out,
                        int64_t *visits_out) {
    int rc = go_validate(s, W);
    if (rc) return rc;
    if (max_passes < 1) return GO_E_ARG;
    const int32_t N = s->n, A = s->A;
    for (int32_t n = 0; n < N; ++n)
        if (pos[n] < 0 || pos[n] + W > s->off[n + 1] - s->off[n]) return GO_E_ARG;
    int32_t aidx[NSLOT];
    alpha_map(s, aidx);
    int64_t bgAll[NSLOT] = {0}, bg[NSLOT];
    int64_t *pfmAll = (int64_t *)calloc((size_t)A * W, sizeof(int64_t));
    int64_t *pfm = (int64_t *)malloc(sizeof(int64_t) * (size_t)A * W);
    double *ppm = (double *)malloc(sizeof(double) * (size_t)A * W);
    int32_t *best = (int32_t *)malloc(sizeof(int32_t) * (size_t)(N ? N : 1));
    for (int32_t m = 0; m < N; ++m) site_contrib(s, aidx, W, m, pos[m], 1, bgAll, pfmAll);
    const double den = (double)(N - 1) + (double)A * pc;
    int32_t passes = 0;
    int64_t visits = 0;
    for (;;) {
        memcpy(best, pos, sizeof(int32_t) * (size_t)N);
        ++passes;
        for (int32_t n = 0; n < N; ++n) {
            if (t_limit > 0 && visits >= t_limit) goto done;
            ++visits;
            memcpy(bg, bgAll, sizeof bg);
            memcpy(pfm, pfmAll, sizeof(int64_t) * (size_t)A * W);
            site_contrib(s, aidx, W, n, pos[n], -1, bg, pfm);
            for (int c = 0; c < A * W; ++c) ppm[c] = ((double)pfm[c] + pc) / den;
            double sc;
            int32_t p;
            rc = go_best_pwms(s, W, pc, n, bg, ppm, &sc, &p);
            if (rc) goto done;
            if (sc > score[n]) { /* fst tmp > fst acc.[n] (.fs:579) */
                score[n] = sc;
                if (p != pos[n]) {
                    site_contrib(s, aidx, W, n, pos[n], -1, bgAll, pfmAll);
                    site_contrib(s, aidx, W, n, p, 1, bgAll, pfmAll);
                }
                pos[n] = p;
            }
        }
        if (memcmp(best, pos, sizeof(int32_t) * (size_t)N) == 0 || passes >= max_passes) break;
    }
done:
    if (passes_out) *passes_out = passes;
    if (visits_out) *visits_out = visits;
    free(pfmAll);
    free(pfm);
    free(ppm);
    free(best);
    return rc;
}

/* ------------------------------------------------------- greedy pass */
/* sign * (the contribution of sequence n's positions to the aggregates C, T) */
static void add_contrib(const go_seqs *s, const int32_t *aidx, int32_t W, int32_t n,
                        const int32_t *cnt, const int32_t *pos, int32_t cap, int64_t sign,
                        int64_t *C, int64_t *T) {
    const uint8_t *sn = s->codes + s->off[n];
    const int64_t Ln = s->off[n + 1] - s->off[n];
    int64_t comp[NSLOT] = {0};
    if (cnt[n] > 0) comp49(sn, Ln, comp);
    for (int i = 0; i < cnt[n]; ++i) {
        const int32_t p = pos[(int64_t)n * cap + i];
        int64_t sc[NSLOT] = {0};
        comp49(sn + p, W, sc);
        for (int a = 0; a < s->A; ++a) {
            const int b = s->alphabet[a] - SLOT0;
            T[a] += sign * (comp[b] - sc[b]);
        }
        for (int j = 0; j < W; ++j) {
            const int a = aidx[sn[p + j] - SLOT0];
            if (a >= 0) C[a * W + j] += sign;
        }
    }
}

/* go_greedy with the aggregates kept up to date by subtraction instead of rebuilt
 * per target: same picks, O(L*W) per target (the timed CPU port of the greedy). */
static int greedy_impl(const go_seqs *s, int32_t motif_amount, int32_t W, double pc,
                       double cutoff, const double *pcv_fixed, int32_t *cnt, int32_t *pos,
                       int32_t cap, double *pwms, int32_t max_passes, int32_t t_limit,
                       int32_t *passes_out, int64_t *visits_out);

int go_greedy_fast(const go_seqs *s, int32_t motif_amount, int32_t W, double pc, double cutoff,
                   int32_t *cnt, int32_t *pos, int32_t cap, double *pwms, int32_t max_passes,
                   int32_t t_limit, int32_t *passes_out, int64_t *visits_out) {
    return greedy_impl(s, motif_amount, W, pc, cutoff, NULL, cnt, pos, cap, pwms, max_passes,
                       t_limit, passes_out, visits_out);
}

int go_greedy_pcv(const go_seqs *s, int32_t W, double pc, double cutoff, const double *pcv49,
                  int32_t *pos, double *pwms, int32_t max_passes, int32_t *passes_out) {
    if (!pcv49) return GO_E_ARG;
    int32_t *cnt = (int32_t *)malloc(sizeof(int32_t) * (size_t)(s->n ? s->n : 1));
    for (int32_t n = 0; n < s->n; ++n) cnt[n] = pos[n] >= 0 ? 1 : 0;
    for (int32_t n = 0; n < s->n; ++n)
        if (pos[n] < 0) pos[n] = 0; /* unused slot of an empty position list */
    int rc = greedy_impl(s, 1, W, pc, cutoff, pcv49, cnt, pos, 1, pwms, max_passes, 0,
                         passes_out, NULL);
    for (int32_t n = 0; n < s->n; ++n)
        if (cnt[n] == 0) pos[n] = -1;
    free(cnt);
    return rc;
}

int go_sweep_pcv(const go_seqs *s, int32_t W, double pc, double cutoff, const double *pcv49,
                 const int32_t *pos, const double *u, int32_t *pos_out, double *pwms_out,
                 double *margin, int32_t *err_index) {
    int rc = go_validate(s, W);
    if (rc) return rc;
    if (!pcv49) return GO_E_ARG;
    const int32_t N = s->n, A = s->A;
    int32_t *cnt = (int32_t *)malloc(sizeof(int32_t) * (size_t)(N ? N : 1));
    int32_t *p1 = (int32_t *)malloc(sizeof(int32_t) * (size_t)(N ? N : 1));
    for (int32_t n = 0; n < N; ++n) {
        cnt[n] = pos[n] >= 0 ? 1 : 0;
        p1[n] = pos[n] >= 0 ? pos[n] : 0;
    }
    int32_t aidx[NSLOT];
    alpha_map(s, aidx);
    int64_t *C = (int64_t *)malloc(sizeof(int64_t) * (size_t)A * W);
    int64_t *Cn = (int64_t *)malloc(sizeof(int64_t) * (size_t)A * W);
    int64_t T[NSLOT];
    scratch_t sc = {(double *)malloc(sizeof(double) * (size_t)max_len(s)),
                    (double *)malloc(sizeof(double) * (size_t)max_len(s)), {0}};
    if ((rc = check_positions(s, W, cnt, p1, 1))) goto done;
    go_counts(s, W, cnt, p1, 1, C, T);
    /* findBestMotifPositionsWithStartPositionsByPCV (.fs:828-853): every target against
     * the snapshot, the caller's pcv for the PWM (.fs:845) and the categories (.fs:847) */
    for (int32_t n = 0; n < N; ++n) {
        int64_t bgc[NSLOT];
        holdout(s, aidx, W, C, T, cnt, p1, 1, n, bgc, Cn);
        cat_t pick;
        double mg = INFINITY;
        rc = score_target(s, aidx, n, W, pc, cutoff, 1, bgc, pcv49, Cn, u[n], 0, 0, &sc, &pick,
                          &mg);
        if (margin) margin[n] = mg;
        if (rc) {
            if (err_index) *err_index = n;
            goto done;
        }
        pos_out[n] = pick.npos ? pick.pos[0] : -1;
        pwms_out[n] = pick.pwms;
    }
done:
    free(cnt);
    free(p1);
    free(C);
    free(Cn);
    free(sc.S);
    free(sc.G);
    free(sc.cats.v);
    return rc;
}

static int greedy_impl(const go_seqs *s, int32_t motif_amount, int32_t W, double pc,
                       double cutoff, const double *pcv_fixed, int32_t *cnt, int32_t *pos,
                       int32_t cap, double *pwms, int32_t max_passes, int32_t t_limit,
                       int32_t *passes_out, int64_t *visits_out) {
    int rc = go_validate(s, W);
    if (rc) return rc;
    if (motif_amount < 1 || motif_amount > GO_MAXM || cap < motif_amount) return GO_E_ARG;
    if ((rc = check_positions(s, W, cnt, pos, cap))) return rc;
    const int32_t N = s->n, A = s->A;
    int32_t aidx[NSLOT];
    alpha_map(s, aidx);
    int64_t Lmax = max_len(s);
    scratch_t sc = {(double *)malloc(sizeof(double) * (size_t)Lmax),
                    (double *)malloc(sizeof(double) * (size_t)Lmax), {0}};
    int64_t *C = (int64_t *)malloc(sizeof(int64_t) * (size_t)A * W);
    int64_t *Cn = (int64_t *)malloc(sizeof(int64_t) * (size_t)A * W);
    int64_t T[NSLOT];
    go_counts(s, W, cnt, pos, cap, C, T);
    int32_t passes = 0;
    int64_t visits = 0;
    int moved = 1;
    while (moved && passes < max_passes) {
        moved = 0;
        ++passes;
        for (int32_t n = 0; n < N; ++n) {
            if (t_limit > 0 && visits >= t_limit) goto done; /* bounded timing sample */
            ++visits;
            int64_t bgc[NSLOT];
            holdout(s, aidx, W, C, T, cnt, pos, cap, n, bgc, Cn);
            cat_t pick;
            rc = score_target(s, aidx, n, W, pc, cutoff, motif_amount, bgc, pcv_fixed, Cn, 0.0, 1,
                              0, &sc, &pick, NULL);
            if (rc) goto done;
            if (pick.pwms > pwms[n]) { /* .fs:923 */
                int same = pick.npos == cnt[n];
                for (int i = 0; i < pick.npos && same; ++i)
                    same = pos[(int64_t)n * cap + i] == pick.pos[i];
                pwms[n] = pick.pwms;
                if (!same) {
                    add_contrib(s, aidx, W, n, cnt, pos, cap, -1, C, T);
                    cnt[n] = pick.npos;
                    for (int i = 0; i < pick.npos; ++i) pos[(int64_t)n * cap + i] = pick.pos[i];
                    add_contrib(s, aidx, W, n, cnt, pos, cap, +1, C, T);
                    moved = 1;
                }
            }
        }
    }
done:
    if (passes_out) *passes_out = passes;
    if (visits_out) *visits_out = visits;
    free(sc.S);
    free(sc.G);
    free(sc.cats.v);
    free(C);
    free(Cn);
    return rc;
}

int go_greedy(const go_seqs *s, int32_t motif_amount, int32_t W, double pc, double cutoff,
              int32_t *cnt, int32_t *pos, int32_t cap, double *pwms, int32_t max_passes,
              int32_t *passes_out) {
    int rc = go_validate(s, W);
    if (rc) return rc;
    if (motif_amount < 1 || motif_amount > GO_MAXM || cap < motif_amount) return GO_E_ARG;
    if ((rc = check_positions(s, W, cnt, pos, cap))) return rc;
    const int32_t N = s->n, A = s->A;
    int32_t aidx[NSLOT];
    alpha_map(s, aidx);
    int64_t Lmax = max_len(s);
    scratch_t sc = {(double *)malloc(sizeof(double) * (size_t)Lmax),
                    (double *)malloc(sizeof(double) * (size_t)Lmax), {0}};
    int64_t *C = (int64_t *)malloc(sizeof(int64_t) * (size_t)A * W);
    int64_t *Cn = (int64_t *)malloc(sizeof(int64_t) * (size_t)A * W);
    int64_t T[NSLOT];
    int32_t *best_cnt = (int32_t *)malloc(sizeof(int32_t) * (size_t)(N ? N : 1));
    int32_t *best_pos = (int32_t *)malloc(sizeof(int32_t) * (size_t)(N ? N : 1) * cap);
    int32_t passes = 0;
    for (;;) {
        memcpy(best_cnt, cnt, sizeof(int32_t) * (size_t)N);
        memcpy(best_pos, pos, sizeof(int32_t) * (size_t)N * cap);
        ++passes;
        for (int32_t n = 0; n < N; ++n) {
            /* others' positions come from the live acc (.fs:891-893): Gauss-Seidel */
            go_counts(s, W, cnt, pos, cap, C, T);
            int64_t bgc[NSLOT];
            holdout(s, aidx, W, C, T, cnt, pos, cap, n, bgc, Cn);
            cat_t pick;
            rc = score_target(s, aidx, n, W, pc, cutoff, motif_amount, bgc, NULL, Cn, 0.0, 1, 0, &sc,
                              &pick, NULL);
            if (rc) goto done;
            if (pick.pwms > pwms[n]) { /* .fs:923 */
                pwms[n] = pick.pwms;
                cnt[n] = pick.npos;
                for (int i = 0; i < pick.npos; ++i) pos[(int64_t)n * cap + i] = pick.pos[i];
            }
        }
        int same = 1;
        for (int32_t n = 0; n < N && same; ++n) {
            if (cnt[n] != best_cnt[n]) same = 0;
            for (int i = 0; i < cnt[n] && same; ++i)
                if (pos[(int64_t)n * cap + i] != best_pos[(int64_t)n * cap + i]) same = 0;
        }
        if (same || passes >= max_passes) break;
    }
done:
    if (passes_out) *passes_out = passes;
    free(sc.S);
    free(sc.G);
    free(sc.cats.v);
    free(C);
    free(Cn);
    free(best_cnt);
    free(best_pos);
    return rc;
}
