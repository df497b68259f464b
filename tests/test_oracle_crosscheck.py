"""The oracle pinned against itself: two independent restatements of GibbsSampling.fs.

oracle/gibbs_oracle.c (C, faithful O(N^2) and hold-one-out modes) and
oracle/gibbs_ref.py (pure-Python literal, list-based) must agree BIT FOR BIT on
every output, on small random inputs covering the reference's edge cases
(non-alphabet symbols, Positions = [], ragged lengths, |A| = 4/5/20, L == W).
"""
import zlib

import numpy as np
import pytest

from conftest import init_positions, make_dataset
from oracle import gibbs_ref as gr
from oracle import oracle_lib as ol


def as_lists(codes, offsets):
    return [list(codes[offsets[i]:offsets[i + 1]]) for i in range(len(offsets) - 1)]


CASES = [
    # N, L, W, alphabet, ragged, extra symbols, none_rate, pc, cutoff
    (12, 30, 6, b"ACGT", False, b"", 0.0, 1e-4, 1.0),
    (10, 40, 5, b"ATGC-", True, b"*", 0.2, 1e-4, 1.0),
    (9, 25, 4, b"ACGT", True, b"N*", 0.3, 0.5, 0.0),
    (6, 40, 8, b"ACDEFGHIKLMNPQRSTVWY", True, b"X*", 0.0, 1e-4, 1.0),
    (5, 7, 7, b"ACGT", False, b"", 0.0, 1e-4, 1.0),       # L == W: one window
    (1, 20, 5, b"ACGT", False, b"", 0.0, 1e-4, 1.0),      # N == 1
    (8, 30, 6, b"ACGT", False, b"", 0.0, 1e-4, -3.0),     # negative cut-off
]


@pytest.mark.parametrize("N,L,W,alpha,ragged,extra,none_rate,pc,cutoff", CASES)
def test_sweep_three_ways(N, L, W, alpha, ragged, extra, none_rate, pc, cutoff):
    seed = zlib.crc32(repr((N, L, W, alpha)).encode()) & 0xffff  # stable across processes
    codes, offsets = make_dataset(N, L, W, alpha, seed=seed, ragged=ragged, extra=extra,
                                  extra_rate=0.05 if extra else 0.0)
    pos = init_positions(offsets, W, seed + 1, none_rate)
    u = np.random.default_rng(seed + 2).random(N)
    S = ol.Seqs(codes, offsets, alpha)
    try:
        p1, w1, m1 = ol.sweep(S, W, pc, cutoff, pos, u, faithful=True)
    except ol.OracleError as e:
        with pytest.raises(IndexError):
            mem = [(0.0, [int(p)] if p >= 0 else []) for p in pos]
            gr.findBestMotifIndicesByWithStartPositions(1, W, pc, cutoff, list(alpha),
                                                        as_lists(codes, offsets), mem, list(u))
        assert e.code == ol.GO_E_ROULETTE_OVERRUN
        return
    p2, w2, m2 = ol.sweep(S, W, pc, cutoff, pos, u, faithful=False)
    assert np.array_equal(p1, p2) and np.array_equal(w1, w2)
    mem = [(0.0, [int(p)] if p >= 0 else []) for p in pos]
    ref = gr.findBestMotifIndicesByWithStartPositions(1, W, pc, cutoff, list(alpha),
                                                      as_lists(codes, offsets), mem, list(u))
    assert [r[1][0] if r[1] else -1 for r in ref] == list(p1)
    assert [r[0] for r in ref] == list(w1)  # bitwise equal binary64


def test_motif_amount_two_matches_python():
    """calculatePWMsForSegmentCombinations with m = 2 (distance check, prefix pruning)."""
    N, L, W = 6, 36, 4
    codes, offsets = make_dataset(N, L, W, seed=5, mut=0.0)
    pos = init_positions(offsets, W, 6)
    u = np.random.default_rng(7).random(N)
    S = ol.Seqs(codes, offsets, b"ACGT")
    (cnt, p2), w, _ = ol.sweep(S, W, 1e-4, 0.5, pos, u, faithful=True, motif_amount=2)
    mem = [(0.0, [int(p)]) for p in pos]
    ref = gr.findBestMotifIndicesByWithStartPositions(2, W, 1e-4, 0.5, list(b"ACGT"),
                                                      as_lists(codes, offsets), mem, list(u))
    for n in range(N):
        assert ref[n][0] == w[n]
        assert list(ref[n][1]) == list(p2[n, :cnt[n]])


@pytest.mark.parametrize("M,cutoff,seed", [(3, 1.0, 15), (2, -2.0, 16), (4, 0.0, 17)])
def test_motif_amount_lists_match_python(M, cutoff, seed):
    """Positions lists in and out (0..M entries per sequence), M = 2..4, both C sweep
    modes and the greedy passes against the literal restatement."""
    N, L, W = 7, 40, 4
    codes, offsets = make_dataset(N, L, W, seed=seed, ragged=True, mut=0.0)
    S = ol.Seqs(codes, offsets, b"ACGT")
    rng = np.random.default_rng(seed + 1)
    lens = np.diff(offsets)
    cnt = rng.integers(0, M + 1, N).astype(np.int32)
    pos = np.full((N, M), -1, np.int32)
    for n in range(N):
        pos[n, :cnt[n]] = rng.integers(0, lens[n] - W + 1, cnt[n])
    u = rng.random(N)
    mem = [(0.0, [int(x) for x in pos[n, :cnt[n]]]) for n in range(N)]
    try:
        ref = gr.findBestMotifIndicesByWithStartPositions(M, W, 1e-4, cutoff, list(b"ACGT"),
                                                          as_lists(codes, offsets), mem, list(u))
    except IndexError:
        with pytest.raises(ol.OracleError):
            ol.sweep_lists(S, M, W, 1e-4, cutoff, cnt, pos, M, u)
        return
    for faithful in (True, False):
        c, p, w = ol.sweep_lists(S, M, W, 1e-4, cutoff, cnt, pos, M, u, faithful=faithful)
        assert [list(p[n, :c[n]]) for n in range(N)] == [list(r[1]) for r in ref]
        assert list(w) == [r[0] for r in ref]
    gc, gp, gw, _ = ol.greedy_lists(S, M, W, 1e-4, cutoff, c, p, M, w)
    rg = gr.findBestMotifIndicesWithStartPositions(M, W, 1e-4, cutoff, list(b"ACGT"),
                                                   as_lists(codes, offsets),
                                                   [(r[0], list(r[1])) for r in ref])
    assert [list(gp[n, :gc[n]]) for n in range(N)] == [list(r[1]) for r in rg]
    assert list(gw) == [r[0] for r in rg]


def test_counts_against_bruteforce():
    codes, offsets = make_dataset(50, 60, 7, seed=8, ragged=True, extra=b"*", extra_rate=0.02)
    pos = init_positions(offsets, 7, 9, 0.2)
    C, T = ol.counts(ol.Seqs(codes, offsets, b"ACGT"), 7, pos)
    Cb = np.zeros((4, 7), np.int64)
    Tb = np.zeros(4, np.int64)
    for n, p in enumerate(pos):
        if p < 0:
            continue
        s = codes[offsets[n]:offsets[n + 1]]
        seg = s[p:p + 7]
        for a, c in enumerate(b"ACGT"):
            Cb[a] += seg == c
            Tb[a] += (s == c).sum() - (seg == c).sum()
    assert np.array_equal(C, Cb) and np.array_equal(T, Tb)


@pytest.mark.parametrize("alpha,W,extra", [(b"ACGT", 5, b""), (b"ATGC-", 6, b"*"),
                                            (b"ACDEFGHIKLMNPQRSTVWY", 6, b"*")])
def test_random_starts_matches_python(alpha, W, extra):
    """getPWMOfRandomStarts + getBestPWMSs with the in-place background drift (Q1)."""
    N = 7
    codes, offsets = make_dataset(N, 30, W, alpha, seed=11, ragged=True, extra=extra,
                                  extra_rate=0.05 if extra else 0.0)
    S = ol.Seqs(codes, offsets, alpha)
    lens = np.diff(offsets)
    rng = np.random.default_rng(12)
    draws = np.zeros((N, N), np.int32)
    for n in range(N):
        for m in range(N):
            draws[n, m] = rng.integers(0, lens[m] - W + 1)
    sc, ps = ol.random_starts(S, W, 1e-4, draws=draws)
    ref = gr.getPWMOfRandomStarts(W, 1e-4, list(alpha), as_lists(codes, offsets),
                                  lambda n, m: int(draws[n, m]))
    assert [r[1] for r in ref] == list(ps)
    assert [r[0] for r in ref] == list(sc)


def test_random_starts_counter_rng_modes():
    """mode 0: fresh draws per target (reference structure); mode 1: one shared vector.
    Both equal the explicit-draw path with the same counter-RNG draws."""
    N, W = 9, 6
    codes, offsets = make_dataset(N, 40, W, seed=13, ragged=True)
    S = ol.Seqs(codes, offsets, b"ACGT")
    lens = np.diff(offsets)
    for mode in (0, 1):
        draws = np.zeros((N, N), np.int32)
        for n in range(N):
            for m in range(N):
                st = ol.stream_init(n) if mode == 0 else ol.STREAM_INIT_SHARED
                draws[n, m] = ol.uniform_int(99, st, m, int(lens[m]) - W + 1)
        a = ol.random_starts(S, W, 1e-4, seed=99, mode=mode)
        b = ol.random_starts(S, W, 1e-4, draws=draws)
        assert np.array_equal(a[1], b[1]) and np.array_equal(a[0], b[0])


def test_greedy_matches_python():
    """findBestMotifIndicesWithStartPositions: Gauss-Seidel passes to convergence."""
    N, W = 8, 6
    codes, offsets = make_dataset(N, 30, W, seed=17, mut=0.1)
    pos = init_positions(offsets, W, 18)
    S = ol.Seqs(codes, offsets, b"ACGT")
    gp, gw, passes = ol.greedy(S, W, 1e-4, 1.0, pos, np.zeros(N))
    mem = [(0.0, [int(p)]) for p in pos]
    ref = gr.findBestMotifIndicesWithStartPositions(1, W, 1e-4, 1.0, list(b"ACGT"),
                                                    as_lists(codes, offsets), mem)
    assert [r[1][0] if r[1] else -1 for r in ref] == list(gp)
    assert [r[0] for r in ref] == list(gw)
    assert passes >= 1


@pytest.mark.parametrize("seed,none_rate", [(0, 0.0), (1, 0.3), (2, 0.0)])
def test_greedy_fast_equals_greedy(seed, none_rate):
    """The incremental CPU port makes the same picks as the per-target rebuild."""
    N, W = 60, 7
    codes, offsets = make_dataset(N, 50, W, seed=31 + seed, ragged=True, mut=0.2)
    pos = init_positions(offsets, W, 32 + seed, none_rate)
    S = ol.Seqs(codes, offsets, b"ACGT")
    a = ol.greedy(S, W, 1e-4, 1.0, pos, np.zeros(N))
    b = ol.greedy_fast(S, W, 1e-4, 1.0, pos, np.zeros(N))
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]) and a[2] == b[2]
    assert b[3] == b[2] * N


@pytest.mark.parametrize("shift,alpha,extra", [(0, b"ACGT", b""), (-1, b"ACGT", b""),
                                               (1, b"ACGT", b""), (0, b"ATGC-", b"*"),
                                               (1, b"ACDEFGHIKLMNPQRSTVWY", b"*")])
def test_site_refine_matches_python(shift, alpha, extra):
    """getBestPWMSsWithStartPositions and the +-1 shifted passes (.fs:483-585)."""
    N, W = 7, 5
    codes, offsets = make_dataset(N, 28, W, alpha, seed=23 + shift, ragged=True, mut=0.1,
                                  extra=extra, extra_rate=0.05 if extra else 0.0)
    S = ol.Seqs(codes, offsets, alpha)
    sc0, p0 = ol.random_starts(S, W, 1e-4, seed=5, mode=0)
    gp, gs, passes = ol.site_refine(S, W, 1e-4, shift, p0, sc0)
    fn = {0: gr.getBestPWMSsWithStartPositions, -1: gr.getLeftShiftedBestPWMSs,
          1: gr.getRightShiftedBestPWMSs}[shift]
    ref = fn(W, 1e-4, list(alpha), as_lists(codes, offsets),
             [(float(s), int(p)) for s, p in zip(sc0, p0)])
    assert [p for _, p in ref] == list(gp)
    assert [s for s, _ in ref] == list(gs)
    assert passes >= 1
    # one Jacobi scan at the final positions: nothing beats the refined scores
    if shift == 0:
        s2, p2 = ol.site_scan(S, W, 1e-4, gp)
        assert not np.any(s2 > gs)


@pytest.mark.parametrize("alpha,extra,seed", [(b"ACGT", b"", 0), (b"ATGC-", b"*", 1),
                                              (b"ACDEFGHIKLMNPQRSTVWY", b"*", 2)])
def test_site_refine_fast_equals_rebuild(alpha, extra, seed):
    """The incremental CPU port of getBestPWMSsWithStartPositions makes the same picks
    and scores as the per-target rebuild, and honours its visit limit."""
    N, W = 50, 6
    codes, offsets = make_dataset(N, 40, W, alpha, seed=61 + seed, ragged=True, mut=0.15,
                                  extra=extra, extra_rate=0.05 if extra else 0.0)
    S = ol.Seqs(codes, offsets, alpha)
    sc0, p0 = ol.random_starts(S, W, 1e-4, seed=9 + seed, mode=1)
    a = ol.site_refine(S, W, 1e-4, 0, p0, sc0)
    b = ol.site_refine_fast(S, W, 1e-4, p0, sc0)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]) and a[2] == b[2]
    assert b[3] == b[2] * N
    c = ol.site_refine_fast(S, W, 1e-4, p0, sc0, t_limit=17)
    assert c[3] == 17


def _pcv49(seed):
    return np.random.default_rng(seed).uniform(0.05, 0.5, 49)


@pytest.mark.parametrize("alpha,extra", [(b"ACGT", b""), (b"ATGC-", b"*")])
def test_fixed_pcv_ppm_initialisers_match_python(alpha, extra):
    """getPWMOfRandomStartsWithBPV (.fs:412-431) and getMotifsWithBestPWMSOfPPM
    (.fs:644-662) with explicit draws."""
    N, W = 7, 5
    codes, offsets = make_dataset(N, 30, W, alpha, seed=41, ragged=True, extra=extra,
                                  extra_rate=0.05 if extra else 0.0)
    S = ol.Seqs(codes, offsets, alpha)
    lens = np.diff(offsets)
    rng = np.random.default_rng(42)
    draws = np.array([[rng.integers(0, lens[m] - W + 1) for m in range(N)] for _ in range(N)],
                     np.int32)
    pcv = _pcv49(43)
    sc, ps = ol.random_starts(S, W, 1e-4, draws=draws, pcv49=pcv)
    ref = gr.getPWMOfRandomStartsWithBPV(W, 1e-4, list(alpha), as_lists(codes, offsets),
                                         list(pcv), lambda n, m: int(draws[n, m]))
    assert [r[1] for r in ref] == list(ps) and [r[0] for r in ref] == list(sc)
    ppm = np.random.default_rng(44).uniform(0.01, 1.0, (49, W))
    sc, ps = ol.random_starts(S, W, 1e-4, draws=draws, ppm49=ppm)
    ref = gr.getMotifsWithBestPWMSOfPPM(W, 1e-4, list(alpha), as_lists(codes, offsets),
                                        [list(r) for r in ppm], lambda n, m: int(draws[n, m]))
    assert [r[1] for r in ref] == list(ps) and [r[0] for r in ref] == list(sc)


@pytest.mark.parametrize("shift", [0, -1, 1])
def test_bpv_site_refine_matches_python(shift):
    """findBestMotifWithStartPosition / getLeft/RightShiftedBestPWMSsWithBPV."""
    N, W = 7, 5
    codes, offsets = make_dataset(N, 28, W, seed=45 + shift, ragged=True, mut=0.1)
    S = ol.Seqs(codes, offsets, b"ACGT")
    pcv = _pcv49(46)
    sc0, p0 = ol.random_starts(S, W, 1e-4, seed=5, mode=0, pcv49=pcv)
    gp, gs, _ = ol.site_refine(S, W, 1e-4, shift, p0, sc0, pcv49=pcv)
    fn = {0: gr.findBestMotifWithStartPosition, -1: gr.getLeftShiftedBestPWMSsWithBPV,
          1: gr.getRightShiftedBestPWMSsWithBPV}[shift]
    ref = fn(W, 1e-4, list(b"ACGT"), as_lists(codes, offsets), list(pcv),
             [(float(s), int(p)) for s, p in zip(sc0, p0)])
    assert [p for _, p in ref] == list(gp) and [s for s, _ in ref] == list(gs)


def test_pcv_motif_sampler_matches_python():
    """findBestMotifPositionsWithStartPositionsByPCV (.fs:828-853) and
    findBestMotifPositionsWithStartPositionByPCV (.fs:788-823), motifAmount = 1."""
    N, W = 8, 6
    codes, offsets = make_dataset(N, 30, W, seed=47, mut=0.1)
    S = ol.Seqs(codes, offsets, b"ACGT")
    pcv = _pcv49(48) / 4.0
    pos = init_positions(offsets, W, 49, 0.2)
    u = np.random.default_rng(50).random(N)
    mem = [(0.0, [int(p)] if p >= 0 else []) for p in pos]
    gp, gw, _ = ol.sweep_pcv(S, W, 1e-4, 1.0, pcv, pos, u)
    ref = gr.findBestMotifPositionsWithStartPositionsByPCV(1, W, 1e-4, 1.0, list(b"ACGT"),
                                                           as_lists(codes, offsets), list(pcv),
                                                           mem, list(u))
    assert [r[1][0] if r[1] else -1 for r in ref] == list(gp)
    assert [r[0] for r in ref] == list(gw)
    hp, hw, passes = ol.greedy_pcv(S, W, 1e-4, 1.0, pcv, gp, gw)
    ref2 = gr.findBestMotifPositionsWithStartPositionByPCV(
        1, W, 1e-4, 1.0, list(b"ACGT"), as_lists(codes, offsets), list(pcv),
        [(float(w), [int(p)] if p >= 0 else []) for p, w in zip(gp, gw)])
    assert [r[1][0] if r[1] else -1 for r in ref2] == list(hp)
    assert [r[0] for r in ref2] == list(hw) and passes >= 1


def test_best_pwms_drift_closed_form():
    """The closed form used by the GPU initialiser (fcv_k = bg0 + (k+1)comp - D_k)
    reproduces the literal in-place mutation of getBestPWMSs (.fs:471-472)."""
    codes, offsets = make_dataset(3, 40, 5, seed=19, extra=b"*", extra_rate=0.05)
    S = ol.Seqs(codes, offsets, b"ACGT")
    rng = np.random.default_rng(20)
    fcv = np.zeros(49, np.int64)
    for c in b"ACGT":
        fcv[c - 42] = rng.integers(50, 90)
    ppm = rng.random((4, 5)) * 0.5 + 0.1
    score, pos = ol.best_pwms(S, 5, 1e-4, 1, fcv, ppm)
    src = codes[offsets[1]:offsets[2]]
    L = len(src)
    comp = np.bincount(src - 42, minlength=49)
    best, bk = 0.0, 0
    D = np.zeros(49, np.int64)
    for k in range(L - 5 + 1):
        D += np.bincount(src[k:k + 5] - 42, minlength=49)
        f = fcv + (k + 1) * comp - D
        tot = float(f.sum()) + 4 * 1e-4
        s = 1.0
        for j in range(5):
            b = src[k + j]
            a = b"ACGT".find(bytes([b]))
            w = 0.0 if a < 0 else ppm[a, j] / ((float(f[b - 42]) + 1e-4) / tot)
            s = s * w
        if s > best:
            best, bk = s, k
    assert pos == bk and score == gr.log2(best)


def test_shard_sweep_equals_full_sweep():
    """The multi-GPU decomposition: per-shard partial aggregates summed, then each shard
    sweeps its own targets -> identical to the single-process sweep."""
    N, W = 40, 7
    codes, offsets = make_dataset(N, 50, W, seed=23, ragged=True)
    pos = init_positions(offsets, W, 24, 0.1)
    u = np.random.default_rng(25).random(N)
    full_p, full_w, _ = ol.sweep(ol.Seqs(codes, offsets, b"ACGT"), W, 1e-4, 1.0, pos, u)
    from gibbssampling_amd.dist import shard_bounds
    bounds = shard_bounds(np.diff(offsets), 3)
    parts = []
    for lo, hi in bounds:
        Sx = ol.Seqs(codes[offsets[lo]:offsets[hi]], offsets[lo:hi + 1] - offsets[lo], b"ACGT")
        parts.append((Sx, *ol.counts(Sx, W, pos[lo:hi])))
    Cg = sum(p[1] for p in parts)
    Tg = sum(p[2] for p in parts)
    out_p, out_w = [], []
    for (lo, hi), (Sx, _, _) in zip(bounds, parts):
        p, w = ol.sweep_shard(Sx, N, W, 1e-4, 1.0, Cg, Tg, pos[lo:hi], u[lo:hi])
        out_p.append(p)
        out_w.append(w)
    assert np.array_equal(np.concatenate(out_p), full_p)
    assert np.array_equal(np.concatenate(out_w), full_w)


def test_oracle_rejects_bad_inputs():
    codes, offsets = make_dataset(5, 20, 5, seed=29)
    S = ol.Seqs(codes, offsets, b"ACGT")
    pos = init_positions(offsets, 5, 30)
    bad = pos.copy()
    bad[2] = 17  # 17 + 5 > 20: getSegment's Array.take throws
    with pytest.raises(ol.OracleError):
        ol.sweep(S, 5, 1e-4, 1.0, bad, np.zeros(5))
    with pytest.raises(ol.OracleError):
        ol.sweep(S, 21, 1e-4, 1.0, pos, np.zeros(5))
    with pytest.raises(ol.OracleError):  # duplicate alphabet symbol
        ol.sweep(ol.Seqs(codes, offsets, b"ACGA"), 5, 1e-4, 1.0, pos, np.zeros(5))
