"""GPU parity of motifAmount >= 2: Positions lists and the
segment combinations of calculatePWMsForSegmentCombinations (.fs:727-742) in the
sweep (.fs:935-970), the greedy passes (.fs:885-929) and doMotifSampling
(.fs:1034-1038), through gs_*_multi, against the oracle (go_sweep_fast /
go_sweep_faithful / go_greedy with lists, cross-checked with the literal Python
restatement in tests/test_oracle_crosscheck.py).

Bar: list lengths and positions (in F# cons order) identical; PWMS within 1e-12
relative (the same binary64 operations; log() may differ in the last ulp between
the device library and glibc).  The reference's own motifAmount = 2 caller is
.fsx:407 (getMotifsWithBestInformationContents 1 2 6 0.0001 1. dnaBases
bioTestsWithMultipleSamples): test_fsx_multiple_samples_amount_two runs that data.
"""
import json
from pathlib import Path

import numpy as np
import pytest

from conftest import init_positions, make_dataset
from oracle import oracle_lib as ol

pytestmark = pytest.mark.gpu

RTOL = 1e-12
GOLDEN = Path(__file__).resolve().parent / "golden"


def random_lists(offsets, W, cap, seed, max_cnt=None):
    """Snapshots with 0..max_cnt positions per sequence (any in-bounds starts)."""
    rng = np.random.default_rng(seed)
    lens = np.diff(offsets)
    N = len(lens)
    max_cnt = cap if max_cnt is None else max_cnt
    cnt = rng.integers(0, max_cnt + 1, N).astype(np.int32)
    pos = np.full((N, cap), -1, np.int32)
    for n in range(N):
        pos[n, :cnt[n]] = rng.integers(0, lens[n] - W + 1, cnt[n])
    return cnt, pos


def check(g, o):
    gc, gp, gw = g[:3]
    oc, op, ow = o[:3]
    bad = np.nonzero(gc != oc)[0]
    assert bad.size == 0, f"list lengths differ at {bad[:10]}"
    for n in range(len(gc)):
        assert list(gp[n, :gc[n]]) == list(op[n, :oc[n]]), f"positions differ at {n}"
    same = gw == ow
    rel = np.abs(gw - ow) / np.maximum(np.abs(ow), 1e-300)
    assert np.all(same | (rel <= RTOL)), f"PWMS rel diff {np.nanmax(rel):.3e}"


SWEEPS = [
    # N, L, W, alphabet, ragged, extra, M, cutoff, seed
    (60, 50, 6, b"ACGT", False, b"", 2, 1.0, 1),
    (80, 90, 8, b"ACGT", True, b"", 2, 0.5, 2),
    (50, 70, 5, b"ACGT", True, b"N*", 3, 1.0, 3),
    (40, 120, 10, b"ACDEFGHIKLMNPQRSTVWY", True, b"X", 2, 1.0, 4),
    (30, 60, 4, b"ATGC-", False, b"*", 4, 2.0, 5),
    (25, 40, 6, b"ACGT", True, b"", 2, -3.0, 6),   # negative cut-off: serial roulette path
    (200, 200, 12, b"ACGT", False, b"", 2, 1.0, 7),
    (5, 12, 12, b"ACGT", False, b"", 2, 1.0, 8),   # L == W: one window, no pairs
]


@pytest.mark.parametrize("N,L,W,alpha,ragged,extra,M,cutoff,seed", SWEEPS)
def test_sweep_multi_matches_oracle(gpu_ctx, N, L, W, alpha, ragged, extra, M, cutoff, seed):
    codes, offsets = make_dataset(N, L, W, alpha, seed=seed, ragged=ragged, extra=extra,
                                  extra_rate=0.04 if extra else 0.0, mut=0.1)
    S = ol.Seqs(codes, offsets, alpha)
    cnt, pos = random_lists(offsets, W, M, seed + 100)
    u = np.random.default_rng(seed + 200).random(N)
    gpu_ctx.set_sequences(codes, offsets, alpha)
    try:
        o = ol.sweep_lists(S, M, W, 1e-4, cutoff, cnt, pos, M, u)
    except ol.OracleError as e:
        with pytest.raises(Exception) as ei:
            gpu_ctx.motif_sweep_multi(M, W, 1e-4, cutoff, cnt, pos, u)
        assert ei.value.status == e.code
        return
    g = gpu_ctx.motif_sweep_multi(M, W, 1e-4, cutoff, cnt, pos, u)
    check(g, o)


def test_sweep_multi_faithful_and_amount_one(gpu_ctx):
    """The list path at motifAmount = 1 equals the ★ sweep kernel; at 2 it equals the
    reference-faithful O(N^2) oracle."""
    N, L, W = 100, 50, 8
    codes, offsets = make_dataset(N, L, W, seed=31, mut=0.1)
    S = ol.Seqs(codes, offsets, b"ACGT")
    pos = init_positions(offsets, W, 32, 0.1)
    u = np.random.default_rng(33).random(N)
    gpu_ctx.set_sequences(codes, offsets, b"ACGT")
    p1, w1 = gpu_ctx.motif_sweep(W, 1e-4, 1.0, pos, u)
    cnt = (pos >= 0).astype(np.int32)
    lst = np.where(pos >= 0, pos, -1).reshape(N, 1).astype(np.int32)
    c2, p2, w2 = gpu_ctx.motif_sweep_multi(1, W, 1e-4, 1.0, cnt, lst, u)
    assert np.array_equal(np.where(c2 > 0, p2[:, 0], -1), p1)
    assert np.array_equal(w2, w1)
    cnt, lst = random_lists(offsets, W, 2, 34)
    g = gpu_ctx.motif_sweep_multi(2, W, 1e-4, 1.0, cnt, lst, u)
    o = ol.sweep_lists(S, 2, W, 1e-4, 1.0, cnt, lst, 2, u, faithful=True)
    check(g, o)


def test_sweep_multi_arena_growth(gpu_ctx):
    """Every window passes (cut-off -1000): the ~3.8k pairs of level 2 (the parents of
    the triples) overflow the first arena (2048 entries) and the targets are rescored
    with a larger one."""
    N, L, W = 12, 90, 2
    codes, offsets = make_dataset(N, L, W, seed=41, mut=0.0)
    S = ol.Seqs(codes, offsets, b"ACGT")
    cnt, pos = random_lists(offsets, W, 3, 42)
    u = np.random.default_rng(43).random(N)
    gpu_ctx.set_sequences(codes, offsets, b"ACGT")
    try:
        o = ol.sweep_lists(S, 3, W, 1e-4, -1000.0, cnt, pos, 3, u)
    except ol.OracleError as e:  # negative weights can run the wheel past its end
        with pytest.raises(Exception) as ei:
            gpu_ctx.motif_sweep_multi(3, W, 1e-4, -1000.0, cnt, pos, u)
        assert ei.value.status == e.code and ei.value.index == e.index
        return
    check(gpu_ctx.motif_sweep_multi(3, W, 1e-4, -1000.0, cnt, pos, u), o)


def test_sweep_multi_capacity_larger_than_amount(gpu_ctx):
    """Input lists longer than motifAmount (cap 3, M = 2) are counted in full."""
    N, L, W = 40, 60, 5
    codes, offsets = make_dataset(N, L, W, seed=51)
    S = ol.Seqs(codes, offsets, b"ACGT")
    cnt, pos = random_lists(offsets, W, 3, 52)
    u = np.random.default_rng(53).random(N)
    gpu_ctx.set_sequences(codes, offsets, b"ACGT")
    g = gpu_ctx.motif_sweep_multi(2, W, 1e-4, 1.0, cnt, pos, u, cap=3)
    o = ol.sweep_lists(S, 2, W, 1e-4, 1.0, cnt, pos, 3, u)
    check((g[0], g[1][:, :3], g[2]), (o[0], o[1][:, :3], o[2]))


def test_sweep_multi_rejects_bad_lists(gpu_ctx):
    N, L, W = 10, 30, 5
    codes, offsets = make_dataset(N, L, W, seed=61)
    gpu_ctx.set_sequences(codes, offsets, b"ACGT")
    cnt = np.ones(N, np.int32)
    pos = np.zeros((N, 2), np.int32)
    pos[3, 0] = L - W + 1  # Array.take past the end (getSegment, .fs:149-153)
    with pytest.raises(ValueError) as ei:
        gpu_ctx.motif_sweep_multi(2, W, 1e-4, 1.0, cnt, pos, np.zeros(N))
    assert ei.value.index == 3
    with pytest.raises(ValueError):
        gpu_ctx.motif_sweep_multi(17, W, 1e-4, 1.0, cnt, np.zeros((N, 17), np.int32), np.zeros(N))


GREEDY = [
    (60, 50, 6, b"ACGT", False, 2, 1.0, 11),
    (50, 80, 8, b"ACGT", True, 3, 1.0, 12),
    (30, 100, 10, b"ACDEFGHIKLMNPQRSTVWY", True, 2, 1.0, 13),
    (40, 40, 5, b"ACGT", True, 2, -1.0, 14),
]


@pytest.mark.parametrize("N,L,W,alpha,ragged,M,cutoff,seed", GREEDY)
def test_greedy_multi_matches_oracle(gpu_ctx, N, L, W, alpha, ragged, M, cutoff, seed):
    codes, offsets = make_dataset(N, L, W, alpha, seed=seed, ragged=ragged, mut=0.1)
    S = ol.Seqs(codes, offsets, alpha)
    cnt, pos = random_lists(offsets, W, M, seed + 100)
    u = np.random.default_rng(seed + 200).random(N)
    c1, p1, w1 = ol.sweep_lists(S, M, W, 1e-4, cutoff, cnt, pos, M, u)  # a sampled motifMem
    gpu_ctx.set_sequences(codes, offsets, alpha)
    g = gpu_ctx.motif_greedy_multi(M, W, 1e-4, cutoff, c1, p1, w1)
    o = ol.greedy_lists(S, M, W, 1e-4, cutoff, c1, p1, M, w1)
    check(g, o)
    assert g[3] == o[3]


def test_greedy_multi_pass_cap(gpu_ctx):
    N, L, W, M = 50, 60, 6, 2
    codes, offsets = make_dataset(N, L, W, seed=71, mut=0.2)
    S = ol.Seqs(codes, offsets, b"ACGT")
    cnt, pos = random_lists(offsets, W, M, 72)
    pw = np.zeros(N)
    gpu_ctx.set_sequences(codes, offsets, b"ACGT")
    for mp in (1, 2):
        g = gpu_ctx.motif_greedy_multi(M, W, 1e-4, 1.0, cnt, pos, pw, max_passes=mp)
        o = ol.greedy_lists(S, M, W, 1e-4, 1.0, cnt, pos, M, pw, max_passes=mp)
        check(g, o)
        assert g[3] == o[3] == mp


@pytest.mark.parametrize("M,init_mode,seed", [(2, 0, 81), (3, 1, 82)])
def test_motif_sampling_multi(gpu_ctx, M, init_mode, seed):
    """doMotifSampling (.fs:1034-1038) with motifAmount M against the oracle's
    composition with the same counter-RNG draws."""
    N, L, W = 60, 60, 6
    codes, offsets = make_dataset(N, L, W, seed=seed, mut=0.1)
    S = ol.Seqs(codes, offsets, b"ACGT")
    gpu_ctx.set_sequences(codes, offsets, b"ACGT")
    g = gpu_ctx.motif_sampling_multi(M, W, 1e-4, 1.0, seed, init_mode=init_mode)
    sc, p = ol.random_starts(S, W, 1e-4, seed=seed, mode=init_mode)
    u = np.array([ol.uniform(seed, ol.stream_sweep(0), n) for n in range(N)])
    cnt = np.ones(N, np.int32)
    lst = np.full((N, M), -1, np.int32)
    lst[:, 0] = p
    c1, p1, w1 = ol.sweep_lists(S, M, W, 1e-4, 1.0, cnt, lst, M, u)
    o = ol.greedy_lists(S, M, W, 1e-4, 1.0, c1, p1, M, w1)
    check(g, o)
    assert g[3] == o[3]


def test_fsx_multiple_samples_amount_two(gpu_ctx):
    """The reference driver's motifAmount = 2 call (.fsx:407) on its own data set
    (bioTestsWithMultipleSamples, .fsx:49-57, W = 6, pc 1e-4, cutOff 1): one
    doMotifSampling repetition on the device equals the oracle's."""
    sets = json.loads((GOLDEN / "fsx_sets.json").read_text())
    seqs = sets["bioTestsWithMultipleSamples"]["seqs"]
    alpha = b"ATGC-"  # dnaBases (.fsx:368-369)
    codes = np.frombuffer("".join(seqs).encode(), np.uint8).copy()
    offsets = np.zeros(len(seqs) + 1, np.int64)
    np.cumsum([len(s) for s in seqs], out=offsets[1:])
    S = ol.Seqs(codes, offsets, alpha)
    N, W, M = len(seqs), 6, 2
    gpu_ctx.set_sequences(codes, offsets, alpha)
    for seed in (1, 2, 3):
        g = gpu_ctx.motif_sampling_multi(M, W, 1e-4, 1.0, seed, init_mode=0)
        sc, p = ol.random_starts(S, W, 1e-4, seed=seed, mode=0)
        u = np.array([ol.uniform(seed, ol.stream_sweep(0), n) for n in range(N)])
        lst = np.full((N, M), -1, np.int32)
        lst[:, 0] = p
        c1, p1, w1 = ol.sweep_lists(S, M, W, 1e-4, 1.0, np.ones(N, np.int32), lst, M, u)
        check(g, ol.greedy_lists(S, M, W, 1e-4, 1.0, c1, p1, M, w1))


def _as_lists(codes, offsets):
    return [list(codes[offsets[i]:offsets[i + 1]]) for i in range(len(offsets) - 1)]


def test_mirror_sweep_and_greedy_amount_two_vs_literal():
    """The Python mirror (MotifSampler.*, same names and arguments as the F#) with
    motifAmount = 2 against the literal list-based restatement oracle/gibbs_ref.py."""
    from gibbssampling_amd.sampler import MotifSampler, createMotifIndex
    from oracle import gibbs_ref as gr
    N, L, W = 8, 36, 4
    codes, offsets = make_dataset(N, L, W, seed=91, mut=0.0)
    srcs = [bytes(codes[offsets[i]:offsets[i + 1]]).decode() for i in range(N)]
    cnt, pos = random_lists(offsets, W, 2, 92)
    mem = [createMotifIndex(0.0, pos[n, :cnt[n]]) for n in range(N)]
    u = np.random.default_rng(93).random(N)
    out = MotifSampler.findBestMotifIndicesByWithStartPositions(2, W, 1e-4, 0.5, "ACGT", srcs,
                                                                mem, u)
    ref = gr.findBestMotifIndicesByWithStartPositions(
        2, W, 1e-4, 0.5, list(b"ACGT"), _as_lists(codes, offsets),
        [(0.0, list(pos[n, :cnt[n]])) for n in range(N)], list(u))
    assert [list(m.Positions) for m in out] == [list(r[1]) for r in ref]
    assert all(abs(m.PWMS - r[0]) <= RTOL * abs(r[0]) for m, r in zip(out, ref))
    g = MotifSampler.findBestMotifIndicesWithStartPositions(2, W, 1e-4, 0.5, "ACGT", srcs, out)
    rg = gr.findBestMotifIndicesWithStartPositions(
        2, W, 1e-4, 0.5, list(b"ACGT"), _as_lists(codes, offsets),
        [(r[0], list(r[1])) for r in ref])
    assert [list(m.Positions) for m in g] == [list(r[1]) for r in rg]
    assert all(abs(m.PWMS - r[0]) <= RTOL * abs(r[0]) for m, r in zip(g, rg))


def test_mirror_bypcv_amount_two_vs_literal():
    """findBestMotifPositionsWithStartPositions(s)ByPCV (.fs:788-853) with motifAmount
    = 2: the caller's pcv in the list path, against the literal restatement."""
    from gibbssampling_amd.sampler import MotifSampler, createMotifIndex
    from oracle import gibbs_ref as gr
    N, L, W = 8, 40, 5
    codes, offsets = make_dataset(N, L, W, seed=95, mut=0.0)
    srcs = [bytes(codes[offsets[i]:offsets[i + 1]]).decode() for i in range(N)]
    pcv = np.zeros(49)
    for c, v in zip(b"ACGT", (0.3, 0.2, 0.2, 0.3)):
        pcv[c - 42] = v
    cnt, pos = random_lists(offsets, W, 2, 96)
    mem = [createMotifIndex(0.0, pos[n, :cnt[n]]) for n in range(N)]
    u = np.random.default_rng(97).random(N)
    out = MotifSampler.findBestMotifPositionsWithStartPositionsByPCV(2, W, 1e-4, 0.5, "ACGT", srcs,
                                                                     pcv, mem, u)
    ref = gr.findBestMotifPositionsWithStartPositionsByPCV(
        2, W, 1e-4, 0.5, list(b"ACGT"), _as_lists(codes, offsets), list(pcv),
        [(0.0, list(pos[n, :cnt[n]])) for n in range(N)], list(u))
    assert [list(m.Positions) for m in out] == [list(r[1]) for r in ref]
    assert all(abs(m.PWMS - r[0]) <= RTOL * abs(r[0]) for m, r in zip(out, ref))
    g = MotifSampler.findBestMotifPositionsWithStartPositionByPCV(2, W, 1e-4, 0.5, "ACGT", srcs,
                                                                  pcv, out)
    rg = gr.findBestMotifPositionsWithStartPositionByPCV(
        2, W, 1e-4, 0.5, list(b"ACGT"), _as_lists(codes, offsets), list(pcv),
        [(r[0], list(r[1])) for r in ref])
    assert [list(m.Positions) for m in g] == [list(r[1]) for r in rg]
    assert all(abs(m.PWMS - r[0]) <= RTOL * abs(r[0]) for m, r in zip(g, rg))


def test_mirror_fsx_407_call():
    """.fsx:407 through the mirror: getMotifsWithBestInformationContents 1 2 6 0.0001 1.
    dnaBases bioTestsWithMultipleSamples (seeded), against the oracle's composition of
    the same repetition loop."""
    from gibbssampling_amd.sampler import MotifSampler, _best_of_repetitions, createMotifIndex
    sets = json.loads((GOLDEN / "fsx_sets.json").read_text())
    seqs = sets["bioTestsWithMultipleSamples"]["seqs"]
    out = MotifSampler.getMotifsWithBestInformationContents(1, 2, 6, 0.0001, 1.0, "ATGC-", seqs,
                                                            seed=5)
    codes = np.frombuffer("".join(seqs).encode(), np.uint8).copy()
    offsets = np.zeros(len(seqs) + 1, np.int64)
    np.cumsum([len(s) for s in seqs], out=offsets[1:])
    S = ol.Seqs(codes, offsets, b"ATGC-")
    N, W, M = len(seqs), 6, 2

    def run(r):
        seed = 5 + r
        sc, p = ol.random_starts(S, W, 1e-4, seed=seed, mode=0)
        u = np.array([ol.uniform(seed, ol.stream_sweep(0), n) for n in range(N)])
        lst = np.full((N, M), -1, np.int32)
        lst[:, 0] = p
        c1, p1, w1 = ol.sweep_lists(S, M, W, 1e-4, 1.0, np.ones(N, np.int32), lst, M, u)
        c2, p2, w2, _ = ol.greedy_lists(S, M, W, 1e-4, 1.0, c1, p1, M, w1)
        return [createMotifIndex(w2[n], p2[n, :c2[n]]) for n in range(N)]
    ref = _best_of_repetitions(1, run, lambda xs: sum(x.PWMS for x in xs),
                               [createMotifIndex(0.0, [])])
    assert [m.Positions for m in out] == [m.Positions for m in ref]
    assert all(abs(a.PWMS - b.PWMS) <= RTOL * abs(b.PWMS) for a, b in zip(out, ref))


@pytest.mark.parametrize("threads", ["64", "1024"])
def test_greedy_multi_workgroup_sizes(threads, monkeypatch):
    """The greedy's workgroup (every wavefront scores the current target) gives the
    same passes at one and at sixteen wavefronts."""
    from gibbssampling_amd import Context
    tuning = {"multi_greedy_threads": float(threads)}
    ctx = Context(0, tuning=tuning)
    try:
        N, L, W, M = 40, 90, 6, 2
        codes, offsets = make_dataset(N, L, W, seed=101, mut=0.1)
        S = ol.Seqs(codes, offsets, b"ACGT")
        cnt, pos = random_lists(offsets, W, M, 102)
        u = np.random.default_rng(103).random(N)
        c1, p1, w1 = ol.sweep_lists(S, M, W, 1e-4, 1.0, cnt, pos, M, u)
        ctx.set_sequences(codes, offsets, b"ACGT")
        g = ctx.motif_greedy_multi(M, W, 1e-4, 1.0, c1, p1, w1)
        o = ol.greedy_lists(S, M, W, 1e-4, 1.0, c1, p1, M, w1)
        check(g, o)
        assert g[3] == o[3]
    finally:
        ctx.close()


@pytest.mark.parametrize("slots", ["1", "7", "64"])
def test_greedy_multi_speculation_widths(slots, monkeypatch):
    """The speculative greedy (visits scored in parallel, committed up to the first
    move) gives the sequential passes at any speculation width."""
    from gibbssampling_amd import Context
    tuning = {"multi_spec_slots": float(slots)}
    ctx = Context(0, tuning=tuning)
    try:
        N, L, W, M = 90, 70, 6, 2
        codes, offsets = make_dataset(N, L, W, seed=111, mut=0.1, ragged=True)
        S = ol.Seqs(codes, offsets, b"ACGT")
        cnt, pos = random_lists(offsets, W, M, 112)
        u = np.random.default_rng(113).random(N)
        c1, p1, w1 = ol.sweep_lists(S, M, W, 1e-4, 1.0, cnt, pos, M, u)
        ctx.set_sequences(codes, offsets, b"ACGT")
        g = ctx.motif_greedy_multi(M, W, 1e-4, 1.0, c1, p1, w1)
        o = ol.greedy_lists(S, M, W, 1e-4, 1.0, c1, p1, M, w1)
        check(g, o)
        assert g[3] == o[3]
    finally:
        ctx.close()


@pytest.mark.parametrize("N", [1, 2, 3])
def test_multi_tiny_sampler(gpu_ctx, N):
    """Edge sizes: one to three sequences (N - 1 = 0 others in normalizePPM at N = 1)."""
    L, W, M = 30, 5, 2
    codes, offsets = make_dataset(N, L, W, seed=120 + N, mut=0.0)
    S = ol.Seqs(codes, offsets, b"ACGT")
    cnt, pos = random_lists(offsets, W, M, 130 + N)
    u = np.random.default_rng(140 + N).random(N)
    gpu_ctx.set_sequences(codes, offsets, b"ACGT")
    try:
        o = ol.sweep_lists(S, M, W, 1e-4, 1.0, cnt, pos, M, u)
    except ol.OracleError as e:
        with pytest.raises(Exception) as ei:
            gpu_ctx.motif_sweep_multi(M, W, 1e-4, 1.0, cnt, pos, u)
        assert ei.value.status == e.code
        return
    g = gpu_ctx.motif_sweep_multi(M, W, 1e-4, 1.0, cnt, pos, u)
    check(g, o)
    gg = gpu_ctx.motif_greedy_multi(M, W, 1e-4, 1.0, g[0], g[1], g[2])
    og = ol.greedy_lists(S, M, W, 1e-4, 1.0, o[0], o[1], M, o[2])
    check(gg, og)
    assert gg[3] == og[3]


def test_list_greedy_amount_one_equals_star_greedy(gpu_ctx):
    """motifAmount = 1 through the list path's speculative greedy equals the ★ engine."""
    N, L, W = 300, 80, 8
    codes, offsets = make_dataset(N, L, W, seed=151, mut=0.15)
    pos = init_positions(offsets, W, 152, 0.1)
    u = np.random.default_rng(153).random(N)
    gpu_ctx.set_sequences(codes, offsets, b"ACGT")
    p1, w1 = gpu_ctx.motif_sweep(W, 1e-4, 1.0, pos, u)
    star = gpu_ctx.motif_greedy(W, 1e-4, 1.0, p1, w1)
    cnt = (p1 >= 0).astype(np.int32)
    lst = np.where(p1 >= 0, p1, -1).reshape(N, 1).astype(np.int32)
    lc, lp, lw, lpass = gpu_ctx.motif_greedy_multi(1, W, 1e-4, 1.0, cnt, lst, w1)
    assert np.array_equal(np.where(lc > 0, lp[:, 0], -1), star[0])
    assert np.array_equal(lw, star[1]) and lpass == star[2]
