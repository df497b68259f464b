"""GPU parity of the greedy refinement:
MotifSampler.findBestMotifIndicesWithStartPositions (.fs:885-929) on the device
(gs_motif_greedy / gs_run_greedy) against the oracle's go_greedy.

Bar: positions and pass counts identical; PWMS within 1e-12 relative (every
product/quotient is the same binary64 operation as the oracle's, log() may differ
in the last ulp between the device library and glibc).  Motif memories come from
an oracle sweep, like doMotifSampling feeds the greedy passes (.fs:1034-1038).
"""
import numpy as np
import pytest

from conftest import init_positions, make_dataset
from oracle import oracle_lib as ol

pytestmark = pytest.mark.gpu

PWMS_RTOL = 1e-12


def check_greedy(g, o):
    gpos, gpw, gpass = g
    opos, opw, opass = o
    bad = np.nonzero(gpos != opos)[0]
    assert bad.size == 0, f"positions differ at {bad[:10]}: {gpos[bad[:5]]} vs {opos[bad[:5]]}"
    assert gpass == opass
    same = gpw == opw
    rel = np.abs(gpw - opw) / np.maximum(np.abs(opw), 1e-300)
    assert np.all(same | (rel <= PWMS_RTOL)), f"PWMS rel diff {np.nanmax(rel):.3e}"


def motif_mem(S, offsets, W, pc, cutoff, seed, none_rate):
    """A sampled motif memory: one oracle sweep from seeded positions."""
    N = len(offsets) - 1
    pos = init_positions(offsets, W, seed, none_rate)
    u = np.random.default_rng(seed + 1).random(N)
    p, w, _ = ol.sweep(S, W, pc, cutoff, pos, u)
    return p, w


SHAPES = [
    (100, 50, 8, b"ACGT", False, 0.0, 0, 1.0),
    (120, 80, 10, b"ACGT", True, 0.2, 1, 1.0),
    (64, 90, 7, b"ATGC-", True, 0.0, 3, 1.0),                        # |A| = 5
    (80, 200, 12, b"ACDEFGHIKLMNPQRSTVWY", False, 0.0, 4, 1.0),      # protein, E > 16
    (30, 1500, 9, b"ACGT", True, 0.1, 5, 1.0),                       # L > 1024: unprefetched staging
    (60, 150, 33, b"ACGT", True, 0.1, 9, 1.0),                       # W > 32
    (3, 20, 20, b"ACGT", False, 0.0, 6, 1.0),                        # L == W: one window
    (1, 30, 6, b"ACGT", False, 0.0, 7, 1.0),                         # N == 1
    (90, 60, 8, b"ACGT", True, 0.0, 11, 1e9),                        # no motif passes the cut-off
    (90, 60, 8, b"ACGT", True, 0.5, 12, -1.0),                       # every window passes
]


@pytest.mark.parametrize("N,L,W,alpha,ragged,none_rate,seed,cutoff", SHAPES)
def test_greedy_matches_oracle(gpu_ctx, N, L, W, alpha, ragged, none_rate, seed, cutoff):
    codes, offsets = make_dataset(N, L, W, alpha, seed=seed, ragged=ragged, mut=0.15)
    S = ol.Seqs(codes, offsets, alpha)
    pc = 1e-4
    pos, pw = motif_mem(S, offsets, W, pc, cutoff, seed + 300, none_rate)
    gpu_ctx.set_sequences(codes, offsets, alpha)
    g = gpu_ctx.motif_greedy(W, pc, cutoff, pos, pw)
    o = ol.greedy(S, W, pc, cutoff, pos, pw)
    check_greedy(g, o)
    # the aggregates left on the device are those of the refined positions
    Cg, Tg = gpu_ctx.counts(W, g[0], len(alpha))
    Co, To = ol.counts(S, W, g[0])
    assert np.array_equal(Cg, Co) and np.array_equal(Tg, To)


@pytest.mark.parametrize("max_passes", [1, 2])
def test_greedy_pass_cap(gpu_ctx, max_passes):
    N, L, W = 150, 80, 9
    codes, offsets = make_dataset(N, L, W, seed=21, mut=0.2)
    S = ol.Seqs(codes, offsets, b"ACGT")
    pos = init_positions(offsets, W, 22)
    pw = np.zeros(N)  # every target accepts its first pick
    gpu_ctx.set_sequences(codes, offsets, b"ACGT")
    g = gpu_ctx.motif_greedy(W, 1e-4, 1.0, pos, pw, max_passes=max_passes)
    o = ol.greedy(S, W, 1e-4, 1.0, pos, pw, max_passes=max_passes)
    check_greedy(g, o)
    assert g[2] == max_passes


@pytest.mark.parametrize("waves", ["1", "3", "8"])
@pytest.mark.parametrize("N,L,W,none_rate", [(203, 60, 8, 0.2), (5, 40, 6, 0.0), (1, 30, 5, 0.0),
                                             (40, 1200, 9, 0.1)])
def test_greedy_speculation_widths(monkeypatch, waves, N, L, W, none_rate):
    """The speculative workgroup (GS_GREEDY_WAVES targets per step) commits exactly the
    sequential loop's results, also when fewer targets than wavefronts share the ring
    and for sequences longer than one prefetch (L > 1024)."""
    from gibbssampling_amd import Context
    codes, offsets = make_dataset(N, L, W, seed=61 + N, ragged=True, mut=0.3)
    S = ol.Seqs(codes, offsets, b"ACGT")
    pos = init_positions(offsets, W, 62, none_rate)
    pw = np.zeros(N)  # many moves in the first passes
    tuning = {"greedy_waves": float(waves)}
    c = Context(0, tuning=tuning)
    try:
        c.set_sequences(codes, offsets, b"ACGT")
        g = c.motif_greedy(W, 1e-4, 1.0, pos, pw)
    finally:
        c.close()
    check_greedy(g, ol.greedy(S, W, 1e-4, 1.0, pos, pw))


def test_greedy_nan_memory_never_accepts(gpu_ctx):
    """PWMS = NaN in motifMem: tmp.PWMS > NaN is false (.fs:923), nothing moves."""
    N, L, W = 40, 60, 8
    codes, offsets = make_dataset(N, L, W, seed=31)
    pos = init_positions(offsets, W, 32)
    pw = np.full(N, np.nan)
    gpu_ctx.set_sequences(codes, offsets, b"ACGT")
    gpos, gpw, passes = gpu_ctx.motif_greedy(W, 1e-4, 1.0, pos, pw)
    assert np.array_equal(gpos, pos) and np.isnan(gpw).all() and passes == 1


def test_resident_pipeline_matches_oracle(gpu_ctx):
    """doMotifSampling's tail on the device: resident sweeps, then gs_run_greedy on the
    same snapshot, against the oracle chain."""
    N, L, W, seed, pc, cutoff = 300, 120, 10, 0xBEEF, 1e-4, 1.0
    codes, offsets = make_dataset(N, L, W, seed=41, mut=0.1)
    pos = init_positions(offsets, W, 42)
    gpu_ctx.set_sequences(codes, offsets, b"ACGT")
    gpu_ctx.set_positions(W, pos)
    gpu_ctx.run_sweeps(pc, cutoff, 2, seed)
    passes, ms = gpu_ctx.run_greedy(pc, cutoff)
    gpos, gpw = gpu_ctx.get_state()
    assert ms > 0.0
    S = ol.Seqs(codes, offsets, b"ACGT")
    p = pos.copy()
    for t in range(2):
        u = np.array([ol.uniform(seed, ol.stream_sweep(t), n) for n in range(N)])
        p, w, _ = ol.sweep(S, W, pc, cutoff, p, u)
    check_greedy((gpos, gpw, passes), ol.greedy(S, W, pc, cutoff, p, w))
    # a further sweep continues from the refined snapshot and its aggregates
    gpu_ctx.run_sweeps(pc, cutoff, 1, seed, first_sweep=2)
    g2, w2 = gpu_ctx.get_state()
    u = np.array([ol.uniform(seed, ol.stream_sweep(2), n) for n in range(N)])
    o2, ow2, _ = ol.sweep(S, W, pc, cutoff, gpos, u)
    assert np.array_equal(g2, o2)


def test_greedy_needs_all_sequences(gpu_ctx):
    from gibbssampling_amd import Context
    from gibbssampling_amd._native import GS_E_UNSUPPORTED, GibbsError
    N, L, W = 50, 40, 6
    codes, offsets = make_dataset(N, L, W, seed=51)
    c = Context(0)
    try:
        o = offsets[:26]
        c.set_sequences(codes[:o[-1]], o, b"ACGT", n_global=N, global_offset=0)
        with pytest.raises(GibbsError) as ei:
            c.motif_greedy(W, 1e-4, 1.0, np.zeros(25, np.int32), np.zeros(25))
        assert ei.value.status == GS_E_UNSUPPORTED
    finally:
        c.close()


@pytest.mark.parametrize("switch", ["1", "16", "0"])
def test_greedy_handover_to_speculative_passes(switch, monkeypatch):
    """The star engine hands the remaining passes to the speculative list path once a
    pass moves few targets (GS_GREEDY_SWITCH): same passes, same snapshot after it
    (positions, PWMS, and the aggregates the next sweeps read)."""
    from gibbssampling_amd import Context
    N, L, W, seed = 800, 120, 9, 61
    codes, offsets = make_dataset(N, L, W, seed=251, mut=0.15, ragged=True)
    S = ol.Seqs(codes, offsets, b"ACGT")
    pos, pw = motif_mem(S, offsets, W, 1e-4, 1.0, 252, 0.1)
    o = ol.greedy(S, W, 1e-4, 1.0, pos, pw)
    tuning = {"greedy_switch": float(switch)}
    c = Context(0, tuning=tuning)
    try:
        c.set_sequences(codes, offsets, b"ACGT")
        g = c.motif_greedy(W, 1e-4, 1.0, pos, pw)
        check_greedy(g, o)
        # doMotifSampling's device pipeline: greedy on the resident snapshot, then sweeps
        c.set_positions(W, pos)
        c.run_sweeps(1e-4, 1.0, 1, seed)
        passes, _ = c.run_greedy(1e-4, 1.0)
        gp, gw = c.get_state()
        c.run_sweeps(1e-4, 1.0, 3, seed, 1)
        after = c.get_state()
    finally:
        c.close()
    ref = Context(0, tuning={"greedy_switch": 0})  # the star engine for every pass
    try:
        ref.set_sequences(codes, offsets, b"ACGT")
        ref.set_positions(W, pos)
        ref.run_sweeps(1e-4, 1.0, 1, seed)
        rpasses, _ = ref.run_greedy(1e-4, 1.0)
        rp, rw = ref.get_state()
        ref.run_sweeps(1e-4, 1.0, 3, seed, 1)
        rafter = ref.get_state()
    finally:
        ref.close()
    assert passes == rpasses and np.array_equal(gp, rp) and np.array_equal(gw, rw)
    assert np.array_equal(after[0], rafter[0]) and np.array_equal(after[1], rafter[1])


@pytest.mark.parametrize("chunk,ratio", [("16", "4"), ("1", "2"), ("64", "16")])
@pytest.mark.parametrize("max_passes", [1, 2, 1000])
def test_greedy_mid_pass_handover(chunk, ratio, max_passes, monkeypatch):
    """The star engine leaves a pass once GS_GREEDY_EXIT_CHUNK visits move fewer than
    chunk / GS_GREEDY_EXIT_RATIO targets; the speculative list path resumes at that
    visit with the pass's moved flag: the sequential passes exactly."""
    from gibbssampling_amd import Context
    N, L, W = 700, 110, 9
    codes, offsets = make_dataset(N, L, W, seed=261, mut=0.15, ragged=True)
    S = ol.Seqs(codes, offsets, b"ACGT")
    pos, pw = motif_mem(S, offsets, W, 1e-4, 1.0, 262, 0.1)
    o = ol.greedy(S, W, 1e-4, 1.0, pos, pw, max_passes=max_passes)
    tuning = {"greedy_exit_chunk": float(chunk), "greedy_exit_ratio": float(ratio)}
    c = Context(0, tuning=tuning)
    try:
        c.set_sequences(codes, offsets, b"ACGT")
        g = c.motif_greedy(W, 1e-4, 1.0, pos, pw, max_passes=max_passes)
    finally:
        c.close()
    check_greedy(g, o)


@pytest.mark.parametrize("coop", ["1", "0", "4096"])
@pytest.mark.parametrize("waves", ["2", "8"])
@pytest.mark.parametrize("N,L,W,alpha,extra", [(400, 90, 8, b"ACGT", b""),
                                               (150, 300, 20, b"ACDEFGHIKLMNPQRSTVWY", b"*")])
def test_greedy_lone_visits(coop, waves, N, L, W, alpha, extra, monkeypatch):
    """The motif greedy's lone-visit mode (every wavefront on one visit, for visits with
    K*W >= GS_GREEDY_COOP) commits exactly the sequential passes."""
    from gibbssampling_amd import Context
    codes, offsets = make_dataset(N, L, W, alpha, seed=271 + N, mut=0.15, ragged=True,
                                  extra=extra, extra_rate=0.04 if extra else 0.0)
    S = ol.Seqs(codes, offsets, alpha)
    pos, pw = motif_mem(S, offsets, W, 1e-4, 1.0, 272, 0.1)
    o = ol.greedy(S, W, 1e-4, 1.0, pos, pw)
    tuning = {"motif_coop": float(coop), "greedy_waves": float(waves), "greedy_switch": float("0")}  # the star engine for every pass
    c = Context(0, tuning=tuning)
    try:
        c.set_sequences(codes, offsets, alpha)
        g = c.motif_greedy(W, 1e-4, 1.0, pos, pw)
    finally:
        c.close()
    check_greedy(g, o)
