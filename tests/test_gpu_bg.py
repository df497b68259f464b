"""GPU parity of the all-background sweep (gs_sweep_bg.hip) against the CPU oracle.

A snapshot is in the all-background state when no window of any sequence can pass the
cut-off (gs_bgregime.h); its sweep (findBestMotifIndicesByWithStartPositions,
GibbsSampling.fs:935-970) is then the roulette over every target's background products
only.  The chain from uniform random starts sits there from its second sweep on.  Bar:
positions identical to the oracle's, PWMS within 1e-12 relative; the same results with
the kernel disabled (bg_mode 0: the DNA / general sweep kernels), with every lane count,
and with every pick forced through the kernel's exact sequential replay.
"""
import numpy as np
import pytest

from conftest import init_positions, make_dataset, uniforms
from oracle import oracle_lib as ol

pytestmark = pytest.mark.gpu

RTOL = 1e-12


def ctx_with(**tuning):
    from gibbssampling_amd import Context
    return Context(0, tuning=tuning)


@pytest.fixture(scope="module")
def ctxs():
    c = {
        "auto": ctx_with(bg_mode=1),  # automatic takes it from 16k targets only
        "G1": ctx_with(bg_mode=1, bg_G=1),
        "G4": ctx_with(bg_mode=1, bg_G=4),
        "G64": ctx_with(bg_mode=1, bg_G=64),
        "dna": ctx_with(bg_mode=1, dna_mode=1),
        "replay": ctx_with(bg_mode=1, bg_G=8, bg_force_replay=1),
        "off": ctx_with(bg_mode=0),
    }
    yield c
    for x in c.values():
        x.close()


def bg_expected(codes, offsets, alpha, W, pc, cutoff):
    """gs_bgregime.h for a snapshot with every position []: C = 0, T = 0, so the
    bound depends on the data alone (the fewest occurrences of a symbol in any
    sequence, the longest sequence)."""
    A = len(alpha)
    N = len(offsets) - 1
    lens = np.diff(offsets)
    cmin = min(int(np.count_nonzero(codes[offsets[n]:offsets[n + 1]] == a))
               for n in range(N) for a in alpha)
    den = (N - 1) + A * pc
    ub = W * np.log2(pc / den)
    lo = (cmin + pc) / (max(int(lens.max()), W) + A * pc)
    return ub - W * np.log2(lo) < cutoff - 1e-6


def same(gpos, gpw, opos, opw, what=""):
    bad = np.nonzero(gpos != opos)[0]
    assert bad.size == 0, f"{what}: {bad.size} positions differ, first {bad[:8]}"
    fin = np.isfinite(opw)
    assert np.array_equal(np.isfinite(gpw), fin)
    rel = np.abs(gpw[fin] - opw[fin]) / np.maximum(np.abs(opw[fin]), 1e-300)
    assert rel.size == 0 or rel.max() <= RTOL, f"{what}: PWMS rel diff {rel.max():.3e}"


SHAPES = [
    # N, L, W, alphabet, ragged, seed
    (100, 50, 8, b"ACGT", False, 0),        # BASELINE config 1
    (300, 120, 12, b"ACGT", True, 2),
    (200, 333, 15, b"ACGT", True, 4),
    (150, 90, 16, b"ACGT", False, 5),       # W = 16
    (120, 60, 2, b"ACGT", True, 7),
    (130, 80, 5, b"GT", False, 8),          # |A| = 2
    (130, 80, 9, b"ACT", True, 9),          # |A| = 3
    (70, 1500, 13, b"ACGT", True, 10),      # many 16-window blocks and chunks per lane
    (3, 20, 16, b"ACGT", False, 11),        # L == W + 4
    (1, 30, 6, b"ACGT", False, 12),         # N == 1
    (65, 40, 4, b"ACGT", True, 13),         # a wavefront of targets plus one
]


@pytest.mark.parametrize("N,L,W,alpha,ragged,seed", SHAPES)
def test_bg_sweep_matches_oracle(ctxs, N, L, W, alpha, ragged, seed):
    """Every position [] (Positions []): the all-background state."""
    codes, offsets = make_dataset(N, L, W, alpha, seed=seed, ragged=ragged)
    S = ol.Seqs(codes, offsets, alpha)
    pos = np.full(N, -1, np.int32)
    u = np.random.default_rng(seed + 200).random(N)
    opos, opw, _ = ol.sweep(S, W, 1e-4, 1.0, pos, u, threads=8)
    assert (opos == -1).all()
    # (admissible when A W >= 2 W + 3: the general kernel's bound scratch)
    engaged = bg_expected(codes, offsets, alpha, W, 1e-4, 1.0) and len(alpha) * W >= 2 * W + 3
    for key, ctx in ctxs.items():
        ctx.set_sequences(codes, offsets, alpha)
        s0 = ctx.stats()
        gpos, gpw = ctx.motif_sweep(W, 1e-4, 1.0, pos, u)
        same(gpos, gpw, opos, opw, key)
        s1 = ctx.stats()
        if key != "off" and engaged:  # the all-background kernel swept it
            assert s1["bg_path"] - s0["bg_path"] == N, key
        if key == "replay" and engaged:
            assert s1["serial_picks"] - s0["serial_picks"] == N


def test_bg_engages_on_fixed_lengths():
    """The bound holds for i.i.d. DNA once N exceeds the sequence length (config 1..4)."""
    for N, L, W, seed in [(100, 50, 8, 0), (500, 200, 12, 1), (2000, 500, 15, 2)]:
        codes, offsets = make_dataset(N, L, W, b"ACGT", seed=seed)
        assert bg_expected(codes, offsets, b"ACGT", W, 1e-4, 1.0)


@pytest.mark.parametrize("pc", [1e-4, 0.5, 1e-12])
def test_bg_pseudocounts(ctxs, pc):
    codes, offsets = make_dataset(300, 120, 11, b"ACGT", seed=31)
    S = ol.Seqs(codes, offsets, b"ACGT")
    pos = np.full(300, -1, np.int32)
    u = np.random.default_rng(32).random(300)
    opos, opw, _ = ol.sweep(S, 11, pc, 1.0, pos, u, threads=8)
    for key, ctx in ctxs.items():
        ctx.set_sequences(codes, offsets, b"ACGT")
        same(*ctx.motif_sweep(11, pc, 1.0, pos, u), opos, opw, key)


def test_bg_not_taken_with_motifs(ctxs):
    """A snapshot whose targets keep motifs is not in the state: the sweep kernels run."""
    codes, offsets = make_dataset(400, 150, 10, b"ACGT", seed=21)
    S = ol.Seqs(codes, offsets, b"ACGT")
    pos = ol.random_starts(S, 10, 1e-4, seed=3, mode=1)[1].astype(np.int32)
    u = np.random.default_rng(22).random(400)
    opos, opw, _ = ol.sweep(S, 10, 1e-4, 1.0, pos, u, threads=8)
    ctx = ctxs["auto"]
    ctx.set_sequences(codes, offsets, b"ACGT")
    s0 = ctx.stats()
    same(*ctx.motif_sweep(10, 1e-4, 1.0, pos, u), opos, opw, "init")
    assert ctx.stats()["bg_path"] - s0["bg_path"] < 400


def oracle_chain(S, W, pc, cutoff, pos, seed, sweeps, n):
    for t in range(sweeps):
        u = uniforms(seed, ol.stream_sweep(t), n)
        pos, pw, _ = ol.sweep(S, W, pc, cutoff, pos, u, threads=8)
    return pos, pw


def run_split(ctx, W, pc, cutoff, pos0, seed, first, rest):
    """A resident chain in two calls: the all-background kernel takes over from the
    second call once the first call's last sweep saw the state."""
    ctx.set_positions(W, pos0)
    ctx.run_sweeps(pc, cutoff, first, seed=seed)
    s0 = ctx.stats()
    ctx.run_sweeps(pc, cutoff, rest, seed=seed, first_sweep=first)
    s1 = ctx.stats()
    pos, pw = ctx.get_state()
    return pos, pw, s1["bg_path"] - s0["bg_path"]


@pytest.mark.parametrize("key", ["auto", "G1", "dna", "off"])
@pytest.mark.parametrize("graph", [0, 1])
def test_bg_chain_from_uniform_starts(ctxs, key, graph):
    """A resident chain from uniform random starts: the first sweeps by the sweep
    kernels, the rest by the all-background kernel; direct launches and graph replay."""
    codes, offsets = make_dataset(3000, 200, 12, b"ACGT", seed=51)
    S = ol.Seqs(codes, offsets, b"ACGT")
    pos0 = init_positions(offsets, 12, seed=52)
    opos, opw = oracle_chain(S, 12, 1e-4, 1.0, pos0, 99, 14, 3000)
    ctx = ctxs[key]
    ctx.set_tuning("graph_mode", graph)
    try:
        ctx.set_sequences(codes, offsets, b"ACGT")
        gpos, gpw, nbg = run_split(ctx, 12, 1e-4, 1.0, pos0, 99, 2, 12)
        same(gpos, gpw, opos, opw, f"{key} graph={graph}")
        if key != "off":
            assert nbg == 12 * 3000, nbg
    finally:
        ctx.set_tuning("graph_mode", -1)


def test_bg_chain_config2(ctxs):
    """BASELINE config 2 (10k x 200, W = 12), 6 sweeps from uniform starts."""
    from gibbssampling_amd import synthetic
    w = synthetic.CONFIGS["cfg2"]
    codes, offsets = synthetic.generate(w)
    S = ol.Seqs(codes, offsets, w.alphabet)
    pos0 = synthetic.initial_positions(w)
    opos, opw = oracle_chain(S, w.W, w.pc, w.cutoff, pos0, 7, 6, w.N)
    ctx = ctxs["auto"]
    ctx.set_sequences(codes, offsets, w.alphabet)
    gpos, gpw, nbg = run_split(ctx, w.W, w.pc, w.cutoff, pos0, 7, 2, 4)
    same(gpos, gpw, opos, opw, "cfg2 chain")
    assert nbg == 4 * w.N


def test_bg_takeover_dropped_by_state_changes(ctxs):
    """Entry points that change the scan or the snapshot drop the takeover: with the
    binary64 scan selected the sweep kernels continue the chain, and new positions
    with motifs are swept by them too; the results stay the oracle's."""
    codes, offsets = make_dataset(2000, 150, 10, b"ACGT", seed=61)
    S = ol.Seqs(codes, offsets, b"ACGT")
    pos0 = init_positions(offsets, 10, seed=62)
    ctx = ctxs["auto"]
    ctx.set_sequences(codes, offsets, b"ACGT")
    try:
        _, _, nbg = run_split(ctx, 10, 1e-4, 1.0, pos0, 5, 2, 2)
        assert nbg == 2 * 2000
        ctx.set_scan_mode(True)
        s0 = ctx.stats()
        ctx.run_sweeps(1e-4, 1.0, 2, seed=5, first_sweep=4)
        assert ctx.stats()["bg_path"] == s0["bg_path"]
        gpos, gpw = ctx.get_state()
        opos, opw = oracle_chain(S, 10, 1e-4, 1.0, pos0, 5, 6, 2000)
        same(gpos, gpw, opos, opw, "exact scan after takeover")
    finally:
        ctx.set_scan_mode(False)
    pos1 = ol.random_starts(S, 10, 1e-4, seed=63, mode=1)[1].astype(np.int32)
    ctx.set_positions(10, pos1)
    s0 = ctx.stats()
    ctx.run_sweeps(1e-4, 1.0, 1, seed=6)
    assert ctx.stats()["bg_path"] - s0["bg_path"] < 2000
    opos, opw = oracle_chain(S, 10, 1e-4, 1.0, pos1, 6, 1, 2000)
    same(*ctx.get_state(), opos, opw, "new snapshot after takeover")


def test_bg_takeover_dropped_by_motif_sweeps(ctxs):
    """the takeover is keyed on (pc, cutOff); a chain that takes it
    over at cutOff 1.0, then places motifs at a lower cutOff, then returns to 1.0
    must not be swept as if still in the state (its aggregates are no longer 0)."""
    codes, offsets = make_dataset(2000, 150, 10, b"ACGT", seed=71)
    S = ol.Seqs(codes, offsets, b"ACGT")
    pos0 = init_positions(offsets, 10, seed=72)
    # cutOff -300 passes every window against the flat PPM of an empty snapshot
    # (log2 S ~ -222 at W = 10): every target takes a motif, the aggregates are non-zero
    cuts = [1.0, 1.0, 1.0, -300.0, 1.0, 1.0]
    pos = pos0
    for t, cut in enumerate(cuts):
        pos, pw, _ = ol.sweep(S, 10, 1e-4, cut, pos, uniforms(8, ol.stream_sweep(t), 2000),
                              threads=8)
        if t == 3:
            assert (pos >= 0).sum() > 1000  # the low cut-off placed motifs
    for key in ("auto", "dna"):
        ctx = ctxs[key]
        ctx.set_sequences(codes, offsets, b"ACGT")
        ctx.set_positions(10, pos0)
        for t, cut in enumerate(cuts):
            ctx.run_sweeps(1e-4, cut, 1, seed=8, first_sweep=t)
        same(*ctx.get_state(), pos, pw, f"{key}: cut-offs {cuts}")
