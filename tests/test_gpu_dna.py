"""GPU parity of the packed-layout sweep kernels (gs_sweep_live.hip, gs_sweep_dna.hip)
against the CPU oracle.

They run every synchronous sweep (findBestMotifIndicesByWithStartPositions,
GibbsSampling.fs:935-970, motifAmount = 1) whose alphabet has at most 4 symbols with no
other symbol in the data and W <= 16.  Bar: positions IDENTICAL to the oracle's (no
tolerance on indices), PWMS within 1e-12 relative (device log vs glibc, the only
non-bit-identical operation), and the general kernel (dna_mode 0) identical too.
Cases cover both sampler regimes: the reference's initialiser state (most picks are
certified motif windows) and uniform random starts (every pick a background
category: the exact binary64 rescan), ragged lengths, alphabets of 2-4 symbols,
every motif width 1..16, Positions = [] snapshots and 1, 2, 4 lanes per sequence.
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
    # the live-chain kernel (gs_sweep_live.hip, the default packed-layout sweep) at
    # every lane count; the older DNA kernel (live_mode 0, dna_mode 1) at its lane
    # counts; the general kernel (dna_mode 0)
    c = {f"live{g}": ctx_with(live_mode=1, live_G=g) for g in (1, 2, 4, 8)}
    # every target through the live kernel's in-wavefront exact rescan
    c["live_rescan"] = ctx_with(live_mode=1, live_force=1)
    c.update({f"dna{g}": ctx_with(dna_mode=1, live_mode=0, dna_G=g) for g in (1, 2, 4)})
    c["general"] = ctx_with(dna_mode=0)
    yield c
    for x in c.values():
        x.close()


def same(gpos, gpw, opos, opw, what=""):
    bad = np.nonzero(gpos != opos)[0]
    assert bad.size == 0, f"{what}: {bad.size} positions differ, first {bad[:8]}"
    fin = np.isfinite(opw)
    assert np.array_equal(np.isfinite(gpw), fin)
    rel = np.abs(gpw[fin] - opw[fin]) / np.maximum(np.abs(opw[fin]), 1e-300)
    assert rel.size == 0 or rel.max() <= RTOL, f"{what}: PWMS rel diff {rel.max():.3e}"


def initialiser_positions(S, W, pc=1e-4, seed=5):
    """getPWMOfRandomStarts (.fs:589-611), shared draws: doMotifSampling's sweep input."""
    return ol.random_starts(S, W, pc, seed=seed, mode=1)[1].astype(np.int32)


SHAPES = [
    # N, L, W, alphabet, ragged, none_rate, seed
    (100, 50, 8, b"ACGT", False, 0.0, 0),        # BASELINE config 1
    (300, 120, 12, b"ACGT", True, 0.1, 2),
    (500, 200, 12, b"ACGT", False, 0.0, 3),
    (200, 333, 15, b"ACGT", True, 0.2, 4),
    (150, 90, 16, b"ACGT", False, 0.0, 5),       # W = 16: every pair group used
    (120, 60, 1, b"ACGT", False, 0.0, 6),        # W = 1
    (120, 60, 2, b"ACGT", True, 0.0, 7),
    (130, 80, 5, b"GT", False, 0.0, 8),          # |A| = 2
    (130, 80, 9, b"ACT", True, 0.1, 9),          # |A| = 3
    (70, 1500, 13, b"ACGT", True, 0.0, 10),      # > 64 windows per lane, many chunks
    (3, 20, 16, b"ACGT", False, 0.0, 11),        # L == W + 4
    (1, 30, 6, b"ACGT", False, 0.0, 12),         # N == 1
    (65, 40, 4, b"ACGT", True, 0.5, 13),         # a tile of 64 plus one
]


@pytest.mark.parametrize("regime", ["init", "uniform"])
@pytest.mark.parametrize("N,L,W,alpha,ragged,none_rate,seed", SHAPES)
def test_dna_sweep_matches_oracle(ctxs, regime, N, L, W, alpha, ragged, none_rate, seed):
    codes, offsets = make_dataset(N, L, W, alpha, seed=seed, ragged=ragged)
    S = ol.Seqs(codes, offsets, alpha)
    if regime == "init":
        pos = initialiser_positions(S, W, seed=seed + 1)
        if none_rate:
            pos[np.random.default_rng(seed).random(N) < none_rate] = -1
    else:
        pos = init_positions(offsets, W, seed + 100, none_rate)
    u = np.random.default_rng(seed + 200).random(N)
    opos, opw, _ = ol.sweep(S, W, 1e-4, 1.0, pos, u, threads=8)
    for key, ctx in ctxs.items():
        ctx.set_sequences(codes, offsets, alpha)
        gpos, gpw = ctx.motif_sweep(W, 1e-4, 1.0, pos, u)
        same(gpos, gpw, opos, opw, f"G={key}")


@pytest.mark.parametrize("cutoff", [-2.0, 0.0, 1.0, 3.0, 8.0])
def test_dna_cutoffs(ctxs, cutoff):
    """Cut-offs from 'every window passes' (negative: negative weights pass too, the
    live kernel hands every target to its exact rescan) to 'almost none does'."""
    from gibbssampling_amd import RouletteOverrunError
    codes, offsets = make_dataset(400, 150, 10, b"ACGT", seed=21)
    S = ol.Seqs(codes, offsets, b"ACGT")
    pos = initialiser_positions(S, 10)
    u = np.random.default_rng(22).random(400)
    try:
        opos, opw, _ = ol.sweep(S, 10, 1e-4, cutoff, pos, u, threads=8)
        oerr = None
    except Exception as e:  # negative weights may overrun the roulette (.fs:752)
        oerr = e
    for key, ctx in ctxs.items():
        ctx.set_sequences(codes, offsets, b"ACGT")
        if oerr is not None:
            with pytest.raises(RouletteOverrunError):
                ctx.motif_sweep(10, 1e-4, cutoff, pos, u)
            continue
        same(*ctx.motif_sweep(10, 1e-4, cutoff, pos, u), opos, opw, f"G={key}")


@pytest.mark.parametrize("pc", [1e-4, 0.5, 1e-12])
def test_dna_pseudocounts(ctxs, pc):
    codes, offsets = make_dataset(300, 120, 11, b"ACGT", seed=31)
    S = ol.Seqs(codes, offsets, b"ACGT")
    pos = initialiser_positions(S, 11, pc=pc)
    u = np.random.default_rng(32).random(300)
    opos, opw, _ = ol.sweep(S, 11, pc, 1.0, pos, u, threads=8)
    for key, ctx in ctxs.items():
        ctx.set_sequences(codes, offsets, b"ACGT")
        same(*ctx.motif_sweep(11, pc, 1.0, pos, u), opos, opw, f"G={key}")


def oracle_chain(S, W, pc, cutoff, pos, seed, sweeps, n):
    """The library's resident chain: sweep t draws u[n] = gs_uniform(seed, stream_sweep(t), n)."""
    st = ol.stream_sweep
    for t in range(sweeps):
        u = uniforms(seed, st(t), n)
        pos, pw, _ = ol.sweep(S, W, pc, cutoff, pos, u, threads=8)
    return pos, pw


@pytest.mark.parametrize("key", ["live1", "live4", "live8", "dna1", "dna4", "general"])
def test_dna_chain_config2(ctxs, key):
    """A 10-sweep resident chain at BASELINE config 2 (10k x 200, W = 12) from the
    initialiser's state: every position of every sweep's output identical."""
    from gibbssampling_amd import synthetic
    w = synthetic.CONFIGS["cfg2"]
    codes, offsets = synthetic.generate(w)
    S = ol.Seqs(codes, offsets, w.alphabet)
    pos0 = initialiser_positions(S, w.W)
    opos, opw = oracle_chain(S, w.W, w.pc, w.cutoff, pos0, 77, 10, w.N)
    ctx = ctxs[key]
    ctx.set_sequences(codes, offsets, w.alphabet)
    gpos, gpw = ctx.motif_run(w.W, w.pc, w.cutoff, 10, 77, pos0)
    same(gpos, gpw, opos, opw, f"chain G={key}")


def test_dna_counts_exact(ctxs):
    """The vector aggregates the DNA sweep leaves equal the oracle's integer counts of
    its output (read back through the replica form)."""
    codes, offsets = make_dataset(2000, 180, 12, b"ACGT", seed=41, ragged=True)
    S = ol.Seqs(codes, offsets, b"ACGT")
    pos = initialiser_positions(S, 12)
    for key in ("live1", "live4", "dna1"):
        ctx = ctxs[key]
        ctx.set_sequences(codes, offsets, b"ACGT")
        ctx.set_positions(12, pos)
        ctx.run_sweeps(1e-4, 1.0, 3, seed=5)
        gpos, _ = ctx.get_state()
        agg = ctx.agg_download().reshape(8, -1).sum(0)
        C, T = ol.counts(S, 12, gpos)
        A = 4
        assert np.array_equal(agg[:A * 12].reshape(A, 12), np.asarray(C).reshape(A, 12)), key
        assert np.array_equal(agg[A * 12:A * 12 + A], np.asarray(T)), key

