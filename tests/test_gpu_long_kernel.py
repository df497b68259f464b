"""GPU parity of the long-sequence sweep kernel (gs_sweep_long.hip)
against the oracle: MotifSampler.findBestMotifIndicesByWithStartPositions
(.fs:935-970) with motifAmount = 1, one 16-lane row a target, exact fixed-point
window scores.  Positions identical (no tolerance on indices), PWMS within 1e-12,
over the shapes it takes: W = 4..16 (pair groups 2..8, an odd W leaving half a
group), sequences up to 16 x 32 windows (the 16- and 32-window lane ranges), ragged
and equal lengths, targets without a motif, the chain from the initialiser's output
(the regime the reference's drivers sweep, .fs:1035-1037), and every target through
the exact rescan.  The engine is told to take the kernel (long_mode 1, dna_mode 1);
each test asserts it ran."""
import numpy as np
import pytest

from conftest import init_positions, make_dataset, uniforms
from oracle import oracle_lib as ol

pytestmark = pytest.mark.gpu

RTOL = 1e-12
TUNING = {"dna_mode": 1, "long_mode": 1}


def same(gpos, gpw, opos, opw, what=""):
    bad = np.nonzero(gpos != opos)[0]
    assert bad.size == 0, f"{what}: {bad.size} positions differ, first {bad[:8]}"
    fin = np.isfinite(opw)
    assert np.array_equal(np.isfinite(gpw), fin), what
    rel = np.abs(gpw[fin] - opw[fin]) / np.maximum(np.abs(opw[fin]), 1e-300)
    assert rel.size == 0 or rel.max() <= RTOL, f"{what}: PWMS rel diff {rel.max():.3e}"


@pytest.fixture(scope="module")
def long_ctx():
    from gibbssampling_amd import Context
    ctx = Context(0, tuning=TUNING)
    yield ctx
    ctx.close()


SHAPES = [
    # N, L, W, ragged, none_rate, seed
    (600, 500, 15, False, 0.0, 21),   # config 3's shape (W = 15: 7 pair groups and a half)
    (700, 500, 15, True, 0.05, 22),   # ragged, some targets without a motif
    (500, 527, 16, True, 0.0, 23),    # the longest sequences the kernel takes (512 windows)
    (800, 300, 12, True, 0.1, 24),    # 16-window lane ranges where every lane's K fits
    (400, 400, 8, False, 0.0, 25),
    (300, 420, 4, True, 0.05, 26),    # the narrowest motif: 2 pair groups
    (257, 290, 13, True, 0.0, 27),    # a last wavefront with one target
    (300, 420, 3, True, 0.05, 28),    # W = 3: one and a half pair groups, padding pairs
    (260, 400, 2, False, 0.0, 29),    # W = 2: a single pair group
]


@pytest.mark.parametrize("N,L,W,ragged,none_rate,seed", SHAPES)
def test_long_sweep_matches_oracle(long_ctx, N, L, W, ragged, none_rate, seed):
    codes, offsets = make_dataset(N, L, W, b"ACGT", seed=seed, ragged=ragged)
    pos = init_positions(offsets, W, seed + 100, none_rate)
    u = np.random.default_rng(seed + 200).random(N)
    long_ctx.set_sequences(codes, offsets, b"ACGT")
    gpos, gpw = long_ctx.motif_sweep(W, 1e-4, 1.0, pos, u)
    assert long_ctx.sweep_kernel_name() == "gs_sweep_long_kernel"
    opos, opw, _ = ol.sweep(ol.Seqs(codes, offsets, b"ACGT"), W, 1e-4, 1.0, pos, u, threads=8)
    same(gpos, gpw, opos, opw, f"W={W} L={L}")


@pytest.mark.parametrize("W,L", [(15, 500), (12, 400), (16, 527)])
def test_long_chain_from_initialiser(long_ctx, W, L):
    """A 4-sweep resident chain from getPWMOfRandomStarts' output (.fs:589-611): every
    target keeps a motif and ~12 % of windows pass the cut-off; each sweep's prologue
    reads the aggregates the previous sweep's last workgroup reduced."""
    N = 1200
    codes, offsets = make_dataset(N, L, W, b"ACGT", seed=60 + W, ragged=True)
    S = ol.Seqs(codes, offsets, b"ACGT")
    pos = ol.random_starts(S, W, 1e-4, seed=5, mode=1)[1].astype(np.int32)
    long_ctx.set_sequences(codes, offsets, b"ACGT")
    gpos, gpw = long_ctx.motif_run(W, 1e-4, 1.0, 4, 91, pos)
    assert long_ctx.sweep_kernel_name() == "gs_sweep_long_kernel"
    opos, opw = pos, None
    for t in range(4):
        u = uniforms(91, ol.stream_sweep(t), N)
        opos, opw, _ = ol.sweep(S, W, 1e-4, 1.0, opos, u, threads=8)
    same(gpos, gpw, opos, opw, f"chain W={W}")
    assert (gpos >= 0).mean() > 0.9


def test_long_every_target_rescanned():
    """live_force: every target through the exact rescan (the path of targets whose pick
    the bound cannot certify) -- the same positions and weights."""
    from gibbssampling_amd import Context
    N, L, W = 300, 450, 15
    codes, offsets = make_dataset(N, L, W, b"ACGT", seed=31, ragged=True)
    pos = init_positions(offsets, W, 32, 0.1)
    u = np.random.default_rng(33).random(N)
    ctx = Context(0, tuning=dict(TUNING, live_force=1))
    try:
        ctx.set_sequences(codes, offsets, b"ACGT")
        gpos, gpw = ctx.motif_sweep(W, 1e-4, 1.0, pos, u)
        assert ctx.sweep_kernel_name() == "gs_sweep_long_kernel"
        assert ctx.stats()["exact_rescans"] >= N
    finally:
        ctx.close()
    opos, opw, _ = ol.sweep(ol.Seqs(codes, offsets, b"ACGT"), W, 1e-4, 1.0, pos, u, threads=8)
    same(gpos, gpw, opos, opw, "forced rescans")


def test_long_uniform_starts_chain():
    """From uniform random starts: the first sweep drops the motifs (no window passes a
    flat PPM), every target a background category through the exact rescan; the chain
    then sits in the all-background state."""
    from gibbssampling_amd import Context
    N, L, W = 500, 480, 14
    codes, offsets = make_dataset(N, L, W, b"ACGT", seed=41, ragged=True)
    pos = init_positions(offsets, W, 42, 0.0)
    ctx = Context(0, tuning=dict(TUNING, bg_mode=0))
    try:
        ctx.set_sequences(codes, offsets, b"ACGT")
        gpos, gpw = ctx.motif_run(W, 1e-4, 1.0, 3, 17, pos)
        assert ctx.sweep_kernel_name() == "gs_sweep_long_kernel"
    finally:
        ctx.close()
    S = ol.Seqs(codes, offsets, b"ACGT")
    opos, opw = pos, None
    for t in range(3):
        opos, opw, _ = ol.sweep(S, W, 1e-4, 1.0, opos, uniforms(17, ol.stream_sweep(t), N), threads=8)
    same(gpos, gpw, opos, opw, "uniform chain")


@pytest.mark.parametrize("W,L,ragged", [(15, 500, False), (12, 420, True), (7, 300, True)])
def test_long_uniform_starts_background_picks(long_ctx, W, L, ragged):
    """The first sweep of a chain from uniform random starts (.fs:1035-1037 without the
    initialiser): against the near-flat PPM of random positions no window passes the
    cut-off, every target's categories are its K background products, and the row's
    background walk (bg_pick) takes them -- the exact rescan only for the few the
    walk's bound cannot certify."""
    N = 900
    codes, offsets = make_dataset(N, L, W, b"ACGT", seed=40 + W, ragged=ragged, planted=False)
    pos = init_positions(offsets, W, 41 + W)
    u = np.random.default_rng(42 + W).random(N)
    long_ctx.set_sequences(codes, offsets, b"ACGT")
    s0 = long_ctx.stats()
    gpos, gpw = long_ctx.motif_sweep(W, 1e-4, 1.0, pos, u)
    s1 = long_ctx.stats()
    assert long_ctx.sweep_kernel_name() == "gs_sweep_long_kernel"
    opos, opw, _ = ol.sweep(ol.Seqs(codes, offsets, b"ACGT"), W, 1e-4, 1.0, pos, u, threads=8)
    assert (opos == -1).mean() > 0.85  # (nearly) every target picks a background category
    same(gpos, gpw, opos, opw, f"uniform W={W}")
    assert s1["exact_rescans"] - s0["exact_rescans"] <= 0.02 * N
