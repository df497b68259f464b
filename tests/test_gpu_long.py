"""Sequences longer than the LDS carves of the site scans: the
initialiser getPWMOfRandomStarts (.fs:589-611, every driver's first stage) and the
site passes keep their D table [(L+1)][A] in HBM once it does not fit the LDS
(protein beyond ~2,000 residues, DNA beyond ~9,600 bases), and the site sampler's
Gauss–Seidel passes (.fs:554-585) run as speculative steps when the star engine's
carve cannot hold a sequence.  The reference has no length limit; neither does this
path.  Bar: the oracle's pipelines, positions identical, scores within 1e-12."""
import numpy as np
import pytest

from conftest import make_dataset
from oracle import oracle_lib as ol

pytestmark = pytest.mark.gpu

CASES = [
    (5, 3000, 20, b"ACDEFGHIKLMNPQRSTVWY"),   # protein, 3k residues
    (3, 20000, 12, b"ACGT"),                   # DNA, 20k bases
]


@pytest.mark.parametrize("N,L,W,alpha", CASES)
def test_long_initialiser_and_site_sampler(gpu_ctx, N, L, W, alpha):
    codes, offsets = make_dataset(N, L, W, alpha, seed=17)
    gpu_ctx.set_sequences(codes, offsets, alpha)
    S = ol.Seqs(codes, offsets, alpha)
    for mode in (0, 1):
        gs, gp = gpu_ctx.random_starts(W, 1e-4, 99, mode)
        os_, op = ol.random_starts(S, W, 1e-4, 99, mode)
        assert np.array_equal(gp, op), f"mode {mode}"
        np.testing.assert_allclose(gs, os_, rtol=1e-12)
    pos, score, _ = gpu_ctx.site_sampling(W, 1e-4, 5)
    sc, p = ol.random_starts(S, W, 1e-4, seed=5, mode=0)
    for shift in (0, -1, 1):
        p, sc, _ = ol.site_refine(S, W, 1e-4, shift, p, sc)
    assert np.array_equal(pos, p)
    np.testing.assert_allclose(score, sc, rtol=1e-12)


@pytest.mark.parametrize("N,L,W,alpha", CASES)
def test_long_motif_sampler(gpu_ctx, N, L, W, alpha):
    codes, offsets = make_dataset(N, L, W, alpha, seed=19)
    gpu_ctx.set_sequences(codes, offsets, alpha)
    S = ol.Seqs(codes, offsets, alpha)
    pos, pwms, _ = gpu_ctx.motif_sampling(W, 1e-4, 1.0, 8)
    _, p0 = ol.random_starts(S, W, 1e-4, seed=8, mode=0)
    u = np.array([ol.uniform(8, ol.stream_sweep(0), n) for n in range(N)])
    p1, w1, _ = ol.sweep(S, W, 1e-4, 1.0, p0, u)
    gp, gw, _ = ol.greedy(S, W, 1e-4, 1.0, p1, w1)
    assert np.array_equal(pos, gp)
    np.testing.assert_allclose(pwms, gw, rtol=1e-12)


@pytest.mark.parametrize("L", [4000, 20000])
def test_long_dna_sweep_live_mode_forced(L):
    """live_mode = 1 ('whenever the packed layout is taken') on sequences whose live
    workgroup cannot fit the LDS at any lane count: the engine takes the
    older packed kernel instead of failing the launch.  A 3-sweep chain equals the
    oracle's, positions identical."""
    from conftest import uniforms
    from gibbssampling_amd import Context
    N, W = 40, 12
    codes, offsets = make_dataset(N, L, W, b"ACGT", seed=23, mut=0.1)
    ctx = Context(0, tuning={"dna_mode": 1, "live_mode": 1})
    ctx.set_sequences(codes, offsets, b"ACGT")
    S = ol.Seqs(codes, offsets, b"ACGT")
    _, p = ol.random_starts(S, W, 1e-4, seed=3, mode=1)
    ctx.set_positions(W, p)
    # (beyond the packed layout's limits the general kernel takes the data)
    assert ctx.sweep_kernel_name() in ("gs_sweep_live_kernel", "gs_sweep_dna_kernel", "gs_sweep_kernel")
    ctx.run_sweeps(1e-4, 1.0, 3, seed=11)
    gp, gw = ctx.get_state()
    for t in range(3):
        p, w, _ = ol.sweep(S, W, 1e-4, 1.0, p, uniforms(11, ol.stream_sweep(t), N))
    ctx.close()
    assert np.array_equal(gp, p)
    np.testing.assert_allclose(gw, w, rtol=1e-12)
