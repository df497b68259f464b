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
