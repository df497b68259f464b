"""The sequential §8(f) rows at BASELINE sizes, whole runs: the greedy refinement
(findBestMotifIndicesWithStartPositions, .fs:885-929) and the site sampler's
Gauss-Seidel refinement (getBestPWMSsWithStartPositions, .fs:554-585) on config 2
(10k x 200 DNA, W = 12) and config 5 (50k x 300 protein, W = 20), against the
oracle's incremental CPU ports (go_greedy_fast / go_site_refine_fast, each
cross-checked with the per-target rebuild in tests/test_oracle_crosscheck.py).

These runs pass through every engine the library switches between (the star
workgroup, lone visits scored by the whole workgroup, the mid-pass hand-over and the
GPU-wide speculative steps).  Bar: positions and pass counts identical; log2 scores
and PWMS within 1e-12 relative (device log vs glibc).
"""
import numpy as np
import pytest

from conftest import make_dataset
from oracle import oracle_lib as ol

pytestmark = pytest.mark.gpu

RTOL = 1e-12
SHAPES = {"cfg2": (10_000, 200, 12, b"ACGT"),
          "cfg5": (50_000, 300, 20, b"ACDEFGHIKLMNPQRSTVWY")}


def close(g, o):
    fin = np.isfinite(o)
    assert np.array_equal(np.isfinite(g), fin)
    rel = np.abs(g[fin] - o[fin]) / np.maximum(np.abs(o[fin]), 1e-300)
    assert rel.size == 0 or rel.max() <= RTOL, f"max rel diff {rel.max():.3e}"


@pytest.fixture(scope="module", params=list(SHAPES))
def data(request):
    N, L, W, alpha = SHAPES[request.param]
    codes, offsets = make_dataset(N, L, W, alpha, seed=5)
    return codes, offsets, W, alpha, ol.Seqs(codes, offsets, alpha)


def test_site_refinement_whole_run(gpu_ctx, data):
    codes, offsets, W, alpha, S = data
    gpu_ctx.set_sequences(codes, offsets, alpha)
    sc0, p0 = gpu_ctx.random_starts(W, 1e-4, 7, 1)
    gp, gs, gpass = gpu_ctx.site_refine(W, 1e-4, 0, p0, sc0)
    op, os_, opass, _ = ol.site_refine_fast(S, W, 1e-4, p0, sc0)
    assert gpass == opass
    bad = np.nonzero(gp != op)[0]
    assert bad.size == 0, f"{bad.size} positions differ, first at {bad[:5]}"
    close(gs, os_)


def test_greedy_whole_run(gpu_ctx, data):
    codes, offsets, W, alpha, S = data
    gpu_ctx.set_sequences(codes, offsets, alpha)
    _, p0 = gpu_ctx.random_starts(W, 1e-4, 7, 1)
    u = np.random.default_rng(11).random(len(offsets) - 1)
    p1, w1 = gpu_ctx.motif_sweep(W, 1e-4, 1.0, p0, u)
    gp, gw, gpass = gpu_ctx.motif_greedy(W, 1e-4, 1.0, p1, w1)
    op, ow, opass, _ = ol.greedy_fast(S, W, 1e-4, 1.0, p1, w1)
    assert gpass == opass
    bad = np.nonzero(gp != op)[0]
    assert bad.size == 0, f"{bad.size} positions differ, first at {bad[:5]}"
    close(gw, ow)


def test_motif_amount_two_sweep_full_size(gpu_ctx):
    """motifAmount = 2 (Positions lists, .fs:727-742) at config 2, whole sweeps: from
    single starts to lists, then lists to lists, against the oracle's list sweep."""
    N, L, W, alpha = SHAPES["cfg2"]
    codes, offsets = make_dataset(N, L, W, alpha, seed=5)
    S = ol.Seqs(codes, offsets, alpha)
    gpu_ctx.set_sequences(codes, offsets, alpha)
    _, p0 = gpu_ctx.random_starts(W, 1e-4, 7, 1)
    M = 2
    cnt = np.ones(N, np.int32)
    lst = np.full((N, M), -1, np.int32)
    lst[:, 0] = p0
    rng = np.random.default_rng(12)
    for _ in range(2):
        u = rng.random(N)
        gc, gp, gw = gpu_ctx.motif_sweep_multi(M, W, 1e-4, 1.0, cnt, lst, u)
        oc, op, ow = ol.sweep_lists(S, M, W, 1e-4, 1.0, cnt, lst, M, u, threads=8)
        assert np.array_equal(gc, oc)
        assert np.array_equal(gp, op[:, :M])
        close(gw, ow)
        cnt, lst = gc, np.ascontiguousarray(gp)
