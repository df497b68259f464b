"""GPU parity of the sweep kernel's four-symbol instantiation (gs_sweep_kernel<WM, 2,
GL, 4>) against the oracle, over the shapes it is chosen for: DNA
without other symbols, W a multiple of 4 up to 32, lane groups of 16 (the four-window
scan, L <= 256), 32 and 64 (longer sequences), ragged and equal lengths (the fixed-stride
offsets), targets without a motif (their PCV logs outside the workgroup table), and a
resident chain whose aggregates come from the previous sweep.  Positions identical,
PWMS within 1e-12 (MotifSampler.findBestMotifIndicesByWithStartPositions, .fs:935-970).
Small N: the general kernel is the one the engine picks (below 64 wavefronts a CU).
"""
import numpy as np
import pytest

from conftest import init_positions, make_dataset, uniforms
from oracle import oracle_lib as ol

pytestmark = pytest.mark.gpu

RTOL = 1e-12


def same(gpos, gpw, opos, opw, what=""):
    bad = np.nonzero(gpos != opos)[0]
    assert bad.size == 0, f"{what}: {bad.size} positions differ, first {bad[:8]}"
    fin = np.isfinite(opw)
    assert np.array_equal(np.isfinite(gpw), fin), what
    rel = np.abs(gpw[fin] - opw[fin]) / np.maximum(np.abs(opw[fin]), 1e-300)
    assert rel.size == 0 or rel.max() <= RTOL, f"{what}: PWMS rel diff {rel.max():.3e}"


SHAPES = [
    # N, L, W, ragged, none_rate, seed
    (400, 60, 4, True, 0.1, 11),      # the narrowest motif, 16-lane groups
    (600, 200, 16, True, 0.05, 12),
    (500, 240, 20, False, 0.0, 13),   # equal lengths: fixed-stride first offsets
    (300, 256, 24, True, 0.1, 14),    # the longest sequence of 16-lane groups
    (200, 400, 28, True, 0.05, 15),   # 32-lane groups (two windows a step)
    (120, 900, 32, False, 0.1, 16),   # 64-lane groups, the widest four-symbol motif
]


@pytest.mark.parametrize("N,L,W,ragged,none_rate,seed", SHAPES)
def test_ek4_sweep_matches_oracle(gpu_ctx, N, L, W, ragged, none_rate, seed):
    codes, offsets = make_dataset(N, L, W, b"ACGT", seed=seed, ragged=ragged)
    pos = init_positions(offsets, W, seed + 100, none_rate)
    u = np.random.default_rng(seed + 200).random(N)
    gpu_ctx.set_sequences(codes, offsets, b"ACGT")
    gpos, gpw = gpu_ctx.motif_sweep(W, 1e-4, 1.0, pos, u)
    opos, opw, _ = ol.sweep(ol.Seqs(codes, offsets, b"ACGT"), W, 1e-4, 1.0, pos, u)
    same(gpos, gpw, opos, opw, f"W={W} L={L}")
    # the four-symbol instantiation is the one that ran (not the EK = 0 kernel)
    launch = gpu_ctx.last_sweep_launch()
    assert launch["ek"] == 4 and launch["waves"] == 4, launch
    assert launch["gl"] == (16 if L <= 256 else 32 if L <= 512 else 64), launch


@pytest.mark.parametrize("W", [16, 32])
def test_ek4_chain_from_initialiser(gpu_ctx, W):
    """A 4-sweep resident chain from getPWMOfRandomStarts' output (.fs:589-611): each
    sweep's prologue reads the aggregates the previous sweep accumulated on the device."""
    N, L = 1500, 180
    codes, offsets = make_dataset(N, L, W, b"ACGT", seed=40 + W, ragged=True)
    S = ol.Seqs(codes, offsets, b"ACGT")
    pos = ol.random_starts(S, W, 1e-4, seed=5, mode=1)[1].astype(np.int32)
    gpu_ctx.set_sequences(codes, offsets, b"ACGT")
    gpos, gpw = gpu_ctx.motif_run(W, 1e-4, 1.0, 4, 91, pos)
    opos, opw = pos, None
    for t in range(4):
        u = uniforms(91, ol.stream_sweep(t), N)
        opos, opw, _ = ol.sweep(S, W, 1e-4, 1.0, opos, u, threads=8)
    same(gpos, gpw, opos, opw, f"chain W={W}")
    assert gpu_ctx.last_sweep_launch()["ek"] == 4
    assert (gpos >= 0).mean() > 0.9  # the chain keeps its motifs (the live aggregates)
