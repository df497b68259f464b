"""GPU parity of gs_sweep_kernel's H = 1 path with its workgroup work counter (kDyn,
gs_sweep.hip: a workgroup's wavefronts take units of G sequences from an LDS counter)
against the oracle: MotifSampler.findBestMotifIndicesByWithStartPositions
(.fs:935-970), motifAmount = 1.

H = 1 is taken for alphabets whose encoded symbol count exceeds 16: protein (config 5,
|A| = 20) and a five-symbol alphabet whose data hold 14 other symbols (E = 19).  The
shapes are ragged (lengths 150-450, several LDS slices' worth of windows apart), hold
targets without a motif (Positions []), and are large enough that every wavefront of
the 12-wavefront workgroups takes several units from the counter (40k protein targets:
20k units of two over 3,072 wavefronts, ~4.5 counter grabs each).  Positions identical
(no tolerance on indices), PWMS within 1e-12 relative.
"""
import numpy as np
import pytest

from conftest import init_positions, make_dataset, uniforms
from oracle import oracle_lib as ol

pytestmark = pytest.mark.gpu

RTOL = 1e-12
PROTEIN = b"ACDEFGHIKLMNPQRSTVWY"


def same(gpos, gpw, opos, opw, what=""):
    bad = np.nonzero(gpos != opos)[0]
    assert bad.size == 0, f"{what}: {bad.size} positions differ, first {bad[:8]}"
    fin = np.isfinite(opw)
    assert np.array_equal(np.isfinite(gpw), fin), what
    rel = np.abs(gpw[fin] - opw[fin]) / np.maximum(np.abs(opw[fin]), 1e-300)
    assert rel.size == 0 or rel.max() <= RTOL, f"{what}: PWMS rel diff {rel.max():.3e}"


def ragged_protein(N, lo, hi, W, seed):
    """Lengths uniform in [lo, hi] (make_dataset draws them in [W, L])."""
    codes, offsets = make_dataset(N, hi, W, PROTEIN, seed=seed, ragged=True)
    lens = np.diff(offsets)
    keep = np.maximum(lens, lo)  # re-cut: lengths in [lo, hi]
    rng = np.random.default_rng(seed + 1)
    a = np.frombuffer(PROTEIN, np.uint8)
    offs = np.zeros(N + 1, np.int64)
    np.cumsum(keep, out=offs[1:])
    out = a[rng.integers(0, len(a), int(offs[-1]))].astype(np.uint8)
    for n in range(N):  # the planted part of each sequence, kept where it fits
        m = min(lens[n], keep[n])
        out[offs[n]:offs[n] + m] = codes[offsets[n]:offsets[n] + m]
    return out, offs


@pytest.mark.parametrize("N,seed", [(40000, 301), (9001, 302)])
def test_kdyn_ragged_protein_sweep(gpu_ctx, N, seed):
    W = 20
    codes, offsets = ragged_protein(N, 150, 450, W, seed)
    pos = init_positions(offsets, W, seed + 100, 0.1)
    u = np.random.default_rng(seed + 200).random(N)
    gpu_ctx.set_sequences(codes, offsets, PROTEIN)
    gpos, gpw = gpu_ctx.motif_sweep(W, 1e-4, 1.0, pos, u)
    assert gpu_ctx.sweep_kernel_name() == "gs_sweep_kernel"
    launch = gpu_ctx.last_sweep_launch()
    assert launch["ek"] == 0 and launch["gl"] >= 32, launch
    opos, opw, _ = ol.sweep(ol.Seqs(codes, offsets, PROTEIN), W, 1e-4, 1.0, pos, u, threads=16)
    same(gpos, gpw, opos, opw, f"protein N={N}")


@pytest.mark.parametrize("waves", [12, 6, 3])
def test_kdyn_workgroup_widths(waves):
    """The counter shared by 12, 6 and 3 wavefronts a workgroup (sweep_waves tuning):
    the first two units of a wavefront are static (wid, wid + waves), the rest grabbed."""
    from gibbssampling_amd import Context
    N, W, seed = 12000, 20, 310 + waves
    codes, offsets = ragged_protein(N, 150, 450, W, seed)
    pos = init_positions(offsets, W, seed + 100, 0.1)
    u = np.random.default_rng(seed + 200).random(N)
    c = Context(0, tuning={"sweep_waves": float(waves)})
    try:
        c.set_sequences(codes, offsets, PROTEIN)
        gpos, gpw = c.motif_sweep(W, 1e-4, 1.0, pos, u)
        assert c.last_sweep_launch()["waves"] == waves
    finally:
        c.close()
    opos, opw, _ = ol.sweep(ol.Seqs(codes, offsets, PROTEIN), W, 1e-4, 1.0, pos, u, threads=16)
    same(gpos, gpw, opos, opw, f"waves={waves}")


def test_kdyn_five_symbols_many_others(gpu_ctx):
    """|A| = 5 (the .fsx's dnaBases ATGC-) with 14 other symbols in the data: E = 19
    encoded symbols, so the H = 1 kernel; raw counts of the others in the PCV (Q3)."""
    N, L, W, seed = 20000, 300, 8, 320
    alpha = b"ATGC-"
    codes, offsets = make_dataset(N, L, W, alpha, seed=seed, ragged=True,
                                  extra=b"BDEFHIJKLMNOPQ", extra_rate=0.03)
    assert len(np.unique(codes)) > 16
    pos = init_positions(offsets, W, seed + 100, 0.1)
    u = np.random.default_rng(seed + 200).random(N)
    gpu_ctx.set_sequences(codes, offsets, alpha)
    gpos, gpw = gpu_ctx.motif_sweep(W, 0.5, 1.0, pos, u)
    launch = gpu_ctx.last_sweep_launch()
    assert launch["ek"] == 0 and launch["gl"] >= 32, launch
    opos, opw, _ = ol.sweep(ol.Seqs(codes, offsets, alpha), W, 0.5, 1.0, pos, u, threads=16)
    same(gpos, gpw, opos, opw, "five symbols + 14 others")


def test_kdyn_chain_from_initialiser(gpu_ctx):
    """A 3-sweep resident chain from getPWMOfRandomStarts' output (.fs:589-611), ragged
    protein: each sweep's counter hands out units of a snapshot the previous sweep's
    workgroups accumulated."""
    N, W = 20000, 20
    codes, offsets = ragged_protein(N, 150, 450, W, 330)
    S = ol.Seqs(codes, offsets, PROTEIN)
    pos = ol.random_starts(S, W, 1e-4, seed=5, mode=1)[1].astype(np.int32)
    gpu_ctx.set_sequences(codes, offsets, PROTEIN)
    gpos, gpw = gpu_ctx.motif_run(W, 1e-4, 1.0, 3, 93, pos)
    opos, opw = pos, None
    for t in range(3):
        u = uniforms(93, ol.stream_sweep(t), N)
        opos, opw, _ = ol.sweep(S, W, 1e-4, 1.0, opos, u, threads=16)
    assert (opos >= 0).mean() > 0.5  # the chain keeps motifs (the init regime)
    same(gpos, gpw, opos, opw, "protein chain")


def test_sweep_waves_above_ceiling_rejected():
    """sweep_waves above the alphabet's ceiling (4 for the pair tables' kernel) is an
    argument error at the sweep, not a silent fall back to the default."""
    from gibbssampling_amd import Context
    from gibbssampling_amd._native import GS_E_ARG, GibbsError
    N, L, W = 200, 100, 8
    codes, offsets = make_dataset(N, L, W, seed=340)
    pos = init_positions(offsets, W, 341)
    u = np.random.default_rng(342).random(N)
    c = Context(0, tuning={"sweep_waves": 6.0, "dna_mode": 0.0})
    try:
        c.set_sequences(codes, offsets, b"ACGT")
        with pytest.raises(GibbsError) as e:
            c.motif_sweep(W, 1e-4, 1.0, pos, u)
        assert e.value.status == GS_E_ARG
    finally:
        c.close()
