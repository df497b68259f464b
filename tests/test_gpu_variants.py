"""GPU parity of the caller's-background / caller's-profile twins (SURVEY §8(f)
rank 3): with gs_set_fixed_pcv every entry point computes its …ByPCV / …WithBPV
twin (.fs:301-459, .fs:788-881), with gs_set_fixed_ppm the initialiser is
getMotifsWithBestPWMSOfPPM (.fs:644-662).  Checked against the oracle's variants
(go_sweep_pcv, go_greedy_pcv, go_random_starts_ex, go_site_refine_ex), which
tests/test_oracle_crosscheck.py pins to literal Python restatements."""
import numpy as np
import pytest

from conftest import init_positions, make_dataset
from oracle import oracle_lib as ol

pytestmark = pytest.mark.gpu

RTOL = 1e-12
# the doMotifSamplingWithPPM mirror test compares the GPU run with an oracle pipeline
# built from the oracle's own sweep; this only checks that pipeline's picks are far
# from a CDF boundary (the data, not a tolerance on the GPU's indices)
ORACLE_MARGIN = 1e-9


def close(g, o):
    g, o = np.asarray(g, np.float64), np.asarray(o, np.float64)
    same = g == o  # also equal infinities (log2 of a zero best score)
    with np.errstate(invalid="ignore"):
        rel = np.abs(g - o) / np.maximum(np.abs(o), 1e-300)
    return bool(np.all(same | (rel <= RTOL)))


def pcv49(alpha, seed):
    rng = np.random.default_rng(seed)
    v = rng.uniform(0.05, 0.6, 49)
    slots = [c - 42 for c in alpha]
    v[slots] = rng.dirichlet(np.ones(len(alpha)))  # a probability vector over the alphabet
    return v


@pytest.fixture
def fixed(gpu_ctx):
    yield gpu_ctx
    gpu_ctx.set_fixed_pcv(None)
    gpu_ctx.set_fixed_ppm(None)


@pytest.mark.parametrize("N,L,W,alpha,extra,cutoff", [
    (200, 80, 10, b"ACGT", b"", 1.0),
    (120, 120, 12, b"ATGC-", b"*", 1.0),
    (80, 150, 9, b"ACDEFGHIKLMNPQRSTVWY", b"", 2.0),
])
@pytest.mark.parametrize("exact", [False, True])
def test_pcv_sweep_and_greedy(fixed, N, L, W, alpha, extra, cutoff, exact):
    codes, offsets = make_dataset(N, L, W, alpha, seed=N + W, ragged=True, mut=0.15, extra=extra,
                                  extra_rate=0.03 if extra else 0.0)
    S = ol.Seqs(codes, offsets, alpha)
    pcv = pcv49(alpha, W)
    pos = init_positions(offsets, W, 3, 0.1)
    u = np.random.default_rng(4).random(N)
    fixed.set_sequences(codes, offsets, alpha)
    fixed.set_fixed_pcv(pcv)
    fixed.set_scan_mode(exact=exact)
    try:
        gp, gw = fixed.motif_sweep(W, 1e-4, cutoff, pos, u)
    finally:
        fixed.set_scan_mode(exact=False)
    op, ow, _ = ol.sweep_pcv(S, W, 1e-4, cutoff, pcv, pos, u)
    bad = np.nonzero(gp != op)[0]
    assert bad.size == 0, f"ByPCV sweep positions differ at {bad[:10]}"
    assert close(gw, ow)
    # the greedy passes with the same pcv, from the oracle's sweep
    hp, hw, hpass = fixed.motif_greedy(W, 1e-4, cutoff, op, ow)
    rp, rw, rpass = ol.greedy_pcv(S, W, 1e-4, cutoff, pcv, op, ow)
    assert np.array_equal(hp, rp) and hpass == rpass and close(hw, rw)


@pytest.mark.parametrize("mode", [0, 1])
def test_bpv_and_ppm_initialisers(fixed, mode):
    N, L, W, alpha = 150, 90, 8, b"ACGT"
    codes, offsets = make_dataset(N, L, W, alpha, seed=11 + mode, ragged=True, mut=0.1)
    S = ol.Seqs(codes, offsets, alpha)
    fixed.set_sequences(codes, offsets, alpha)
    pcv = pcv49(alpha, 12)
    fixed.set_fixed_pcv(pcv)
    gs, gp = fixed.random_starts(W, 1e-4, 77, mode)
    os_, op = ol.random_starts(S, W, 1e-4, seed=77, mode=mode, pcv49=pcv)
    assert np.array_equal(gp, op) and close(gs, os_)
    fixed.set_fixed_pcv(None)
    ppm = np.random.default_rng(13).uniform(0.01, 1.0, (49, W))
    fixed.set_fixed_ppm(ppm, W)
    gs, gp = fixed.random_starts(W, 1e-4, 78, mode)
    os_, op = ol.random_starts(S, W, 1e-4, seed=78, mode=mode, ppm49=ppm)
    assert np.array_equal(gp, op) and close(gs, os_)


@pytest.mark.parametrize("shift", [0, -1, 1])
def test_bpv_site_refinements(fixed, shift):
    N, L, W, alpha = 120, 70, 8, b"ATGC-"
    codes, offsets = make_dataset(N, L, W, alpha, seed=21 + shift, ragged=True, mut=0.1,
                                  extra=b"*", extra_rate=0.03)
    S = ol.Seqs(codes, offsets, alpha)
    pcv = pcv49(alpha, 22)
    sc0, p0 = ol.random_starts(S, W, 1e-4, seed=23, mode=1, pcv49=pcv)
    fixed.set_sequences(codes, offsets, alpha)
    fixed.set_fixed_pcv(pcv)
    gp, gs, gpass = fixed.site_refine(W, 1e-4, shift, p0, sc0)
    op, os_, opass = ol.site_refine(S, W, 1e-4, shift, p0, sc0, pcv49=pcv)
    assert np.array_equal(gp, op) and gpass == opass and close(gs, os_)


def test_settings_lifecycle(fixed):
    from gibbssampling_amd._native import ArgumentError
    N, L, W = 30, 40, 6
    codes, offsets = make_dataset(N, L, W, seed=31)
    S = ol.Seqs(codes, offsets, b"ACGT")
    fixed.set_sequences(codes, offsets, b"ACGT")
    fixed.set_fixed_ppm(np.full((49, W), 0.25), W)
    with pytest.raises(ArgumentError):
        fixed.random_starts(W + 1, 1e-4, 1, 1)  # the PPM belongs to another motifLength
    # gs_set_sequences resets both settings: the plain initialiser again
    fixed.set_sequences(codes, offsets, b"ACGT")
    gs, gp = fixed.random_starts(W, 1e-4, 5, 1)
    os_, op = ol.random_starts(S, W, 1e-4, seed=5, mode=1)
    assert np.array_equal(gp, op) and close(gs, os_)


def test_python_mirror_variants():
    """SiteSampler.doSiteSamplingWithBPV / doSiteSamplingWithPPM and
    MotifSampler.doMotifSamplingWithPPM against the oracle compositions."""
    from gibbssampling_amd import MotifSampler, SiteSampler
    N, L, W, pc, cutoff, seed = 60, 70, 8, 1e-4, 1.0, 4321
    codes, offsets = make_dataset(N, L, W, b"ACGT", seed=41, mut=0.1)
    sources = [bytes(codes[offsets[i]:offsets[i + 1]]) for i in range(N)]
    S = ol.Seqs(codes, offsets, b"ACGT")
    pcv = pcv49(b"ACGT", 42)
    ppm = np.random.default_rng(43).uniform(0.01, 1.0, (49, W))

    res = SiteSampler.doSiteSamplingWithBPV(W, pc, "ACGT", sources, pcv, seed=seed)
    sc, p = ol.random_starts(S, W, pc, seed=seed, mode=0, pcv49=pcv)
    for shift in (0, -1, 1):
        p, sc, _ = ol.site_refine(S, W, pc, shift, p, sc, pcv49=pcv)
    assert [q for _, q in res] == list(p) and close([s for s, _ in res], sc)

    res = SiteSampler.doSiteSamplingWithPPM(W, pc, "ACGT", sources, ppm, seed=seed)
    sc, p = ol.random_starts(S, W, pc, seed=seed, mode=0, ppm49=ppm)
    for shift in (0, -1, 1):
        p, sc, _ = ol.site_refine(S, W, pc, shift, p, sc)
    assert [q for _, q in res] == list(p) and close([s for s, _ in res], sc)

    mi = MotifSampler.doMotifSamplingWithPPM(1, W, pc, cutoff, "ACGT", sources, ppm, seed=seed)
    sc, p = ol.random_starts(S, W, pc, seed=seed, mode=0, ppm49=ppm)
    u = np.array([ol.uniform(seed, ol.stream_sweep(0), n) for n in range(N)])
    p1, w1, margin = ol.sweep(S, W, pc, cutoff, p, u)
    assert (margin > ORACLE_MARGIN).all()
    op, ow, _ = ol.greedy(S, W, pc, cutoff, p1, w1)
    assert [m.Positions[0] if m.Positions else -1 for m in mi] == list(op)
    assert close([m.PWMS for m in mi], ow)
