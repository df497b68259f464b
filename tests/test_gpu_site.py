"""GPU parity of the site sampler's scans and refinements:
gs_site_scan (getBestPWMSs of every target, .fs:462-479), gs_site_refine
(getBestPWMSsWithStartPositions .fs:554-585, getLeftShiftedBestPWMSs .fs:519-550,
getRightShiftedBestPWMSs .fs:483-517) and gs_site_sampling (doSiteSampling,
.fs:697-701) against the oracle (go_site_scan / go_site_refine / go_random_starts).

Bar: positions and pass counts identical; log2 scores within 1e-12 relative (the
binary64 products/quotients are the reference's, log() may differ in the last
ulp between the device library and glibc).
"""
import numpy as np
import pytest

from conftest import make_dataset
from oracle import oracle_lib as ol

pytestmark = pytest.mark.gpu

RTOL = 1e-12


def check_scores(g, o):
    same = g == o  # (equal infinities included: their difference would be NaN)
    diff = np.where(same, 0.0, g - np.where(same, 0.0, o))
    rel = np.abs(diff) / np.maximum(np.abs(np.where(same, 1.0, o)), 1e-300)
    assert np.all(same | (rel <= RTOL)), f"score rel diff {np.nanmax(rel[~same]):.3e}"


SHAPES = [
    (60, 50, 8, b"ACGT", False, b"", 0),
    (80, 90, 10, b"ACGT", True, b"", 1),
    (50, 70, 7, b"ATGC-", True, b"*", 2),                          # non-alphabet symbols
    (40, 120, 9, b"ACDEFGHIKLMNPQRSTVWY", True, b"*X", 3),         # protein, E > 16
    (12, 1300, 12, b"ACGT", True, b"", 4),                         # long sequences
    (3, 20, 20, b"ACGT", False, b"", 5),                           # L == W
    (2, 30, 6, b"ACGT", False, b"", 6),                            # N == 2
]


def dataset(N, L, W, alpha, ragged, extra, seed):
    codes, offsets = make_dataset(N, L, W, alpha, seed=seed, ragged=ragged, mut=0.15,
                                  extra=extra, extra_rate=0.04 if extra else 0.0)
    return codes, offsets, ol.Seqs(codes, offsets, alpha)


@pytest.mark.parametrize("N,L,W,alpha,ragged,extra,seed", SHAPES)
def test_site_scan_matches_oracle(gpu_ctx, N, L, W, alpha, ragged, extra, seed):
    codes, offsets, S = dataset(N, L, W, alpha, ragged, extra, seed)
    lens = np.diff(offsets)
    r = (np.random.default_rng(seed + 7).random(N) * (lens - W + 1)).astype(np.int32)
    gpu_ctx.set_sequences(codes, offsets, alpha)
    gs, gp = gpu_ctx.site_scan(W, 1e-4, r)
    os_, op = ol.site_scan(S, W, 1e-4, r)
    assert np.array_equal(gp, op)
    check_scores(gs, os_)


@pytest.mark.parametrize("shift", [0, -1, 1])
@pytest.mark.parametrize("N,L,W,alpha,ragged,extra,seed", SHAPES[:5])
def test_site_refine_matches_oracle(gpu_ctx, shift, N, L, W, alpha, ragged, extra, seed):
    codes, offsets, S = dataset(N, L, W, alpha, ragged, extra, seed)
    sc0, p0 = ol.random_starts(S, W, 1e-4, seed=seed + 11, mode=0)
    gpu_ctx.set_sequences(codes, offsets, alpha)
    gp, gs, gpass = gpu_ctx.site_refine(W, 1e-4, shift, p0, sc0)
    op, os_, opass = ol.site_refine(S, W, 1e-4, shift, p0, sc0)
    assert np.array_equal(gp, op), f"positions differ at {np.nonzero(gp != op)[0][:10]}"
    assert gpass == opass
    check_scores(gs, os_)


@pytest.mark.parametrize("waves", ["1", "2", "8"])
@pytest.mark.parametrize("N,L,W,alpha,extra", [(150, 70, 8, b"ACGT", b""),
                                               (6, 40, 6, b"ATGC-", b"*"),
                                               (30, 1100, 10, b"ACGT", b""),
                                               (40, 90, 9, b"ACDEFGHIKLMNPQRSTVWY", b"*")])
def test_site_greedy_speculation_widths(monkeypatch, waves, N, L, W, alpha, extra):
    """getBestPWMSsWithStartPositions on the speculative engine (GS_GREEDY_WAVES
    targets per step) commits exactly the sequential passes."""
    from gibbssampling_amd import Context
    codes, offsets, S = dataset(N, L, W, alpha, True, extra, 71 + N)
    sc0, p0 = ol.random_starts(S, W, 1e-4, seed=72, mode=1)
    tuning = {"greedy_waves": float(waves)}
    c = Context(0, tuning=tuning)
    try:
        c.set_sequences(codes, offsets, alpha)
        gp, gs, gpass = c.site_refine(W, 1e-4, 0, p0, sc0)
    finally:
        c.close()
    op, os_, opass = ol.site_refine(S, W, 1e-4, 0, p0, sc0)
    assert np.array_equal(gp, op) and gpass == opass
    check_scores(gs, os_)


@pytest.mark.parametrize("coop,dt16,rate", [("0", "0", "0"), ("0", "1", "0.5"), ("1", "0", "0"),
                                            ("1", "1", "0.5"), ("1", "1", "0.1"),
                                            ("1", "1", "0.35")])  # the shipped default
@pytest.mark.parametrize("N,L,W,alpha,extra,waves", [
    (300, 80, 9, b"ACGT", b"", "8"),
    (120, 300, 20, b"ACDEFGHIKLMNPQRSTVWY", b"*", "4"),            # K > 64 * waves
    (40, 3400, 20, b"ACGT", b"", "2"),                             # L * W >= 2^16: int32 D
    (20, 25, 12, b"ATGC-", b"*", "8"),                             # K < 16
])
def test_site_greedy_coop_and_d_table(monkeypatch, coop, dt16, rate, N, L, W, alpha, extra,
                                      waves):
    """The site engine's lone-visit mode (every wavefront on one visit, GS_SITE_COOP)
    and its two-byte D table (GS_SITE_DT16) commit exactly the sequential passes; the
    random starts make the first passes move-heavy, so lone visits are frequent."""
    from gibbssampling_amd import Context
    codes, offsets, S = dataset(N, L, W, alpha, True, extra, 91 + N)
    sc0, p0 = ol.random_starts(S, W, 1e-4, seed=92, mode=1)
    tuning = {"site_coop": float(coop), "site_dt16": float(dt16), "coop_rate": float(rate), "greedy_waves": float(waves), "site_switch": float("0")}  # site_switch 0: the in-workgroup engine for every pass
    c = Context(0, tuning=tuning)
    try:
        c.set_sequences(codes, offsets, alpha)
        gp, gs, gpass = c.site_refine(W, 1e-4, 0, p0, sc0)
    finally:
        c.close()
    op, os_, opass = ol.site_refine(S, W, 1e-4, 0, p0, sc0)
    assert np.array_equal(gp, op) and gpass == opass
    check_scores(gs, os_)


@pytest.mark.parametrize("shift", [0, -1, 1])
def test_site_refine_pass_cap(gpu_ctx, shift):
    codes, offsets, S = dataset(100, 60, 8, b"ACGT", True, b"", 21)
    p0 = np.zeros(100, np.int32)
    sc0 = np.full(100, -np.inf)  # every target takes its first scan
    gpu_ctx.set_sequences(codes, offsets, b"ACGT")
    g = gpu_ctx.site_refine(8, 1e-4, shift, p0, sc0, max_passes=1)
    o = ol.site_refine(S, 8, 1e-4, shift, p0, sc0, max_passes=1)
    assert np.array_equal(g[0], o[0]) and g[2] == o[2] == 1
    check_scores(g[1], o[1])


@pytest.mark.parametrize("init_mode", [0, 1])
def test_site_sampling_pipeline(gpu_ctx, init_mode):
    """doSiteSampling end to end on the device vs the oracle's composition."""
    N, L, W, seed = 90, 80, 9, 1234
    codes, offsets, S = dataset(N, L, W, b"ACGT", True, b"", 31)
    gpu_ctx.set_sequences(codes, offsets, b"ACGT")
    gp, gs, gpasses = gpu_ctx.site_sampling(W, 1e-4, seed, init_mode)
    sc, p = ol.random_starts(S, W, 1e-4, seed=seed, mode=init_mode)
    passes = []
    for shift in (0, -1, 1):
        p, sc, k = ol.site_refine(S, W, 1e-4, shift, p, sc)
        passes.append(k)
    assert np.array_equal(gp, p)
    assert list(gpasses) == passes
    check_scores(gs, sc)


def test_site_positions_validated(gpu_ctx):
    from gibbssampling_amd._native import ArgumentError
    codes, offsets, S = dataset(10, 30, 6, b"ACGT", False, b"", 41)
    gpu_ctx.set_sequences(codes, offsets, b"ACGT")
    bad = np.zeros(10, np.int32)
    bad[3] = -1  # Positions = [] has no site-sampler meaning
    with pytest.raises(ArgumentError):
        gpu_ctx.site_scan(6, 1e-4, bad)
    bad[3] = 25  # 25 + 6 > 30
    with pytest.raises(ArgumentError):
        gpu_ctx.site_refine(6, 1e-4, 0, bad, np.zeros(10))


@pytest.mark.parametrize("switch,slots", [("1", "256"), ("1", "3"), ("16", "256"), ("0", "256")])
@pytest.mark.parametrize("N,L,W,alpha,extra", [(300, 90, 8, b"ACGT", b""),
                                               (40, 90, 9, b"ACDEFGHIKLMNPQRSTVWY", b"*")])
def test_site_greedy_handover_to_speculative_steps(monkeypatch, switch, slots, N, L, W, alpha,
                                                   extra):
    """Once a pass moves fewer than N / GS_SITE_SWITCH starts, the remaining passes of
    getBestPWMSsWithStartPositions run as speculative steps (visits scanned in parallel,
    committed up to the first move): the sequential passes exactly."""
    from gibbssampling_amd import Context
    codes, offsets, S = dataset(N, L, W, alpha, True, extra, 81 + N)
    sc0, p0 = ol.random_starts(S, W, 1e-4, seed=82, mode=1)
    tuning = {"site_switch": float(switch), "multi_spec_slots": float(slots)}
    c = Context(0, tuning=tuning)
    try:
        c.set_sequences(codes, offsets, alpha)
        gp, gs, gpass = c.site_refine(W, 1e-4, 0, p0, sc0)
        # the pipeline after it (shifted passes) sees the refined starts' aggregates
        gl, gls, glp = c.site_refine(W, 1e-4, -1, gp, gs)
    finally:
        c.close()
    op, os_, opass = ol.site_refine(S, W, 1e-4, 0, p0, sc0)
    assert np.array_equal(gp, op) and gpass == opass
    check_scores(gs, os_)
    ol_, ols, olp = ol.site_refine(S, W, 1e-4, -1, op, os_)
    assert np.array_equal(gl, ol_) and glp == olp


@pytest.mark.parametrize("chunk,switch", [("16", "4"), ("16", "1"), ("64", "16"), ("1", "2")])
@pytest.mark.parametrize("N,L,W,alpha,extra", [(500, 90, 8, b"ACGT", b""),
                                               (200, 120, 10, b"ACDEFGHIKLMNPQRSTVWY", b"*")])
@pytest.mark.parametrize("max_passes", [1, 2, 1000])
def test_site_greedy_mid_pass_handover(monkeypatch, chunk, switch, N, L, W, alpha, extra,
                                       max_passes):
    """The star engine leaves a pass once GS_SITE_EXIT_CHUNK visits move fewer than
    chunk / GS_SITE_EXIT_RATIO starts; the speculative steps resume at that visit with the
    pass's moved flag, and the pass cap counts the split pass once."""
    from gibbssampling_amd import Context
    codes, offsets, S = dataset(N, L, W, alpha, True, extra, 101 + N)
    sc0, p0 = ol.random_starts(S, W, 1e-4, seed=102, mode=1)
    tuning = {"site_exit_chunk": float(chunk), "site_exit_ratio": float(switch), "site_switch": float(switch)}
    c = Context(0, tuning=tuning)
    try:
        c.set_sequences(codes, offsets, alpha)
        gp, gs, gpass = c.site_refine(W, 1e-4, 0, p0, sc0, max_passes=max_passes)
    finally:
        c.close()
    op, os_, opass = ol.site_refine(S, W, 1e-4, 0, p0, sc0, max_passes=max_passes)
    assert np.array_equal(gp, op) and gpass == opass
    check_scores(gs, os_)
