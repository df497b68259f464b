"""GPU parity: libgibbs_hip.so against the CPU oracle on the same seeded inputs.

Bar (BASELINE.json north_star): integer count matrices bit-exact; positions
identical (no tolerance on indices: a pick the binary32 bound cannot certify is
taken in binary64 exactly as the reference does); PWMS within 1e-5 relative (we
hold them to 1e-12: every product and quotient is the same IEEE binary64 operation,
only log() may differ in the last ulp between the device math library and glibc).
"""
import numpy as np
import pytest

from conftest import init_positions, make_dataset
from oracle import oracle_lib as ol

pytestmark = pytest.mark.gpu

PWMS_RTOL = 1e-12


def check_sweep(gpos, gpw, opos, opw, margin=None):
    bad = np.nonzero(gpos != opos)[0]
    assert bad.size == 0, f"{bad.size} positions differ, first {bad[:10]}"
    rel = np.abs(gpw - opw) / np.maximum(np.abs(opw), 1e-300)
    same_inf = (gpw == opw)
    assert np.all(same_inf | (rel <= PWMS_RTOL)), f"PWMS rel diff {rel.max():.3e}"


def run_case(ctx, codes, offsets, alpha, W, pc, cutoff, pos, u):
    ctx.set_sequences(codes, offsets, alpha)
    gpos, gpw = ctx.motif_sweep(W, pc, cutoff, pos, u)
    opos, opw, margin = ol.sweep(ol.Seqs(codes, offsets, alpha), W, pc, cutoff, pos, u)
    check_sweep(gpos, gpw, opos, opw, margin)
    return gpos, gpw


@pytest.fixture
def exact_scan(gpu_ctx):
    """Run a test with the binary64-for-every-window scan, then restore the default."""
    gpu_ctx.set_scan_mode(exact=True)
    yield gpu_ctx
    gpu_ctx.set_scan_mode(exact=False)


SHAPES = [
    (100, 50, 8, b"ACGT", False, 0.0, 0),        # BASELINE config 1
    (100, 50, 8, b"ACGT", True, 0.2, 1),
    (300, 120, 12, b"ACGT", True, 0.1, 2),
    (64, 90, 7, b"ATGC-", True, 0.0, 3),         # dnaBases of the .fsx (|A| = 5)
    (200, 300, 20, b"ACDEFGHIKLMNPQRSTVWY", False, 0.0, 4),  # protein (config 5 shape, small N)
    (50, 700, 15, b"ACGT", True, 0.3, 5),        # long sequences, > 64 windows per chunk
    (3, 20, 20, b"ACGT", False, 0.0, 6),         # L == W: a single window
    (1, 30, 6, b"ACGT", False, 0.0, 7),          # N == 1: den = |A|*pc
    (40, 2000, 9, b"ACGT", True, 0.0, 8),        # > 4096 windows: > 64 windows per lane
    (60, 200, 33, b"ACGT", True, 0.1, 9),        # W > 32 (8-wide unroll classes)
]


@pytest.mark.parametrize("N,L,W,alpha,ragged,none_rate,seed", SHAPES)
def test_sweep_matches_oracle(gpu_ctx, N, L, W, alpha, ragged, none_rate, seed):
    codes, offsets = make_dataset(N, L, W, alpha, seed=seed, ragged=ragged)
    pos = init_positions(offsets, W, seed + 100, none_rate)
    u = np.random.default_rng(seed + 200).random(N)
    run_case(gpu_ctx, codes, offsets, alpha, W, 1e-4, 1.0, pos, u)


@pytest.mark.parametrize("N,L,W,alpha,ragged,none_rate,seed", SHAPES)
def test_exact_scan_matches_oracle(exact_scan, N, L, W, alpha, ragged, none_rate, seed):
    codes, offsets = make_dataset(N, L, W, alpha, seed=seed, ragged=ragged)
    pos = init_positions(offsets, W, seed + 100, none_rate)
    u = np.random.default_rng(seed + 200).random(N)
    run_case(exact_scan, codes, offsets, alpha, W, 1e-4, 1.0, pos, u)


def test_fastmath_error_model(gpu_ctx):
    """The certified scan budgets 2^-22 for the device log2/exp2 errors; the measured
    worst cases must sit well inside that budget."""
    from gibbssampling_amd import _native
    el, ee = gpu_ctx.fastmath_check()
    assert 0 <= el <= _native.LOG2_ERR_BUDGET / 2, el
    assert 0 <= ee <= _native.EXP2_ERR_BUDGET / 2, ee


@pytest.mark.parametrize("W,alpha,pc", [(12, b"ACGT", 1e-4), (8, b"ATGC-", 0.5),
                                        (20, b"ACDEFGHIKLMNPQRSTVWY", 1e-4)])
def test_certified_equals_exact_chain(gpu_ctx, W, alpha, pc):
    """Certified binary32 scan and binary64 scan give bit-identical chains."""
    N, L, seed = 3000, 240, 4242
    codes, offsets = make_dataset(N, L, W, alpha, seed=111, ragged=True, mut=0.15,
                                  extra=b"*", extra_rate=0.002)
    pos = init_positions(offsets, W, 112, 0.1)
    gpu_ctx.set_sequences(codes, offsets, alpha)
    s0 = gpu_ctx.stats()
    got = gpu_ctx.motif_run(W, pc, 1.0, 8, seed, pos)
    s1 = gpu_ctx.stats()
    gpu_ctx.set_scan_mode(exact=True)
    try:
        ref = gpu_ctx.motif_run(W, pc, 1.0, 8, seed, pos)
    finally:
        gpu_ctx.set_scan_mode(exact=False)
    assert np.array_equal(got[0], ref[0])
    assert np.array_equal(got[1], ref[1])
    # the certified path decides nearly every sequence on its own
    assert s1["exact_rescans"] - s0["exact_rescans"] <= 0.01 * 8 * N


@pytest.mark.parametrize("group_lanes", ["16", "32", "64"])
def test_lane_groups_partial_iterations(group_lanes, monkeypatch):
    """Several sequences per wavefront (lane groups of 16/32/64): with the grid capped
    at one workgroup per CU, wavefronts run many iterations and the last one is
    partly empty (its idle groups hold other groups' descriptors)."""
    from gibbssampling_amd import Context
    N, L, W = 1024 * 40 + 7, 60, 8
    codes, offsets = make_dataset(N, L, W, seed=131, ragged=True)
    pos = init_positions(offsets, W, 132, 0.1)
    u = np.random.default_rng(133).random(N)
    tuning = {"blocks_per_cu_cap": float("1"), "group_lanes": float(group_lanes)}
    c = Context(0, tuning=tuning)
    try:
        gpos, gpw = run_case(c, codes, offsets, b"ACGT", W, 1e-4, 1.0, pos, u)
    finally:
        c.close()


def test_cutoff_on_window_scores(gpu_ctx):
    """Cut-offs placed exactly on (and next to) window scores of the targets: the
    binary32 scan's band must hand every such window to the binary64 fold."""
    N, L, W = 60, 80, 8
    codes, offsets = make_dataset(N, L, W, seed=121, mut=0.05)
    pos = init_positions(offsets, W, 122)
    S = ol.Seqs(codes, offsets, b"ACGT")
    u = np.random.default_rng(123).random(N)
    d = ol.target_detail(S, W, 1e-4, pos, 3)
    l2 = np.log(np.asarray(d["S"], np.float64)) / np.log(2.0)
    for cut in (float(np.sort(l2)[-3]), float(np.nextafter(np.sort(l2)[-5], -np.inf)),
                float(np.median(l2))):
        run_case(gpu_ctx, codes, offsets, b"ACGT", W, 1e-4, cut, pos, u)


@pytest.mark.parametrize("cutoff", [0.0, 1.0, 5.0, 1e9, -1.0])
def test_sweep_cutoffs(gpu_ctx, cutoff):
    codes, offsets = make_dataset(150, 80, 8, seed=11, mut=0.05)
    pos = init_positions(offsets, 8, 12)
    u = np.random.default_rng(13).random(150)
    try:
        run_case(gpu_ctx, codes, offsets, b"ACGT", 8, 1e-4, cutoff, pos, u)
    except Exception as e:  # negative weights may legitimately overrun in both
        from gibbssampling_amd import RouletteOverrunError
        assert isinstance(e, RouletteOverrunError) and cutoff < 0


def test_non_alphabet_symbols(gpu_ctx):
    """'*' (Ter, .fsx:63), 'N' and '-' outside the alphabet: PWM 0, raw-count PCV (Q3)."""
    codes, offsets = make_dataset(120, 100, 8, seed=21, extra=b"*N-", extra_rate=0.03,
                                  ragged=True)
    pos = init_positions(offsets, 8, 22, 0.1)
    u = np.random.default_rng(23).random(120)
    run_case(gpu_ctx, codes, offsets, b"ACGT", 8, 1e-4, 1.0, pos, u)


def test_pseudocounts(gpu_ctx):
    codes, offsets = make_dataset(80, 60, 6, seed=31)
    pos = init_positions(offsets, 6, 32)
    u = np.random.default_rng(33).random(80)
    for pc in (1e-4, 0.5, 1.0, 3.0):
        run_case(gpu_ctx, codes, offsets, b"ACGT", 6, pc, 1.0, pos, u)


def test_counts_exact(gpu_ctx):
    for seed, (N, L, W, alpha) in enumerate([(100, 50, 8, b"ACGT"), (500, 200, 12, b"ACGT"),
                                              (300, 300, 20, b"ACDEFGHIKLMNPQRSTVWY")]):
        codes, offsets = make_dataset(N, L, W, alpha, seed=seed, ragged=True, extra=b"*",
                                      extra_rate=0.01)
        pos = init_positions(offsets, W, seed, 0.2)
        gpu_ctx.set_sequences(codes, offsets, alpha)
        Cg, Tg = gpu_ctx.counts(W, pos, len(alpha))
        Co, To = ol.counts(ol.Seqs(codes, offsets, alpha), W, pos)
        assert np.array_equal(Cg, Co)
        assert np.array_equal(Tg, To)


def test_boundary_u_uses_exact_fallback(gpu_ctx):
    """u placed exactly on a CDF boundary forces the serial exact path."""
    codes, offsets = make_dataset(40, 40, 6, seed=41)
    pos = init_positions(offsets, 6, 42)
    S = ol.Seqs(codes, offsets, b"ACGT")
    # boundaries: cumulative normalised background weights of target 0
    d = ol.target_detail(S, 6, 1e-4, pos, 0)
    G = d["G"]
    tot = 0.0
    for g in G:
        tot = tot + g
    acc = 0.0
    for g in G[:5]:
        acc = acc + g / tot
    u = np.random.default_rng(43).random(40)
    u[0] = acc  # exactly the left edge of category 5 (if nothing passes the cut-off)
    before = gpu_ctx.stats()
    run_case(gpu_ctx, codes, offsets, b"ACGT", 6, 1e-4, 1e9, pos, u)
    after = gpu_ctx.stats()
    assert after["exact_rescans"] >= before["exact_rescans"] + 1
    assert after["serial_picks"] >= before["serial_picks"] + 1


def test_overrun_raises(gpu_ctx):
    from gibbssampling_amd import RouletteOverrunError
    codes, offsets = make_dataset(30, 40, 6, seed=51)
    pos = init_positions(offsets, 6, 52)
    u = np.random.default_rng(53).random(30)
    u[7] = 2.0  # beyond every category: the reference's list index overruns
    gpu_ctx.set_sequences(codes, offsets, b"ACGT")
    with pytest.raises(RouletteOverrunError) as ei:
        gpu_ctx.motif_sweep(6, 1e-4, 1.0, pos, u)
    assert ei.value.index == 7
    with pytest.raises(ol.OracleError):
        ol.sweep(ol.Seqs(codes, offsets, b"ACGT"), 6, 1e-4, 1.0, pos, u)


def test_argument_errors(gpu_ctx):
    from gibbssampling_amd import ArgumentError
    codes, offsets = make_dataset(10, 30, 6, seed=61)
    gpu_ctx.set_sequences(codes, offsets, b"ACGT")
    pos = init_positions(offsets, 6, 62)
    u = np.zeros(10)
    bad = pos.copy()
    bad[3] = 25  # 25 + 6 > 30
    with pytest.raises(ArgumentError):
        gpu_ctx.motif_sweep(6, 1e-4, 1.0, bad, u)
    with pytest.raises(ArgumentError):
        gpu_ctx.motif_sweep(31, 1e-4, 1.0, pos, u)
    with pytest.raises(ArgumentError):
        gpu_ctx.set_sequences(codes, offsets, b"ACGA")
    with pytest.raises(ArgumentError):
        gpu_ctx.set_sequences(np.full(30, 33, np.uint8), np.array([0, 30]), b"ACGT")


def test_chained_sweeps_match_oracle(gpu_ctx):
    """gs_run_sweeps: device-resident chain with counter-RNG uniforms."""
    N, L, W, seed = 400, 150, 10, 0xC0FFEE
    codes, offsets = make_dataset(N, L, W, seed=71, mut=0.1)
    pos = init_positions(offsets, W, 72)
    gpu_ctx.set_sequences(codes, offsets, b"ACGT")
    gpos, gpw = gpu_ctx.motif_run(W, 1e-4, 1.0, 6, seed, pos)
    S = ol.Seqs(codes, offsets, b"ACGT")
    p = pos.copy()
    for t in range(6):
        u = np.array([ol.uniform(seed, ol.stream_sweep(t), n) for n in range(N)])
        p, w, _ = ol.sweep(S, W, 1e-4, 1.0, p, u)
    assert np.array_equal(gpos, p)
    np.testing.assert_allclose(gpw, w, rtol=PWMS_RTOL)


def test_counter_rng_matches_oracle():
    from gibbssampling_amd import _native
    for (s, st, i) in [(0, 0, 0), (1, _native.stream_sweep(3), 12345), (2**64 - 1, 7, 2**40)]:
        assert _native.uniform(s, st, i) == ol.uniform(s, st, i)


def test_two_shards_bit_identical(gpu_ctx):
    """The multi-GPU decomposition on one device: two shard contexts with host-staged
    aggregate exchange reproduce the single-context chain bit for bit."""
    from gibbssampling_amd import Context
    N, L, W, seed = 1000, 120, 10, 99
    codes, offsets = make_dataset(N, L, W, seed=91, ragged=True, mut=0.1)
    pos = init_positions(offsets, W, 92)
    gpu_ctx.set_sequences(codes, offsets, b"ACGT")
    ref_pos, ref_pw = gpu_ctx.motif_run(W, 1e-4, 1.0, 4, seed, pos)
    cut = 437
    shards = []
    for lo, hi in [(0, cut), (cut, N)]:
        c = Context(0)
        o = offsets[lo:hi + 1] - offsets[lo]
        c.set_sequences(codes[offsets[lo]:offsets[hi]], o, b"ACGT", n_global=N, global_offset=lo)
        shards.append((c, lo, hi))

    def exchange():
        tot = sum(c.agg_download() for c, _, _ in shards)
        for c, _, _ in shards:
            c.agg_upload(tot)

    for c, lo, hi in shards:
        c.set_positions(W, pos[lo:hi])
    exchange()
    for t in range(4):
        for c, _, _ in shards:
            c.run_sweeps(1e-4, 1.0, 1, seed, t)
        exchange()
    got_pos = np.concatenate([c.get_state()[0] for c, _, _ in shards])
    got_pw = np.concatenate([c.get_state()[1] for c, _, _ in shards])
    assert np.array_equal(got_pos, ref_pos)
    assert np.array_equal(got_pw, ref_pw)
    for c, _, _ in shards:
        c.close()


@pytest.mark.parametrize("mode,N,L,W,alpha", [
    (0, 60, 50, 8, b"ACGT"),
    (0, 40, 120, 10, b"ATGC-"),
    (1, 2000, 200, 12, b"ACGT"),
    (1, 300, 300, 20, b"ACDEFGHIKLMNPQRSTVWY"),
])
def test_random_starts_match_oracle(gpu_ctx, mode, N, L, W, alpha):
    codes, offsets = make_dataset(N, L, W, alpha, seed=101, ragged=True, extra=b"*",
                                  extra_rate=0.005)
    gpu_ctx.set_sequences(codes, offsets, alpha)
    gs, gp = gpu_ctx.random_starts(W, 1e-4, 12345, mode)
    t1 = N if mode == 0 or N <= 400 else 400
    os_, op = ol.random_starts(ol.Seqs(codes, offsets, alpha), W, 1e-4, 12345, mode, t1=t1)
    assert np.array_equal(gp[:t1], op[:t1])
    np.testing.assert_allclose(gs[:t1], os_[:t1], rtol=PWMS_RTOL)


@pytest.mark.parametrize("N,L,W,alpha,extra", [
    (5, 60, 6, b"ATGC-", b""),
    (3, 300, 12, b"ACGT", b"*N"),
    (4, 250, 20, b"ACDEFGHIKLMNPQRSTVWY", b""),
    (2, 9, 12, b"ACGT", b""),            # L < W: (log2 0., 0) without a window
])
def test_best_pwms_matches_oracle(gpu_ctx, N, L, W, alpha, extra):
    """getBestPWMSs (.fs:462-479) against a caller's FrequencyCompositeVector and PPM,
    the background drifting window after window (quirk Q1)."""
    rng = np.random.default_rng(123 + W)
    codes, offsets = make_dataset(N, max(L, W), W, alpha, seed=7, extra=extra, extra_rate=0.01)
    if L < W:
        codes = codes.reshape(N, -1)[:, :L].reshape(-1).copy()
        offsets = np.arange(0, N * L + 1, L, dtype=np.int64)
    gpu_ctx.set_sequences(codes, offsets, alpha)
    S = ol.Seqs(codes, offsets, alpha)
    for n in range(N):
        fcv = np.zeros(49, np.int64)
        for a in alpha:
            fcv[a - 42] = rng.integers(50, 5000)
        fcv[ord("*") - 42] = rng.integers(0, 30)
        ppm = np.zeros((49, W))
        for a in alpha:
            ppm[a - 42] = rng.random(W) + 1e-3
        ppm /= ppm.sum(0, keepdims=True)
        # the oracle takes the PPM by alphabet index, the library by slot (49 x W)
        want = ol.best_pwms(S, W, 1e-4, n, fcv, ppm[[a - 42 for a in alpha]])
        got = gpu_ctx.best_pwms(W, 1e-4, n, fcv, ppm)
        if L < W:
            assert want == (-np.inf, 0) and got == want
            continue
        assert got[1] == want[1]
        assert got[0] == want[0] or abs(got[0] - want[0]) <= PWMS_RTOL * abs(want[0])
