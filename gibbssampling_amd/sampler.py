"""Host-side mirror of the reference's F# entry points for the hot path.

Same names, argument order and meaning as GibbsSampling.fs; the work runs in
libgibbs_hip.so on the GPU.  Error behaviour follows the .NET exceptions the
reference raises (see _native.py for the mapping).
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Callable, Sequence

import numpy as np

from . import _native
from .bioarray import alphabet_codes, pack


@dataclass(frozen=True)
class MotifIndex:
    """MotifSampler.MotifIndex (.fs:712-716)."""
    PWMS: float
    Positions: tuple


def createMotifIndex(pwms: float, pos) -> MotifIndex:       # .fs:719-723
    return MotifIndex(float(pwms), tuple(int(p) for p in pos))


#: the reference loops until a pass moves nothing (.fs:886-888, .fs:556-559); the
#: mirror's default pass cap is effectively unbounded, and a run that reaches an
#: explicit cap warns instead of passing for converged
UNBOUNDED = 2**31 - 1


def _passes(passes: int, max_passes: int) -> None:
    if max_passes < UNBOUNDED and passes >= max_passes:
        import warnings
        warnings.warn(f"refinement stopped at max_passes={max_passes}; the last pass may "
                      "still have moved positions (the reference loops until none moves)",
                      RuntimeWarning, stacklevel=3)


_contexts: dict[int, _native.Context] = {}


def context(device: int = 0) -> _native.Context:
    if device not in _contexts:
        _contexts[device] = _native.Context(device)
    return _contexts[device]


class _Bound:
    """Keeps the (sources, alphabet) last handed to a context to avoid re-uploads."""

    def __init__(self, ctx: _native.Context):
        self.ctx = ctx
        self.key = None

    def bind(self, alphabet, sources) -> None:
        codes, offsets = pack(sources)
        alpha = alphabet_codes(alphabet)
        key = (alpha, offsets.tobytes(), hash(codes.tobytes()))
        if key != self.key:
            self.ctx.set_sequences(codes, offsets, alpha)
            self.key = key


_bound: dict[int, _Bound] = {}


def _bind(alphabet, sources, device: int) -> _native.Context:
    if device not in _bound:
        _bound[device] = _Bound(context(device))
    _bound[device].bind(alphabet, sources)
    return _bound[device].ctx


def _uniforms(rnd, n: int) -> np.ndarray:
    """The n NextDouble() draws of `let rnd = new System.Random()` (.fs:936)."""
    if rnd is None:
        return np.random.default_rng().random(n)
    if isinstance(rnd, np.random.Generator):
        return rnd.random(n)
    if callable(rnd):
        return np.array([float(rnd()) for _ in range(n)], np.float64)
    if hasattr(rnd, "NextDouble"):
        return np.array([float(rnd.NextDouble()) for _ in range(n)], np.float64)
    u = np.asarray(rnd, np.float64)
    if u.shape != (n,):
        raise _native.ArgumentError(_native.GS_E_ARG, "need one uniform per sequence")
    return u


def _single_positions(motifMem: Sequence[MotifIndex]) -> np.ndarray:
    pos = np.empty(len(motifMem), np.int32)
    for i, m in enumerate(motifMem):
        pos[i] = m.Positions[0] if m.Positions else -1
    return pos


class MotifSampler:
    """MotifSampler module (.fs:709-1038): the hot-path entry points."""

    @staticmethod
    def findBestMotifIndicesByWithStartPositions(motifAmount: int, motifLength: int,
                                                 pseudoCount: float, cutOff: float, alphabet,
                                                 sources, motifMem: Sequence[MotifIndex],
                                                 rnd=None, device: int = 0) -> list[MotifIndex]:
        """One synchronous stochastic sweep (.fs:935-970).  motifAmount = 1 with single
        positions runs the ★ sweep kernel; otherwise the Positions-list path."""
        if len(motifMem) != len(sources):
            raise _native.ArgumentError(_native.GS_E_ARG, "motifMem and sources differ in length")
        ctx = _bind(alphabet, sources, device)
        u = _uniforms(rnd, len(sources))
        if _is_single(motifAmount, motifMem):
            pos_out, pwms = ctx.motif_sweep(motifLength, pseudoCount, cutOff,
                                            _single_positions(motifMem), u)
            return _motif_indices(pos_out, pwms)
        cap, cnt, pos = _lists(motifAmount, motifMem)
        co, po, pw = ctx.motif_sweep_multi(motifAmount, motifLength, pseudoCount, cutOff, cnt,
                                           pos, u, cap)
        return _motif_lists(co, po, pw)

    @staticmethod
    def runSweeps(motifLength: int, pseudoCount: float, cutOff: float, alphabet, sources,
                  motifMem: Sequence[MotifIndex], sweeps: int, seed: int, first_sweep: int = 0,
                  device: int = 0) -> list[MotifIndex]:
        """`sweeps` chained sweeps on the device (uniforms from the counter RNG)."""
        ctx = _bind(alphabet, sources, device)
        pos, pwms = ctx.motif_run(motifLength, pseudoCount, cutOff, sweeps, seed,
                                  _single_positions(motifMem), first_sweep)
        return _motif_indices(pos, pwms)

    @staticmethod
    def findBestMotifIndicesWithStartPositions(motifAmount: int, motifLength: int,
                                               pseudoCount: float, cutOff: float, alphabet,
                                               sources, motifMem: Sequence[MotifIndex],
                                               max_passes: int = UNBOUNDED,
                                               device: int = 0) -> list[MotifIndex]:
        """Greedy passes until no position moves (.fs:885-929)."""
        if len(motifMem) != len(sources):
            raise _native.ArgumentError(_native.GS_E_ARG, "motifMem and sources differ in length")
        ctx = _bind(alphabet, sources, device)
        pwms = np.array([m.PWMS for m in motifMem], np.float64)
        if _is_single(motifAmount, motifMem):
            pos, pwms, np_ = ctx.motif_greedy(motifLength, pseudoCount, cutOff,
                                              _single_positions(motifMem), pwms, max_passes)
            _passes(np_, max_passes)
            return _motif_indices(pos, pwms)
        cap, cnt, pos = _lists(motifAmount, motifMem)
        co, po, pw, np_ = ctx.motif_greedy_multi(motifAmount, motifLength, pseudoCount, cutOff,
                                                 cnt, pos, pwms, max_passes, cap)
        _passes(np_, max_passes)
        return _motif_lists(co, po, pw)

    @staticmethod
    def doMotifSampling(motifAmount: int, motifLength: int, pseudoCount: float, cutOff: float,
                        alphabet, sources, seed: int | None = None, init_mode: int = 0,
                        device: int = 0) -> list[MotifIndex]:
        """getPWMOfRandomStarts |> one sweep |> greedy passes (.fs:1034-1038), on the
        device.  seed None draws a fresh one (the reference's time-seeded Randoms)."""
        ctx = _bind(alphabet, sources, device)
        return _sampling(ctx, motifAmount, motifLength, pseudoCount, cutOff, _seed(seed),
                         init_mode)

    @staticmethod
    def getMotifsWithBestInformationContents(numberOfRepetitions: int, motifAmount: int,
                                             motifLength: int, pseudoCount: float,
                                             cutOff: float, alphabet, sources,
                                             seed: int | None = None, init_mode: int = 0,
                                             device: int = 0) -> list[MotifIndex]:
        """Repeated doMotifSampling keeping the run of largest Σ PWMS (.fs:973-998);
        run r uses seed + r."""
        base = _seed(seed)
        return _best_of_repetitions(
            numberOfRepetitions,
            lambda r: MotifSampler.doMotifSampling(motifAmount, motifLength, pseudoCount,
                                                   cutOff, alphabet, sources, base + r,
                                                   init_mode, device),
            lambda xs: sum(x.PWMS for x in xs), [createMotifIndex(0.0, [])])

    # ---- the caller's background (…ByPCV, .fs:788-881) and profile (…OfPPM) twins
    @staticmethod
    def findBestMotifPositionsWithStartPositionsByPCV(motifAmount: int, motifLength: int,
                                                      pseudoCount: float, cutOff: float,
                                                      alphabet, sources, pcv,
                                                      motifMem: Sequence[MotifIndex], rnd=None,
                                                      device: int = 0) -> list[MotifIndex]:
        """One stochastic sweep with the caller's pcv (.fs:828-853)."""
        ctx = _bind(alphabet, sources, device)
        with _fixed(ctx, pcv=pcv):
            return MotifSampler.findBestMotifIndicesByWithStartPositions(
                motifAmount, motifLength, pseudoCount, cutOff, alphabet, sources, motifMem, rnd,
                device)

    @staticmethod
    def findBestMotifPositionsWithStartPositionByPCV(motifAmount: int, motifLength: int,
                                                     pseudoCount: float, cutOff: float,
                                                     alphabet, sources, pcv,
                                                     motifMem: Sequence[MotifIndex],
                                                     max_passes: int = UNBOUNDED,
                                                     device: int = 0) -> list[MotifIndex]:
        """The greedy passes with the caller's pcv (.fs:788-823)."""
        ctx = _bind(alphabet, sources, device)
        with _fixed(ctx, pcv=pcv):
            return MotifSampler.findBestMotifIndicesWithStartPositions(
                motifAmount, motifLength, pseudoCount, cutOff, alphabet, sources, motifMem,
                max_passes, device)

    @staticmethod
    def findBestInormationContentContainingMotifsWithPCV(numberOfRepetitions: int,
                                                          motifAmount: int, motifLength: int,
                                                          pseudoCount: float, cutOff: float,
                                                          alphabet, sources, pcv,
                                                          seed: int | None = None,
                                                          device: int = 0) -> list[MotifIndex]:
        """Repetitions of getPWMOfRandomStartsWithBPV |> ByPCV sweep |> ByPCV greedy
        (.fs:856-881); run r uses seed + r."""
        ctx = _bind(alphabet, sources, device)
        base = _seed(seed)

        def run(r):
            with _fixed(ctx, pcv=pcv):
                return _sampling(ctx, motifAmount, motifLength, pseudoCount, cutOff, base + r, 0)
        return _best_of_repetitions(numberOfRepetitions, run, lambda xs: sum(x.PWMS for x in xs),
                                    [createMotifIndex(0.0, [])])

    @staticmethod
    def doMotifSamplingWithPPM(motifAmount: int, motifLength: int, pseudoCount: float,
                               cutOff: float, alphabet, sources, positionProbabilityMatrix,
                               seed: int | None = None, device: int = 0) -> list[MotifIndex]:
        """getMotifsWithBestPWMSOfPPM |> sweep |> greedy passes (.fs:1028-1032)."""
        ctx = _bind(alphabet, sources, device)
        with _fixed(ctx, ppm=positionProbabilityMatrix, W=motifLength):
            return _sampling(ctx, motifAmount, motifLength, pseudoCount, cutOff, _seed(seed), 0)

    @staticmethod
    def getBestPWMSsOfPPM(numberOfRepetitions: int, motifAmount: int, motifLength: int,
                          pseudoCount: float, cutOff: float, alphabet, sources,
                          positionProbabilityMatrix, seed: int | None = None,
                          device: int = 0) -> list[MotifIndex]:
        """Repetitions of doMotifSamplingWithPPM (.fs:1001-1026); run r uses seed + r."""
        base = _seed(seed)
        return _best_of_repetitions(
            numberOfRepetitions,
            lambda r: MotifSampler.doMotifSamplingWithPPM(
                motifAmount, motifLength, pseudoCount, cutOff, alphabet, sources,
                positionProbabilityMatrix, base + r, device),
            lambda xs: sum(x.PWMS for x in xs), [createMotifIndex(0.0, [])])


class _fixed:
    """Sets the caller's pcv / ppm on a context for the duration of one call."""

    def __init__(self, ctx, pcv=None, ppm=None, W=None):
        self.ctx, self.pcv, self.ppm, self.W = ctx, pcv, ppm, W

    def __enter__(self):
        if self.pcv is not None:
            self.ctx.set_fixed_pcv(np.asarray(self.pcv, np.float64))
        if self.ppm is not None:
            self.ctx.set_fixed_ppm(np.asarray(self.ppm, np.float64), self.W)
        return self.ctx

    def __exit__(self, *exc):
        if self.pcv is not None:
            self.ctx.set_fixed_pcv(None)
        if self.ppm is not None:
            self.ctx.set_fixed_ppm(None)
        return False


def _is_single(motifAmount: int, motifMem: Sequence[MotifIndex]) -> bool:
    """motifAmount = 1 and no list longer than one: the ★ kernels' snapshot form."""
    return motifAmount == 1 and all(len(m.Positions) <= 1 for m in motifMem)


def _lists(motifAmount: int, motifMem: Sequence[MotifIndex]):
    """MotifIndex[] -> (cap, cnt[N], pos[N, cap]) in F# list order."""
    if not 1 <= motifAmount <= 16:
        raise _native.ArgumentError(_native.GS_E_ARG, "motifAmount must be in [1, 16]")
    cap = max([motifAmount] + [len(m.Positions) for m in motifMem])
    cnt = np.array([len(m.Positions) for m in motifMem], np.int32)
    pos = np.full((len(motifMem), cap), -1, np.int32)
    for i, m in enumerate(motifMem):
        pos[i, :len(m.Positions)] = m.Positions
    return cap, cnt, pos


def _sampling(ctx, motifAmount, motifLength, pseudoCount, cutOff, seed, init_mode):
    """doMotifSampling on the device: the ★ kernels for motifAmount = 1, else the
    Positions-list path."""
    if motifAmount == 1:
        pos, pwms, _ = ctx.motif_sampling(motifLength, pseudoCount, cutOff, seed, init_mode,
                                          UNBOUNDED)
        return _motif_indices(pos, pwms)
    co, po, pw, _ = ctx.motif_sampling_multi(motifAmount, motifLength, pseudoCount, cutOff, seed,
                                             init_mode, UNBOUNDED)
    return _motif_lists(co, po, pw)


def _motif_indices(pos, pwms) -> list[MotifIndex]:
    return [createMotifIndex(w, [] if p < 0 else [p]) for p, w in zip(pos, pwms)]


def _motif_lists(cnt, pos, pwms) -> list[MotifIndex]:
    return [createMotifIndex(w, pos[n, :cnt[n]]) for n, w in enumerate(pwms)]


def _seed(seed: int | None) -> int:
    if seed is None:
        return int.from_bytes(os.urandom(8), "little")
    return int(seed) & (2**64 - 1)


def _best_of_repetitions(numberOfRepetitions: int, run: Callable[[int], list], ic: Callable,
                         initial_best: list) -> list:
    """The repetition loop shared by getMotifsWithBestInformationContent(s)
    (.fs:615-640, .fs:973-998): stop after numberOfRepetitions or when a run equals
    the best; a run whose Σ score beats the best replaces it (one step later)."""
    n, acc, best = 0, [], initial_best
    while True:
        if n > numberOfRepetitions or acc == best:
            return best
        if ic(acc) > ic(best):
            n, acc, best = n + 1, [], (best if not acc else acc)
        else:
            n, acc = n + 1, run(n)


class SiteSampler:
    """SiteSampler module (.fs:298-707): the initialiser used by every driver."""

    @staticmethod
    def getPWMOfRandomStarts(motifLength: int, pseudoCount: float, alphabet, sources,
                             seed: int = 0, mode: int = 0, device: int = 0):
        """.fs:589-611 -> [(log2 best score, start)].  mode 0: every target draws its own
        starts for all others (the reference's O(N^2) structure); mode 1: one shared vector."""
        ctx = _bind(alphabet, sources, device)
        score, pos = ctx.random_starts(motifLength, pseudoCount, seed, mode)
        return _pairs(score, pos)

    @staticmethod
    def _refine(shift: int, motifLength: int, pseudoCount: float, alphabet, sources,
                startPositions, max_passes: int, device: int):
        if len(startPositions) != len(sources):
            raise _native.ArgumentError(_native.GS_E_ARG,
                                        "startPositions and sources differ in length")
        ctx = _bind(alphabet, sources, device)
        score = np.array([s for s, _ in startPositions], np.float64)
        pos = np.array([p for _, p in startPositions], np.int32)
        pos, score, np_ = ctx.site_refine(motifLength, pseudoCount, shift, pos, score, max_passes)
        _passes(np_, max_passes)
        return _pairs(score, pos)

    @staticmethod
    def getBestPWMSsWithStartPositions(motifLength: int, pseudoCount: float, alphabet, sources,
                                       startPositions, max_passes: int = UNBOUNDED, device: int = 0):
        """Gauss–Seidel passes over the live positions (.fs:554-585)."""
        return SiteSampler._refine(0, motifLength, pseudoCount, alphabet, sources,
                                   startPositions, max_passes, device)

    @staticmethod
    def getLeftShiftedBestPWMSs(motifLength: int, pseudoCount: float, alphabet, sources,
                                startPositions, max_passes: int = UNBOUNDED, device: int = 0):
        """Passes with the others one position upstream (.fs:519-550)."""
        return SiteSampler._refine(-1, motifLength, pseudoCount, alphabet, sources,
                                   startPositions, max_passes, device)

    @staticmethod
    def getRightShiftedBestPWMSs(motifLength: int, pseudoCount: float, alphabet, sources,
                                 startPositions, max_passes: int = UNBOUNDED, device: int = 0):
        """Passes with the others one position downstream (.fs:483-517)."""
        return SiteSampler._refine(1, motifLength, pseudoCount, alphabet, sources,
                                   startPositions, max_passes, device)

    @staticmethod
    def doSiteSampling(motifLength: int, pseudoCount: float, alphabet, sources,
                       seed: int | None = None, init_mode: int = 0, device: int = 0):
        """getPWMOfRandomStarts |> getBestPWMSsWithStartPositions |> left |> right
        shifted passes (.fs:697-701), on the device."""
        ctx = _bind(alphabet, sources, device)
        pos, score, _ = ctx.site_sampling(motifLength, pseudoCount, _seed(seed), init_mode,
                                          UNBOUNDED)
        return _pairs(score, pos)

    @staticmethod
    def getMotifsWithBestInformationContent(numberOfRepetitions: int, motifLength: int,
                                            pseudoCount: float, alphabet, sources,
                                            seed: int | None = None, init_mode: int = 0,
                                            device: int = 0):
        """Repeated doSiteSampling keeping the run of largest Σ score (.fs:615-640);
        run r uses seed + r."""
        base = _seed(seed)
        return _best_of_repetitions(
            numberOfRepetitions,
            lambda r: SiteSampler.doSiteSampling(motifLength, pseudoCount, alphabet, sources,
                                                 base + r, init_mode, device),
            lambda xs: sum(s for s, _ in xs), [(0.0, 0)])

    # ---- the caller's background (…WithBPV, .fs:301-459, .fs:691-695) and profile
    # (…OfPPM, .fs:644-689, .fs:703-707) twins
    @staticmethod
    def getPWMOfRandomStartsWithBPV(motifLength: int, pseudoCount: float, alphabet, sources,
                                    pcv, seed: int = 0, mode: int = 0, device: int = 0):
        """.fs:412-431: random starts, the others' PPM, getBestPWMSsWithBPV."""
        ctx = _bind(alphabet, sources, device)
        with _fixed(ctx, pcv=pcv):
            score, pos = ctx.random_starts(motifLength, pseudoCount, seed, mode)
        return _pairs(score, pos)

    @staticmethod
    def _refine_bpv(shift, motifLength, pseudoCount, alphabet, sources, pcv, startPositions,
                    max_passes, device):
        ctx = _bind(alphabet, sources, device)
        with _fixed(ctx, pcv=pcv):
            return SiteSampler._refine(shift, motifLength, pseudoCount, alphabet, sources,
                                       startPositions, max_passes, device)

    @staticmethod
    def findBestMotifWithStartPosition(motifLength: int, pseudoCount: float, alphabet, sources,
                                       pcv, startPositions, max_passes: int = UNBOUNDED,
                                       device: int = 0):
        """Gauss–Seidel passes with the caller's pcv (.fs:381-409)."""
        return SiteSampler._refine_bpv(0, motifLength, pseudoCount, alphabet, sources, pcv,
                                       startPositions, max_passes, device)

    @staticmethod
    def getLeftShiftedBestPWMSsWithBPV(motifLength: int, pseudoCount: float, alphabet, sources,
                                       pcv, startPositions, max_passes: int = UNBOUNDED,
                                       device: int = 0):
        """.fs:350-378."""
        return SiteSampler._refine_bpv(-1, motifLength, pseudoCount, alphabet, sources, pcv,
                                       startPositions, max_passes, device)

    @staticmethod
    def getRightShiftedBestPWMSsWithBPV(motifLength: int, pseudoCount: float, alphabet, sources,
                                        pcv, startPositions, max_passes: int = UNBOUNDED,
                                        device: int = 0):
        """.fs:318-347."""
        return SiteSampler._refine_bpv(1, motifLength, pseudoCount, alphabet, sources, pcv,
                                       startPositions, max_passes, device)

    @staticmethod
    def doSiteSamplingWithBPV(motifLength: int, pseudoCount: float, alphabet, sources, pcv,
                              seed: int | None = None, init_mode: int = 0, device: int = 0):
        """.fs:691-695: every stage with the caller's pcv."""
        ctx = _bind(alphabet, sources, device)
        with _fixed(ctx, pcv=pcv):
            pos, score, _ = ctx.site_sampling(motifLength, pseudoCount, _seed(seed), init_mode,
                                          UNBOUNDED)
        return _pairs(score, pos)

    @staticmethod
    def getMotifsWithBestInformationContentWithBPV(numberOfRepetitions: int, motifLength: int,
                                                   pseudoCount: float, alphabet, sources, pcv,
                                                   seed: int | None = None, init_mode: int = 0,
                                                   device: int = 0):
        """.fs:434-459; run r uses seed + r."""
        base = _seed(seed)
        return _best_of_repetitions(
            numberOfRepetitions,
            lambda r: SiteSampler.doSiteSamplingWithBPV(motifLength, pseudoCount, alphabet,
                                                        sources, pcv, base + r, init_mode, device),
            lambda xs: sum(s for s, _ in xs), [(0.0, 0)])

    @staticmethod
    def getMotifsWithBestPWMSOfPPM(motifLength: int, pseudoCount: float, alphabet, sources,
                                   positionProbabilityMatrix, seed: int = 0, mode: int = 0,
                                   device: int = 0):
        """.fs:644-662: the random starts give the background, the caller's PPM scores."""
        ctx = _bind(alphabet, sources, device)
        with _fixed(ctx, ppm=positionProbabilityMatrix, W=motifLength):
            score, pos = ctx.random_starts(motifLength, pseudoCount, seed, mode)
        return _pairs(score, pos)

    @staticmethod
    def doSiteSamplingWithPPM(motifLength: int, pseudoCount: float, alphabet, sources,
                              positionProbabilityMatrix, seed: int | None = None,
                              init_mode: int = 0, device: int = 0):
        """.fs:703-707: getMotifsWithBestPWMSOfPPM |> the three refinements."""
        ctx = _bind(alphabet, sources, device)
        with _fixed(ctx, ppm=positionProbabilityMatrix, W=motifLength):
            pos, score, _ = ctx.site_sampling(motifLength, pseudoCount, _seed(seed), init_mode,
                                          UNBOUNDED)
        return _pairs(score, pos)

    @staticmethod
    def getBestInformationContentOfPPM(numberOfRepetitions: int, motifLength: int,
                                       pseudoCount: float, alphabet, sources,
                                       positionProbabilityMatrix, seed: int | None = None,
                                       init_mode: int = 0, device: int = 0):
        """.fs:664-689; run r uses seed + r."""
        base = _seed(seed)
        return _best_of_repetitions(
            numberOfRepetitions,
            lambda r: SiteSampler.doSiteSamplingWithPPM(motifLength, pseudoCount, alphabet,
                                                        sources, positionProbabilityMatrix,
                                                        base + r, init_mode, device),
            lambda xs: sum(s for s, _ in xs), [(0.0, 0)])


def _pairs(score, pos) -> list[tuple[float, int]]:
    return [(float(s), int(p)) for s, p in zip(score, pos)]
