"""Pure-Python literal restatement of GibbsSampling/GibbsSampling.fs.

TEST INFRASTRUCTURE ONLY: used by tests/ to cross-check the C restatement
(oracle/gibbs_oracle.c) bit for bit on small inputs.  Written independently of
the C file, function by function after the F# source, keeping its data flow
(lists, folds, in-place mutation where the F# mutates).  Parity against
reference-produced numbers is UNPINNED (the F# cannot run here and ships no
golden vectors) -- see oracle/gibbs_oracle.h.

Symbols are ASCII codes (BioItem.symbol), slot = code - 42 (.fs:16-17).
All floats are Python floats (IEEE binary64); math.log is the C library log.
"""
from __future__ import annotations

import math

NSLOT = 49


def log2(x: float) -> float:
    """FSharpAux.Math.log2 = Math.Log(x, 2.0) = Log(x)/Log(2.0)."""
    if x == 0.0:
        return -math.inf
    if x < 0.0 or x != x:
        return math.nan
    if x == math.inf:
        return math.inf
    return math.log(x) / 0.6931471805599453


def idx(sym: int) -> int:
    return sym - 42


# ---------------------------------------------------------------- CompositeVector
def createFCVOf(res):                                    # .fs:60-62
    v = [0] * NSLOT
    for b in res:
        v[idx(b)] += 1
    return v


def fuseFrequencyVectors(alphabet, vectors):             # .fs:65-70
    out = [0] * NSLOT
    for v in vectors:
        for a in alphabet:
            out[idx(a)] += v[idx(a)]
    return out


def createFCVWithout(W, position, res):                  # .fs:73-76
    return createFCVOf(list(res[0:position]) + list(res[position + W:]))


def increaseInPlaceFCVOf(res, fcv):                      # .fs:79-81 (mutates)
    for b in res:
        fcv[idx(b)] += 1
    return fcv


def substractSegmentCountsFrom(seg, fcv):                # .fs:84-88 (aliases fcv)
    for b in seg:
        fcv[idx(b)] = fcv[idx(b)] - 1 if fcv[idx(b)] - 1 > 0 else 0
    return fcv


def checked_int32_sum(v):
    s = 0
    for x in v:
        s += x
        if s > 2**31 - 1 or s < -(2**31):
            raise OverflowError("Array.sum overflow")
    return s


def createNormalizedPCVOfFCV(alphabet, pc, fcv):         # .fs:115-120
    pcv = [float(x) for x in fcv]
    total = float(checked_int32_sum(fcv)) + float(len(alphabet)) * pc
    for a in alphabet:
        pcv[idx(a)] = (pcv[idx(a)] + pc) / total
    return pcv


def bg_segment_score(pcv, items):                        # .fs:123-124
    v = 1.0
    for b in items:
        v = v * pcv[idx(b)]
    return v


# ---------------------------------------------------------------- PositionMatrix
def ceckForDistance(width, items):                       # .fs:129-140
    if len(items) <= 1:
        return True
    for n in range(len(items) - 1):
        for i in range(n + 1, len(items)):
            if not abs(items[n] - items[i]) > width:
                return False
    return True


def getSegment(W, source, start):                        # .fs:149-153
    if start < 0 or start + W > len(source):
        raise IndexError("getSegment")
    return list(source[start:start + W])


def createPFMOf(seg):                                    # .fs:211-215
    m = [[0] * len(seg) for _ in range(NSLOT)]
    for j, b in enumerate(seg):
        m[idx(b)][j] += 1
    return m


def fusePositionFrequencyMatrices(W, mats):              # .fs:218-226
    out = [[0] * W for _ in range(NSLOT)]
    for m in mats:
        for r in range(NSLOT):
            for c in range(len(m[r])):
                out[r][c] += m[r][c]
    return out


def createPPMOf(pfm):                                    # .fs:249-251
    return [[float(x) for x in row] for row in pfm]


def normalizePPM(source_count, alphabet, pc, ppm):       # .fs:255-261 (mutates)
    total = float(source_count) + float(len(alphabet)) * pc
    for a in alphabet:
        row = ppm[idx(a)]
        for j in range(len(row)):
            row[j] = (row[j] + pc) / total
    return ppm


def createPositionWeightMatrix(alphabet, pcv, ppm):      # .fs:282-287
    W = len(ppm[0])
    pwm = [[0.0] * W for _ in range(NSLOT)]
    for a in alphabet:
        for j in range(W):
            pwm[idx(a)][j] = ppm[idx(a)][j] / pcv[idx(a)]
    return pwm


def pwm_segment_score(pwm, items):                       # .fs:290-293
    v = 1.0
    for j, b in enumerate(items):
        v = v * pwm[idx(b)][j]
    return v


# ---------------------------------------------------------------- SiteSampler
def getBestPWMSs(W, alphabet, pc, source, fcv, ppm):     # .fs:462-479 (mutates fcv)
    high, hi = 0.0, 0
    n = 0
    while n + W <= len(source):
        seg = list(source[n:n + W])
        pcv = createNormalizedPCVOfFCV(
            alphabet, pc, substractSegmentCountsFrom(seg, increaseInPlaceFCVOf(source, fcv)))
        pwm = createPositionWeightMatrix(alphabet, pcv, ppm)
        tmp = pwm_segment_score(pwm, seg)
        if tmp > high:
            high, hi = tmp, n
        n += 1
    return log2(high), hi


def getPWMOfRandomStarts(W, pc, alphabet, sources, draws):   # .fs:589-611
    """draws(n, m) -> start of the m-th other sequence for target n."""
    out = []
    N = len(sources)
    for n in range(N):
        others = [m for m in range(N) if m != n]
        starts = [draws(n, m) for m in others]
        fcv = fuseFrequencyVectors(
            alphabet, [createFCVWithout(W, p, sources[m]) for m, p in zip(others, starts)])
        ppm = normalizePPM(N - 1, alphabet, pc, createPPMOf(fusePositionFrequencyMatrices(
            W, [createPFMOf(getSegment(W, sources[m], p)) for m, p in zip(others, starts)])))
        out.append(getBestPWMSs(W, alphabet, pc, sources[n], fcv, ppm))
    return out


def _site_scan_with(W, pc, alphabet, sources, n, starts):
    """The body shared by .fs:489-507, .fs:525-542 and .fs:560-577: getBestPWMSs of
    sequence n with every other sequence m at starts[m]."""
    N = len(sources)
    others = [m for m in range(N) if m != n]
    fcv = fuseFrequencyVectors(
        alphabet, [createFCVWithout(W, starts[m], sources[m]) for m in others])
    ppm = normalizePPM(N - 1, alphabet, pc, createPPMOf(fusePositionFrequencyMatrices(
        W, [createPFMOf(getSegment(W, sources[m], starts[m])) for m in others])))
    return getBestPWMSs(W, alphabet, pc, sources[n], fcv, ppm)


def _site_passes(W, pc, alphabet, sources, start, starts_of):
    """loop n acc bestMotif of the three refinements: acc[n] takes tmp when fst tmp >
    fst acc[n]; a pass ends by comparing positions with the pass-start copy."""
    acc = list(start)
    while True:
        best = list(acc)
        for n in range(len(sources)):
            tmp = _site_scan_with(W, pc, alphabet, sources, n, starts_of(acc, best))
            if tmp[0] > acc[n][0]:
                acc[n] = tmp
        if [p for _, p in acc] == [p for _, p in best]:
            return acc


def getBestPWMSsWithStartPositions(W, pc, alphabet, sources, start):   # .fs:554-585
    return _site_passes(W, pc, alphabet, sources, start,
                        lambda acc, best: [p for _, p in acc])


def getLeftShiftedBestPWMSs(W, pc, alphabet, sources, start):          # .fs:519-550
    return _site_passes(W, pc, alphabet, sources, start,
                        lambda acc, best: [p - 1 if p > 0 else p for _, p in best])


def getRightShiftedBestPWMSs(W, pc, alphabet, sources, start):         # .fs:483-517
    return _site_passes(W, pc, alphabet, sources, start,
                        lambda acc, best: [p + 1 if p <= len(sources[m]) - W - 1 else p
                                           for m, (_, p) in enumerate(best)])


# ------------------------------------------- SiteSampler, fixed pcv / fixed ppm twins
def getBestPWMSsWithBPV(W, alphabet, source, pcv, ppm):   # .fs:301-313
    high, hi = 0.0, 0
    n = 0
    while n + W <= len(source):
        seg = list(source[n:n + W])
        pwm = createPositionWeightMatrix(alphabet, pcv, ppm)
        tmp = pwm_segment_score(pwm, seg)
        if tmp > high:
            high, hi = tmp, n
        n += 1
    return log2(high), hi


def _others_ppm(W, pc, alphabet, sources, n, starts):
    N = len(sources)
    others = [m for m in range(N) if m != n]
    return normalizePPM(N - 1, alphabet, pc, createPPMOf(fusePositionFrequencyMatrices(
        W, [createPFMOf(getSegment(W, sources[m], starts[m])) for m in others])))


def getPWMOfRandomStartsWithBPV(W, pc, alphabet, sources, pcv, draws):   # .fs:412-431
    N = len(sources)
    out = []
    for n in range(N):
        starts = {m: draws(n, m) for m in range(N) if m != n}
        out.append(getBestPWMSsWithBPV(W, alphabet, sources[n], pcv,
                                       _others_ppm(W, pc, alphabet, sources, n, starts)))
    return out


def getMotifsWithBestPWMSOfPPM(W, pc, alphabet, sources, ppm, draws):     # .fs:644-662
    """The random starts only give the background; the caller's PPM scores."""
    N = len(sources)
    out = []
    for n in range(N):
        others = [m for m in range(N) if m != n]
        fcv = fuseFrequencyVectors(
            alphabet, [createFCVWithout(W, draws(n, m), sources[m]) for m in others])
        out.append(getBestPWMSs(W, alphabet, pc, sources[n], fcv, [list(r) for r in ppm]))
    return out


def _site_passes_bpv(W, pc, alphabet, sources, pcv, start, starts_of):
    acc = list(start)
    while True:
        best = list(acc)
        for n in range(len(sources)):
            ppm = _others_ppm(W, pc, alphabet, sources, n, starts_of(acc, best))
            tmp = getBestPWMSsWithBPV(W, alphabet, sources[n], pcv, ppm)
            if tmp[0] > acc[n][0]:
                acc[n] = tmp
        if [p for _, p in acc] == [p for _, p in best]:
            return acc


def findBestMotifWithStartPosition(W, pc, alphabet, sources, pcv, start):   # .fs:381-409
    return _site_passes_bpv(W, pc, alphabet, sources, pcv, start,
                            lambda acc, best: [p for _, p in acc])


def getLeftShiftedBestPWMSsWithBPV(W, pc, alphabet, sources, pcv, start):   # .fs:350-378
    return _site_passes_bpv(W, pc, alphabet, sources, pcv, start,
                            lambda acc, best: [p - 1 if p > 0 else p for _, p in best])


def getRightShiftedBestPWMSsWithBPV(W, pc, alphabet, sources, pcv, start):  # .fs:318-347
    return _site_passes_bpv(W, pc, alphabet, sources, pcv, start,
                            lambda acc, best: [p + 1 if p <= len(sources[m]) - W - 1 else p
                                               for m, (_, p) in enumerate(best)])


# ---------------------------------------------------------------- MotifSampler
def calculatePWMsForSegmentCombinations(cutoff, width, m, items):   # .fs:727-742
    out = []

    def loop(prob, positions, size, rest):
        if rest:
            x, xs = rest[0], rest[1:]
            if size > 0:
                if ceckForDistance(width, [x[1]] + positions):
                    if log2(x[0] * prob) > cutoff:
                        loop(x[0] * prob, [x[1]] + positions, size - 1, xs)
            if size >= 0:
                loop(prob, positions, size, xs)
        elif size == 0:
            out.append((log2(prob), positions))

    loop(1.0, [], m, items)
    return out


def rouletteWheelSelection(pick, items):                 # .fs:746-754
    total = 0.0
    for it in items:
        total = total + it[0]
    norm = [it[0] / total for it in items]
    acc, n = 0.0, 0
    while True:
        if n >= len(items):
            raise IndexError("roulette overrun")
        if acc <= pick and pick <= acc + norm[n]:
            return items[n]
        acc, n = acc + norm[n], n + 1


def calculateNormalizedSegmentScores(cutoff, amount, W, source, pcv, pwm):   # .fs:759-784
    segs = [(list(source[n:n + W]), n) for n in range(len(source) - W + 1)]
    scores = [(pwm_segment_score(pwm, s), k) for s, k in segs]
    bg = [(bg_segment_score(pcv, s), []) for s, _ in segs]
    cats = list(bg)
    for m in range(1, amount + 1):
        cats += calculatePWMsForSegmentCombinations(cutoff, W, m, scores)
    return cats


def _target_pwm(W, pc, alphabet, sources, mem, n):
    """Shared rebuild of .fs:940-965 / .fs:891-916 for target n against snapshot mem."""
    N = len(sources)
    others = [m for m in range(N) if m != n]
    fcvs = [createFCVWithout(W, p, sources[m]) for m in others for p in mem[m][1]]
    pcv = createNormalizedPCVOfFCV(
        alphabet, pc, increaseInPlaceFCVOf(sources[n], fuseFrequencyVectors(alphabet, fcvs)))
    pfms = [createPFMOf(getSegment(W, sources[m], p)) for m in others for p in mem[m][1]]
    ppm = normalizePPM(N - 1, alphabet, pc, createPPMOf(fusePositionFrequencyMatrices(W, pfms)))
    return pcv, createPositionWeightMatrix(alphabet, pcv, ppm)


def findBestMotifIndicesByWithStartPositions(amount, W, pc, cutoff, alphabet, sources, mem, u):
    """.fs:935-970.  mem: list of (PWMS, [positions]); u: list of NextDouble draws."""
    out = []
    for n in range(len(sources)):
        pcv, pwm = _target_pwm(W, pc, alphabet, sources, mem, n)
        cats = calculateNormalizedSegmentScores(cutoff, amount, W, sources[n], pcv, pwm)
        out.append(rouletteWheelSelection(u[n], cats))
    return out


def _target_pwm_pcv(W, pc, alphabet, sources, mem, n, pcv):
    """.fs:795-813 / .fs:835-845: the others' PPM with the caller's pcv."""
    N = len(sources)
    others = [m for m in range(N) if m != n]
    pfms = [createPFMOf(getSegment(W, sources[m], p)) for m in others for p in mem[m][1]]
    ppm = normalizePPM(N - 1, alphabet, pc, createPPMOf(fusePositionFrequencyMatrices(W, pfms)))
    return createPositionWeightMatrix(alphabet, pcv, ppm)


def findBestMotifPositionsWithStartPositionsByPCV(amount, W, pc, cutoff, alphabet, sources, pcv,
                                                  mem, u):                # .fs:828-853
    out = []
    for n in range(len(sources)):
        pwm = _target_pwm_pcv(W, pc, alphabet, sources, mem, n, pcv)
        cats = calculateNormalizedSegmentScores(cutoff, amount, W, sources[n], pcv, pwm)
        out.append(rouletteWheelSelection(u[n], cats))
    return out


def findBestMotifPositionsWithStartPositionByPCV(amount, W, pc, cutoff, alphabet, sources, pcv,
                                                 mem, max_passes=1000):   # .fs:788-823
    acc = [(p, list(ps)) for p, ps in mem]
    for _ in range(max_passes):
        best = [list(ps) for _, ps in acc]
        for n in range(len(sources)):
            pwm = _target_pwm_pcv(W, pc, alphabet, sources, acc, n, pcv)
            cats = calculateNormalizedSegmentScores(cutoff, amount, W, sources[n], pcv, pwm)
            top = cats[0]
            for c in cats[1:]:
                if c[0] > top[0] or (top[0] != top[0] and c[0] == c[0]):
                    top = c
            if top[0] > acc[n][0]:
                acc[n] = top
        if [ps for _, ps in acc] == best:
            return acc
    return acc


def findBestMotifIndicesWithStartPositions(amount, W, pc, cutoff, alphabet, sources, mem,
                                           max_passes=1000):
    """.fs:885-929 greedy Gauss-Seidel passes until positions stop changing."""
    acc = [(p, list(ps)) for p, ps in mem]
    for _ in range(max_passes):
        best = [list(ps) for _, ps in acc]
        for n in range(len(sources)):
            pcv, pwm = _target_pwm(W, pc, alphabet, sources, acc, n)
            cats = calculateNormalizedSegmentScores(cutoff, amount, W, sources[n], pcv, pwm)
            top = cats[0]
            for c in cats[1:]:          # stable sortByDescending |> head (NaN ranks last)
                if c[0] > top[0] or (top[0] != top[0] and c[0] == c[0]):
                    top = c
            if top[0] > acc[n][0]:
                acc[n] = top
        if [ps for _, ps in acc] == best:
            return acc
    return acc
