"""Host-side driver logic of the Python mirror (no GPU): the repetition loop of
getMotifsWithBestInformationContent(s) (.fs:615-640, .fs:973-998)."""
import numpy as np
import pytest

from gibbssampling_amd.sampler import _best_of_repetitions, _seed


def fsharp_loop(numberOfRepetitions, run, ic, initial):
    """Literal transcription of `let rec loop n acc bestPWMS` (.fs:974-998)."""
    def loop(n, acc, best):
        if n > numberOfRepetitions:
            return best
        if acc == best:
            return best
        if ic(acc) > ic(best):
            return loop(n + 1, [], best if len(acc) == 0 else acc)
        return loop(n + 1, run(n), best)
    return loop(0, [], initial)


@pytest.mark.parametrize("reps", [0, 1, 2, 5, 9])
@pytest.mark.parametrize("seed", [0, 1, 2])
def test_repetition_loop_matches_fsharp(reps, seed):
    rng = np.random.default_rng(seed)
    runs = {}

    def run(n):
        if n not in runs:
            runs[n] = [(float(x), int(i)) for i, x in enumerate(rng.random(3) * 4)]
        return runs[n]

    ic = lambda xs: sum(s for s, _ in xs)  # noqa: E731
    a = _best_of_repetitions(reps, run, ic, [(0.0, 0)])
    b = fsharp_loop(reps, run, ic, [(0.0, 0)])
    assert a == b


def test_repetition_loop_stops_on_equal_run():
    """A run equal to the best ends the loop (acc = bestPWMS)."""
    same = [(2.0, 1)]
    calls = []

    def run(n):
        calls.append(n)
        return list(same)

    out = _best_of_repetitions(10, run, lambda xs: sum(s for s, _ in xs), [(0.0, 0)])
    assert out == same and calls == [0, 2]


def test_seed_normalisation():
    assert _seed(5) == 5 and _seed(-1) == 2**64 - 1
    assert 0 <= _seed(None) < 2**64


def test_motif_index_lists_roundtrip():
    """MotifIndex[] <-> (cnt, pos[N, cap]) keeps the F# list order."""
    from gibbssampling_amd.sampler import _lists, _motif_lists, _is_single, createMotifIndex
    mem = [createMotifIndex(1.5, [7, 2]), createMotifIndex(0.1, []), createMotifIndex(2.0, [3])]
    cap, cnt, pos = _lists(2, mem)
    assert cap == 2 and list(cnt) == [2, 0, 1] and list(pos[0]) == [7, 2]
    back = _motif_lists(cnt, pos, np.array([m.PWMS for m in mem]))
    assert back == mem
    assert not _is_single(1, mem) and _is_single(1, mem[1:]) and not _is_single(2, mem[1:])
    cap, _, _ = _lists(1, mem)  # lists longer than motifAmount widen the capacity
    assert cap == 2
