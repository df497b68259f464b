"""Golden vectors (tests/golden/*.npz, made by tests/golden/make_golden.py).

CPU: the oracle still reproduces every committed vector bit for bit (regression
pin of the checker).  GPU: libgibbs_hip.so reproduces them (positions exact,
PWMS within 1e-12 relative; integer aggregates exact).
"""
from pathlib import Path

import numpy as np
import pytest

from oracle import oracle_lib as ol

GOLDEN = Path(__file__).resolve().parent / "golden"
SWEEPS = sorted(p.stem for p in GOLDEN.glob("*_sweep.npz"))
STARTS = sorted(p.stem for p in GOLDEN.glob("*_starts.npz"))


def load(name):
    return dict(np.load(GOLDEN / f"{name}.npz"))  # allow_pickle=False (default)


def alpha_of(f):
    return bytes(f["alphabet"].tobytes())


@pytest.mark.parametrize("name", SWEEPS)
def test_oracle_reproduces_sweep(name):
    f = load(name)
    S = ol.Seqs(f["codes"], f["offsets"], alpha_of(f))
    p, w, _ = ol.sweep(S, int(f["W"]), float(f["pc"]), float(f["cutoff"]), f["pos_in"], f["u"])
    assert np.array_equal(p, f["pos_out"]) and np.array_equal(w, f["pwms_out"])
    C, T = ol.counts(S, int(f["W"]), f["pos_in"])
    assert np.array_equal(C, f["C"]) and np.array_equal(T, f["T"])
    for t in f["detail_targets"]:
        d = ol.target_detail(S, int(f["W"]), float(f["pc"]), f["pos_in"], int(t))
        for k in ("bgc", "pcv", "pwm", "S", "G"):
            assert np.array_equal(d[k], f[f"t{t}_{k}"]), (t, k)


@pytest.mark.parametrize("name", STARTS)
def test_oracle_reproduces_starts(name):
    f = load(name)
    S = ol.Seqs(f["codes"], f["offsets"], alpha_of(f))
    sc, ps = ol.random_starts(S, int(f["W"]), float(f["pc"]), seed=int(f["seed"]),
                              mode=int(f["mode"]))
    assert np.array_equal(ps, f["pos"]) and np.array_equal(sc, f["score"])


def test_oracle_reproduces_chain():
    f = load("cfg1_chain5")
    S = ol.Seqs(f["codes"], f["offsets"], alpha_of(f))
    p = f["pos_in"]
    for t in range(int(f["sweeps"])):
        u = np.array([ol.uniform(int(f["seed"]), ol.stream_sweep(t), n) for n in range(S.n)])
        p, w, _ = ol.sweep(S, int(f["W"]), float(f["pc"]), float(f["cutoff"]), p, u)
    assert np.array_equal(p, f["pos_out"]) and np.array_equal(w, f["pwms_out"])


def test_fsx_fixture_shapes():
    """The parsed .fsx data sets have the shapes SURVEY.md §4 lists."""
    import json
    sets = json.loads((GOLDEN / "fsx_sets.json").read_text())
    assert [len(s) for s in sets["tests"]["seqs"]] == [21] * 4
    assert len(sets["dataSet"]["seqs"]) == 62
    assert sum(len(s) for s in sets["dataSet"]["seqs"]) == 29616
    assert sets["bioTestsII"]["seqs"][2].endswith("*")  # Ter symbol, .fsx:63
    assert [s.find("CACGTG") for s in sets["tests"]["seqs"]] == [10, 9, 5, 14]


# ----------------------------------------------------------------- GPU side
@pytest.mark.gpu
@pytest.mark.parametrize("name", SWEEPS)
def test_gpu_reproduces_sweep(gpu_ctx, name):
    f = load(name)
    gpu_ctx.set_sequences(f["codes"], f["offsets"], alpha_of(f))
    p, w = gpu_ctx.motif_sweep(int(f["W"]), float(f["pc"]), float(f["cutoff"]), f["pos_in"],
                               f["u"])
    assert np.array_equal(p, f["pos_out"])
    np.testing.assert_allclose(w, f["pwms_out"], rtol=1e-12)
    C, T = gpu_ctx.counts(int(f["W"]), f["pos_in"], len(alpha_of(f)))
    assert np.array_equal(C, f["C"]) and np.array_equal(T, f["T"])


@pytest.mark.gpu
@pytest.mark.parametrize("name", STARTS)
def test_gpu_reproduces_starts(gpu_ctx, name):
    f = load(name)
    gpu_ctx.set_sequences(f["codes"], f["offsets"], alpha_of(f))
    sc, ps = gpu_ctx.random_starts(int(f["W"]), float(f["pc"]), int(f["seed"]), int(f["mode"]))
    assert np.array_equal(ps, f["pos"])
    np.testing.assert_allclose(sc, f["score"], rtol=1e-12)


@pytest.mark.gpu
def test_gpu_reproduces_chain(gpu_ctx):
    f = load("cfg1_chain5")
    gpu_ctx.set_sequences(f["codes"], f["offsets"], alpha_of(f))
    p, w = gpu_ctx.motif_run(int(f["W"]), float(f["pc"]), float(f["cutoff"]), int(f["sweeps"]),
                             int(f["seed"]), f["pos_in"])
    assert np.array_equal(p, f["pos_out"])
    np.testing.assert_allclose(w, f["pwms_out"], rtol=1e-12)
