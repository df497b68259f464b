import os
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libgibbs_hip.so)")
    config.addinivalue_line("markers", "slow: larger CPU case")


def make_dataset(N, L, W, alpha=b"ACGT", seed=0, planted=True, ragged=False, extra=b"",
                 extra_rate=0.0, mut=0.25):
    """Synthetic sequences: i.i.d. symbols over `alpha`, optionally one mutated copy of a
    random consensus W-mer per sequence (BASELINE.md synthetic inputs); `extra` symbols
    (non-alphabet codes) sprinkled at `extra_rate`; ragged lengths in [W, L]."""
    rng = np.random.default_rng(seed)
    a = np.frombuffer(alpha, np.uint8)
    lens = rng.integers(W, L + 1, N) if ragged else np.full(N, L)
    offsets = np.zeros(N + 1, np.int64)
    np.cumsum(lens, out=offsets[1:])
    codes = a[rng.integers(0, len(a), int(offsets[-1]))].astype(np.uint8)
    if planted:
        cons = a[rng.integers(0, len(a), W)]
        starts = offsets[:-1] + (rng.random(N) * (lens - W + 1)).astype(np.int64)
        motif = np.tile(cons, (N, 1))
        flip = rng.random((N, W)) < mut
        motif[flip] = a[rng.integers(0, len(a), int(flip.sum()))]
        idx = starts[:, None] + np.arange(W)[None, :]
        codes[idx] = motif
    if extra and extra_rate > 0:
        e = np.frombuffer(extra, np.uint8)
        hit = rng.random(codes.size) < extra_rate
        codes[hit] = e[rng.integers(0, len(e), int(hit.sum()))]
    return codes, offsets


def init_positions(offsets, W, seed=1, none_rate=0.0):
    rng = np.random.default_rng(seed)
    lens = np.diff(offsets)
    pos = (rng.random(len(lens)) * (lens - W + 1)).astype(np.int32)
    if none_rate:
        pos[rng.random(len(lens)) < none_rate] = -1
    return pos


@pytest.fixture(scope="session")
def gpu_ctx():
    from gibbssampling_amd import Context
    ctx = Context(0)
    yield ctx
    ctx.close()


_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _mix64(z):
    z = z + np.uint64(0x9E3779B97F4A7C15)
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def uniforms(seed, stream, n, first=0):
    """gs_uniform(seed, stream, i) for i in [first, first + n), vectorised (the
    library's and the oracle's counter RNG, gs_common.h / gibbs_oracle.c)."""
    with np.errstate(over="ignore"):
        i = np.arange(first, first + n, dtype=np.uint64)
        h = _mix64(np.uint64(seed) ^ _mix64(np.uint64(stream) ^ _mix64(i)))
    return (h >> np.uint64(11)).astype(np.float64) * 2.0 ** -53
