"""Synthetic workloads of BASELINE.json (BASELINE.md §2 'Synthetic inputs').

i.i.d. uniform symbols over the alphabet, one planted copy of a random consensus
W-mer per sequence with per-symbol mutation probability 0.25, fixed seeds
(data 0x6B5A1D, init +1).  Sequence n's content depends only on (seed, n), so a
rank can generate exactly its own shard.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from .bioarray import ACGT, AMINO20

DATA_SEED = 0x6B5A1D


@dataclass(frozen=True)
class Workload:
    name: str
    N: int
    L: int
    W: int
    alphabet: bytes
    pc: float = 1e-4      # pseudoCount of GibbsSampling.fsx:384,407
    cutoff: float = 1.0   # cutOff of GibbsSampling.fsx:407

    @property
    def K(self) -> int:
        return self.L - self.W + 1


CONFIGS = {
    "cfg1": Workload("cfg1: 100 DNA seqs x 50bp, W=8", 100, 50, 8, ACGT),
    "cfg2": Workload("cfg2: 10k DNA seqs x 200bp, W=12", 10_000, 200, 12, ACGT),
    "cfg3": Workload("cfg3: 100k DNA seqs x 500bp, W=15", 100_000, 500, 15, ACGT),
    "cfg4": Workload("cfg4: 1M DNA seqs x 200bp, W=12", 1_000_000, 200, 12, ACGT),
    "cfg5": Workload("cfg5: protein 50k seqs x 300aa, W=20", 50_000, 300, 20, AMINO20),
}


def generate(w: Workload, lo: int = 0, hi: int | None = None, seed: int = DATA_SEED,
             mutation: float = 0.25):
    """Sequences [lo, hi) of workload w: (codes uint8, offsets int64)."""
    hi = w.N if hi is None else hi
    n = hi - lo
    a = np.frombuffer(w.alphabet, np.uint8)
    cons = a[np.random.default_rng(seed).integers(0, len(a), w.W)]
    # per-sequence streams keyed by global index, generated in blocks
    codes = np.empty(n * w.L, np.uint8)
    block = 4096  # absolute blocks: a shard [lo, hi) sees the same data as the full set
    for B in range(lo // block * block, hi, block):
        rng = np.random.default_rng([seed, B])
        m = min(block, w.N - B)
        x = a[rng.integers(0, len(a), m * w.L)].reshape(m, w.L)
        starts = rng.integers(0, w.L - w.W + 1, m)
        motif = np.tile(cons, (m, 1))
        flip = rng.random((m, w.W)) < mutation
        motif[flip] = a[rng.integers(0, len(a), int(flip.sum()))]
        x[np.arange(m)[:, None], starts[:, None] + np.arange(w.W)[None, :]] = motif
        s0, s1 = max(lo, B), min(hi, B + m)
        codes[(s0 - lo) * w.L:(s1 - lo) * w.L] = x[s0 - B:s1 - B].reshape(-1)
    offsets = np.arange(0, n * w.L + 1, w.L, dtype=np.int64)
    return codes, offsets


def initial_positions(w: Workload, lo: int = 0, hi: int | None = None, seed: int = DATA_SEED + 1):
    """Uniform start positions in [0, L-W] (initial positions uniform)."""
    hi = w.N if hi is None else hi
    out = np.empty(hi - lo, np.int32)
    block = 4096
    for B in range(lo // block * block, hi, block):
        rng = np.random.default_rng([seed, B])
        m = min(block, w.N - B)
        v = rng.integers(0, w.L - w.W + 1, m)
        s0, s1 = max(lo, B), min(hi, B + m)
        out[s0 - lo:s1 - lo] = v[s0 - B:s1 - B]
    return out
