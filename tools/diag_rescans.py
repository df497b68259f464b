#!/usr/bin/env python3
"""Fallback statistics of the certified scan on BASELINE shapes and on the test
datasets: how often a sequence needed the binary64 rescan, and why."""
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

from gibbssampling_amd import _native, synthetic  # noqa: E402
from conftest import init_positions, make_dataset  # noqa: E402


def run(ctx, name, codes, offsets, alpha, W, pc, cutoff, pos, sweeps):
    ctx.set_sequences(codes, offsets, alpha)
    s0 = ctx.stats()
    ctx.motif_run(W, pc, cutoff, sweeps, 4242, pos)
    s1 = ctx.stats()
    d = {k: s1[k] - s0[k] for k in s1}
    d["per_sequence_sweep"] = d["exact_rescans"] / (sweeps * (len(offsets) - 1))
    return name, d


def main():
    ctx = _native.Context(0)
    out = {}
    for name in ("cfg2", "cfg3", "cfg5"):
        w = synthetic.CONFIGS[name]
        codes, offsets = synthetic.generate(w)
        k, d = run(ctx, name, codes, offsets, w.alphabet, w.W, w.pc, w.cutoff,
                   synthetic.initial_positions(w), 10)
        out[k] = d
    for W, alpha, pc in [(12, b"ACGT", 1e-4), (8, b"ATGC-", 0.5)]:
        N, L = 3000, 240
        codes, offsets = make_dataset(N, L, W, alpha, seed=111, ragged=True, mut=0.15,
                                      extra=b"*", extra_rate=0.002)
        pos = init_positions(offsets, W, 112, 0.1)
        k, d = run(ctx, f"test_{W}_{alpha.decode()}", codes, offsets, alpha, W, pc, 1.0, pos, 8)
        out[k] = d
        codes, offsets = make_dataset(N, L, W, alpha, seed=111, ragged=True, mut=0.15)
        k, d = run(ctx, f"test_{W}_{alpha.decode()}_noextra", codes, offsets, alpha, W, pc, 1.0,
                   pos, 8)
        out[k] = d
    ctx.close()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
