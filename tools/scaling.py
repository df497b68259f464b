#!/usr/bin/env python3
"""Sweep-kernel time versus N (fixed L, W) in both scan modes: separates the fixed
per-launch cost from the per-sequence cost.  Usage: tools/scaling.py [L] [W] [A]"""
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

from gibbssampling_amd import _native  # noqa: E402
from conftest import init_positions, make_dataset  # noqa: E402


def kernel_us(ctx, W, pos, sweeps=20):
    ctx.set_positions(W, pos)
    ctx.run_sweeps(1e-4, 1.0, 3, seed=1)
    ctx.synchronize()
    ctx.profile(True)
    ctx.profile_read()
    ctx.run_sweeps(1e-4, 1.0, sweeps, seed=1, first_sweep=3)
    ctx.synchronize()
    kms, nk, _, _ = ctx.profile_read()
    ctx.profile(False)
    return round(1000 * kms / max(nk, 1), 2)


def main():
    L = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    W = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    alpha = b"ACGT" if len(sys.argv) <= 3 else sys.argv[3].encode()
    ctx = _native.Context(0)
    out = {}
    for N in (1024, 2500, 5000, 10000, 20000, 40000, 80000):
        codes, offsets = make_dataset(N, L, W, alpha, seed=5, mut=0.2)
        pos = init_positions(offsets, W, 6)
        ctx.set_sequences(codes, offsets, alpha)
        row = {}
        for exact in (False, True):
            ctx.set_scan_mode(exact)
            row["exact" if exact else "certified"] = kernel_us(ctx, W, pos)
        ctx.set_scan_mode(False)
        out[N] = row
    ctx.close()
    print(json.dumps({"L": L, "W": W, "alphabet": alpha.decode(), "kernel_us": out}))


if __name__ == "__main__":
    main()
