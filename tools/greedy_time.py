"""Time the greedy refinement (gs_run_greedy, .fs:885-929) on a BASELINE shape after
a few resident sweeps; prints one JSON line (passes, kernel ms, µs per target visit).

    python tools/greedy_time.py --shape cfg2 --sweeps 5
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))

from conftest import init_positions, make_dataset  # noqa: E402

SHAPES = {"cfg1": (100, 50, 8, b"ACGT"), "cfg2": (10_000, 200, 12, b"ACGT"),
          "cfg3": (100_000, 500, 15, b"ACGT"), "cfg5": (50_000, 300, 20, b"ACDEFGHIKLMNPQRSTVWY")}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="cfg2")
    ap.add_argument("--sweeps", type=int, default=5)
    ap.add_argument("--max-passes", type=int, default=1000)
    ap.add_argument("--oracle", action="store_true", help="also time + check the oracle greedy")
    args = ap.parse_args()
    from gibbssampling_amd import Context
    N, L, W, alpha = SHAPES[args.shape]
    codes, offsets = make_dataset(N, L, W, alpha, seed=5)
    pos = init_positions(offsets, W, 6)
    ctx = Context(0)
    ctx.set_sequences(codes, offsets, alpha)
    ctx.set_positions(W, pos)
    ctx.run_sweeps(1e-4, 1.0, args.sweeps, 7)
    p0, w0 = ctx.get_state()
    t0 = time.perf_counter()
    passes, ms = ctx.run_greedy(1e-4, 1.0, args.max_passes)
    wall = (time.perf_counter() - t0) * 1e3
    gp, gw = ctx.get_state()
    out = {"shape": args.shape, "N": N, "L": L, "W": W, "sweeps": args.sweeps, "passes": passes,
           "kernel_ms": ms, "wall_ms": wall, "us_per_target_visit": ms * 1e3 / (passes * N),
           "moved_vs_sweep": int((gp != p0).sum())}
    if args.oracle:
        from oracle import oracle_lib as ol
        S = ol.Seqs(codes, offsets, alpha)
        # pwms of the resident snapshot: the sweep's own
        t1 = time.perf_counter()
        op, ow, opass = ol.greedy(S, W, 1e-4, 1.0, p0, w0, max_passes=args.max_passes)
        out["oracle_s"] = time.perf_counter() - t1
        out["oracle_passes"] = opass
        out["positions_equal"] = bool(np.array_equal(op, gp))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
