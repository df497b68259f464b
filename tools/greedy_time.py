"""Time the greedy refinement (gs_run_greedy, .fs:885-929) on a BASELINE shape in
the doMotifSampling setting (random starts -> one sweep -> greedy), and count the
moves of each pass; prints one JSON line.

    python tools/greedy_time.py --shape cfg2 [--oracle]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))

from conftest import make_dataset  # noqa: E402

SHAPES = {"cfg1": (100, 50, 8, b"ACGT"), "cfg2": (10_000, 200, 12, b"ACGT"),
          "cfg3": (100_000, 500, 15, b"ACGT"), "cfg5": (50_000, 300, 20, b"ACDEFGHIKLMNPQRSTVWY")}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="cfg2")
    ap.add_argument("--init-mode", type=int, default=1)
    ap.add_argument("--max-passes", type=int, default=1000)
    ap.add_argument("--per-pass", type=int, default=6, help="count moves of the first k passes")
    ap.add_argument("--oracle", action="store_true", help="also check the oracle greedy")
    ap.add_argument("--waves", type=int, default=0, help="tuning greedy_waves (0: library default)")
    args = ap.parse_args()
    from gibbssampling_amd import Context
    N, L, W, alpha = SHAPES[args.shape]
    pc, cutoff, seed = 1e-4, 1.0, 7
    codes, offsets = make_dataset(N, L, W, alpha, seed=5)
    ctx = Context(0, tuning={"greedy_waves": args.waves} if args.waves else None)
    ctx.set_sequences(codes, offsets, alpha)
    t0 = time.perf_counter()
    sc, p0 = ctx.random_starts(W, pc, seed, args.init_mode)
    t_init = time.perf_counter() - t0
    ctx.set_positions(W, p0)
    ctx.run_sweeps(pc, cutoff, 1, seed)
    p1, w1 = ctx.get_state()
    t0 = time.perf_counter()
    passes, ms = ctx.run_greedy(pc, cutoff, args.max_passes)
    wall = (time.perf_counter() - t0) * 1e3
    gp, gw = ctx.get_state()
    moves = []
    prev = p1
    for k in range(1, min(passes, args.per_pass) + 1):
        pk, _, _ = ctx.motif_greedy(W, pc, cutoff, p1, w1, max_passes=k)
        moves.append(int((pk != prev).sum()))
        prev = pk
    out = {"shape": args.shape, "N": N, "L": L, "W": W, "init_mode": args.init_mode,
           "init_s": t_init, "passes": passes, "kernel_ms": ms, "wall_ms": wall,
           "us_per_target_visit": ms * 1e3 / (passes * N), "moves_per_pass": moves,
           "moved_total": int((gp != p1).sum())}
    if args.oracle:
        from oracle import oracle_lib as ol
        S = ol.Seqs(codes, offsets, alpha)
        t1 = time.perf_counter()
        op, ow, opass = ol.greedy(S, W, pc, cutoff, p1, w1, max_passes=args.max_passes)
        out["oracle_s"] = time.perf_counter() - t1
        out["oracle_passes"] = opass
        out["positions_equal"] = bool(np.array_equal(op, gp))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
