#!/usr/bin/env python3
"""Phase costs of the live-chain sweep kernel by subtraction (timing experiments).

Each library variant is built with -DGS_EXP=<bits> (gs_sweep_live.hip: phases
skipped, no rescans); every measurement is ONE sweep from the same snapshot (the
initialiser's output), so that a variant's wrong outputs do not change the next
sweep's input.  Prints per (config, variant) the median device microseconds of a
sweep over --reps repetitions.

    python tools/phase_exp.py --configs cfg4 --libs libgibbs_hip.so,libgibbs_hip_x1.so
"""
import argparse
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from gibbssampling_amd import Context, synthetic  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="cfg2,cfg3,cfg4")
    ap.add_argument("--libs", default="libgibbs_hip.so")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--tuning", default="", help="NAME=v,NAME=v (gs_set_tuning fields)")
    ap.add_argument("--regime", default="init", choices=["init", "uniform"],
                    help="the snapshot swept: the initialiser's output or uniform random starts")
    a = ap.parse_args()
    tun = {k: float(v) for k, v in (kv.split("=") for kv in a.tuning.split(",") if kv)}
    for cfg in a.configs.split(","):
        w = synthetic.CONFIGS[cfg]
        codes, offsets = synthetic.generate(w)
        for lib in a.libs.split(","):
            ctx = Context(0, str(ROOT / "gibbssampling_amd" / lib), tuning=tun)
            ctx.set_sequences(codes, offsets, w.alphabet)
            if a.regime == "uniform":
                p0 = synthetic.initial_positions(w)
            else:
                _, p0 = ctx.random_starts(w.W, w.pc, seed=synthetic.DATA_SEED + 1, mode=1)
            ts = []
            for r in range(a.reps + 2):
                ctx.set_positions(w.W, p0)
                ctx.synchronize()
                ctx.region_begin()
                ctx.run_sweeps(w.pc, w.cutoff, 1, seed=synthetic.DATA_SEED + 2, first_sweep=0)
                ms = ctx.region_end()
                if r >= 2:
                    ts.append(ms * 1e3)
            ctx.close()
            print(json.dumps({"cfg": cfg, "lib": lib, "regime": a.regime, "us_median": float(np.median(ts)),
                              "us_min": float(np.min(ts))}), flush=True)


if __name__ == "__main__":
    main()
