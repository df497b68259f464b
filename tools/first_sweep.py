#!/usr/bin/env python3
"""The first sweep of a chain from uniform random starts, timed alone (HIP events around
one gs_run_sweeps call of one sweep, after a warm-up chain on the same context so that
code objects are loaded): the sweep kernel's cost when no window passes the cut-off
(every target's categories are its background products).  One JSON line per (config,
library): microseconds of that sweep (median of --reps), and the exact rescans it took.
"""
from __future__ import annotations

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
    ap.add_argument("--configs", default="cfg3")
    ap.add_argument("--libs", default="")
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    for cfg in a.configs.split(","):
        w = synthetic.CONFIGS[cfg]
        codes, offsets = synthetic.generate(w)
        for lib in (a.libs.split(",") if a.libs else [None]):
            ctx = Context(0, lib)
            ctx.set_sequences(codes, offsets, w.alphabet)
            pos = synthetic.initial_positions(w)
            ts, rx = [], []
            for r in range(a.reps + 1):
                ctx.set_positions(w.W, pos)
                kname = ctx.sweep_kernel_name()
                s0 = ctx.stats()
                ctx.synchronize()
                ctx.region_begin()
                ctx.run_sweeps(w.pc, w.cutoff, 1, seed=synthetic.DATA_SEED + 2 + r, first_sweep=0)
                ms = ctx.region_end()
                s1 = ctx.stats()
                if r:  # (the first: code objects loading)
                    ts.append(ms * 1e3)
                    rx.append(s1["exact_rescans"] - s0["exact_rescans"])
            p, _ = ctx.get_state()
            print(json.dumps({"cfg": cfg, "lib": Path(lib).name if lib else "libgibbs_hip.so",
                              "kernel": kname, "first_sweep_us": float(np.median(ts)),
                              "all_us": [round(x, 1) for x in ts], "exact_rescans": rx,
                              "keep_motif_after": float((p >= 0).mean())}), flush=True)
            ctx.close()


if __name__ == "__main__":
    main()
