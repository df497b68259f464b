#!/usr/bin/env python3
"""Sweep timing in the two sampler regimes, per BASELINE config.

'uniform': the snapshot is uniform random starts.  After one sweep every sequence
picks a background category (measured: 0 of 10k keep a motif at cfg2), so the
chain sits in the absorbing all-background state.
'init': the snapshot is doMotifSampling's own input, getPWMOfRandomStarts
(.fs:589-611, shared-draw mode) -- the regime the reference's drivers run the
sweep in (every sequence keeps a motif; ~12 % of windows pass the cut-off).

Prints one JSON line per (config, regime): kernel microseconds per sweep (HIP
events around the timed region), fallback counters, fraction of sequences that
keep a motif.
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


def start_positions(ctx, w, regime):
    if regime == "uniform":
        return synthetic.initial_positions(w)
    _, pos = ctx.random_starts(w.W, w.pc, seed=synthetic.DATA_SEED + 1, mode=1)
    return pos


_DATA = {}


def run(cfg, regime, steps, warmup, lib=None, tuning=None):
    w = synthetic.CONFIGS[cfg]
    if cfg not in _DATA:
        _DATA.clear()
        _DATA[cfg] = synthetic.generate(w)
    codes, offsets = _DATA[cfg]
    ctx = Context(0, lib, tuning=tuning)
    ctx.set_sequences(codes, offsets, w.alphabet)
    pos = start_positions(ctx, w, regime)
    ctx.set_positions(w.W, pos)
    ctx.run_sweeps(w.pc, w.cutoff, warmup, seed=synthetic.DATA_SEED + 2, first_sweep=0)
    ctx.synchronize()
    s0 = ctx.stats()
    ctx.region_begin()
    ctx.run_sweeps(w.pc, w.cutoff, steps, seed=synthetic.DATA_SEED + 2, first_sweep=warmup)
    ms = ctx.region_end() / steps
    s1 = ctx.stats()
    p, pw = ctx.get_state()
    rec = {"cfg": cfg, "regime": regime, "lib": Path(lib).name if lib else "libgibbs_hip.so", "tuning": tuning or {}, "N": w.N, "L": w.L, "W": w.W,
           "us_per_sweep": ms * 1e3,
           "GBps_alg": w.N * (w.L + 24) / (ms * 1e-3) / 1e9,
           "keep_motif": float((p >= 0).mean()), "mean_pwms": float(pw.mean()),
           "fallbacks_per_sweep": {k: (s1[k] - s0[k]) / steps for k in s1}}
    ctx.close()
    print(json.dumps(rec), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="cfg2,cfg3")
    ap.add_argument("--regimes", default="init,uniform")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--libs", default="", help="comma-separated library variants (A/B)")
    ap.add_argument("--tunings", default="", help="';'-separated tuning specs NAME=v,NAME=v (A/B)")
    ap.add_argument("--shapes", default="", help="extra DNA shapes N:L:W, run as configs sN_L_W")
    a = ap.parse_args()
    for sh in filter(None, a.shapes.split(",")):
        n, l, w = (int(x) for x in sh.split(":"))
        synthetic.CONFIGS[f"s{n}_{l}_{w}"] = synthetic.Workload(f"{n} DNA seqs x {l}bp, W={w}", n, l, w,
                                                                 synthetic.CONFIGS["cfg2"].alphabet)
    for cfg in a.configs.split(","):
        for reg in a.regimes.split(","):
            for lib in (a.libs.split(",") if a.libs else [None]):
                for t in (a.tunings.split(";") if a.tunings else [""]):
                    tun = {k: float(v) for k, v in (kv.split("=") for kv in t.split(",") if kv)}
                    run(cfg, reg, a.steps, a.warmup, lib, tun)


if __name__ == "__main__":
    main()
