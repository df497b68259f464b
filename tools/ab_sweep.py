#!/usr/bin/env python3
"""A/B of the sweep kernel's per-sweep device time between library builds on one box:
    python tools/ab_sweep.py cfg2 lib_a.so lib_b.so ...   (rounds interleaved)
    python tools/ab_sweep.py cfg2 lib.so lib.so@GS_GROUP_LANES=16,GS_SWEEP_WAVES=2
(an @-suffix sets tuning fields, gs_set_tuning, for that variant's context only)
Each measurement: 200 resident sweeps between two stream events (as bench.py)."""
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from gibbssampling_amd import _native, synthetic  # noqa: E402


def per_sweep_us(variant, w, codes, offsets, pos, steps=200):
    lib, _, knobs = variant.partition("@")
    ctx = _native.Context(0, lib, tuning=_native.tuning_spec(knobs))
    ctx.set_sequences(codes, offsets, w.alphabet)
    ctx.set_positions(w.W, pos)
    ctx.run_sweeps(w.pc, w.cutoff, 5, seed=9)
    ctx.synchronize()
    ctx.region_begin()
    ctx.run_sweeps(w.pc, w.cutoff, steps, seed=9, first_sweep=5)
    ms = ctx.region_end()
    out = ctx.get_state()
    ctx.close()
    return 1000.0 * ms / steps, out


def main():
    cfg = sys.argv[1]
    libs = sys.argv[2:]
    w = synthetic.CONFIGS[cfg]
    codes, offsets = synthetic.generate(w)
    pos = synthetic.initial_positions(w)
    res = {lib: [] for lib in libs}
    ref = None
    for rnd in range(int(os.environ.get("AB_ROUNDS", "3"))):
        for lib in libs:
            us, st = per_sweep_us(lib, w, codes, offsets, pos)
            res[lib].append(round(us, 2))
            if ref is None:
                ref = st
            same = bool((st[0] == ref[0]).all() and (st[1] == ref[1]).all())
            print(f"round {rnd} {Path(lib).name}: {us:.2f} us/sweep identical={same}",
                  file=sys.stderr, flush=True)
    print(json.dumps({"config": cfg, "us_per_sweep": {Path(k).name: v for k, v in res.items()}}))


if __name__ == "__main__":
    main()
