#!/usr/bin/env python3
"""Per-sweep device time of the first sweeps of a chain (warm-up effects): config 2,
uniform starts, `--warmup` sweeps, then 60 single-sweep calls each timed by HIP
events on the library stream."""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from gibbssampling_amd import Context, synthetic  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "cfg2"
warm = int(sys.argv[2]) if len(sys.argv) > 2 else 5
w = synthetic.CONFIGS[cfg]
codes, offsets = synthetic.generate(w)
ctx = Context(0)
ctx.set_sequences(codes, offsets, w.alphabet)
ctx.set_positions(w.W, synthetic.initial_positions(w))
ctx.run_sweeps(w.pc, w.cutoff, warm, seed=3)
ctx.synchronize()
us = []
for t in range(60):
    ctx.region_begin()
    ctx.run_sweeps(w.pc, w.cutoff, 1, seed=3, first_sweep=warm + t)
    us.append(round(ctx.region_end() * 1e3, 1))
print(json.dumps({"cfg": cfg, "warmup": warm, "us": us, "stats": ctx.stats()}))
