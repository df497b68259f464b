"""Per-pass cost of the site sampler's Gauss-Seidel refinement (getBestPWMSsWithStartPositions,
.fs:554-585) at cfg2 (or cfg5: `python tools/site_passes.py cfg5`): cumulative time for
1..P passes from the same starts, and the positions each pass moves."""
import sys, time
sys.path.insert(0, '.'); sys.path.insert(0, 'tests')
import numpy as np
from conftest import make_dataset
from gibbssampling_amd import Context

N, L, W, AL = {"cfg2": (10000, 200, 12, b"ACGT"),
               "cfg5": (50000, 300, 20, b"ACDEFGHIKLMNPQRSTVWY")}[sys.argv[1] if len(sys.argv) > 1 else "cfg2"]
codes, offsets = make_dataset(N, L, W, AL, seed=5)
ctx = Context(0)
ctx.set_sequences(codes, offsets, AL)
sc, p = ctx.random_starts(W, 1e-4, 7, 1)
ctx.site_refine(W, 1e-4, 0, p, sc, max_passes=1)  # warm-up
prev = p
for k in range(1, 10):
    t = time.perf_counter()
    q, s, passes = ctx.site_refine(W, 1e-4, 0, p, sc, max_passes=k)
    dt = (time.perf_counter() - t) * 1e3
    print(f"passes<={k}: {dt:.1f} ms, ran {passes}, moved vs previous cap {int((q != prev).sum())}")
    prev = q
    if passes < k:
        break
