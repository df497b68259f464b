#!/usr/bin/env python3
"""Per-step phase cycles of the greedy kernel (gs_greedy.hip) from the diagnostic
stamps build, in the doMotifSampling setting of tools/greedy_time.py.

    make -C gibbssampling_amd/csrc stamps && python tools/greedy_stamps.py cfg2
The stamps build's absolute times are not quoted anywhere (only phase shares).
"""
import ctypes as C
import json
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

from conftest import make_dataset  # noqa: E402
from gibbssampling_amd import _native  # noqa: E402

PHASES = ["prologue", "prefetch issue", "score tail", "ring store", "barrier A", "commit",
          "barrier B", "score: holdout+pcv", "score: tab", "score: scan", "score: argmax"]
SLOTS = 16
SHAPES = {"cfg2": (10_000, 200, 12, b"ACGT"), "cfg5": (50_000, 300, 20, b"ACDEFGHIKLMNPQRSTVWY")}


def main():
    lib_path = ROOT / "gibbssampling_amd" / "libgibbs_hip_stamps.so"
    out = {}
    site = "--site" in sys.argv  # getBestPWMSsWithStartPositions instead of the motif greedy
    for name in [x for x in sys.argv[1:] if not x.startswith("--")] or ["cfg2"]:
        N, L, W, alpha = SHAPES[name]
        codes, offsets = make_dataset(N, L, W, alpha, seed=5)
        ctx = _native.Context(0, lib_path)
        f = ctx.lib.gs_debug_stamps
        f.argtypes = [C.c_void_p, C.c_void_p, C.c_int32]
        buf = np.zeros(SLOTS, np.uint64)
        ctx.set_sequences(codes, offsets, alpha)
        sc, p0 = ctx.random_starts(W, 1e-4, 7, 1)
        ctx.set_positions(W, p0)
        ctx.run_sweeps(1e-4, 1.0, 1, 7)
        ctx.synchronize()
        f(ctx.h, buf.ctypes.data, 1)  # drop the sweep's stamps
        if site:
            f(ctx.h, buf.ctypes.data, 1)
            _, _, passes = ctx.site_refine(W, 1e-4, 0, p0, sc)
        else:
            passes, ms = ctx.run_greedy(1e-4, 1.0)
        f(ctx.h, buf.ctypes.data, 1)
        wave_steps = max(float(buf[SLOTS - 1]), 1.0)
        res = {p: round(float(buf[i]) / wave_steps, 1) for i, p in enumerate(PHASES)}
        res.update({"passes": passes, "wave_steps": wave_steps,
                    "waves": os.environ.get("GS_GREEDY_WAVES", "16")})
        out[name] = res
        ctx.close()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
