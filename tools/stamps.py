#!/usr/bin/env python3
"""Phase shares of the sweep kernel from the diagnostic stamps build.

Loads gibbssampling_amd/libgibbs_hip_stamps.so (make -C gibbssampling_amd/csrc stamps),
runs a few sweeps per config and prints the per-phase cycle shares.  The stamps
build's absolute times are not quoted anywhere (its fences forbid overlap).
"""
import ctypes as C
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from gibbssampling_amd import _native, synthetic  # noqa: E402

PHASES = ["startup", "stage", "holdout+pcv", "log tables", "window scan", "pick", "fold",
          "rescans", "result", "accumulate", "batch end", "flush"]
SLOTS = 16  # gs_common.h kStampSlots: phases, then the sequence count


def main():
    lib_path = ROOT / "gibbssampling_amd" / "libgibbs_hip_stamps.so"
    out = {}
    for spec in sys.argv[1:] or ["cfg2", "cfg3", "cfg5"]:
        name, _, regime = spec.partition(":")  # cfg2:init = the initialiser's output
        w = synthetic.CONFIGS[name]
        codes, offsets = synthetic.generate(w)
        ctx = _native.Context(0, lib_path)
        f = ctx.lib.gs_debug_stamps
        f.argtypes = [C.c_void_p, C.c_void_p, C.c_int32]
        buf = np.zeros(SLOTS, np.uint64)
        ctx.set_sequences(codes, offsets, w.alphabet)
        if regime == "init":
            ctx.set_positions(w.W, ctx.random_starts(w.W, w.pc, seed=synthetic.DATA_SEED + 1, mode=1)[1])
        else:
            ctx.set_positions(w.W, synthetic.initial_positions(w))
        ctx.run_sweeps(w.pc, w.cutoff, 5, seed=1)
        ctx.synchronize()
        f(ctx.h, buf.ctypes.data, 1)
        ctx.run_sweeps(w.pc, w.cutoff, 10, seed=1, first_sweep=5)
        ctx.synchronize()
        f(ctx.h, buf.ctypes.data, 1)
        tot = float(buf[:len(PHASES)].sum())
        res = {p: round(float(buf[i]) / tot, 4) for i, p in enumerate(PHASES)}
        res["cycles_per_wave_iteration"] = tot / max(float(buf[SLOTS - 1]), 1.0)
        out[spec] = res
        ctx.close()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
