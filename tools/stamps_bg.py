#!/usr/bin/env python3
"""Phase shares of the all-background sweep kernel (gs_sweep_bg.hip) from the stamps
build (make -C gibbssampling_amd/csrc stamps): the chain from uniform random starts,
3 sweeps to reach the all-background state, then 10 stamped sweeps.  Prints the
per-phase cycle shares and the cycles per wavefront (the stamps build's fences
forbid overlap, so absolute times are not quoted).
Usage: tools/stamps_bg.py [cfg[:NAME=v,...]] ..."""
import ctypes as C
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from gibbssampling_amd import _native, synthetic  # noqa: E402

PHASES = ["prologue", "target setup", "pass-1 walk", "scan + certify", "pass-2 walk",
          "fold + stores", "tail", "tile top"]
SLOTS = 16


def main():
    lib = ROOT / "gibbssampling_amd" / "libgibbs_hip_stamps.so"
    out = {}
    for spec in sys.argv[1:] or ["cfg2", "cfg4"]:
        name, _, tun = spec.partition(":")
        tuning = {k: float(v) for k, v in (kv.split("=") for kv in tun.split(",") if kv)}
        tuning.setdefault("bg_mode", 1)
        w = synthetic.CONFIGS[name]
        codes, offsets = synthetic.generate(w)
        ctx = _native.Context(0, lib, tuning=tuning)
        f = ctx.lib.gs_debug_stamps
        f.argtypes = [C.c_void_p, C.c_void_p, C.c_int32]
        buf = np.zeros(SLOTS, np.uint64)
        ctx.set_sequences(codes, offsets, w.alphabet)
        ctx.set_positions(w.W, synthetic.initial_positions(w))
        ctx.run_sweeps(w.pc, w.cutoff, 3, seed=1)
        ctx.synchronize()
        f(ctx.h, buf.ctypes.data, 1)
        ctx.run_sweeps(w.pc, w.cutoff, 10, seed=1, first_sweep=3)
        ctx.synchronize()
        f(ctx.h, buf.ctypes.data, 1)
        tot = float(buf[:len(PHASES)].sum())
        res = {p: round(float(buf[i]) / tot, 4) for i, p in enumerate(PHASES)}
        res["cycles_per_wave"] = tot / max(float(buf[SLOTS - 1]), 1.0)
        # diagnostics per wavefront pass: the find walk's range, its hit offset, walkers
        res["find_range_max"] = float(buf[8]) / max(float(buf[SLOTS - 1]), 1.0)
        res["find_hit_max"] = float(buf[9]) / max(float(buf[SLOTS - 1]), 1.0)
        res["walkers"] = float(buf[10]) / max(float(buf[SLOTS - 1]), 1.0)
        out[spec] = res
        ctx.close()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
