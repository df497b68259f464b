#!/usr/bin/env python3
"""Phase shares of the live-chain sweep kernel (gs_sweep_live.hip) from the stamps build.

make -C gibbssampling_amd/csrc stamps builds libgibbs_hip_stamps.so; this runs sweeps
from the initialiser's state (doMotifSampling's input) and prints the per-phase
cycle shares per wavefront and the cycles per tile (64 sequences, or 64/G).  The
stamps build's absolute times are not quoted (its s_memtime fences forbid overlap).
"""
import ctypes as C
import json
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from gibbssampling_amd import _native, synthetic  # noqa: E402

PHASES = ["prologue", "descriptors+pcv", "scan", "refine", "totals+pick", "fold",
          "why", "stores", "aggregates C", "aggregates T + wave_sync", "rescans"]
ORDER = [0, 1, 2, 3, 4, 5, 7, 8, 9, 10, 6]  # stamp slot of each phase above
SLOTS = 16


def main():
    lib_path = ROOT / "gibbssampling_amd" / "libgibbs_hip_stamps.so"
    out = {}
    for spec in sys.argv[1:] or ["cfg2", "cfg3", "cfg4"]:
        name, _, regime = spec.partition(":")  # cfg3:uniform = uniform random starts
        w = synthetic.CONFIGS[name]
        codes, offsets = synthetic.generate(w)
        tun = {"live_mode": 1, "dna_mode": 1}
        if os.environ.get("LIVE_G"):  # lanes per target (default: the engine's choice)
            tun["live_G"] = int(os.environ["LIVE_G"])
        ctx = _native.Context(0, lib_path, tuning=tun)
        f = ctx.lib.gs_debug_stamps
        f.argtypes = [C.c_void_p, C.c_void_p, C.c_int32]
        buf = np.zeros(SLOTS, np.uint64)
        ctx.set_sequences(codes, offsets, w.alphabet)
        if regime == "uniform":
            p0 = synthetic.initial_positions(w)
        else:
            _, p0 = ctx.random_starts(w.W, w.pc, seed=synthetic.DATA_SEED + 1, mode=1)
        ctx.set_positions(w.W, p0)
        ctx.run_sweeps(w.pc, w.cutoff, 3, seed=1)
        ctx.synchronize()
        f(ctx.h, buf.ctypes.data, 1)
        st0 = ctx.stats()
        ctx.run_sweeps(w.pc, w.cutoff, 10, seed=1, first_sweep=3)
        ctx.synchronize()
        f(ctx.h, buf.ctypes.data, 1)
        tot = float(buf[:SLOTS - 1].sum())
        res = {p: round(float(buf[ORDER[i]]) / tot, 4) for i, p in enumerate(PHASES)}
        res["cycles_per_tile"] = tot / max(float(buf[SLOTS - 1]), 1.0)
        st = ctx.stats()
        nres = max(st["exact_rescans"] - st0["exact_rescans"], 1)
        res["exact_rescans_10_sweeps"] = nres
        out[spec] = res
        ctx.close()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
