#!/usr/bin/env python3
"""Per-wavefront timeline (stamps build, TLINE marks) of the live sweep on one
strong-scaling shard of config 4: N / world targets swept as rank 0 of a world-size
sampler would (n_global = N; the GLOBAL snapshot uploaded).  Diagnostic only.

usage: tools/timeline_shard.py [world] [tuning NAME=v,...]
"""
import ctypes as C
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from gibbssampling_amd import _native, synthetic  # noqa: E402
sys.path.insert(0, str(ROOT / "tools"))
from timeline import MARKS, WAVES, summarize  # noqa: E402
from shard_probe import snapshots  # noqa: E402


def main():
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    tun = {k: float(v) for k, v in (kv.split("=") for kv in (sys.argv[2] if len(sys.argv) > 2 else "").split(",") if kv)}
    w = synthetic.CONFIGS["cfg4"]
    codes, offsets = synthetic.generate(w)
    seed = synthetic.DATA_SEED + 2
    snaps = snapshots(w, codes, offsets, "init", 3, 3, seed)
    lo, hi = 0, w.N // world
    import os
    lib_path = ROOT / "gibbssampling_amd" / os.environ.get("GS_TL_LIB", "libgibbs_hip_stamps.so")
    ctx = _native.Context(0, lib_path, tuning=tun)
    f = ctx.lib.gs_debug_timeline
    f.argtypes = [C.c_void_p, C.c_void_p, C.c_int32]
    ctx.set_sequences(codes[offsets[lo]:offsets[hi]], offsets[lo:hi + 1] - offsets[lo], w.alphabet,
                      n_global=w.N, global_offset=lo)
    buf = np.zeros((WAVES, MARKS), np.uint64)
    runs = []
    for (t, p0, agg, p1) in snaps:
        ctx.set_positions(w.W, p0[lo:hi])
        ctx.agg_upload(agg)
        ctx.synchronize()
        f(ctx.h, buf.ctypes.data, WAVES)
        ctx.run_sweeps(w.pc, w.cutoff, 1, seed=seed, first_sweep=t)
        ctx.synchronize()
        f(ctx.h, buf.ctypes.data, WAVES)
        got, _ = ctx.get_state()
        rec = summarize(buf.copy())
        rec["positions_match"] = bool(np.array_equal(got, p1[lo:hi]))
        runs.append(rec)
    print(json.dumps({"world": world, "tuning": tun, "kernel": ctx.sweep_kernel_name(), "runs": runs[1:]}, indent=1))
    ctx.close()


if __name__ == "__main__":
    main()
