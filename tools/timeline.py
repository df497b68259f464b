#!/usr/bin/env python3
"""Per-wavefront timeline of one sweep launch from the diagnostic stamps build.

Loads gibbssampling_amd/libgibbs_hip_stamps.so (make -C gibbssampling_amd/csrc stamps),
runs a chain in the given regime, then reads the TLINE marks (global 100 MHz clock)
of the last launch: when wavefronts start, reach each mark and exit, relative to the
first wavefront's start.  Diagnostic only: the stamps build's times are not quoted.

usage: tools/timeline.py cfg2:init [cfg5:init ...]
"""
import ctypes as C
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from gibbssampling_amd import _native, synthetic  # noqa: E402

MARKS = 8     # gs_common.h kTlMarks
WAVES = 16384  # gs_common.h kTlWaves
TICK_US = 0.01  # s_memrealtime: 100 MHz


def summarize(tl):
    live = tl[tl[:, 0] != 0]
    if len(live) == 0:
        return {"waves": 0, "nonzero_entries": int((tl != 0).sum())}
    t0 = live[:, 0].min()
    out = {"waves": int(len(live))}
    for i in range(MARKS):
        col = live[:, i]
        col = col[col != 0]
        if len(col) == 0:
            continue
        rel = (col.astype(np.float64) - t0) * TICK_US
        out[f"m{i}"] = [round(float(np.percentile(rel, q)), 2) for q in (0, 10, 50, 90, 100)]
    # per-wave spans between consecutive reached marks (median)
    spans = {}
    for i in range(1, MARKS):
        ok = (live[:, i] != 0) & (live[:, i - 1] != 0)
        if ok.any():
            spans[f"m{i - 1}->m{i}"] = round(float(np.median((live[ok, i] - live[ok, i - 1]) * TICK_US)), 2)
    out["median_spans_us"] = spans
    last = np.max(live[:, 1:], axis=1)
    out["wave_life_us"] = [round(float(np.percentile((last - live[:, 0]) * TICK_US, q)), 2)
                           for q in (10, 50, 90, 100)]
    return out


def main():
    import os
    lib_path = ROOT / "gibbssampling_amd" / os.environ.get("GS_TL_LIB", "libgibbs_hip_stamps.so")
    res = {}
    for spec in sys.argv[1:] or ["cfg2:init"]:
        name, _, regime = spec.partition(":")
        w = synthetic.CONFIGS[name]
        codes, offsets = synthetic.generate(w)
        tun = {k: float(v) for k, v in (kv.split("=") for kv in os.environ.get("TL_TUNING", "").split(",") if kv)}
        ctx = _native.Context(0, lib_path, tuning=tun)
        f = ctx.lib.gs_debug_timeline
        f.argtypes = [C.c_void_p, C.c_void_p, C.c_int32]
        ctx.set_sequences(codes, offsets, w.alphabet)
        if regime == "init":
            ctx.set_positions(w.W, ctx.random_starts(w.W, w.pc, seed=synthetic.DATA_SEED + 1, mode=1)[1])
        else:
            ctx.set_positions(w.W, synthetic.initial_positions(w))
        ctx.run_sweeps(w.pc, w.cutoff, 5, seed=1)
        ctx.synchronize()
        buf = np.zeros((WAVES, MARKS), np.uint64)
        runs = []
        st = np.zeros(16, np.uint64)
        fs = ctx.lib.gs_debug_stamps
        fs.argtypes = [C.c_void_p, C.c_void_p, C.c_int32]
        for r in range(3):
            rc0 = f(ctx.h, buf.ctypes.data, WAVES)  # clears
            ctx.run_sweeps(w.pc, w.cutoff, 1, seed=1, first_sweep=5 + r)
            ctx.synchronize()
            rc1 = f(ctx.h, buf.ctypes.data, WAVES)
            fs(ctx.h, st.ctypes.data, 1)
            rec = summarize(buf.copy())
            rec.update(rc=[rc0, rc1], stamp_sum=int(st[:12].sum()), stamp_seqs=int(st[15]),
                       stamp_share=[round(float(x) / max(1, float(st[:12].sum())), 4) for x in st[:12]])
            runs.append(rec)
        if os.environ.get("TL_RAW"):  # the last launch's raw marks, for per-wave analysis
            np.save(os.environ["TL_RAW"] + f"_{name}.npy", buf)
        res[spec] = {"kernel": ctx.sweep_kernel_name(), "runs": runs}
        ctx.close()
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
