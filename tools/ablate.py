#!/usr/bin/env python3
"""Time the sweep kernel of several builds (ablation variants are timing-only: their
outputs are wrong by construction).  Usage: tools/ablate.py lib1.so lib2.so ..."""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from gibbssampling_amd import _native, synthetic  # noqa: E402


def time_lib(lib, name, sweeps=20, exact=False):
    w = synthetic.CONFIGS[name]
    codes, offsets = synthetic.generate(w)
    ctx = _native.Context(0, lib)
    if exact:
        ctx.set_scan_mode(exact=True)
    ctx.set_sequences(codes, offsets, w.alphabet)
    ctx.set_positions(w.W, synthetic.initial_positions(w))
    ctx.run_sweeps(w.pc, w.cutoff, 3, seed=1)
    ctx.synchronize()
    ctx.profile(True)
    ctx.profile_read()
    ctx.run_sweeps(w.pc, w.cutoff, sweeps, seed=1, first_sweep=3)
    try:
        ctx.synchronize()
        err = None
    except Exception as e:  # ablated builds may trip the roulette
        err = str(e)[:60]
    kms, nk, _, _ = ctx.profile_read()
    ctx.close()
    return {"kernel_us": round(1000 * kms / max(nk, 1), 2), "err": err}


def main():
    libs = sys.argv[1:] or [str(ROOT / "gibbssampling_amd" / "libgibbs_hip.so")]
    out = {}
    for lib in libs:
        out[Path(lib).name] = {c: time_lib(lib, c) for c in ("cfg2", "cfg3", "cfg5")}
        out[Path(lib).name + " (exact scan)"] = {c: time_lib(lib, c, exact=True)
                                                 for c in ("cfg2", "cfg3", "cfg5")}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
