#!/usr/bin/env python3
"""Run a fixed number of sweeps of one BASELINE config (for rocprofv3 runs).
Usage: tools/run_cfg.py <cfg> [sweeps] [lib.so]"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from gibbssampling_amd import _native, synthetic  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "cfg3"
    sweeps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    lib = sys.argv[3] if len(sys.argv) > 3 else None
    w = synthetic.CONFIGS[name]
    codes, offsets = synthetic.generate(w)
    ctx = _native.Context(0, lib)
    ctx.set_sequences(codes, offsets, w.alphabet)
    ctx.set_positions(w.W, synthetic.initial_positions(w))
    ctx.run_sweeps(w.pc, w.cutoff, sweeps, seed=synthetic.DATA_SEED + 2)
    pos, pw = ctx.get_state()
    print(name, "sweeps", sweeps, "motif fraction", float((pos >= 0).mean()),
          "fallbacks", ctx.stats())
    ctx.close()


if __name__ == "__main__":
    main()
