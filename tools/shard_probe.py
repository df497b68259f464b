#!/usr/bin/env python3
"""Per-rank sweep time of BASELINE config 4's strong-scaling shards on one GPU.

Rank 0's shard of world = 1, 2, 4, 8 (N / world sequences of one sampler of global
N = 1M, no communicator): the device time per sweep each rank spends before the
aggregate all-reduce, in both start regimes.  With the all-reduce's own time (the
one-rank RCCL bench's allreduce_ms) it predicts the driver's strong-scaling curve.

    python tools/shard_probe.py [--worlds 1,2,4,8] [--steps 30]
"""
import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from gibbssampling_amd import Context, synthetic  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="cfg4")
    ap.add_argument("--regimes", default="uniform,init")
    ap.add_argument("--tunings", default="", help="';'-separated NAME=v,NAME=v specs (A/B)")
    a = ap.parse_args()
    w = synthetic.CONFIGS[a.config]
    for world in [int(x) for x in a.worlds.split(",")]:
        lo, hi = 0, w.N // world
        codes, offsets = synthetic.generate(w, lo, hi)
        for t in (a.tunings.split(";") if a.tunings else [""]):
            tun = {k: float(v) for k, v in (kv.split("=") for kv in t.split(",") if kv)}
            run_shard(a, w, world, lo, hi, codes, offsets, tun)


def run_shard(a, w, world, lo, hi, codes, offsets, tun):
        ctx = Context(0, tuning=tun)
        ctx.set_sequences(codes, offsets, w.alphabet, n_global=w.N, global_offset=lo)
        for regime in a.regimes.split(","):
            if regime == "uniform":
                pos = synthetic.initial_positions(w, lo, hi)
            else:
                pos = ctx.random_starts(w.W, w.pc, seed=synthetic.DATA_SEED + 1, mode=1)[1]
            ctx.set_positions(w.W, pos)
            ctx.run_sweeps(w.pc, w.cutoff, a.warmup, seed=synthetic.DATA_SEED + 2, first_sweep=0)
            ctx.synchronize()
            ctx.region_begin()
            ctx.run_sweeps(w.pc, w.cutoff, a.steps, seed=synthetic.DATA_SEED + 2, first_sweep=a.warmup)
            ms = ctx.region_end() / a.steps
            print(json.dumps({"config": w.name, "world": world, "n_local": hi - lo, "regime": regime,
                              "tuning": tun, "us_per_sweep": ms * 1e3}), flush=True)
        ctx.close()


if __name__ == "__main__":
    main()
