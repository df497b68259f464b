#!/usr/bin/env python3
"""Per-rank sweep time of a BASELINE config's strong-scaling shards, on one GPU.

A multi-GPU sweep is: every rank sweeps its contiguous shard of the targets against
the GLOBAL snapshot aggregates, then the ranks all-reduce the new aggregates
(.fs:940-942: every target reads only the snapshot).  This probe reproduces the first
part exactly without a communicator:

1. the whole sampler (world 1) runs the chain from doMotifSampling's input
   (getPWMOfRandomStarts' shared draws, .fs:1035-1037) or from uniform starts, and
   the snapshot before each measured sweep is kept (positions + global aggregates);
2. rank 0's shard of world = 1, 2, 4, 8 (N / world targets, n_global = N) is given
   each snapshot -- its slice of the positions, the GLOBAL aggregates uploaded -- and
   sweeps it once; the sweep kernel's device time is taken from the library's
   per-launch events, and the shard's new positions are checked against the whole
   sampler's (bit-identical: the same snapshot, the same counter-RNG uniforms).

With the all-reduce's own time (the one-rank RCCL bench's allreduce_ms) the rows
predict the driver's strong-scaling curve: speedup(world) = t(1) / (t(world) + ar).

    python tools/shard_probe.py [--config cfg4] [--worlds 1,2,4,8] [--steps 8]
"""
import argparse
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from gibbssampling_amd import Context, synthetic  # noqa: E402


def snapshots(w, codes, offsets, regime, warmup, steps, seed):
    """The whole sampler's chain: the snapshots (positions, aggregates) before the
    sweeps warmup .. warmup + steps - 1, and the positions after each."""
    ctx = Context(0)
    ctx.set_sequences(codes, offsets, w.alphabet)
    if regime == "uniform":
        pos = synthetic.initial_positions(w)
    else:
        pos = ctx.random_starts(w.W, w.pc, seed=synthetic.DATA_SEED + 1, mode=1)[1]
    ctx.set_positions(w.W, pos)
    if warmup:
        ctx.run_sweeps(w.pc, w.cutoff, warmup, seed=seed, first_sweep=0)
    snaps = []
    for t in range(warmup, warmup + steps):
        p0, _ = ctx.get_state()
        agg = ctx.agg_download()
        ctx.run_sweeps(w.pc, w.cutoff, 1, seed=seed, first_sweep=t)
        p1, _ = ctx.get_state()
        snaps.append((t, p0, agg, p1))
    ctx.close()
    return snaps


def shard_time(w, codes, offsets, lo, hi, snaps, seed, tun, exchange=False):
    ctx = Context(0, tuning=tun)
    ctx.set_sequences(codes[offsets[lo]:offsets[hi]], offsets[lo:hi + 1] - offsets[lo], w.alphabet,
                      n_global=w.N, global_offset=lo)
    if exchange:
        # the in-kernel exchange opened on this rank alone: the timed sweep includes its
        # last workgroup's stores and polls (not the xGMI hop to peers, nor their skew)
        ctx.exchange_open([ctx.exchange_handle()], 0)
    times, same, kernel = [], True, None
    for r, (t, p0, agg, p1) in enumerate(snaps):
        ctx.set_positions(w.W, p0[lo:hi])
        ctx.agg_upload(agg)  # the global snapshot (the all-reduced aggregates)
        kernel = ctx.sweep_kernel_name()
        ctx.synchronize()
        ctx.profile(True)
        ctx.run_sweeps(w.pc, w.cutoff, 1, seed=seed, first_sweep=t)
        ms, n, _, _ = ctx.profile_read()
        ctx.profile(False)
        got, _ = ctx.get_state()
        same &= bool(np.array_equal(got, p1[lo:hi]))
        if r > 0 and n > 0:  # the first launch pays the code-object load
            times.append(ms / n)
    ctx.close()
    return float(np.median(times)) * 1e3 if times else None, same, kernel


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="cfg4")
    ap.add_argument("--regimes", default="init")
    ap.add_argument("--tunings", default="", help="';'-separated NAME=v,NAME=v specs (A/B)")
    ap.add_argument("--exchange", action="store_true",
                    help="time the shard's sweep with a one-rank in-kernel exchange open")
    a = ap.parse_args()
    w = synthetic.CONFIGS[a.config]
    codes, offsets = synthetic.generate(w)
    seed = synthetic.DATA_SEED + 2
    for regime in a.regimes.split(","):
        snaps = snapshots(w, codes, offsets, regime, a.warmup, a.steps + 1, seed)
        keep = float(np.mean([(s[1] >= 0).mean() for s in snaps]))
        for world in [int(x) for x in a.worlds.split(",")]:
            lo, hi = 0, w.N // world
            for t in (a.tunings.split(";") if a.tunings else [""]):
                tun = {k: float(v) for k, v in (kv.split("=") for kv in t.split(",") if kv)}
                us, same, kernel = shard_time(w, codes, offsets, lo, hi, snaps, seed, tun, a.exchange)
                print(json.dumps({"config": w.name, "regime": regime, "world": world, "n_local": hi - lo,
                                  "kernel": kernel, "tuning": tun, "exchange": a.exchange, "us_per_sweep_kernel": us,
                                  "keep_motif": keep, "positions_match_whole_sampler": same}), flush=True)


if __name__ == "__main__":
    main()
