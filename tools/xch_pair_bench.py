#!/usr/bin/env python3
"""Two processes on the box's one GPU, each holding half of a config (contiguous shards,
dist.shard_bounds), sweeping concurrently with the in-kernel aggregate exchange open
(gs_exchange_*): the chain of `steps` sweeps in one gs_run_sweeps call a rank, timed
between gloo barriers, against the whole config swept by one process.  Both ranks'
final positions are gathered and compared with the one-process chain (bit-identical).
The two ranks share the GPU's CUs, so the pair's sweep is not faster than the whole
one; the difference is what running as two exchanging processes costs (the exchange's
stores and polls, the two kernels' skew).  Diagnostic (not the bench line).

usage: tools/xch_pair_bench.py [--config cfg4] [--steps 20]
"""
import argparse
import json
import os
import socket
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _init(w, codes, offsets):
    """getPWMOfRandomStarts' output for the whole config (the init regime's snapshot)."""
    from gibbssampling_amd import Context, synthetic
    c = Context(0)
    c.set_sequences(codes, offsets, w.alphabet)
    pos = c.random_starts(w.W, w.pc, seed=synthetic.DATA_SEED + 1, mode=1)[1]
    c.close()
    return pos


def _worker(rank, world, port, cfg, steps, out_dir):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from gibbssampling_amd import Context, synthetic
        from gibbssampling_amd.dist import open_exchange, shard_bounds
        w = synthetic.CONFIGS[cfg]
        codes, offsets = synthetic.generate(w)
        pos = _init(w, codes, offsets)
        lo, hi = shard_bounds(np.diff(offsets), world)[rank]
        ctx = Context(0)
        ctx.set_sequences(codes[offsets[lo]:offsets[hi]], offsets[lo:hi + 1] - offsets[lo], w.alphabet,
                          n_global=w.N, global_offset=lo)
        err = open_exchange(ctx, rank, world)
        assert err == "", err
        ctx.set_positions(w.W, pos[lo:hi])
        agg = torch.from_numpy(ctx.agg_download())
        dist.all_reduce(agg)  # the snapshot's aggregates (set from outside: the caller's)
        ctx.agg_upload(agg.numpy())
        ctx.synchronize()
        seed = synthetic.DATA_SEED + 2
        ctx.run_sweeps(w.pc, w.cutoff, 2, seed=seed, first_sweep=0)  # warmup (code objects)
        ctx.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        ctx.run_sweeps(w.pc, w.cutoff, steps, seed=seed, first_sweep=2)
        ctx.synchronize()
        dist.barrier()
        dt = time.perf_counter() - t0
        p, _ = ctx.get_state()
        np.savez(os.path.join(out_dir, f"pair{rank}.npz"), p=p, dt=dt, kernel=ctx.sweep_kernel_name(),
                 rescans=ctx.stats()["exact_rescans"])
        ctx.exchange_close()
        ctx.close()
    finally:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg4")
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    import tempfile

    import torch.multiprocessing as mp

    from gibbssampling_amd import Context, synthetic
    w = synthetic.CONFIGS[a.config]
    # the whole config in one process, the same chain
    codes, offsets = synthetic.generate(w)
    pos = _init(w, codes, offsets)
    c = Context(0)
    c.set_sequences(codes, offsets, w.alphabet)
    c.set_positions(w.W, pos)
    seed = synthetic.DATA_SEED + 2
    c.run_sweeps(w.pc, w.cutoff, 2, seed=seed, first_sweep=0)
    c.synchronize()
    t0 = time.perf_counter()
    c.run_sweeps(w.pc, w.cutoff, a.steps, seed=seed, first_sweep=2)
    c.synchronize()
    one = time.perf_counter() - t0
    ref, _ = c.get_state()
    kernel1 = c.sweep_kernel_name()
    c.close()
    del codes, offsets
    with tempfile.TemporaryDirectory() as d:
        ctx = mp.get_context("spawn")
        port = _free_port()
        procs = [ctx.Process(target=_worker, args=(r, 2, port, a.config, a.steps, d)) for r in range(2)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(timeout=600)
        codes_ok = all(p.exitcode == 0 for p in procs)
        parts = [np.load(os.path.join(d, f"pair{r}.npz")) for r in range(2)] if codes_ok else []
    rec = {"config": a.config, "steps": a.steps, "one_process_us_per_sweep": one / a.steps * 1e6,
           "one_process_kernel": kernel1, "exit_codes": [p.exitcode for p in procs]}
    if parts:
        got = np.concatenate([x["p"] for x in parts])
        rec.update({"pair_us_per_sweep": max(float(x["dt"]) for x in parts) / a.steps * 1e6,
                    "pair_kernel": str(parts[0]["kernel"]),
                    "pair_rescans": [int(x["rescans"]) for x in parts],
                    "positions_match_one_process": bool(np.array_equal(got, ref))})
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
