#!/usr/bin/env python3
"""Where the bench's fixed cost goes: the timed region of bench.py (config 2, init
regime) split into host enqueue, device region and the synchronisations around it,
at 20 and 200 steps.  Prints one JSON object.
"""
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    import torch

    from gibbssampling_amd import Context, synthetic
    torch.cuda.set_device(0)
    w = synthetic.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "cfg2"]
    codes, offsets = synthetic.generate(w)
    ctx = Context(0)
    ctx.set_sequences(codes, offsets, w.alphabet)
    pos = ctx.random_starts(w.W, w.pc, seed=synthetic.DATA_SEED + 1, mode=1)[1]
    ctx.set_positions(w.W, pos)
    ctx.run_sweeps(w.pc, w.cutoff, 5, seed=synthetic.DATA_SEED + 2)
    ctx.synchronize()
    out = {"workload": w.name}
    first = 5
    for steps in (20, 20, 200, 20):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ctx.region_begin()
        t1 = time.perf_counter()
        ctx.run_sweeps(w.pc, w.cutoff, steps, seed=synthetic.DATA_SEED + 2, first_sweep=first)
        t2 = time.perf_counter()
        region_ms = ctx.region_end()
        t3 = time.perf_counter()
        torch.cuda.synchronize()
        t4 = time.perf_counter()
        ctx.synchronize()
        first += steps
        rec = {"steps": steps, "region_us_per_step": region_ms * 1e3 / steps,
               "elapsed_us_per_step": (t4 - t0) * 1e6 / steps,
               "fixed_us": (t4 - t0) * 1e6 - region_ms * 1e3,
               "region_begin_us": (t1 - t0) * 1e6, "enqueue_us": (t2 - t1) * 1e6,
               "region_end_wait_us": (t3 - t2) * 1e6, "torch_sync_us": (t4 - t3) * 1e6}
        out.setdefault("runs", []).append(rec)
    # an empty region: the events alone
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ctx.region_begin()
    ms = ctx.region_end()
    torch.cuda.synchronize()
    out["empty_region"] = {"region_us": ms * 1e3, "elapsed_us": (time.perf_counter() - t0) * 1e6}
    ctx.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
