#!/usr/bin/env python3
"""Headline benchmark: Gibbs sweeps (iterations) per second and W-mer windows
scored per second on BASELINE.json's configuration (10k x 200 bp DNA, W = 12).

A step is one synchronous sweep (MotifSampler.findBestMotifIndicesByWithStartPositions,
GibbsSampling.fs:935-970) over every sequence, inputs resident in HBM.  With N GPUs
(torch.distributed.run, one rank per GPU) every rank holds a 10k x 200 shard of one
global sampler (weak scaling) and the ranks all-reduce the count aggregates over
RCCL once per sweep.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import subprocess
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E, MI355X_MICROARCH.md chip table
METRIC = "Gibbs iters/sec and W-mer windows scored/sec, 10k×200bp DNA, W=12"


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def cpu_baseline(w, codes, offsets, pos, budget_s: float):
    """The reference-faithful O(N^2) CPU restatement (oracle, 1 thread) on a bounded
    sample of targets of one sweep, extrapolated per window; plus the hold-one-out
    OpenMP restatement on the full sweep for context."""
    from oracle import oracle_lib as ol  # checker / baseline only

    S = ol.Seqs(codes, offsets, w.alphabet)
    u = np.random.default_rng(7).random(len(pos))
    t = time.perf_counter()
    ol.sweep(S, w.W, w.pc, w.cutoff, pos, u, faithful=True, t0=0, t1=4)
    per_target = (time.perf_counter() - t) / 4
    n_t = int(max(4, min(len(pos), budget_s / max(per_target, 1e-9))))
    t = time.perf_counter()
    ol.sweep(S, w.W, w.pc, w.cutoff, pos, u, faithful=True, t0=0, t1=n_t)
    dt = time.perf_counter() - t
    faithful = n_t * w.K / dt
    threads = os.cpu_count() or 1
    threads = min(threads, 16)
    t = time.perf_counter()
    ol.sweep(S, w.W, w.pc, w.cutoff, pos, u, faithful=False, threads=threads)
    dt2 = time.perf_counter() - t
    fast = len(pos) * w.K / dt2
    return {
        "value": faithful, "unit": "windows/s", "cores": 1, "kind": "port",
        "sample": f"{n_t} of {len(pos)} targets of one sweep, reference-faithful O(N^2) rebuild "
                  f"(oracle/gibbs_oracle.c go_sweep_faithful), {dt:.1f}s, extrapolated per window; "
                  f"iters/s = {faithful / (len(pos) * w.K):.3e}",
        "cpu_model": cpu_model(),
        "optimized": {"value": fast, "unit": "windows/s", "cores": threads,
                      "kind": "port (hold-one-out, OpenMP)",
                      "sample": f"one full sweep, {dt2:.2f}s"},
    }


TRAFFIC_FILE = ROOT / "profiles" / "traffic_gs_sweep_kernel_{cfg}.json"


def pmc_traffic(cfg: str):
    """roofline.traffic: HBM bytes per gs_sweep_kernel launch from the committed PMC
    passes of this same command (tools/pmc_traffic.sh: FETCH_SIZE x 2 + WRITE_SIZE,
    the gfx950 corrections of MI355X_MICROARCH.md), used only while the kernel's
    sources hash to the profiled ones; otherwise None."""
    p = Path(str(TRAFFIC_FILE).format(cfg=cfg))
    if not p.exists():
        return None, None
    sys.path.insert(0, str(ROOT / "tools"))
    try:
        from pmc_traffic import source_hash
        rec = json.loads(p.read_text())
        if rec.get("source_sha256") != source_hash(ROOT):
            return None, f"{p.relative_to(ROOT)} is stale (kernel sources changed)"
        return float(rec["traffic_bytes_per_launch"]), str(p.relative_to(ROOT))
    except (OSError, ValueError, KeyError, ImportError) as e:
        return None, f"{p.name}: {e}"


def run_workload(ctx, w, lo, hi, steps, warmup, dist_ctx=None, dispatch_sample=16):
    """Times `steps` back-to-back resident sweeps.  Returns (elapsed_s, max over
    ranks; kernel_ms = device time per sweep from two HIP events on the library's
    stream around the timed region; dispatch, a dict of per-dispatch event averages
    from `dispatch_sample` extra sweeps after the timed region (each event-attached
    dispatch completes with a release and widens the gap behind it by ~5 us, so the
    timed region carries no per-launch events))."""
    import torch

    from gibbssampling_amd import synthetic

    pos = synthetic.initial_positions(w, lo, hi)
    ctx.set_positions(w.W, pos)
    ctx.run_sweeps(w.pc, w.cutoff, warmup, seed=synthetic.DATA_SEED + 2, first_sweep=0)
    # with a communicator the chain replays as hipGraphs: capture it before the clock
    ctx.prepare_sweeps(w.pc, w.cutoff, seed=synthetic.DATA_SEED + 2)
    ctx.synchronize()
    if dist_ctx is not None:
        dist_ctx.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ctx.region_begin()
    ctx.run_sweeps(w.pc, w.cutoff, steps, seed=synthetic.DATA_SEED + 2, first_sweep=warmup)
    region_ms = ctx.region_end()
    ctx.synchronize()
    torch.cuda.synchronize()
    if dist_ctx is not None:
        dist_ctx.barrier()
    elapsed = time.perf_counter() - t0
    if dist_ctx is not None:
        elapsed = dist_ctx.max(elapsed)
    dispatch = {}
    if dispatch_sample:
        ctx.profile(True)
        ctx.profile_read()
        ctx.run_sweeps(w.pc, w.cutoff, dispatch_sample, seed=synthetic.DATA_SEED + 2,
                       first_sweep=warmup + steps)
        ctx.synchronize()
        kms, nk, arms, nar = ctx.profile_read()
        ctx.profile(False)
        dispatch = {"kernel_ms": kms / max(nk, 1), "launches": nk}
        if nar:
            dispatch["allreduce_ms"] = arms / nar
    return elapsed, region_ms / steps, dispatch


class Dist:
    def __init__(self):
        import torch
        import torch.distributed as dist
        self.dist = dist
        self.rank = int(os.environ["RANK"])
        self.world = int(os.environ["WORLD_SIZE"])
        self.local = int(os.environ.get("LOCAL_RANK", self.rank))
        torch.cuda.set_device(self.local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", self.local))
        self.gloo = dist.new_group(backend="gloo")
        self.torch = torch

    def barrier(self):
        self.dist.barrier(group=self.gloo)

    def max(self, x: float) -> float:
        t = self.torch.tensor([x], dtype=self.torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX, group=self.gloo)
        return float(t.item())

    def bcast_bytes(self, b: bytes | None) -> bytes:
        obj = [b]
        self.dist.broadcast_object_list(obj, src=0, group=self.gloo)
        return obj[0]


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="cfg2", help="workload per rank (cfg1..cfg5)")
    ap.add_argument("--cpu-budget", type=float, default=12.0,
                    help="seconds of reference-faithful CPU work for cpu_baseline")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--extra", action="store_true",
                    help="also time the scan kernel at the long-sequence shape (cfg3)")
    args = ap.parse_args()

    # The one JSON line is the only thing on stdout: libraries (RCCL's version banner,
    # gloo) print to fd 1, so fd 1 points at stderr for the run and the result goes to
    # the saved original stdout.
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)

    import torch

    from gibbssampling_amd import Context, synthetic
    from gibbssampling_amd.synthetic import Workload

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        print("bench.py --gpus N>1 must be launched by torch.distributed.run (one rank per GPU)",
              file=sys.stderr)
        return 2
    # under torch.distributed.run every rank (also a single one) joins the RCCL path
    dist_ctx = Dist() if "WORLD_SIZE" in os.environ else None
    rank = dist_ctx.rank if dist_ctx else 0
    world = dist_ctx.world if dist_ctx else 1
    device = dist_ctx.local if dist_ctx else 0
    if not dist_ctx:
        torch.cuda.set_device(0)

    base = synthetic.CONFIGS[args.config]
    w = Workload(base.name, base.N * world, base.L, base.W, base.alphabet, base.pc, base.cutoff)
    lo, hi = rank * base.N, (rank + 1) * base.N
    codes, offsets = synthetic.generate(w, lo, hi)

    ctx = Context(device)
    ctx.set_sequences(codes, offsets, w.alphabet, n_global=w.N, global_offset=lo)
    if dist_ctx:
        uid = dist_ctx.bcast_bytes(Context.unique_id() if rank == 0 else None)
        ctx.comm_init(uid, world, rank)

    elapsed, kernel_ms, dispatch = run_workload(ctx, w, lo, hi, args.steps, args.warmup, dist_ctx)
    ms_per_step = elapsed * 1e3 / args.steps
    iters = args.steps / elapsed
    windows = w.N * w.K * iters
    fallbacks = ctx.stats()

    bytes_launch = base.N * (w.L + 24)  # scan kernel N*(L+24) per launch
    achieved = bytes_launch / (kernel_ms * 1e-3) / 1e9
    traffic, traffic_src = pmc_traffic(args.config) if world == 1 else (None, None)
    roofline = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                "traffic_unit": "bytes per launch", "traffic_source": traffic_src,
                "kernel": "gs_sweep_kernel", "kernel_ms": kernel_ms,
                "kernel_ms_source": "HIP events around the timed region / steps",
                "dispatch_event_ms": dispatch.get("kernel_ms"),
                "bytes_per_launch": bytes_launch}
    out = {
        "metric": METRIC,
        "value": windows,
        "unit": "windows/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (i.i.d. uniform symbols + one planted mutated W-mer per sequence)",
        "config": {"workload": w.name + (f" per rank, global N={w.N}" if world > 1 else ""),
                   "N": w.N, "L": w.L, "W": w.W, "alphabet": w.alphabet.decode(),
                   "pseudoCount": w.pc, "cutOff": w.cutoff, "motifAmount": 1,
                   "parallelism": f"sequences sharded over {world} GPU(s)"},
        "iters_per_sec": iters,
        "roofline": roofline,
        "fallbacks": fallbacks,  # cumulative over warmup + timed sweeps
    }
    if "allreduce_ms" in dispatch:
        out["allreduce_ms"] = dispatch["allreduce_ms"]

    if rank == 0 and world == 1 and args.extra and args.config == "cfg2":
        # the scan kernel at the long-sequence shape (BASELINE config 3)
        w3 = synthetic.CONFIGS["cfg3"]
        c3, o3 = synthetic.generate(w3)
        ctx3 = Context(device)
        ctx3.set_sequences(c3, o3, w3.alphabet)
        e3, k3, d3 = run_workload(ctx3, w3, 0, w3.N, 20, 3, None, dispatch_sample=4)
        b3 = w3.N * (w3.L + 24)
        a3 = b3 / (k3 * 1e-3) / 1e9
        out["roofline_cfg3"] = {"bound": "hbm", "achieved": a3, "peak": HBM_PEAK_GBS,
                                "unit": "GB/s", "frac": a3 / HBM_PEAK_GBS, "kernel_ms": k3,
                                "dispatch_event_ms": d3.get("kernel_ms"),
                                "iters_per_sec": 20 / e3,
                                "windows_per_sec": w3.N * w3.K * 20 / e3}
        ctx3.close()
        del c3, o3

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        pos = synthetic.initial_positions(w, lo, hi)
        out["cpu_baseline"] = cpu_baseline(w, codes, offsets, pos, args.cpu_budget)
        out["speedup_vs_cpu_baseline"] = windows / out["cpu_baseline"]["value"]

    ctx.close()
    if rank == 0:
        sys.stdout.flush()
        os.write(json_fd, (json.dumps(out) + "\n").encode())
    if dist_ctx:
        dist_ctx.dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
