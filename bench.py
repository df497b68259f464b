#!/usr/bin/env python3
"""Headline benchmark: Gibbs sweeps (iterations) per second and W-mer windows
scored per second on BASELINE.json's configuration (10k x 200 bp DNA, W = 12).

A step is one synchronous sweep (MotifSampler.findBestMotifIndicesByWithStartPositions,
GibbsSampling.fs:935-970) over every sequence, inputs resident in HBM.  One GPU:
BASELINE config 2 (10k x 200, W = 12), with config 3's scan (roofline_cfg3) and
config 4 whole on the GPU (cfg4: the strong-scaling base) beside it.  N GPUs
(torch.distributed.run, one rank per GPU): BASELINE config 4 (1M x 200, W = 12)
split over the ranks (strong scaling), one RCCL all-reduce of the count aggregates
per sweep.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import hashlib
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
    # the hold-one-out port on the host cores this job may use (the GPU box grants a
    # 16-core share, OMP_NUM_THREADS; os.cpu_count() there reports the whole machine)
    threads = min(os.cpu_count() or 1, int(os.environ.get("OMP_NUM_THREADS", "16") or 16))
    ol.sweep(S, w.W, w.pc, w.cutoff, pos, u, faithful=False, threads=threads)  # warm
    nsw, p = 20, pos
    t = time.perf_counter()
    for _ in range(nsw):
        p, _, _ = ol.sweep(S, w.W, w.pc, w.cutoff, p, u, faithful=False, threads=threads)
    dt2 = time.perf_counter() - t
    fast = nsw * len(pos) * w.K / dt2
    return {
        "value": faithful, "unit": "windows/s", "cores": 1, "kind": "port",
        "sample": f"{n_t} of {len(pos)} targets of one sweep, reference-faithful O(N^2) rebuild "
                  f"(oracle/gibbs_oracle.c go_sweep_faithful), {dt:.1f}s, extrapolated per window; "
                  f"iters/s = {faithful / (len(pos) * w.K):.3e}",
        "cpu_model": cpu_model(),
        "optimized": {"value": fast, "unit": "windows/s", "cores": threads,
                      "kind": "port (hold-one-out, OpenMP)",
                      "iters_per_sec": nsw / dt2,
                      "sample": f"{nsw} chained full sweeps from the same start, {dt2:.2f}s, "
                                f"{threads} OpenMP threads (nproc {os.cpu_count()})"},
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


PMC_RECORD_DIRS = ("r6", "r5", "r4", "r3", "r2")  # newest first


def pmc_record(cfg: str, regime: str):
    """The committed per-launch PMC record of the config's dominant sweep kernel in
    that regime (tools/pmc_regime.sh + tools/pmc_record.py): HBM traffic and the
    VALU-issue roofline, used only while the kernels' sources hash to the profiled
    ones; otherwise None."""
    cands = [ROOT / "profiles" / d / f"pmc_{cfg}_{regime}.json" for d in PMC_RECORD_DIRS]
    cands = [p for p in cands if p.exists()]
    if not cands:
        return None
    p = cands[0]
    sys.path.insert(0, str(ROOT / "tools"))
    try:
        from pmc_record import source_hash
        rec = json.loads(p.read_text())
        if rec.get("source_sha256") != source_hash(ROOT):
            return {"source": str(p.relative_to(ROOT)), "stale": True}
        return {"source": str(p.relative_to(ROOT)), "kernel": rec["kernel"],
                "kernel_us_under_pmc": rec["avg_duration_ns_under_pmc"] * 1e-3,
                "traffic_bytes_per_launch": rec.get("traffic_bytes_per_launch"),
                "valu": rec.get("valu"), "wave_cycle_split": rec.get("wave_cycle_split")}
    except (OSError, ValueError, KeyError, ImportError) as e:
        return {"source": p.name, "error": str(e)}


def start_positions(ctx, w, lo, hi, regime):
    """'uniform': uniform random starts (SURVEY §8(d) synthetic inputs; after one sweep
    every pick is a background category and the sampler stays in that state);
    'init': getPWMOfRandomStarts' output (.fs:589-611, shared draws, on the GPU), the
    snapshot doMotifSampling hands to the sweep (most picks are motif windows)."""
    from gibbssampling_amd import synthetic
    if regime == "uniform":
        return synthetic.initial_positions(w, lo, hi)
    return ctx.random_starts(w.W, w.pc, seed=synthetic.DATA_SEED + 1, mode=1)[1]


def run_workload(ctx, w, lo, hi, steps, warmup, dist_ctx=None, dispatch_sample=16,
                 regime="uniform"):
    """Times `steps` back-to-back resident sweeps.  Returns (elapsed_s, max over
    ranks; kernel_ms = device time per sweep from two HIP events on the library's
    stream around the timed region; dispatch, a dict of per-dispatch event averages
    from `dispatch_sample` extra sweeps after the timed region (each event-attached
    dispatch completes with a release and widens the gap behind it by ~5 us, so the
    timed region carries no per-launch events))."""
    import torch

    from gibbssampling_amd import synthetic

    pos = start_positions(ctx, w, lo, hi, regime)
    ctx.set_positions(w.W, pos)
    exchange = None
    if dist_ctx is not None and ctx.exchange_is_open():
        # the in-kernel exchange, checked on the warmup chain: every rank's sweeps ran and
        # every rank holds the same global aggregates, else the chain is restarted over
        # RCCL (the exchange's first run across GPUs is this one: a failure is reported
        # in the line, not fatal)
        err = ""
        try:
            ctx.run_sweeps(w.pc, w.cutoff, max(warmup, 2), seed=synthetic.DATA_SEED + 2, first_sweep=0)
            ctx.synchronize()
            agg = ctx.agg_download()
        except Exception as e:  # noqa: BLE001 (any failure of the exchange: fall back)
            err, agg = f"{type(e).__name__}: {e}", None
        ok = dist_ctx.sum_ints([0 if err else 1])[0] == dist_ctx.world
        if ok:
            h = int.from_bytes(hashlib.sha256(agg.tobytes()).digest()[:3], "little")  # (exact in binary64)
            ok = dist_ctx.sum_ints([h])[0] == h * dist_ctx.world and dist_ctx.max(h) == h
            err = err or ("" if ok else "ranks' aggregates differ after the warmup chain")
        exchange = "ipc" if ok else "rccl (ipc failed on the warmup chain: " + (err or "another rank") + ")"
        if not ok:
            try:
                ctx.exchange_close()
            except Exception:  # noqa: BLE001 (closed or not, the RCCL chain restarts below)
                pass
            ctx.set_positions(w.W, pos)  # (also clears the device error of a timed-out exchange)
    nwarm = max(warmup, 2) if exchange == "ipc" else warmup  # (the checked chain's sweeps)
    if exchange != "ipc":
        ctx.run_sweeps(w.pc, w.cutoff, warmup, seed=synthetic.DATA_SEED + 2, first_sweep=0)
    # with a communicator the chain replays as hipGraphs: capture it before the clock
    ctx.prepare_sweeps(w.pc, w.cutoff, seed=synthetic.DATA_SEED + 2)
    ctx.synchronize()
    # the snapshot the timed chain starts from (the CPU baseline sweeps the same one)
    pos0, _ = ctx.get_state()
    s0 = ctx.stats()
    if dist_ctx is not None:
        dist_ctx.barrier()
    torch.cuda.synchronize()
    # the region's start event is instrumentation, not sweep work: recorded (and its
    # host call paid) before the clock starts; the stop event (recorded without a
    # wait) and the device synchronize stay inside, the events are read after it
    ctx.region_begin()
    t0 = time.perf_counter()
    ctx.run_sweeps(w.pc, w.cutoff, steps, seed=synthetic.DATA_SEED + 2, first_sweep=nwarm)
    ctx.region_stop()  # the stop event, recorded without a wait of its own
    torch.cuda.synchronize()
    if dist_ctx is not None:
        dist_ctx.barrier()
    elapsed = time.perf_counter() - t0
    region_ms = ctx.region_end()  # the events' time (the clock has stopped; no wait left)
    ctx.synchronize()  # the sticky device error check (after the clock: not sweep work)
    if dist_ctx is not None:
        elapsed = dist_ctx.max(elapsed)
    pos1, _ = ctx.get_state()
    s1 = ctx.stats()
    n_loc = max(1, len(pos0))
    kept = [int((pos0 >= 0).sum()), int((pos1 >= 0).sum()), s1["bg_picks"] - s0["bg_picks"],
            s1["exact_rescans"] - s0["exact_rescans"], len(pos0)]
    if dist_ctx is not None:
        kept = dist_ctx.sum_ints(kept)
    n_all = max(1, kept[4])
    # a collapsed chain (every pick a background category, no window PWM-scored)
    # shows here: keep_motif ~0, bg_picks_per_target ~1
    chain = {"keep_motif_start": kept[0] / n_all, "keep_motif": kept[1] / n_all,
             "bg_picks_per_target_sweep": kept[2] / (n_all * steps),
             "rescans_per_sweep": kept[3] / steps, "start_pos": pos0 if n_loc else None}
    dispatch = {}
    if dispatch_sample:
        ctx.profile(True)
        ctx.profile_read()
        ctx.run_sweeps(w.pc, w.cutoff, dispatch_sample, seed=synthetic.DATA_SEED + 2,
                       first_sweep=nwarm + steps)
        ctx.synchronize()
        kms, nk, arms, nar = ctx.profile_read()
        ctx.profile(False)
        dispatch = {"kernel_ms": kms / max(nk, 1), "launches": nk}
        if nar:
            dispatch["allreduce_ms"] = arms / nar
    dispatch["chain"] = chain
    if exchange is not None:
        dispatch["exchange"] = exchange
    return elapsed, region_ms / steps, dispatch


def side_record(device, cfg, steps, warmup, regimes=("init", "uniform")):
    """One GPU, a whole BASELINE config, in the given start regimes: the figures the
    headline line carries beside its own (config 3: the HBM-bound long-sequence scan;
    config 4: the one-GPU base of the strong-scaling curve; config 5: protein; config
    2 uniform: the collapsed all-background chain, for the record)."""
    from gibbssampling_amd import Context, synthetic
    w = synthetic.CONFIGS[cfg]
    codes, offsets = synthetic.generate(w)
    ctx = Context(device)
    ctx.set_sequences(codes, offsets, w.alphabet)
    del codes
    rec = {"workload": w.name, "N": w.N, "L": w.L, "W": w.W,
           "kernel": None, "bytes_per_launch": w.N * (w.L + 24)}
    for regime in regimes:
        e, k, d = run_workload(ctx, w, 0, w.N, steps, warmup, None, dispatch_sample=0,
                               regime=regime)
        ch = dict(d["chain"])
        ch.pop("start_pos", None)
        rec["kernel"] = ctx.sweep_kernel_name()
        # the all-background state (every sweep after the first from uniform starts)
        # is swept by gs_sweep_bg_kernel, the sweep kernel then only exits
        bg = ch["bg_picks_per_target_sweep"] >= 1.0
        a = w.N * (w.L + 24) / (k * 1e-3) / 1e9
        rec[regime] = {"iters_per_sec": steps / e, "windows_per_sec": w.N * w.K * steps / e,
                       "ms_per_step": e * 1e3 / steps, "kernel_ms": k,
                       "kernel": "gs_sweep_bg_kernel" if bg else ctx.sweep_kernel_name(),
                       "hbm": {"achieved": a, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                               "frac": a / HBM_PEAK_GBS}, **ch}
        pmc = pmc_record(cfg, regime)
        if pmc:
            rec[regime]["pmc"] = pmc
    ctx.close()
    return rec


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

    def sum_ints(self, xs):
        t = self.torch.tensor(xs, dtype=self.torch.int64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM, group=self.gloo)
        return [int(v) for v in t.tolist()]

    def bcast_bytes(self, b: bytes | None) -> bytes:
        obj = [b]
        self.dist.broadcast_object_list(obj, src=0, group=self.gloo)
        return obj[0]


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default=None,
                    help="workload (cfg1..cfg5); default cfg2 on one GPU, cfg4 on several")
    ap.add_argument("--scaling", choices=["strong", "weak"], default=None,
                    help="strong: the config's N split over the ranks (default for cfg4); "
                         "weak: every rank a whole config-sized shard")
    ap.add_argument("--regime", choices=["uniform", "init"], default="init",
                    help="start positions of the timed chain (see start_positions); "
                         "init = getPWMOfRandomStarts' output, the snapshot the reference's "
                         "doMotifSampling sweeps (.fs:1035-1037)")
    ap.add_argument("--cpu-budget", type=float, default=12.0,
                    help="seconds of reference-faithful CPU work for cpu_baseline")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--exchange", choices=["auto", "rccl", "ipc"], default="auto",
                    help="the aggregate vector's per-sweep exchange between ranks: an RCCL "
                         "all-reduce after each sweep, or summed inside the live/long sweep's "
                         "last workgroup over HIP IPC (gs_exchange_open; checked on the warmup "
                         "chain, RCCL if that fails); auto = ipc with several ranks, else rccl")
    ap.add_argument("--no-side", action="store_true",
                    help="skip the config-3 roofline and config-4 records on one GPU")
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

    cfg = args.config or ("cfg2" if world == 1 else "cfg4")
    scaling = args.scaling or ("strong" if cfg == "cfg4" else "weak")
    base = synthetic.CONFIGS[cfg]
    if scaling == "strong":
        # one sampler of the config's N sequences, contiguous equal shards
        w = base
        lo, hi = rank * w.N // world, (rank + 1) * w.N // world
    else:
        w = Workload(base.name, base.N * world, base.L, base.W, base.alphabet, base.pc,
                     base.cutoff)
        lo, hi = rank * base.N, (rank + 1) * base.N
    codes, offsets = synthetic.generate(w, lo, hi)

    ctx = Context(device)
    ctx.set_sequences(codes, offsets, w.alphabet, n_global=w.N, global_offset=lo)
    if dist_ctx:
        uid = dist_ctx.bcast_bytes(Context.unique_id() if rank == 0 else None)
        ctx.comm_init(uid, world, rank)
        xch_err = None
        if args.exchange == "ipc" or (args.exchange == "auto" and world > 1):
            from gibbssampling_amd.dist import open_exchange
            xch_err = open_exchange(ctx, rank, world, dist_ctx.gloo)

    elapsed, kernel_ms, dispatch = run_workload(ctx, w, lo, hi, args.steps, args.warmup,
                                                dist_ctx, regime=args.regime)
    chain = dispatch.pop("chain")
    start_pos = chain.pop("start_pos")
    ms_per_step = elapsed * 1e3 / args.steps
    iters = args.steps / elapsed
    windows = w.N * w.K * iters
    fallbacks = ctx.stats()
    # the kernel that swept the timed chain: the all-background kernel once the chain
    # is in that state (from uniform starts, every sweep after the first), else the
    # sweep kernel
    bg_timed = chain["bg_picks_per_target_sweep"] >= 1.0
    kernel_name = "gs_sweep_bg_kernel" if bg_timed else ctx.sweep_kernel_name()

    bytes_launch = (hi - lo) * (w.L + 24)  # scan kernel N*(L+24) per launch
    achieved = bytes_launch / (kernel_ms * 1e-3) / 1e9
    traffic, traffic_src, valu = None, None, None
    if world == 1:
        rec = pmc_record(cfg, args.regime)
        if rec and not rec.get("stale") and rec.get("kernel") == kernel_name:
            traffic, traffic_src, valu = rec.get("traffic_bytes_per_launch"), rec["source"], rec.get("valu")
        elif kernel_name == "gs_sweep_kernel":
            traffic, traffic_src = pmc_traffic(cfg)
    roofline = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                "traffic_unit": "bytes per launch", "traffic_source": traffic_src,
                "kernel": kernel_name, "kernel_ms": kernel_ms,
                "valu": valu,  # the second roofline: VALU issue (committed PMC record)
                "kernel_ms_source": "HIP events around the timed region / steps (rank 0)",
                "dispatch_event_ms": dispatch.get("kernel_ms"),
                "bytes_per_launch": bytes_launch}
    xch = ("the count aggregates summed in each sweep's last workgroup over HIP IPC"
           if dispatch.get("exchange") == "ipc" else "one RCCL all-reduce of the count aggregates per sweep")
    par = f"{w.N} sequences split over {world} GPU(s), {xch}" if world > 1 else "one GPU"
    if dist_ctx and world == 1:
        par = f"one GPU, one-rank communicator, {xch}"
    out = {
        "metric": METRIC,
        "value": windows,
        "unit": "windows/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "f64 (outputs binary64-exact; windows filtered by certified int16/int32 fixed-point and binary32 bounds)",
        "data": "synthetic (i.i.d. uniform symbols + one planted mutated W-mer per sequence)",
        "config": {"workload": w.name + (f" per rank, global N={w.N}"
                                         if scaling == "weak" and world > 1 else ""),
                   "N": w.N, "L": w.L, "W": w.W, "alphabet": w.alphabet.decode(),
                   "pseudoCount": w.pc, "cutOff": w.cutoff, "motifAmount": 1,
                   "start_regime": args.regime, "parallelism": par},
        "iters_per_sec": iters,
        # keep_motif: targets holding a motif at the end of the timed chain (a chain
        # collapsed into the all-background state scores no window: ~0)
        "chain": chain,
        "roofline": roofline,
        "fallbacks": fallbacks,  # cumulative over warmup + timed sweeps
    }
    if "allreduce_ms" in dispatch:
        out["allreduce_ms"] = dispatch["allreduce_ms"]
    if "exchange" in dispatch:
        out["exchange"] = dispatch["exchange"]
    elif dist_ctx and xch_err:
        out["exchange"] = f"rccl (the IPC exchange did not open: {xch_err})"
    ctx.close()
    del codes, offsets

    if rank == 0 and world == 1 and not args.no_side and cfg == "cfg2":
        # the HBM-bound long-sequence scan (config 3), the strong-scaling base (config
        # 4, whole on one GPU), protein (config 5), each from getPWMOfRandomStarts'
        # output and from uniform starts; config 2 from uniform starts (collapsed)
        out["roofline_cfg3"] = side_record(device, "cfg3", 20, 3)
        out["cfg4"] = side_record(device, "cfg4", 20, 3)
        out["cfg5"] = side_record(device, "cfg5", 20, 3, regimes=("init",))
        out["cfg2_uniform"] = side_record(device, "cfg2", args.steps, args.warmup,
                                          regimes=("uniform",))

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        codes, offsets = synthetic.generate(w, lo, hi)
        # like for like: the CPU sweeps the snapshot the timed GPU chain started from
        pos = start_pos if start_pos is not None else synthetic.initial_positions(w, lo, hi)
        out["cpu_baseline"] = cpu_baseline(w, codes, offsets, pos, args.cpu_budget)
        out["cpu_baseline"]["start_regime"] = args.regime
        out["speedup_vs_cpu_baseline"] = windows / out["cpu_baseline"]["value"]
        out["speedup_vs_cpu_optimized"] = windows / out["cpu_baseline"]["optimized"]["value"]

    if rank == 0:
        sys.stdout.flush()
        os.write(json_fd, (json.dumps(out) + "\n").encode())
    if dist_ctx:
        dist_ctx.dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
