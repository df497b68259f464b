#!/usr/bin/env python3
"""A/B of the site sampler's Gauss-Seidel refinement (getBestPWMSsWithStartPositions,
.fs:554-585) between tuning-field variants (gs_set_tuning), interleaved, on BASELINE shapes:

    python tools/site_ab.py cfg2,cfg5 GS_SITE_COOP=0 GS_SITE_COOP=1 ...
    python tools/site_ab.py cfg5 lib=gibbssampling_amd/libgibbs_hip_prev.so ""
    AB_ROW=greedy python tools/site_ab.py cfg2,cfg5 ...   (the motif greedy instead:
    findBestMotifIndicesWithStartPositions .fs:885-929 after one sweep from the starts)

Each variant: a fresh context (knobs are read at creation), shared random starts,
the whole refinement timed around the C call; positions must agree across variants."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.join(os.path.dirname(__file__), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from conftest import make_dataset  # noqa: E402

SHAPES = {"cfg2": (10_000, 200, 12, b"ACGT"), "cfg5": (50_000, 300, 20, b"ACDEFGHIKLMNPQRSTVWY")}


def run(variant, codes, offsets, alpha, W):
    from gibbssampling_amd import Context
    from gibbssampling_amd._native import tuning_spec
    lib = None
    knobs = []
    for kv in filter(None, variant.split(",")):
        k, v = kv.split("=", 1)
        if k == "lib":  # another build of the library
            lib = os.path.join(ROOT, v)
        else:
            knobs.append(kv)
    ctx = Context(0, lib, tuning=tuning_spec(",".join(knobs)))
    try:
        ctx.set_sequences(codes, offsets, alpha)
        sc, p = ctx.random_starts(W, 1e-4, 7, 1)
        if os.environ.get("AB_ROW") == "greedy":
            ctx.set_positions(W, p)
            ctx.run_sweeps(1e-4, 1.0, 1, 7)
            q0, w0 = ctx.get_state()
            t = time.perf_counter()
            q, s, passes = ctx.motif_greedy(W, 1e-4, 1.0, q0, w0)
            return (time.perf_counter() - t) * 1e3, q, passes
        t = time.perf_counter()
        q, s, passes = ctx.site_refine(W, 1e-4, 0, p, sc)
        return (time.perf_counter() - t) * 1e3, q, passes
    finally:
        ctx.close()


def main():
    cfgs = sys.argv[1].split(",")
    variants = sys.argv[2:] or [""]
    out = {}
    for name in cfgs:
        N, L, W, alpha = SHAPES[name]
        codes, offsets = make_dataset(N, L, W, alpha, seed=5)
        res = {v: [] for v in variants}
        ref = None
        for rnd in range(int(os.environ.get("AB_ROUNDS", "2"))):
            for v in variants:
                ms, q, passes = run(v, codes, offsets, alpha, W)
                if ref is None:
                    ref = q
                same = bool(np.array_equal(q, ref))
                res[v].append(round(ms, 1))
                print(f"{name} round {rnd} [{v}]: {ms:.1f} ms, {passes} passes, same={same}",
                      file=sys.stderr, flush=True)
                if not same:
                    raise SystemExit(f"{name} [{v}]: positions differ from the first variant")
        out[name] = res
    print(json.dumps(out))


if __name__ == "__main__":
    main()
