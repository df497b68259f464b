"""Measurement of the motifAmount >= 2 row: the Positions-list
sweep (gs_motif_sweep_multi), greedy passes (gs_motif_greedy_multi) and
doMotifSampling (gs_motif_sampling_multi) at BASELINE shapes, beside the CPU
restatement on a bounded sample (one thread).

    python tools/multi_bench.py cfg2 [cfg5] > profiles/r1/multi/rows_multi.json

GPU times are wall-clock around each C call (uploads, aggregates and arena
allocation included); run under `rocprofv3 --kernel-trace --stats` for the kernels'
own durations.  CPU: go_sweep_fast (hold-one-out, 1 thread) on the whole sweep, and
the incremental greedy port go_greedy_fast on its first `lim` visits.
"""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.join(os.path.dirname(__file__), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from conftest import make_dataset  # noqa: E402

SHAPES = {"cfg1": (100, 50, 8, b"ACGT"), "cfg2": (10_000, 200, 12, b"ACGT"),
          "cfg5": (50_000, 300, 20, b"ACDEFGHIKLMNPQRSTVWY")}
PC, CUTOFF, SEED = 1e-4, 1.0, 7


def wall(fn):
    t = time.perf_counter()
    r = fn()
    return r, (time.perf_counter() - t) * 1e3


def main():
    from gibbssampling_amd import Context
    from oracle import oracle_lib as ol
    out = {}
    M = int(os.environ.get("GS_MOTIF_AMOUNT", "2"))
    for name in sys.argv[1:] or ["cfg2"]:
        N, L, W, alpha = SHAPES[name]
        codes, offsets = make_dataset(N, L, W, alpha, seed=5)
        S = ol.Seqs(codes, offsets, alpha)
        ctx = Context(0)
        ctx.set_sequences(codes, offsets, alpha)
        res = {"N": N, "L": L, "W": W, "A": len(alpha), "motifAmount": M}
        sc, p = ctx.random_starts(W, PC, SEED, 1)
        cnt = np.ones(N, np.int32)
        lst = np.full((N, M), -1, np.int32)
        lst[:, 0] = p
        u0 = np.array([ol.uniform(SEED, ol.stream_sweep(0), n) for n in range(N)])
        u1 = np.array([ol.uniform(SEED, ol.stream_sweep(1), n) for n in range(N)])
        # sweep 0 from the single starts, then sweep 1 from its lists (timed)
        c1, p1, w1 = ctx.motif_sweep_multi(M, W, PC, CUTOFF, cnt, lst, u0)
        (c2, p2, w2), ms = wall(lambda: ctx.motif_sweep_multi(M, W, PC, CUTOFF, c1, p1, u1))
        (_, _, _), ms_b = wall(lambda: ctx.motif_sweep_multi(M, W, PC, CUTOFF, c1, p1, u1))
        t0 = time.perf_counter()
        oc, op, ow = ol.sweep_lists(S, M, W, PC, CUTOFF, c1, p1, M, u1, threads=1)
        cms = (time.perf_counter() - t0) * 1e3
        same = bool(np.array_equal(oc, c2) and np.array_equal(op[:, :M], p2)
                    and np.allclose(ow, w2, rtol=1e-12, atol=0))
        print(f"{name}: sweep gpu {ms:.2f} ms cpu {cms:.0f} ms", file=sys.stderr, flush=True)
        res["sweep"] = {"gpu_ms": min(ms, ms_b), "cpu_ms_holdout_1thread": cms,
                        "windows": int(N * (L - W + 1)),
                        "list_lengths": np.bincount(c2, minlength=M + 1).tolist(),
                        "identical_to_oracle": same}
        # greedy passes from sweep 1's motif memory
        (gc, gp, gw, passes), gms = wall(
            lambda: ctx.motif_greedy_multi(M, W, PC, CUTOFF, c2, p2, w2))
        print(f"{name}: greedy gpu {gms:.1f} ms, {passes} passes", file=sys.stderr, flush=True)
        lim = 20_000 if N > 1000 else N * 50
        cc, cp, cw = c2.copy(), np.ascontiguousarray(p2).copy(), w2.copy()
        ps, vis = C.c_int32(), C.c_int64()
        t0 = time.perf_counter()
        rc = ol.lib().go_greedy_fast(C.byref(S.s), M, W, PC, CUTOFF, ol._p(cc), ol._p(cp), M,
                                     ol._p(cw), 1000, lim, C.byref(ps), C.byref(vis))
        cgms = (time.perf_counter() - t0) * 1e3
        assert rc == 0
        visits = passes * N
        res["greedy"] = {"gpu_ms": gms, "passes": passes, "visits": visits,
                         "gpu_us_per_visit": gms * 1e3 / visits,
                         "cpu_us_per_visit": cgms * 1e3 / max(vis.value, 1),
                         "cpu_sample_visits": int(vis.value)}
        _, ms = wall(lambda: ctx.motif_sampling_multi(M, W, PC, CUTOFF, SEED, 1))
        res["doMotifSampling_ms"] = ms
        ctx.close()
        out[name] = res
        print(json.dumps({name: res}), file=sys.stderr)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
