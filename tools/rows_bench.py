"""Measurement of the §8(f) rows beside the sweep:
GPU time of each entry point at a BASELINE shape, and the CPU restatement timed on
a bounded sample of the same work (single thread), one JSON object per shape.

    python tools/rows_bench.py cfg2 cfg5 > profiles/r1/rows.json

Rows: greedy refinement (gs_run_greedy after doMotifSampling's sweep), site scan
(one getBestPWMSs pass over all targets), the site sampler's refinements
(Gauss–Seidel and the ±1 shifted Jacobi passes), the exact / shared random-start
initialiser, and the two end-to-end drivers.  CPU samples: the incremental greedy
port (go_greedy_fast, first `visits` target visits), the faithful site scan and
initialiser (go_site_scan / go_random_starts, first `targets` targets, scaled by
N / targets: every target costs the same O(N·L) there).
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.join(os.path.dirname(__file__), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from conftest import make_dataset  # noqa: E402

SHAPES = {"cfg2": (10_000, 200, 12, b"ACGT"), "cfg3": (100_000, 500, 15, b"ACGT"),
          "cfg5": (50_000, 300, 20, b"ACDEFGHIKLMNPQRSTVWY")}
PC, CUTOFF, SEED = 1e-4, 1.0, 7


def wall(fn):
    t = time.perf_counter()
    r = fn()
    ms = (time.perf_counter() - t) * 1e3
    print(f"  step {ms:.1f} ms", file=sys.stderr, flush=True)  # progress for long runs
    return r, ms


def main():
    from gibbssampling_amd import Context
    from oracle import oracle_lib as ol
    out = {}
    for name in sys.argv[1:] or ["cfg2"]:
        N, L, W, alpha = SHAPES[name]
        codes, offsets = make_dataset(N, L, W, alpha, seed=5)
        S = ol.Seqs(codes, offsets, alpha)
        ctx = Context(0)
        ctx.set_sequences(codes, offsets, alpha)
        res = {"N": N, "L": L, "W": W, "A": len(alpha)}
        # --- initialiser (getPWMOfRandomStarts): shared draws and the exact O(N^2) mode
        ctx.random_starts(W, PC, SEED, 1)  # warm-up (module load)
        (sc1, p1), ms1 = wall(lambda: ctx.random_starts(W, PC, SEED, 1))
        (sc0, p0), ms0 = wall(lambda: ctx.random_starts(W, PC, SEED, 0))
        tgt = 4 if N > 20_000 else 16
        _, cms = wall(lambda: ol.random_starts(S, W, PC, seed=SEED, mode=0, t0=0, t1=tgt))
        res["random_starts"] = {"gpu_ms_shared": ms1, "gpu_ms_exact": ms0,
                                "cpu_ms_exact_extrapolated": cms * N / tgt,
                                "cpu_sample_targets": tgt}
        # --- site scan: one Jacobi getBestPWMSs pass at the shared starts
        ctx.site_scan(W, PC, p1)
        (ss, sp), ms = wall(lambda: ctx.site_scan(W, PC, p1))
        _, cms = wall(lambda: ol.site_scan(S, W, PC, p1, 0, tgt))
        res["site_scan"] = {"gpu_ms": ms, "cpu_ms_extrapolated": cms * N / tgt,
                            "cpu_sample_targets": tgt}
        # --- site refinements from the shared starts
        rows = {}
        p, s = p1, sc1
        for shift, key in ((0, "gauss_seidel"), (-1, "left_shift"), (1, "right_shift")):
            (p, s, passes), ms = wall(lambda: ctx.site_refine(W, PC, shift, p, s))
            rows[key] = {"gpu_ms": ms, "passes": passes}
            if shift == 0:
                gs_p, gs_s = p, s
        # CPU: the incremental port of getBestPWMSsWithStartPositions on a sample of
        # visits; the whole refinement (and a bitwise comparison) when it is short
        (_, _, _, cvis), cms = wall(lambda: ol.site_refine_fast(S, W, PC, p1, sc1, t_limit=5000))
        gsr = rows["gauss_seidel"]
        gsr.update(visits=gsr["passes"] * N, gpu_us_per_visit=gsr["gpu_ms"] * 1e3 / (gsr["passes"] * N),
                   cpu_us_per_visit=cms * 1e3 / max(cvis, 1), cpu_sample_visits=cvis,
                   moved=int((gs_p != p1).sum()))
        if gsr["cpu_us_per_visit"] * gsr["visits"] < 120e6:
            (cp, cs, cpass, cvis), cms = wall(lambda: ol.site_refine_fast(S, W, PC, p1, sc1))
            # positions and passes exactly; scores are log2 values (device log vs glibc:
            # the tests' 1e-12 relative)
            fin = np.isfinite(cs)
            rel = np.abs(cs[fin] - gs_s[fin]) / np.maximum(np.abs(cs[fin]), 1e-300)
            gsr.update(cpu_ms_full=cms, cpu_visits_full=cvis,
                       positions_identical=bool(np.array_equal(cp, gs_p)),
                       positions_differing=int((cp != gs_p).sum()),
                       passes_equal=bool(cpass == gsr["passes"]),
                       score_max_rel_diff=float(rel.max()) if rel.size else 0.0,
                       score_inf_equal=bool(np.array_equal(np.isfinite(cs), np.isfinite(gs_s))))
        res["site_refine"] = rows
        # --- greedy refinement after doMotifSampling's sweep
        ctx.set_positions(W, p1)
        ctx.run_sweeps(PC, CUTOFF, 1, SEED)
        q, w = ctx.get_state()
        passes, kms = ctx.run_greedy(PC, CUTOFF)
        gq, gw = ctx.get_state()
        visits = passes * N
        lim = 20_000
        (_, _, _, cvis), cms = wall(lambda: ol.greedy_fast(S, W, PC, CUTOFF, q, w, t_limit=lim))
        res["greedy"] = {"gpu_kernel_ms": kms, "passes": passes, "visits": visits,
                         "gpu_us_per_visit": kms * 1e3 / visits,
                         "cpu_us_per_visit": cms * 1e3 / max(cvis, 1),
                         "cpu_sample_visits": cvis,
                         "moved": int((gq != q).sum())}
        # --- end-to-end drivers
        _, ms = wall(lambda: ctx.motif_sampling(W, PC, CUTOFF, SEED, 1))
        res["doMotifSampling_ms"] = ms
        _, ms = wall(lambda: ctx.site_sampling(W, PC, SEED, 1))
        res["doSiteSampling_ms"] = ms
        ctx.close()
        out[name] = res
        print(json.dumps({name: res}), file=sys.stderr)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
