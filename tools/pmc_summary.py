#!/usr/bin/env python3
"""Per-dispatch PMC summary of a tools/pmc_cfg.sh run: averages over the sweep
dispatches of one kernel (default gs_sweep_kernel: all its dispatches but the first,
the counts-only pass; gs_sweep_dna_kernel: every dispatch).
Usage: tools/pmc_summary.py <dir> [kernel-name]"""
import csv, sys, collections
from pathlib import Path
d = Path(sys.argv[1])
kname = sys.argv[2] if len(sys.argv) > 2 else "gs_sweep_kernel"
skip_first = kname == "gs_sweep_kernel"
vals = collections.defaultdict(list)
for p in sorted(list(d.glob("p*/run_counter_collection.csv")) + list(d.glob("*_SIZE/run_counter_collection.csv"))):
    rows = list(csv.DictReader(open(p)))
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    names = {}
    for r in rows:
        if kname + "<" not in r["Kernel_Name"] and kname + "(" not in r["Kernel_Name"]:
            continue
        per[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    for i, disp in enumerate(sorted(per)):
        if i == 0 and skip_first:
            continue  # the aggregate (counts-only) pass
        for k, v in per[disp].items():
            vals[k].append(v)
out = {k: sum(v) / len(v) for k, v in vals.items()}
for k in sorted(out):
    print(f"{k:24s} {out[k]:.4g}")
