"""Durations and dispatch gaps of one kernel from a rocprofv3 --kernel-trace CSV:
    python tools/kernel_gaps.py gpurun_out/prof/<...>_kernel_trace.csv gs_sweep_kernel
Prints count, mean duration and the median / mean gap between consecutive
launches of that kernel (end of one to start of the next), in microseconds."""
import csv
import json
import sys

import numpy as np


def main():
    path, name = sys.argv[1], sys.argv[2]
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            if name in r["Kernel_Name"]:
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    rows.sort()
    s = np.array([a for a, _ in rows], np.float64)
    e = np.array([b for _, b in rows], np.float64)
    dur = (e - s) / 1e3
    gap = (s[1:] - e[:-1]) / 1e3
    gap = gap[gap < 1000.0]  # drop host pauses between phases
    print(json.dumps({"kernel": name, "count": len(rows), "mean_us": float(dur.mean()),
                      "median_gap_us": float(np.median(gap)) if gap.size else None,
                      "mean_gap_us": float(gap.mean()) if gap.size else None}))


if __name__ == "__main__":
    main()
