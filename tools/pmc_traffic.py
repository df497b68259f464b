#!/usr/bin/env python3
"""HBM traffic per gs_sweep_kernel launch from two rocprofv3 PMC passes
(tools/pmc_traffic.sh), corrected as MI355X_MICROARCH.md § HBM prescribes:

- FETCH_SIZE / WRITE_SIZE are in KiB, from the L2's memory-side request counters;
- on gfx950 FETCH_SIZE reports half the bytes of a wide (16 B per lane) coalesced
  read — the kernel's sequence loads are exactly that (uint4 per lane), so the
  read bytes are 2 x FETCH_SIZE (its 4/8-byte descriptor and aggregate loads are
  uncalibrated and counted the same way);
- WRITE_SIZE is taken as is.

Averages over the sweep dispatches of the run (the first gs_sweep_kernel dispatch
is the counts-only pass of gs_state_set_positions and is skipped).  Writes one JSON
object carrying the SHA-256 of the kernel's sources, which bench.py checks before it
reports the figure as roofline.traffic.

    python tools/pmc_traffic.py <fetch_dir> <write_dir> <workload> > profiles/.../traffic.json
"""
import csv
import hashlib
import json
import re
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
SOURCES = ["gibbssampling_amd/csrc/gs_sweep.hip", "gibbssampling_amd/csrc/gs_common.h",
           "gibbssampling_amd/csrc/gs_wave.h", "gibbssampling_amd/csrc/gs_fold.h",
           "gibbssampling_amd/csrc/gs_stamps.h", "gibbssampling_amd/csrc/Makefile"]


def _code_only(text: str) -> str:
    """Source without comments and blank-line / indentation differences: a comment
    edit keeps a recorded measurement valid, a code edit does not."""
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    text = re.sub(r"//[^\n]*", "", text)
    text = re.sub(r"(?m)^\s*#(?!\s*(include|define|if|ifdef|ifndef|elif|else|endif|undef|pragma)).*$",
                  "", text)  # Makefile comments
    return "\n".join(ln.strip() for ln in text.splitlines() if ln.strip())


def _sweep_part(path: str, text: str) -> str:
    """gs_common.h also declares the other kernels' argument structs: keep what the
    sweep kernel compiles against (everything up to the greedy kernel's block)."""
    if path.endswith("gs_common.h"):
        cut = text.find("// findBestMotifIndicesWithStartPositions (.fs:885-929) and its site-sampler twin")
        if cut > 0:
            text = text[:cut]
    return text


def source_hash(root: Path = ROOT) -> str:
    h = hashlib.sha256()
    for s in SOURCES:
        h.update(s.encode())
        h.update(_code_only(_sweep_part(s, (root / s).read_text())).encode())
    return h.hexdigest()


def per_dispatch(d: Path, counter: str) -> list[float]:
    vals = {}
    for p in sorted(d.rglob("*counter_collection.csv")):
        for r in csv.DictReader(open(p)):
            if "gs_sweep_kernel" in r["Kernel_Name"] and r["Counter_Name"] == counter:
                k = (p, int(r["Dispatch_Id"]))
                vals[k] = vals.get(k, 0.0) + float(r["Counter_Value"])
    v = [vals[k] for k in sorted(vals)]
    return v[1:]  # skip the counts-only dispatch


def main():
    fetch_dir, write_dir, workload = Path(sys.argv[1]), Path(sys.argv[2]), sys.argv[3]
    f = per_dispatch(fetch_dir, "FETCH_SIZE")
    w = per_dispatch(write_dir, "WRITE_SIZE")
    if not f or not w:
        sys.exit("no gs_sweep_kernel dispatches with FETCH_SIZE / WRITE_SIZE found")
    fk, wk = sum(f) / len(f), sum(w) / len(w)
    out = {"kernel": "gs_sweep_kernel", "workload": workload,
           "fetch_size_kib_per_launch": fk, "write_size_kib_per_launch": wk,
           "launches": [len(f), len(w)],
           "traffic_bytes_per_launch": (2.0 * fk + wk) * 1024.0,
           "correction": "read bytes = 2 x FETCH_SIZE (gfx950, 16 B/lane streaming reads); "
                         "write bytes = WRITE_SIZE; KiB -> bytes",
           "source_sha256": source_hash()}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
