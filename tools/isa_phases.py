#!/usr/bin/env python3
"""Static instruction accounting of the sweep kernel: compiles gs_sweep.hip with
-DGS_MARKS (phase labels as ISA comments) and counts VALU / SALU / LDS / VMEM
instructions per labelled segment for one kernel instantiation.  Loops are
counted once (static), so the numbers are per pass through straight-line code.
Usage: tools/isa_phases.py [WM] [H] [GL]"""
import collections
import re
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
SRC = ROOT / "gibbssampling_amd" / "csrc"


def classify(op):
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_"):
        return "salu" if not op.startswith(("s_waitcnt", "s_cbranch", "s_branch", "s_nop",
                                             "s_barrier", "s_load", "s_buffer")) else "sctl"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    return None


def main():
    wm = sys.argv[1] if len(sys.argv) > 1 else "16"
    h = sys.argv[2] if len(sys.argv) > 2 else "2"
    gl = sys.argv[3] if len(sys.argv) > 3 else "16"
    with tempfile.TemporaryDirectory() as td:
        out = Path(td) / "k.s"
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                        "-ffp-contract=off", "-DGS_MARKS", "--cuda-device-only", "-S",
                        str(SRC / "gs_sweep.hip"), "-o", str(out)], check=True)
        text = out.read_text()
    name = f"_Z15gs_sweep_kernelILi{wm}ELi{h}ELi{gl}EEvN2gs9SweepArgsE:"
    body = text[text.index(name):]
    body = body[:body.index(".Lfunc_end")]
    seg = "entry"
    counts = collections.OrderedDict()
    for line in body.splitlines():
        m = re.search(r";GSMARK (\S+)", line)
        if m:
            seg = m.group(1)
            continue
        t = line.strip().split()
        if not t or t[0].startswith((".", ";")) or t[0].endswith(":"):
            continue
        c = classify(t[0])
        if c:
            counts.setdefault(seg, collections.Counter())[c] += 1
    print(f"gs_sweep_kernel<{wm},{h}> static instruction counts by phase (first occurrence order)")
    print(f"{'phase':12s} {'valu':>6s} {'salu':>6s} {'sctl':>6s} {'lds':>6s} {'vmem':>6s}")
    for k, c in counts.items():
        print(f"{k:12s} {c['valu']:6d} {c['salu']:6d} {c['sctl']:6d} {c['lds']:6d} {c['vmem']:6d}")


if __name__ == "__main__":
    main()
