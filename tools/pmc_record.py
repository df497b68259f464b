#!/usr/bin/env python3
"""Per-launch PMC record of the dominant sweep kernel of one (config, regime) from
tools/pmc_regime.sh's passes, for bench.py's second roofline and its traffic figure.

For each pass the dispatches of the kernel that takes the most time are joined with
their counters (Dispatch_Id); early-exit dispatches (shorter than a third of the
longest: the all-background kernel's no-op in the init regime, the sweep kernel's
exit in the all-background state) are dropped.  Derived, per launch:

- traffic: read_factor x FETCH_SIZE + write_factor x WRITE_SIZE (KiB -> B): for the
  live kernel the factors calibrated on its own access pattern (profiles/r3/
  calib_live.json: 1.94 / 1.99 and 1.0), else MI355X_MICROARCH.md's gfx950 x2 for
  16-byte-per-lane reads; with the live kernel's minimum bytes by source beside it;
- valu: SQ_INSTS_VALU wave-instructions / the pass's own average duration, against
  the chip's issue peak 256 CUs x 4 SIMDs x 2.4 GHz / 2 cycles per wave64 VALU
  instruction (MI355X_MICROARCH.md cycle table: v_fma_f32 wave64 2 cycles per SIMD);
- the wave-cycle split SQ_ACTIVE_INST_VALU / SQ_WAIT_ANY / SQ_WAIT_INST_ANY over
  SQ_WAVE_CYCLES (all quad-cycles).

The record carries the SHA-256 of the sweep kernels' sources (the general and the
packed-layout ones) and of the engine that routes sweeps to them and sizes their grids
(gs_engine.cpp), comment-stripped; bench.py reports it only while they match.

    python tools/pmc_record.py gpurun_out/pmc_cfg3_init cfg3 init [kernel] > profiles/pmc_cfg3_init.json
"""
import collections
import csv
import hashlib
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "tools"))
from pmc_traffic import _code_only  # noqa: E402

SOURCES = ["gibbssampling_amd/csrc/gs_sweep_live.hip", "gibbssampling_amd/csrc/gs_sweep.hip",
           "gibbssampling_amd/csrc/gs_sweep_ek4.hip",
           "gibbssampling_amd/csrc/gs_engine.cpp",
           "gibbssampling_amd/csrc/gs_sweep_dna.hip", "gibbssampling_amd/csrc/gs_sweep_bg.hip",
           "gibbssampling_amd/csrc/gs_sweep_long.hip",
           "gibbssampling_amd/csrc/gs_bgregime.h", "gibbssampling_amd/csrc/gs_common.h",
           "gibbssampling_amd/csrc/gs_wave.h", "gibbssampling_amd/csrc/gs_fold.h",
           "gibbssampling_amd/csrc/gs_pick.h", "gibbssampling_amd/csrc/Makefile"]
VALU_PEAK = 256 * 4 * 2.4e9 / 2  # wave64 VALU instructions per second, whole chip
SWEEP_KERNELS = ("gs_sweep_live_kernel", "gs_sweep_dna_kernel", "gs_sweep_long_kernel",
                 "gs_sweep_bg_kernel", "gs_sweep_kernel")


def source_hash(root: Path = ROOT) -> str:
    h = hashlib.sha256()
    for s in SOURCES:
        h.update(s.encode())
        h.update(_code_only((root / s).read_text()).encode())
    return h.hexdigest()


CALIB_LIVE = ROOT / "profiles" / "r3" / "calib_live.json"
CALIB_SWEEP = ROOT / "profiles" / "r4" / "calib_sweep.json"
CALIB_LONG = ROOT / "profiles" / "r5" / "calib_long.json"
# round 6: recalibrated at the kernels' current launch shapes (tools/calib/run_calib_r6.sh:
# the general kernel's 625 x 4 and 256 x 12 grids, the live kernel's work-counter grid);
# a shape missing there falls back to the older record
CALIB_R6 = {"sweep": ROOT / "profiles" / "r6" / "calib_sweep.json",
            "live": ROOT / "profiles" / "r6" / "calib_live.json"}


def _calib(kind: str, old: Path, key: str):
    new = CALIB_R6[kind]
    if new.exists():
        c = json.load(open(new))
        if key in c:
            return c[key]["known_over_counter_bytes"], f"profiles/r6/{new.name}"
    return json.load(open(old))[key]["known_over_counter_bytes"], f"profiles/{old.parent.name}/{old.name}"
SHAPE_N = {"cfg3": "100000", "cfg4": "1000000"}
SWEEP_SHAPE_N = {"cfg2": "10000", "cfg5": "50000"}


def read_write_factors(kern: str, cfg: str):
    """Bytes per counted byte, calibrated on the kernel family's own global access
    pattern at the config's shape: the general sweep kernel's (lane groups staging
    byte sequences, tools/calib/calib_sweep.hip: configs 2 and 5), the packed-layout
    kernels' (one or a few lanes a target streaming 2-bit words, tools/calib/
    calib_live.hip: configs 3 and 4 -- the live kernel's own pattern, the closest one
    measured for the round-2 packed and the all-background kernels); otherwise
    MI355X_MICROARCH.md's gfx950 correction for 16-byte-per-lane reads (x2).
    Writes are the raw WRITE_SIZE (factor 1.0) throughout: the calibration kernels'
    write patterns (per-workgroup flush atomics at grids other than the real kernel's)
    gave factors that put corrected writes below the outputs the kernel must store."""
    if kern == "gs_sweep_long_kernel" and CALIB_LONG.exists() and cfg == "cfg3":
        c = json.load(open(CALIB_LONG))
        return (c["FETCH_SIZE_100000"]["known_over_counter_bytes"], 1.0,
                "reads: profiles/r5/calib_long.json (shape N=100000: the kernel's own pattern, its grid); "
                "writes: raw WRITE_SIZE")
    if kern == "gs_sweep_kernel" and CALIB_SWEEP.exists() and cfg in SWEEP_SHAPE_N:
        n = SWEEP_SHAPE_N[cfg]
        f, src = _calib("sweep", CALIB_SWEEP, f"FETCH_SIZE_{n}")
        return (f, 1.0, f"reads: {src} (shape N={n}: the kernel's own pattern); writes: raw WRITE_SIZE")
    if kern in ("gs_sweep_live_kernel", "gs_sweep_dna_kernel", "gs_sweep_bg_kernel") and CALIB_LIVE.exists() \
            and cfg in SHAPE_N:
        n = SHAPE_N[cfg]
        own = kern == "gs_sweep_live_kernel"
        f, src = _calib("live", CALIB_LIVE, f"FETCH_SIZE_{n}")
        return (f, 1.0, f"reads: {src} (shape N={n}: " +
                ("the kernel's own pattern" if own else "the packed-layout pattern of the live kernel") +
                "); writes: raw WRITE_SIZE")
    return 2.0, 1.0, "MI355X_MICROARCH.md HBM: 2 x FETCH_SIZE for 16 B/lane streaming reads (uncalibrated mix)"


def attribution(kern: str, cfg: str):
    """The packed-layout kernels' minimum HBM bytes per launch by source."""
    if kern not in ("gs_sweep_live_kernel", "gs_sweep_long_kernel"):
        return None
    sys.path.insert(0, str(ROOT))
    from gibbssampling_amd import synthetic
    w = synthetic.CONFIGS[cfg]
    words = ((w.L + 15) // 16 + 3) // 4 * 4  # packed words a sequence, padded to 4
    rec = {"descriptors": w.N * 16, "packed_words": w.N * 4 * words, "outputs": w.N * 12,
           "note": "descriptors: len, pos_in (4 B), pkoff (8 B); packed_words: 2-bit symbols padded to "
                   "16-byte multiples; outputs: pos_out (4 B), pwms_out (8 B); aggregates and counters < 1 KB"}
    if kern == "gs_sweep_long_kernel":
        rec["note"] += ("; the long kernel's work counters: one device-scope atomic a pair of batches of four "
                        "targets (N / 8, plus a last grab a wavefront), each counted by WRITE_SIZE as a partial "
                        "line (~55 B) though it stays at the memory side")
    return rec


def kernel_of(name: str):
    for k in SWEEP_KERNELS:
        if k + "<" in name or k + "(" in name:
            return k
    return None


def load_pass(d: Path):
    durs = {}
    for p in d.rglob("*kernel_trace.csv"):
        for r in csv.DictReader(open(p)):
            k = kernel_of(r["Kernel_Name"])
            if k:
                durs[int(r["Dispatch_Id"])] = (k, int(r["End_Timestamp"]) - int(r["Start_Timestamp"]),
                                               r["Kernel_Name"])
    ctr = collections.defaultdict(lambda: collections.defaultdict(float))
    for p in d.rglob("*counter_collection.csv"):
        for r in csv.DictReader(open(p)):
            i = int(r["Dispatch_Id"])
            if i in durs:
                ctr[i][r["Counter_Name"]] += float(r["Counter_Value"])
    return durs, ctr


def main():
    d, cfg, regime = Path(sys.argv[1]), sys.argv[2], sys.argv[3]
    passes = [load_pass(p) for p in sorted(d.glob("p*")) if p.is_dir()]
    tot = collections.Counter()
    for durs, _ in passes:
        for k, t, _n in durs.values():
            tot[k] += t
    # the kernel named on the command line (the regime's steady-state sweep), else the
    # one that took the most time
    kern = sys.argv[4] if len(sys.argv) > 4 and sys.argv[4] in tot else tot.most_common(1)[0][0]
    # ... and of its instantiations the one that took the most time: the snapshot's
    # aggregate launches (gs_sweep_kernel mode 1, the EK = 0 instantiation beside the
    # four-symbol sweep) are not the sweep (a round-5 record averaged two of them in)
    inst = collections.Counter()
    for durs, _ in passes:
        for k, t, n in durs.values():
            if k == kern:
                inst[n] += t
    name = inst.most_common(1)[0][0]
    vals = collections.defaultdict(list)
    durations = []
    for durs, ctr in passes:
        mx = max((t for k, t, n in durs.values() if n == name), default=0)
        keep = [i for i, (k, t, n) in durs.items() if n == name and t >= mx / 3]
        pd = [durs[i][1] for i in keep]
        for i in keep:
            for c, v in ctr[i].items():
                vals[c].append(v)
        if pd:
            durations.append(sum(pd) / len(pd))
    avg = {c: sum(v) / len(v) for c, v in vals.items()}
    # the median of the passes' means: one pass's dispatches can run long under the
    # profiler (a cfg2 record once averaged 40.8 us against 15.9 in every other)
    dur_ns = sorted(durations)[len(durations) // 2] if len(durations) % 2 else \
        sum(sorted(durations)[len(durations) // 2 - 1:len(durations) // 2 + 1]) / 2
    rec = {"workload": cfg, "regime": regime, "kernel": kern, "instantiation": name,
           "avg_duration_ns_under_pmc": dur_ns,
           "counters_per_launch": avg, "source_sha256": source_hash(),
           "method": "tools/pmc_regime.sh + tools/pmc_record.py"}
    if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
        rf, wf, how = read_write_factors(kern, cfg)
        rec["traffic_bytes_per_launch"] = (rf * avg["FETCH_SIZE"] + wf * avg["WRITE_SIZE"]) * 1024
        rec["traffic_correction"] = {"read_factor": rf, "write_factor": wf, "source": how}
        att = attribution(kern, cfg)
        if att:
            att["measured_read_bytes"] = rf * avg["FETCH_SIZE"] * 1024
            att["measured_write_bytes"] = wf * avg["WRITE_SIZE"] * 1024
            rec["attribution"] = att
    if "SQ_INSTS_VALU" in avg:
        rate = avg["SQ_INSTS_VALU"] / (dur_ns * 1e-9)
        rec["valu"] = {"achieved": rate, "peak": VALU_PEAK, "unit": "wave64 VALU instr/s",
                       "frac": rate / VALU_PEAK}
    wc = avg.get("SQ_WAVE_CYCLES")
    if wc:
        rec["wave_cycle_split"] = {k: avg[k] / wc for k in ("SQ_ACTIVE_INST_VALU", "SQ_WAIT_ANY",
                                                          "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY")
                                   if k in avg}
    json.dump(rec, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
