#!/usr/bin/env bash
# Round-6 read-factor calibrations at the sweep kernels' current launch shapes (known
# bytes vs FETCH_SIZE / WRITE_SIZE, one counter a rocprofv3 pass):
#   general sweep (calib_sweep): config 2 (10k x 200, 625 workgroups x 4 wavefronts),
#     config 5 (50k x 300, 20 symbols, 256 x 12 = 3,072 wavefronts, round 5 on);
#   live sweep (calib_live): config 4 (1M x 200, W = 12) with the work counters' shape
#     (512 workgroups x 8 wavefronts, a tile's grab one device atomic).
# Writes gpurun_out/calib_r6/{calib_sweep,calib_live}.json.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
OUT=gpurun_out/calib_r6
rm -rf $OUT && mkdir -p $OUT
run() {  # name counter binary args...
  local name=$1 c=$2; shift 2
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc $c -d $OUT/${name}_$c -o run --output-format csv -- "$@" > $OUT/${name}_$c.log 2>&1
}
for c in FETCH_SIZE WRITE_SIZE; do
  run sweep_10000 $c tools/calib/calib_sweep 10000 200 16 4 52 10 4 625 || exit $?
  run sweep_50000 $c tools/calib/calib_sweep 50000 300 32 20 420 10 12 256 || exit $?
  run live_1000000 $c tools/calib/calib_live 1000000 200 12 10 8 512 || exit $?
done
python3 - <<'PY'
import csv, glob, json
O = "gpurun_out/calib_r6"
def rec(prefix, kname):
    out = {}
    for path in sorted(glob.glob(f"{O}/{prefix}_*_*/run_counter_collection.csv")):
        key = path.split("/")[-2]            # e.g. sweep_10000_FETCH_SIZE
        _, n, *cn = key.split("_")
        c = "_".join(cn)
        vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path)) if kname in r["Kernel_Name"]]
        known = json.loads(open(f"{O}/{key}.log").read().strip().splitlines()[-1])
        kib = sum(vals[1:]) / max(1, len(vals) - 1)
        k = "bytes_read_per_launch" if c == "FETCH_SIZE" else "bytes_written_per_launch"
        out[f"{c}_{n}"] = {"counter_kib_per_launch": kib, "known_bytes": known[k],
                           "known_over_counter_bytes": known[k] / (kib * 1024),
                           "launch": {"waves_per_block": known.get("waves_per_block"), "grid": known.get("grid")}}
    return out
sw = {"method": "tools/calib/calib_sweep.hip under tools/calib/run_calib_r6.sh: one rocprofv3 --pmc pass per counter, 10 launches, the first dropped, at the general sweep kernel's own launch shapes",
      "shapes": {"10000": "cfg2: 10k x 200, W=12, 16 lanes a sequence, 625 x 4 wavefronts",
                 "50000": "cfg5: 50k x 300, W=20, 20 symbols, 32 lanes, 256 x 12 = 3,072 wavefronts"}}
sw.update(rec("sweep", "calib_sweep"))
lv = {"method": "tools/calib/calib_live.hip (work-counter launch: calib_live_ctr_kernel) under tools/calib/run_calib_r6.sh",
      "shapes": {"1000000": "cfg4: 1M x 200, W=12, one lane a target, 512 x 8 wavefronts, tiles from a device counter"}}
lv.update(rec("live", "calib_live"))
json.dump(sw, open(f"{O}/calib_sweep.json", "w"), indent=1)
json.dump(lv, open(f"{O}/calib_live.json", "w"), indent=1)
print(json.dumps(sw, indent=1)); print(json.dumps(lv, indent=1))
PY
