#!/usr/bin/env bash
# FETCH_SIZE / WRITE_SIZE of the general sweep kernel's global access pattern
# (calib_sweep.hip) at config 2's shape (10k x 200, 16 lanes a sequence, DNA) and
# config 5's (50k x 300, 32 lanes, 20 symbols): known bytes vs counters, one counter a
# pass, each at the sweep kernel's own launch shape (config 2: 625 workgroups of 4
# wavefronts; config 5: 256 of 12, round 5 on).  Output under gpurun_out/calib_sweep/.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
OUT=gpurun_out/calib_sweep
rm -rf $OUT && mkdir -p $OUT
for shape in "10000 200 16 4 52 4 625" "50000 300 32 20 420 12 256"; do
  set -- $shape
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 60 rocprofv3 --kernel-trace --pmc $c -d $OUT/${c}_$1 -o run --output-format csv \
      -- tools/calib/calib_sweep $1 $2 $3 $4 $5 10 $6 $7 > $OUT/${c}_$1.log 2>&1 || exit $?
  done
done
python3 - <<'PY'
import csv, glob, json
out = {"method": "tools/calib/calib_sweep.hip (the general sweep kernel's global loads and stores, known byte counts) under tools/calib/run_calib_sweep.sh: one rocprofv3 --pmc pass per counter, 10 launches, the first dropped",
       "shapes": {"10000": "cfg2: 10k x 200, W=12, 16 lanes a sequence, 625 workgroups x 4 wavefronts", "50000": "cfg5: 50k x 300, W=20, 20 symbols, 32 lanes, 256 workgroups x 12 wavefronts (3,072)"}}
for path in sorted(glob.glob("gpurun_out/calib_sweep/*_*/run_counter_collection.csv")):
    key = path.split("/")[-2]
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path)) if "calib_sweep" in r["Kernel_Name"]]
    known = json.loads(open("gpurun_out/calib_sweep/%s.log" % key).read().strip().splitlines()[-1])
    kib = sum(vals[1:]) / max(1, len(vals) - 1)
    k = "bytes_read_per_launch" if key.startswith("FETCH") else "bytes_written_per_launch"
    out[key] = {"counter_kib_per_launch": kib, "known_bytes": known[k], "known_over_counter_bytes": known[k] / (kib * 1024)}
print(json.dumps(out, indent=1))
PY
