#!/usr/bin/env bash
# FETCH_SIZE / WRITE_SIZE of the calibration pattern at the bench's size (resident)
# and past the Infinity Cache (streaming).  Output under gpurun_out/calib/.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
OUT=gpurun_out/calib
rm -rf $OUT && mkdir -p $OUT
for n in 10000 2000000; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 60 rocprofv3 --kernel-trace --pmc $c -d $OUT/${c}_$n -o run --output-format csv \
      -- tools/calib/calib_read $n 200 20 > $OUT/${c}_$n.log 2>&1 || exit $?
  done
done
python3 - <<'PY'
import csv, glob, json
out = {}
for path in sorted(glob.glob("gpurun_out/calib/*_*/run_counter_collection.csv")):
    key = path.split("/")[-2]
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path)) if "calib_read" in r["Kernel_Name"]]
    out[key] = {"per_launch_kib": sum(vals[1:]) / max(1, len(vals) - 1), "first_kib": vals[0] if vals else None}
print(json.dumps(out, indent=1))
PY
