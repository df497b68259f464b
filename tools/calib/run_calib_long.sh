#!/usr/bin/env bash
# FETCH_SIZE / WRITE_SIZE of the long-sequence kernel's global access pattern (calib_long.hip)
# at config 3's shape (100k x 500, W = 15), the kernel's 3,072-wavefront grid: known
# bytes vs counters, one counter a pass.  Output under gpurun_out/calib_long/.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
OUT=gpurun_out/calib_long
rm -rf $OUT && mkdir -p $OUT
for shape in "100000 500 15"; do
  set -- $shape
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 60 rocprofv3 --kernel-trace --pmc $c -d $OUT/${c}_$1 -o run --output-format csv \
      -- tools/calib/calib_long $1 $2 $3 10 > $OUT/${c}_$1.log 2>&1 || exit $?
  done
done
python3 - <<'PY'
import csv, glob, json
out = {}
for path in sorted(glob.glob("gpurun_out/calib_long/*_*/run_counter_collection.csv")):
    key = path.split("/")[-2]
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path)) if "calib_long" in r["Kernel_Name"]]
    known = json.loads(open("gpurun_out/calib_long/%s.log" % key).read().strip().splitlines()[-1])
    kib = sum(vals[1:]) / max(1, len(vals) - 1)
    k = "bytes_read_per_launch" if key.startswith("FETCH") else "bytes_written_per_launch"
    out[key] = {"counter_kib_per_launch": kib, "known_bytes": known[k], "known_over_counter_bytes": known[k] / (kib * 1024)}
print(json.dumps(out, indent=1))
PY
