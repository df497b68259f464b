#!/usr/bin/env bash
# FETCH_SIZE / WRITE_SIZE of the live kernel's global access pattern (calib_live.hip)
# at config 4's shape (1M x 200, W = 12) and config 3's (100k x 500, W = 15): known
# bytes vs counters, one counter a pass.  Output under gpurun_out/calib_live/.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
OUT=gpurun_out/calib_live
rm -rf $OUT && mkdir -p $OUT
for shape in "1000000 200 12" "100000 500 15"; do
  set -- $shape
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 60 rocprofv3 --kernel-trace --pmc $c -d $OUT/${c}_$1 -o run --output-format csv \
      -- tools/calib/calib_live $1 $2 $3 10 > $OUT/${c}_$1.log 2>&1 || exit $?
  done
done
python3 - <<'PY'
import csv, glob, json
out = {}
for path in sorted(glob.glob("gpurun_out/calib_live/*_*/run_counter_collection.csv")):
    key = path.split("/")[-2]
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path)) if "calib_live" in r["Kernel_Name"]]
    known = json.loads(open("gpurun_out/calib_live/%s.log" % key).read().strip().splitlines()[-1])
    kib = sum(vals[1:]) / max(1, len(vals) - 1)
    k = "bytes_read_per_launch" if key.startswith("FETCH") else "bytes_written_per_launch"
    out[key] = {"counter_kib_per_launch": kib, "known_bytes": known[k], "known_over_counter_bytes": known[k] / (kib * 1024)}
print(json.dumps(out, indent=1))
PY
