#!/usr/bin/env bash
# HBM traffic of the bench's sweep kernel: two PMC passes (FETCH_SIZE, WRITE_SIZE:
# TCC budget 4, so one per run), kernel trace only, on the bench command itself.
# Result: gpurun_out/traffic_<cfg>.json (copy it to profiles/<round>/).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
CFG=${1:-cfg2}
OUT=gpurun_out/traffic_$CFG
rm -rf $OUT && mkdir -p $OUT
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $c -d $OUT/$c -o run --output-format csv \
    -- python3 bench.py --config $CFG --steps 20 --warmup 3 --no-cpu-baseline --no-side > $OUT/$c.log 2>&1 || exit $?
done
python3 tools/pmc_traffic.py $OUT/FETCH_SIZE $OUT/WRITE_SIZE $CFG > gpurun_out/traffic_$CFG.json && cat gpurun_out/traffic_$CFG.json
