#!/usr/bin/env bash
# instruction-fetch counters of gs_sweep_kernel at cfg2 init (separate passes, kernel trace only)
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
OUT=gpurun_out/pmc_icache
mkdir -p $OUT
i=0
for set in "SQ_WAVES SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" \
           "SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $set -d $OUT/p$i -o run --output-format csv -- python3 tools/regime_bench.py --configs cfg2 --regimes init --steps 10 --warmup 2 > $OUT/p$i.log 2>&1 || { tail -5 $OUT/p$i.log; exit 1; }
done
python3 tools/pmc_summary.py $OUT gs_sweep_kernel | tee $OUT/summary.txt
