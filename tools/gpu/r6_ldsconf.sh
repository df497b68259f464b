# LDS bank-conflict attribution for the live kernel at config 4 (diagnostic builds with
# phases skipped, GS_EXP; their results are not the sweep's): one PMC pass each.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/ldsconf
mkdir -p $OUT
for lib in ${LIBS:-libgibbs_hip.so libgibbs_hip_exp1.so libgibbs_hip_exp4.so}; do
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS \
    -d $OUT/$lib -o run --output-format csv -- python3 tools/regime_bench.py --configs ${CFG:-cfg4} --regimes init --steps 10 --warmup 2 \
    --libs gibbssampling_amd/$lib > $OUT/$lib.log 2>&1 || exit $?
  python3 tools/pmc_summary.py $OUT/$lib ${KERNEL:-gs_sweep_live_kernel} > $OUT/$lib.txt || exit 1
  echo "== $lib"; cat $OUT/$lib.txt; tail -1 $OUT/$lib.log | cut -c1-200
done
