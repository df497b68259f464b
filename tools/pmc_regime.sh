#!/usr/bin/env bash
# PMC counter passes (separate rocprofv3 runs, kernel-trace only) of a sweep kernel (KERNEL, default the live one)
# kernel for one config and start regime; summaries land in gpurun_out/pmc_<cfg>_<regime>/.
# usage: [KERNEL=k] [TUNINGS='live_G=4'] [SUFFIX=_g4] tools/pmc_regime.sh cfg3 init
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
CFG=${1:-cfg3}
REG=${2:-init}
OUT=gpurun_out/pmc_${CFG}_${REG}${SUFFIX:-}
mkdir -p $OUT
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $set -d $OUT/p$i -o run --output-format csv -- python3 tools/regime_bench.py --configs $CFG --regimes $REG --steps 10 --warmup 2 ${TUNINGS:+--tunings "$TUNINGS"} > $OUT/p$i.log 2>&1 || exit $?
done
python3 tools/pmc_summary.py $OUT ${KERNEL:-gs_sweep_live_kernel} > $OUT/summary.txt
echo ok
