#!/usr/bin/env bash
# Round-4 evidence, part 2: FETCH/WRITE calibration of the general sweep kernel's access
# pattern (configs 2 and 5), then the PMC passes and records of every config's dominant
# kernel in the init regime (the records use the calibration: it is copied into
# profiles/r4/ on the box before tools/pmc_record.py runs).
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/calib/run_calib_sweep.sh > gpurun_out/calib_sweep.json 2> gpurun_out/calib_sweep.err || { tail -20 gpurun_out/calib_sweep.err; exit 1; }
cp gpurun_out/calib_sweep.json profiles/r4/calib_sweep.json
for cr in ${PMC_SETS:-"cfg2 init" "cfg5 init" "cfg4 init" "cfg3 init"}; do
  set -- $cr
  k=gs_sweep_kernel; [ $1 = cfg4 ] && k=gs_sweep_live_kernel; [ $1 = cfg3 ] && k=gs_sweep_dna_kernel
  KERNEL=$k bash tools/pmc_regime.sh $1 $2 || exit $?
  python3 tools/pmc_record.py gpurun_out/pmc_$1_$2 $1 $2 > gpurun_out/pmc_$1_$2.json || exit $?
  echo "$1 $2 recorded"
done
echo final-b-ok
