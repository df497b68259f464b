#!/usr/bin/env bash
# Round-4 evidence for the current sources: GPU tests, smoke, bench (1 GPU, plain and
# one-rank torchrun), rocprofv3 kernel stats of the bench, then the PMC records of the
# headline (config 2 init) and the side configs.  Every step has its own limit; the
# first failure ends the run.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
TAG=${TAG:-r4final}
TAG=$TAG bash tools/gpu_round.sh || exit $?
for cr in ${PMC_SETS:-"cfg2 init" "cfg4 init" "cfg3 init" "cfg5 init"}; do
  set -- $cr
  k=gs_sweep_kernel; [ $1 = cfg4 ] && k=gs_sweep_live_kernel; [ $1 = cfg3 ] && k=gs_sweep_dna_kernel
  KERNEL=$k bash tools/pmc_regime.sh $1 $2 || exit $?
  python3 tools/pmc_record.py gpurun_out/pmc_$1_$2 $1 $2 > gpurun_out/pmc_$1_$2.json || exit $?
done
echo final-ok
