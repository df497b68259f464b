# Round-5 evidence: the long-sequence kernel's read calibration on its own access
# pattern (tools/calib/calib_long.hip), then the PMC passes of the init-regime sweeps of
# configs 3 (long kernel) and 5 (protein, general kernel) and their summaries.
# Usage: bash tools/gpu/r5_evidence.sh
set -o pipefail
bash tools/calib/run_calib_long.sh > gpurun_out/calib_long.json || exit $?
KERNEL=gs_sweep_long_kernel bash tools/pmc_regime.sh cfg3 init || exit $?
KERNEL=gs_sweep_kernel bash tools/pmc_regime.sh cfg5 init || exit $?
echo done
