# Round-5 evidence for the long-sequence kernel at config 3: its read calibration on
# its own access pattern (tools/calib/calib_long.hip), then the PMC passes of the
# init-regime sweep (routed automatically) and their record.  Usage: bash tools/gpu/r5_evidence.sh
set -o pipefail
bash tools/calib/run_calib_long.sh > gpurun_out/calib_long.json || exit $?
KERNEL=gs_sweep_long_kernel bash tools/pmc_regime.sh cfg3 init || exit $?
echo done
