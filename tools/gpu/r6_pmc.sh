# Round-6 PMC records of the dominant sweep kernels (tools/pmc_regime.sh passes, then
# tools/pmc_record.py with the current sources' hash) for the (config, regime) pairs
# given as cfg:regime:kernel.  Records land in gpurun_out/r6pmc/ (copied to profiles/r6/).
# Usage: bash tools/gpu/r6_pmc.sh cfg2:init:gs_sweep_kernel cfg3:init:gs_sweep_long_kernel ...
set -o pipefail
mkdir -p gpurun_out/r6pmc
for spec in "$@"; do
  IFS=: read -r cfg reg kern <<< "$spec"
  rm -rf gpurun_out/pmc_${cfg}_${reg}
  KERNEL=$kern bash tools/pmc_regime.sh $cfg $reg || exit $?
  python3 tools/pmc_record.py gpurun_out/pmc_${cfg}_${reg} $cfg $reg $kern > gpurun_out/r6pmc/pmc_${cfg}_${reg}.json || exit $?
  cp gpurun_out/pmc_${cfg}_${reg}/summary.txt gpurun_out/r6pmc/pmc_${cfg}_${reg}_summary.txt
  rm -rf gpurun_out/pmc_${cfg}_${reg}/p*/
done
echo done
