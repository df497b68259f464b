# PMC records (tools/pmc_regime.sh passes + tools/pmc_record.py) for the given configs.
# Usage: TAG=x CFGS="cfg4 cfg3" bash tools/gpu/pmc.sh
set -o pipefail
TAG=${TAG:-pmc}
mkdir -p gpurun_out/$TAG
for cfg in ${CFGS:-cfg4}; do
  bash tools/pmc_regime.sh $cfg ${REGIME:-init} || exit $?
  python3 tools/pmc_record.py gpurun_out/pmc_${cfg}_${REGIME:-init} $cfg ${REGIME:-init} > gpurun_out/$TAG/pmc_${cfg}_${REGIME:-init}.json || exit $?
  head -40 gpurun_out/$TAG/pmc_${cfg}_${REGIME:-init}.json
done
