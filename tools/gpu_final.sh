#!/usr/bin/env bash
# End-of-session GPU run: the round script (tests, smoke, bench, RCCL bench, rocprof
# stats), then the PMC records of configs 3/4 in both regimes and the headline's
# HBM traffic.  Every step has its own limit; the first failure ends the run.
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${TAG:-r2final}
TAG=$TAG bash tools/gpu_round.sh || exit $?
for cr in "cfg3 uniform" "cfg3 init" "cfg4 uniform" "cfg4 init"; do
  bash tools/pmc_regime.sh $cr || exit $?
done
bash tools/pmc_traffic.sh cfg2 || exit $?
echo final-ok
