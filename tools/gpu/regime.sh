# Sweep timing per config / regime / tuning (tools/regime_bench.py) on the GPU.
# Usage: TAG=x ARGS="--configs cfg2 --tunings 'live_G=1;live_G=8'" bash tools/gpu/regime.sh
set -o pipefail
TAG=${TAG:-regime}
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
eval timeout -k 10 ${RB_TIMEOUT:-400} python -u tools/regime_bench.py $ARGS > $OUT/regime.jsonl 2> $OUT/regime.err
rc=$?; echo "rc=$rc"; cat $OUT/regime.jsonl | cut -c1-400; exit $rc
