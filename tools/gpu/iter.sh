# One iteration on the GPU: selected parity tests, regime timings, optional stamps.
# Usage: TAG=x TESTS="tests/test_gpu_dna.py" ARGS="--configs cfg2,cfg3,cfg4 --regimes init" STAMPS=1 bash tools/gpu/iter.sh
set -o pipefail
TAG=${TAG:-iter}
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
export PYTHONUNBUFFERED=1
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-300} python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -5 $OUT/pytest.log
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
eval timeout -k 10 ${RB_TIMEOUT:-300} python -u tools/regime_bench.py $ARGS > $OUT/regime.jsonl 2> $OUT/regime.err
rc=$?; echo "regime rc=$rc"; cut -c1-260 $OUT/regime.jsonl
if [ $rc -ne 0 ]; then exit $rc; fi
if [ -n "${STAMPS:-}" ]; then
  timeout -k 10 200 python -u tools/stamps_live.py ${STAMP_CFGS:-cfg2 cfg3 cfg4} > $OUT/stamps.json 2> $OUT/stamps.err
  rc=$?; echo "stamps rc=$rc"; cat $OUT/stamps.json
fi
exit $rc
