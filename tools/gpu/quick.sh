# Quick GPU check: a chosen test selection, then an optional bench line.
# Usage: TAG=x TESTS="tests/test_gpu_dna.py" BENCH_ARGS="--no-side" bash tools/gpu/quick.sh
set -o pipefail
TAG=${TAG:-quick}
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 ${TEST_TIMEOUT:-300} python -u -m pytest ${TESTS:-tests/test_gpu_dna.py} -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 $OUT/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
if [ -n "${BENCH_ARGS:-}" ]; then
  timeout -k 10 300 python bench.py $BENCH_ARGS > $OUT/bench.json 2> $OUT/bench.err; rc=$?
  echo "bench rc=$rc"; tail -c 1500 $OUT/bench.json
fi
exit $rc
