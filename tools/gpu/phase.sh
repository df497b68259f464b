# Parity tests of the shipped library, then the phase-subtraction timings.
# Usage: TAG=x TESTS="..." LIBS="libgibbs_hip.so,libgibbs_hip_x1.so" CFGS=cfg2,cfg3,cfg4 bash tools/gpu/phase.sh
set -o pipefail
TAG=${TAG:-phase}
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
export PYTHONUNBUFFERED=1
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-300} python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -5 $OUT/pytest.log
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
timeout -k 10 ${PX_TIMEOUT:-400} python -u tools/phase_exp.py --configs ${CFGS:-cfg2,cfg3,cfg4} --libs ${LIBS} > $OUT/phase.jsonl 2> $OUT/phase.err
rc=$?; echo "phase rc=$rc"; cat $OUT/phase.jsonl; exit $rc
