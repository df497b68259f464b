# Round-6 GPU step: the -m gpu tests named by $TESTS (default: the whole suite), then
# optional init-regime A/B sweeps: $CFGS configs over the comma-separated $LIBS
# libraries and/or the ';'-separated $TUNINGS, $REPS times.  Usage (repo root):
#   TAG=r6a TESTS="tests/test_gpu_kdyn.py" CFGS=cfg2,cfg5 LIBS=a.so,b.so bash tools/gpu/r6.sh
set -o pipefail
OUT=gpurun_out/${TAG:-r6}
mkdir -p $OUT
export PYTHONUNBUFFERED=1
if [ "${TESTS:-tests}" != "none" ]; then
  timeout -k 10 ${TEST_LIMIT:-600} python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
  rc=$?; tail -3 $OUT/pytest_gpu.log; if [ $rc -ne 0 ]; then grep -E "FAIL|Error" $OUT/pytest_gpu.log | head -20; exit $rc; fi
fi
if [ -n "${CFGS:-}" ]; then
  for rep in $(seq ${REPS:-2}); do
    timeout -k 10 ${AB_LIMIT:-300} python -u tools/regime_bench.py --configs $CFGS --regimes ${REGIMES:-init} --steps ${STEPS:-30} --warmup 3 ${LIBS:+--libs $LIBS} ${TUNINGS:+--tunings "$TUNINGS"} >> $OUT/ab.jsonl || exit 1
  done
  python3 - $OUT <<'PY'
import json, sys
for l in open(f"{sys.argv[1]}/ab.jsonl"):
    r = json.loads(l); print(r["cfg"], r["regime"], r["lib"], r["tuning"], round(r["us_per_sweep"], 2), r["fallbacks_per_sweep"]["exact_rescans"], r["keep_motif"])
PY
fi
