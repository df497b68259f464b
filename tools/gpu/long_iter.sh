# Long-sequence kernel iteration: its parity tests, then config 3 / 4 init-regime sweep
# times (A/B over LIBS).  Usage: TAG=x [LIBS=a.so,b.so] [FULL=1] bash tools/gpu/long_iter.sh
set -o pipefail
TAG=${TAG:-long}
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest ${TESTS:-tests/test_gpu_long_kernel.py} -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|Error|assert" $OUT/pytest.log | head -30
if [ $rc -ne 0 ]; then tail -30 $OUT/pytest.log; exit $rc; fi
if [ -n "${FULL:-}" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
  rc=$?; echo "full pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log
  if [ $rc -ne 0 ]; then grep -E "FAIL|Error" $OUT/pytest_gpu.log | head; exit $rc; fi
fi
for rep in 1 2; do
timeout -k 10 300 python -u tools/regime_bench.py --configs cfg3 --regimes init --steps 30 --warmup 3 ${LIBS:+--libs "$LIBS"} \
  --tunings "${CFG3_TUNINGS:-long_mode=-1;long_mode=0}" >> $OUT/regime.jsonl 2>> $OUT/regime.err || { tail $OUT/regime.err; exit 1; }
done
timeout -k 10 300 python -u tools/regime_bench.py --configs cfg4 --regimes init --steps 30 --warmup 3 ${LIBS:+--libs "$LIBS"} \
  >> $OUT/regime.jsonl 2>> $OUT/regime.err || { tail $OUT/regime.err; exit 1; }
python3 - $OUT/regime.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    r = json.loads(l); print(r["cfg"], r["lib"], r["tuning"], round(r["us_per_sweep"], 2), r["keep_motif"], {k: v for k, v in r["fallbacks_per_sweep"].items() if v})
PY
