# Live-kernel iteration: the full GPU suite, then config 3 / 4 init-regime sweep times
# by kernel and lane count, and the stamps build's phase shares at config 3 (G = 4).
# Usage: TAG=x bash tools/gpu/live_iter.sh
set -o pipefail
TAG=${TAG:-live}
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" $OUT/pytest_gpu.log | head -20; exit $rc; fi
timeout -k 10 300 python -u tools/regime_bench.py --configs cfg3 --regimes init --steps 20 --warmup 3 \
  --tunings "${CFG3_TUNINGS:-live_mode=0;live_mode=1,live_G=2;live_mode=1,live_G=4}" > $OUT/regime.jsonl 2> $OUT/regime.err || { tail $OUT/regime.err; exit 1; }
timeout -k 10 300 python -u tools/regime_bench.py --configs cfg4 --regimes init --steps 20 --warmup 3 >> $OUT/regime.jsonl 2>> $OUT/regime.err || { tail $OUT/regime.err; exit 1; }
cut -c1-250 $OUT/regime.jsonl
LIVE_G=4 timeout -k 10 200 python -u tools/stamps_live.py cfg3 cfg4 > $OUT/stamps_live.json 2> $OUT/stamps_live.err && cat $OUT/stamps_live.json
