# Round 6: the done counter without L2 writeback fences (GS_NOFENCE variant: returning
# flush atomics, replicas read by atomics) vs the fenced build vs HEAD-of-round, config 2
# init regime with the handed-over tables; then the GPU tests on the variant.
set -o pipefail
OUT=gpurun_out/${TAG:-r6nf}
mkdir -p $OUT
export PYTHONUNBUFFERED=1
D=gibbssampling_amd
L=$D/libgibbs_hip.so,$D/libgibbs_hip_nofence.so,$D/libgibbs_hip_base6.so
for rep in 1 2 3; do
timeout -k 10 300 python -u tools/regime_bench.py --configs ${CFGS:-cfg2} --regimes init --steps 100 --warmup 5 --libs $L >> $OUT/ab.jsonl || exit 1
done
python3 - $OUT <<'PY'
import json, sys
for l in open(f"{sys.argv[1]}/ab.jsonl"):
    r = json.loads(l); print(r["cfg"], r["lib"], r["tuning"], round(r["us_per_sweep"], 2), r["fallbacks_per_sweep"]["exact_rescans"])
PY
cp $D/libgibbs_hip_nofence.so $D/libgibbs_hip.so
timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; if [ $rc -ne 0 ]; then grep -E "FAIL|Error" $OUT/pytest_gpu.log | head -20; exit $rc; fi
