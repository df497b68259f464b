# Round-5 A/B of the long kernel: its GPU tests on the working tree's library, then
# config 3 init / uniform sweeps against the HEAD build (libgibbs_hip_base5.so:
# `make -C gibbssampling_amd/csrc variant NAME=base5` on the HEAD sources first).
set -o pipefail
OUT=gpurun_out/abl
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_long_kernel.py tests/test_golden.py tests/test_gpu_dist_gloo.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; if [ $rc -ne 0 ]; then grep -E "FAIL|Error" $OUT/pytest.log | head; exit $rc; fi
L=gibbssampling_amd/libgibbs_hip.so,gibbssampling_amd/libgibbs_hip_base5.so
for rep in 1 2; do
timeout -k 10 300 python -u tools/regime_bench.py --configs cfg3 --regimes init,uniform --steps 30 --warmup 3 --libs $L >> $OUT/ab.jsonl || exit 1
done
python3 - $OUT <<'PY'
import json, sys
for l in open(f"{sys.argv[1]}/ab.jsonl"):
    r = json.loads(l); print(r["cfg"], r.get("regime"), r["lib"], round(r["us_per_sweep"], 2), r["fallbacks_per_sweep"])
PY
