# Round-5 A/B of the general kernel: the full GPU suite on the working tree's library,
# then config 5 / 2 init-regime sweeps against the HEAD build (libgibbs_hip_base5.so:
# `make -C gibbssampling_amd/csrc variant NAME=base5` on the HEAD sources first).
set -o pipefail
OUT=gpurun_out/${TAG:-ab5}
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; if [ $rc -ne 0 ]; then grep -E "FAIL|Error" $OUT/pytest_gpu.log | head; exit $rc; fi
L=gibbssampling_amd/libgibbs_hip.so,gibbssampling_amd/libgibbs_hip_base5.so
for rep in 1 2; do
timeout -k 10 300 python -u tools/regime_bench.py --configs cfg5,cfg2 --regimes init --steps 30 --warmup 3 --libs $L >> $OUT/ab.jsonl || exit 1
done
python3 - $OUT <<'PY'
import json, sys
for l in open(f"{sys.argv[1]}/ab.jsonl"):
    r = json.loads(l); print(r["cfg"], r["lib"], round(r["us_per_sweep"], 2), r["fallbacks_per_sweep"]["exact_rescans"])
PY
