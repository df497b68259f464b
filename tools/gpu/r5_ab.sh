# Round-5 A/B: the full GPU suite on the working tree's library, then config 3 / 5 /
# 2 init-regime sweeps against the HEAD build (libgibbs_hip_base5.so) and graph mode.
set -o pipefail
OUT=gpurun_out/${TAG:-r5ab}
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; if [ $rc -ne 0 ]; then grep -E "FAIL|Error" $OUT/pytest_gpu.log | head; exit $rc; fi
L=gibbssampling_amd/libgibbs_hip.so,gibbssampling_amd/libgibbs_hip_base5.so
for rep in 1 2; do
timeout -k 10 300 python -u tools/regime_bench.py --configs cfg3,cfg5,cfg2 --regimes init --steps 30 --warmup 3 --libs $L >> $OUT/ab.jsonl || exit 1
done
timeout -k 10 300 python -u tools/regime_bench.py --configs cfg2,cfg3 --regimes init --steps 100 --warmup 5 --tunings "graph_mode=0;graph_mode=1" >> $OUT/graph.jsonl || exit 1
timeout -k 10 300 python -u tools/regime_bench.py --configs cfg2,cfg4 --regimes init --steps 30 --warmup 3 --tunings "dna_mode=1,long_mode=1;dna_mode=1,long_mode=1,long_waves=8" >> $OUT/cfg2long.jsonl || exit 1
python3 - $OUT <<'PY'
import json, sys
for f in ("ab", "graph", "cfg2long"):
    for l in open(f"{sys.argv[1]}/{f}.jsonl"):
        r = json.loads(l); print(f, r["cfg"], r["lib"], r["tuning"], round(r["us_per_sweep"], 2), r["fallbacks_per_sweep"]["exact_rescans"])
PY
