# Round 6: done counters without the L2 writeback (default build) vs -DGS_L2_FENCE
# (libgibbs_hip_fence.so) vs HEAD-of-round (libgibbs_hip_base6.so): the GPU suite, the
# init-regime sweeps of configs 2-5, config 3's first sweep from uniform starts, and
# config 4's world-1/8 shards.
set -o pipefail
OUT=gpurun_out/${TAG:-r6nf2}
mkdir -p $OUT
export PYTHONUNBUFFERED=1
D=gibbssampling_amd
if [ "${TESTS:-tests}" != "none" ]; then
timeout -k 10 700 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; if [ $rc -ne 0 ]; then grep -E "FAIL|Error" $OUT/pytest_gpu.log | head -20; exit $rc; fi
fi
L=$D/libgibbs_hip.so,$D/libgibbs_hip_fence.so,$D/libgibbs_hip_base6.so
for rep in 1 2; do
timeout -k 10 400 python -u tools/regime_bench.py --configs ${CFGS:-cfg2,cfg3,cfg4,cfg5} --regimes init --steps 30 --warmup 3 --libs $L >> $OUT/ab.jsonl || exit 1
done
timeout -k 10 300 python -u tools/first_sweep.py --configs cfg3 --libs $D/libgibbs_hip.so,$D/libgibbs_hip_base6.so > $OUT/first.jsonl || exit 1
timeout -k 10 400 python -u tools/shard_probe.py --config cfg4 --worlds 1,8 --steps 6 > $OUT/shard.jsonl 2> $OUT/shard.err || { tail -5 $OUT/shard.err; exit 1; }
python3 - $OUT <<'PY'
import json, sys
for l in open(f"{sys.argv[1]}/ab.jsonl"):
    r = json.loads(l); print(r["cfg"], r["lib"], r["tuning"], round(r["us_per_sweep"], 2), r["fallbacks_per_sweep"]["exact_rescans"])
for l in open(f"{sys.argv[1]}/first.jsonl"):
    print(l.strip())
for l in open(f"{sys.argv[1]}/shard.jsonl"):
    d = json.loads(l); print(d["world"], d["tuning"], round(d["us_per_sweep_kernel"], 1), d["positions_match_whole_sampler"], d["keep_motif"])
PY
