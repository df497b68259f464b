# Round 6: exchange tests, then the shard probe with and without the one-rank exchange.
set -o pipefail
OUT=gpurun_out/${TAG:-r6xch3}
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests/test_gpu_exchange.py tests/test_gpu_long_kernel.py tests/test_gpu_dist_gloo.py tests/test_gpu_dist.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for x in "" "--exchange"; do
  timeout -k 10 300 python -u tools/shard_probe.py --config cfg4 --worlds ${WORLDS:-1,8} --steps 6 $x >> $OUT/shard.jsonl 2>> $OUT/shard.err || exit 1
done
python3 -c "
import json
for l in open('$OUT/shard.jsonl'):
    r = json.loads(l); print(r['world'], r['exchange'], round(r['us_per_sweep_kernel'], 1), r['positions_match_whole_sampler'])"
