# Round 6: the in-kernel aggregate exchange.  Its GPU tests, then one-rank torchrun
# benches (a real one-rank RCCL communicator) of configs 4 and 3 with the per-sweep RCCL
# all-reduce vs the exchange (bench.py --exchange rccl|ipc), REPS times alternating.
set -o pipefail
OUT=gpurun_out/${TAG:-r6xch}
mkdir -p $OUT
export PYTHONUNBUFFERED=1
if [ "${TESTS:-tests/test_gpu_exchange.py tests/test_gpu_dist.py tests/test_gpu_dist_gloo.py}" != "none" ]; then
  timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_gpu_exchange.py tests/test_gpu_dist.py tests/test_gpu_dist_gloo.py} -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
  rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
fi
port=29611
for rep in $(seq ${REPS:-2}); do
  for cfg in ${CFGS:-cfg4 cfg3}; do
    for x in rccl ipc; do
      port=$((port + 1))
      timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
        --master-port $port bench.py --gpus 1 --steps ${STEPS:-60} --warmup 5 --config $cfg --exchange $x \
        --no-side --no-cpu-baseline > $OUT/bench_${cfg}_${x}_$rep.json 2> $OUT/bench_${cfg}_${x}_$rep.log || exit 1
      python3 -c "import json,sys; r=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], round(r['ms_per_step']*1e3,2), round(r['roofline']['kernel_ms']*1e3,2), r.get('allreduce_ms'))" $OUT/bench_${cfg}_${x}_$rep.json $cfg $x
    done
  done
done
