# Multi-GPU evidence on one GPU: the distributed tests, the init-regime shard probe
# (rank 0's shard of world 1/2/4/8 against the global snapshot) and a one-rank RCCL
# bench line (allreduce_ms).  Usage: TAG=x bash tools/gpu/dist.sh
set -o pipefail
TAG=${TAG:-dist}
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_dist_gloo.py tests/test_gpu_bg.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python -u tools/shard_probe.py --config ${SP_CFG:-cfg4} --worlds 1,2,4,8 --regimes init > $OUT/shard_probe.jsonl 2> $OUT/shard_probe.err
rc=$?; echo "shard rc=$rc"; cat $OUT/shard_probe.jsonl
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps ${STEPS:-50} --warmup 5 --config ${BCFG:-cfg4} > $OUT/bench_rccl1.json 2> $OUT/bench_rccl1.err
rc=$?; echo "bench rc=$rc"; tail -c 1500 $OUT/bench_rccl1.json; exit $rc
