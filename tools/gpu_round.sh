#!/usr/bin/env bash
# One GPU-box session: parity tests, smoke, bench (1 GPU, plain and under torchrun),
# rocprofv3 kernel trace.  Every GPU step has its own time limit; steps are chained
# with && (the script stops at the first failure).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out
TAG=${TAG:-r1}
mkdir -p $OUT
echo "== pytest -m gpu" && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > $OUT/pytest_gpu_$TAG.log 2>&1; rc=$?; tail -5 $OUT/pytest_gpu_$TAG.log; [ $rc -eq 0 ] || exit $rc
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1 && cat $OUT/smoke_$TAG.log && \
echo "== bench" && timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err && cat $OUT/bench_$TAG.json && \
echo "== bench torchrun (1 rank, RCCL path)" && timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 100 --warmup 3 --no-cpu-baseline > $OUT/bench_tr_$TAG.json 2> $OUT/bench_tr_$TAG.err && cat $OUT/bench_tr_$TAG.json && \
echo "== rocprof" && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_$TAG -o run --output-format csv -- python3 bench.py --steps 100 --warmup 3 --no-cpu-baseline > $OUT/rocprof_$TAG.log 2>&1 && \
find $OUT/prof_$TAG -name "*stats*" | head && echo done
