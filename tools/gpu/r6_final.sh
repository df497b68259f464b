# Round 6 final evidence on the final sources: the GPU suite, smoke(), the default bench
# line (with the r6 PMC records in profiles/r6), rocprofv3 kernel stats of the headline
# bench, the strong-scaling shard probe.  Output under gpurun_out/r6final/.
set -o pipefail
export PYTHONUNBUFFERED=1
OUT=$PWD/gpurun_out/r6final
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1
timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-side > $OUT/bench_20steps.json 2> $OUT/bench_20steps.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-side --no-cpu-baseline --steps 200 > $OUT/bench_prof.json 2> $OUT/prof.err || exit 1
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u tools/shard_probe.py --config cfg4 --worlds 1,2,4,8 --steps 6 > $OUT/shard.jsonl 2> $OUT/shard.err || exit 1
timeout -k 10 300 python -u tools/shard_probe.py --config cfg4 --worlds 1,8 --steps 6 --exchange >> $OUT/shard.jsonl 2>> $OUT/shard.err || exit 1
cat $OUT/bench.json
