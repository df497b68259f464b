# One GPU call: the -m gpu tests, smoke(), the default bench line and a rocprofv3
# kernel-stats pass of the headline bench.  Usage (repo root): TAG=r3s2 bash tools/gpu/run_all.sh
# Test failures (pytest exit 1) do not stop the call; anything else does.
set -o pipefail
TAG=${TAG:-run}
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err && \
cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --no-side --no-cpu-baseline --steps 200 > $OUT/bench_prof.json 2> $OUT/prof.err
rc=$?; echo "rc=$rc"; exit $rc
