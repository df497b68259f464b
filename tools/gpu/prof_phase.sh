# rocprofv3 kernel trace of tools/phase_exp.py (one config, given libraries).
# Usage: TAG=x LIBS=libgibbs_hip.so CFGS=cfg4 bash tools/gpu/prof_phase.sh
set -o pipefail
TAG=${TAG:-profphase}
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/phase_exp.py --configs ${CFGS:-cfg4} --libs ${LIBS} --reps ${REPS:-10} --tuning "${TUNING:-}" > $OUT/phase.jsonl 2> $OUT/prof.err
rc=$?; echo "rc=$rc"; cat $OUT/phase.jsonl; find $OUT/prof -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-200 | head -30; exit $rc
