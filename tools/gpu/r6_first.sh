# Round 6: config 3's first sweep from uniform starts under rocprofv3 (kernel trace):
# which kernels the timed sweep runs and how long each takes.
set -o pipefail
OUT=gpurun_out/${TAG:-r6first}
mkdir -p $OUT
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/first_sweep.py --configs cfg3 --reps 3 > $GRAFT_REPO_ROOT/$OUT/first.jsonl || exit 1
cd $GRAFT_REPO_ROOT
cat $OUT/first.jsonl
python3 - $OUT <<'PY'
import csv, glob, sys
for f in glob.glob(f"{sys.argv[1]}/prof/**/*kernel_stats.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        print(row["Name"][:70], row["Calls"], row["AverageNs"], row["MaxNs"])
PY
