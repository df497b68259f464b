# Round 6: the four-symbol sweep's handed-over workgroup tables.  The GPU suite on the
# working tree's library, then config 2 init-regime sweeps: handoff (default) vs the
# HEAD-of-round build (libgibbs_hip_base6.so), and the table kernel before every sweep
# (ftab_mode=1) under rocprofv3 (the sweep kernel's own time with its tables given).
set -o pipefail
OUT=gpurun_out/${TAG:-r6ftab}
mkdir -p $OUT
export PYTHONUNBUFFERED=1
if [ "${TESTS:-tests}" != "none" ]; then
timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; if [ $rc -ne 0 ]; then grep -E "FAIL|Error" $OUT/pytest_gpu.log | head -20; exit $rc; fi
fi
L=gibbssampling_amd/libgibbs_hip.so,gibbssampling_amd/libgibbs_hip_base6.so
for rep in 1 2 3; do
timeout -k 10 300 python -u tools/regime_bench.py --configs cfg2 --regimes init --steps 100 --warmup 5 --libs $L >> $OUT/ab.jsonl || exit 1
timeout -k 10 300 python -u tools/regime_bench.py --configs cfg2 --regimes init --steps 100 --warmup 5 --tunings "ftab_mode=1" >> $OUT/ab.jsonl || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof_tk -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/regime_bench.py --configs cfg2 --regimes init --steps 100 --warmup 5 --tunings "ftab_mode=1" > $GRAFT_REPO_ROOT/$OUT/prof_tk.jsonl || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof_ho -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/regime_bench.py --configs cfg2 --regimes init --steps 100 --warmup 5 > $GRAFT_REPO_ROOT/$OUT/prof_ho.jsonl || exit 1
cd $GRAFT_REPO_ROOT
python3 - $OUT <<'PY'
import json, sys, glob, csv
for l in open(f"{sys.argv[1]}/ab.jsonl"):
    r = json.loads(l); print(r["cfg"], r["lib"], r["tuning"], round(r["us_per_sweep"], 2), r["fallbacks_per_sweep"]["exact_rescans"])
for t in ("prof_tk", "prof_ho"):
    for f in glob.glob(f"{sys.argv[1]}/{t}/**/*kernel_stats.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if "sweep" in row["Name"]:
                print(t, row["Name"][:60], row["Calls"], row["AverageNs"])
PY
