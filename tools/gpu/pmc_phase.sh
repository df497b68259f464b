# Instruction counts per phase variant (GS_EXP libraries) of the live kernel, one config.
# Usage: TAG=x LIBS=a.so,b.so CFG=cfg4 bash tools/gpu/pmc_phase.sh
set -o pipefail
TAG=${TAG:-pmcphase}
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for lib in $(echo $LIBS | tr ',' ' '); do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $OUT/$lib -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/phase_exp.py --configs ${CFG:-cfg4} --libs $lib --reps 3 > $OUT/$lib.log 2>&1 || exit $?
done
python3 - $OUT <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
for d in sorted(glob.glob(out + "/*.so")):
    f = glob.glob(d + "/**/*counter_collection.csv", recursive=True)
    if not f: continue
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f[0])):
        if "sweep_live" in r["Kernel_Name"]:
            per[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    ids = sorted(per)[1:]  # drop the first launch
    avg = {k: sum(per[i][k] for i in ids) / len(ids) for k in per[ids[0]]} if ids else {}
    print(d.split("/")[-1], {k: round(v / 1e6, 3) for k, v in sorted(avg.items())})
PY
