# Round 6: cfg5 with odd prefix-sum chunks (H = 1): LDS conflicts (one PMC pass a
# library) and the A/B timing, then the protein parity tests.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/h1q
mkdir -p $OUT
for lib in libgibbs_hip.so libgibbs_hip_prev.so; do
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT \
    -d $OUT/$lib -o run --output-format csv -- python3 tools/regime_bench.py --configs cfg5 --regimes init --steps 10 --warmup 2 \
    --libs gibbssampling_amd/$lib > $OUT/$lib.log 2>&1 || exit $?
done
python3 - <<'PY'
import csv, collections
for lib in ("libgibbs_hip.so", "libgibbs_hip_prev.so"):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(f"gpurun_out/h1q/{lib}/run_counter_collection.csv")):
        if "gs_sweep_kernel<20, 1, 32" in r["Kernel_Name"]:
            d[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(lib, {k: f"{sum(v[2:]) / max(1, len(v) - 2):.3g}" for k, v in d.items()})
PY
TAG=h1q TESTS='tests/test_gpu_kdyn.py tests/test_gpu_fullsize_sweep.py' CFGS=cfg5 LIBS=gibbssampling_amd/libgibbs_hip.so,gibbssampling_amd/libgibbs_hip_prev.so REPS=3 bash tools/gpu/r6.sh
