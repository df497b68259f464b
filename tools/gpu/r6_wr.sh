# Round 6: WRITE_SIZE / FETCH_SIZE passes (rocprofv3, kernel trace only, one counter a
# pass) of the shipped build for the configs given, init regime.  Per-dispatch values
# land in gpurun_out/$TAG/<cfg>/.
set -o pipefail
OUT=gpurun_out/${TAG:-r6wr}
for cfg in "$@"; do
  mkdir -p $OUT/$cfg
  for c in WRITE_SIZE FETCH_SIZE; do
    timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $c -d $OUT/$cfg/$c -o run --output-format csv -- python3 tools/regime_bench.py --configs $cfg --regimes init --steps 6 --warmup 2 > $OUT/$cfg/$c.log 2>&1 || exit 1
  done
done
python3 - $OUT "$@" <<'PY'
import csv, collections, sys
out = sys.argv[1]
for cfg in sys.argv[2:]:
    for c in ("WRITE_SIZE", "FETCH_SIZE"):
        per = collections.OrderedDict()
        for r in csv.DictReader(open(f"{out}/{cfg}/{c}/run_counter_collection.csv")):
            n = r["Kernel_Name"]
            if "sweep" not in n: continue
            key = (int(r["Dispatch_Id"]), n.split("(")[0][:48])
            per[key] = per.get(key, 0.0) + float(r["Counter_Value"])
        print(cfg, c, [(k[1], round(v)) for k, v in per.items()])
PY
