# Kernel-argument placement A/B: HIP_FORCE_DEV_KERNARG unset / 1 / 0, config 2 and 3
# init-regime sweeps and the bench line (each run its own process).
set -o pipefail
OUT=gpurun_out/kernarg
mkdir -p $OUT
export PYTHONUNBUFFERED=1
for rep in 1 2; do
for v in unset 1 0; do
  if [ $v = unset ]; then E=""; else E="HIP_FORCE_DEV_KERNARG=$v"; fi
  env $E timeout -k 10 200 python -u tools/regime_bench.py --configs cfg2,cfg3 --regimes init --steps 100 --warmup 5 > $OUT/rb_$v.jsonl || exit 1
  env $E timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 > $OUT/bench_$v.json 2> $OUT/bench_$v.err || exit 1
  python3 - $OUT $v <<'PY'
import json, sys
o, v = sys.argv[1], sys.argv[2]
for l in open(f"{o}/rb_{v}.jsonl"):
    r = json.loads(l); print("kernarg", v, r["cfg"], round(r["us_per_sweep"], 2))
b = json.loads(open(f"{o}/bench_{v}.json").read().strip().splitlines()[-1])
print("kernarg", v, "bench", b["ms_per_step"] * 1000, b["roofline"]["achieved"])
PY
done
done
