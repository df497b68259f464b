# A/B of live-kernel library variants at configs 3 (G = 4) and 4, init regime, then the
# PMC passes of the current library at config 3 G = 4.  Usage: TAG=x LIBS="a.so,b.so" bash tools/gpu/ab_live.sh
set -o pipefail
TAG=${TAG:-ablive}
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
export PYTHONUNBUFFERED=1
for rep in 1 2; do
timeout -k 10 300 python -u tools/regime_bench.py --configs cfg3 --regimes init --steps 30 --warmup 3 --libs "$LIBS" \
  --tunings "live_mode=1,live_G=4" >> $OUT/regime.jsonl 2>> $OUT/regime.err || { tail $OUT/regime.err; exit 1; }
timeout -k 10 300 python -u tools/regime_bench.py --configs cfg4 --regimes init --steps 30 --warmup 3 --libs "$LIBS" \
  >> $OUT/regime.jsonl 2>> $OUT/regime.err || { tail $OUT/regime.err; exit 1; }
done
python3 - $OUT/regime.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    r = json.loads(l); print(r["cfg"], r["lib"], r["tuning"], round(r["us_per_sweep"], 2), r["fallbacks_per_sweep"]["exact_rescans"])
PY
if [ -n "${PMC:-}" ]; then
KERNEL=gs_sweep_live_kernel TUNINGS="live_mode=1,live_G=4" SUFFIX=_live4 bash tools/pmc_regime.sh cfg3 init && \
mv gpurun_out/pmc_cfg3_init_live4 $OUT/ && cat $OUT/pmc_cfg3_init_live4/summary.txt
fi
