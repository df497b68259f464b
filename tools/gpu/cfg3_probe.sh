# Config 3 (100k x 500, W = 15, init regime) on the packed-layout kernels: sweep times by
# kernel and lane count, then PMC passes of the live kernel at G = 4 and the DNA kernel.
# Usage: TAG=x bash tools/gpu/cfg3_probe.sh
set -o pipefail
TAG=${TAG:-cfg3}
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u tools/regime_bench.py --configs cfg3 --regimes init --steps 20 --warmup 3 \
  --tunings "live_mode=0;live_mode=0,dna_G=2;live_mode=0,dna_G=4;live_mode=1,live_G=2;live_mode=1,live_G=4;live_mode=1,live_G=8" \
  > $OUT/regime.jsonl 2> $OUT/regime.err || { tail $OUT/regime.err; exit 1; }
cut -c1-300 $OUT/regime.jsonl
KERNEL=gs_sweep_live_kernel TUNINGS="live_mode=1,live_G=4" SUFFIX=_live4 bash tools/pmc_regime.sh cfg3 init && \
KERNEL=gs_sweep_dna_kernel TUNINGS="live_mode=0" SUFFIX=_dna bash tools/pmc_regime.sh cfg3 init && \
mv gpurun_out/pmc_cfg3_init_live4 gpurun_out/pmc_cfg3_init_dna $OUT/ && cat $OUT/pmc_*/summary.txt
timeout -k 10 200 python -u tools/stamps_dna.py cfg3 > $OUT/stamps_dna.json 2> $OUT/stamps_dna.err && cat $OUT/stamps_dna.json && \
LIVE_G=4 timeout -k 10 200 python -u tools/stamps_live.py cfg3 > $OUT/stamps_live4.json 2> $OUT/stamps_live4.err && cat $OUT/stamps_live4.json
