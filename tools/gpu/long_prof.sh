# Long-kernel profile at config 3 (init regime): the timeline variant's per-wave marks
# (first iteration's phases), then the PMC passes.  Usage: TAG=x bash tools/gpu/long_prof.sh
set -o pipefail
TAG=${TAG:-longprof}
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
export PYTHONUNBUFFERED=1
TL_TUNING="dna_mode=1,long_mode=1" GS_TL_LIB=libgibbs_hip_tl.so timeout -k 10 200 python -u tools/timeline.py cfg3:init > $OUT/timeline.json 2> $OUT/timeline.err || { tail $OUT/timeline.err; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/timeline.json'))
for k,v in d.items():
    r=v['runs'][-1] if isinstance(v,dict) and 'runs' in v else v
    print(k, json.dumps(r)[:1500])
"
KERNEL=gs_sweep_long_kernel TUNINGS="dna_mode=1,long_mode=1" SUFFIX=_long bash tools/pmc_regime.sh cfg3 init && \
mv gpurun_out/pmc_cfg3_init_long $OUT/ && cat $OUT/pmc_cfg3_init_long/summary.txt
