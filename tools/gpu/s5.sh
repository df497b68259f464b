#!/usr/bin/env bash
# round 4 session 3: config 2 init prologue timeline (TLP marks) and the sweep kernel's
# PMC passes for the current library
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/s5
mkdir -p $O
GS_TL_LIB=libgibbs_hip_tlp.so timeout -k 10 240 python tools/timeline.py cfg2:init > $O/timeline_pro.json 2> $O/timeline.err || { tail -20 $O/timeline.err; exit 1; }
python - <<'P'
import json
d=json.load(open('gpurun_out/s5/timeline_pro.json'))
for k,v in d.items():
    for r in v['runs'][-1:]:
        print(k, {x:r[x] for x in r if x.startswith("m") or x in ("wave_life_us",)})
P
KERNEL=gs_sweep_kernel bash tools/pmc_regime.sh cfg2 init || exit 1
cat gpurun_out/pmc_cfg2_init/summary.txt
