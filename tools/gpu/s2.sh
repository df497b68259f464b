#!/usr/bin/env bash
# round 4 session 2: cfg2/cfg5 per-wavefront timelines (stamps build)
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/s2
mkdir -p $O
timeout -k 10 240 python tools/timeline.py cfg2:init cfg5:init > $O/timeline.json 2> $O/timeline.err || { tail -20 $O/timeline.err; exit 1; }
python - <<'P'
import json
d=json.load(open('gpurun_out/s2/timeline.json'))
for k,v in d.items():
    r=v['runs'][-1]
    print(k, v["kernel"], {x:r[x] for x in r if x.startswith("m") or x in ("wave_life_us","waves","stamp_share")})
P
