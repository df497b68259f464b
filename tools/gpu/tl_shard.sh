#!/usr/bin/env bash
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/tl_shard
mkdir -p $O
for wl in 8 1; do
GS_TL_LIB=libgibbs_hip_tl.so timeout -k 10 300 python tools/timeline_shard.py $wl > $O/w$wl.json 2> $O/w$wl.err || { tail -20 $O/w$wl.err; exit 1; }
python -c "
import json
d=json.load(open('$O/w$wl.json'))
r=d['runs'][-1]
print(d['world'], d['kernel'], {x:r[x] for x in r if x.startswith('m') or x in ('wave_life_us','waves','positions_match')})
"
done
