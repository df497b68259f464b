#!/usr/bin/env bash
# world-8 shard of config 4 (init regime): live-kernel lane counts / waves per workgroup
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/shard8
mkdir -p $O
timeout -k 10 400 python tools/shard_probe.py --config cfg4 --worlds 8 --steps 6 \
  --tunings ";live_G=1;live_G=2;live_G=4;live_G=8;live_G=2,live_waves=4;live_G=4,live_waves=4;live_G=2,live_waves=2;live_G=1,live_waves=4" \
  > $O/probe.jsonl 2> $O/probe.err || { tail -20 $O/probe.err; exit 1; }
python -c "
import json
for l in open('$O/probe.jsonl'):
    d=json.loads(l); print(d['world'], d['tuning'], round(d['us_per_sweep_kernel'],1), d['positions_match_whole_sampler'], d['keep_motif'])
"
