#!/usr/bin/env bash
# round 4: the driver's 20-step bench line (host clock vs the region's events), three runs
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/s7
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-side --no-cpu-baseline > $O/bench20_$i.json 2> $O/bench20_$i.err || { tail -20 $O/bench20_$i.err; exit 1; }
done
python -c "
import json
for i in (1,2,3):
    d=json.load(open('$O/bench20_%d.json' % i)); r=d['roofline']
    print(i, round(d['ms_per_step']*1e3,2), round(r['kernel_ms']*1e3,2), round(d['ms_per_step']/r['kernel_ms'],3), r['traffic'], r['frac'])
"
