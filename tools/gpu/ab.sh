#!/usr/bin/env bash
# A/B of library variants on regime chains: tools/gpu/ab.sh OUT CONFIGS REGIMES LIBS [STEPS]
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 500 python tools/regime_bench.py --configs $2 --regimes $3 --libs $4 --steps ${5:-100} > $O/ab.jsonl 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
python -c "
import json
for l in open('$O/ab.jsonl'):
    d=json.loads(l); f=d['fallbacks_per_sweep']
    print(d['cfg'], d['regime'], d['lib'], round(d['us_per_sweep'],2), 'keep', round(d['keep_motif'],4), {k:v for k,v in f.items() if v and k!='bg_path'})
"
