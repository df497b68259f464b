#!/usr/bin/env bash
# round 4: fixed-point motif scan — parity subset, then cfg2/cfg5 init timing + rescans
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/s3
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize_sweep.py tests/test_golden.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 python tools/regime_bench.py --configs cfg2,cfg5 --regimes init,uniform --steps 100 > $O/regime.jsonl 2> $O/regime.err || { tail -20 $O/regime.err; exit 1; }
python -c "
import json
for l in open('$O/regime.jsonl'):
    d=json.loads(l); f=d['fallbacks_per_sweep']
    print(d['cfg'], d['regime'], round(d['us_per_sweep'],2), 'keep', d['keep_motif'], {k:v for k,v in f.items() if v})
"
