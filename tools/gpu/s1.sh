#!/usr/bin/env bash
# round 4 session 1: GPU tests, overhead probe, timelines, the driver's bench line
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/s1
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 120 python tools/overhead_probe.py > $O/overhead.json 2> $O/overhead.err || exit 1
cat $O/overhead.json
timeout -k 10 180 python tools/timeline.py cfg2:init cfg5:init cfg2:uniform > $O/timeline.json 2> $O/timeline.err || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err || exit 1
python -c "import json;d=json.load(open('$O/bench20.json'));print(d['ms_per_step'], d['roofline']['kernel_ms'])"
