#!/usr/bin/env bash
# live-kernel parity tests, then config 4 A/B and the world-8 shard
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/live_check
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_dna.py tests/test_gpu_long.py tests/test_gpu_fullsize_sweep.py tests/test_gpu_bg.py tests/test_gpu_dist_gloo.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
