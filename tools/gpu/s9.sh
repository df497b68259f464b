#!/usr/bin/env bash
# round 4, final sources: the four-symbol kernel's and the multi-rank parity tests
# (empty shard included), the driver's 20-step bench line, then the calibration and
# PMC records (tools/gpu/final_r4b.sh)
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/s9
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_ek4.py tests/test_gpu_dist_gloo.py tests/test_gpu_dist.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash tools/gpu/s7.sh || exit 1
bash tools/gpu/final_r4b.sh || exit 1
