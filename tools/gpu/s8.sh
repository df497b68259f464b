#!/usr/bin/env bash
# round 4: the four-symbol kernel's parity tests, then the driver's 20-step bench line
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/s8
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_ek4.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
bash tools/gpu/s7.sh
