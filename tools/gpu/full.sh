#!/usr/bin/env bash
# full GPU test suite into gpurun_out/$1/
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/${1:-full}
mkdir -p $O
timeout -k 10 540 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
