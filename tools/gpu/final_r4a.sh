#!/usr/bin/env bash
# Round-4 evidence, part 1: GPU tests, smoke, bench (1 GPU, plain and one-rank
# torchrun), rocprofv3 kernel stats of the bench (tools/gpu_round.sh, TAG r4final).
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
TAG=${TAG:-r4final} bash tools/gpu_round.sh || exit $?
echo final-a-ok
