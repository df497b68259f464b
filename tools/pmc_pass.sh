#!/bin/bash
# One rocprofv3 PMC pass over the regime bench (one config, initialiser regime).
# usage: tools/pmc_pass.sh <outdir> <config> <kernel regex> <counters...>
out=$1; cfg=$2; rx=$3; shift 3
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-include-regex "$rx" --output-format csv \
    -d "$GRAFT_REPO_ROOT/gpurun_out/$out" -o pmc -- \
    python3 "$GRAFT_REPO_ROOT/tools/regime_bench.py" --configs "$cfg" --regimes init --steps 10 --warmup 2
