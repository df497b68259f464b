#!/bin/bash
# Run GPU steps in order; stop at the first one that faults, aborts, segfaults or
# times out (exit 124/134/137/139 or > 128), continue past ordinary test failures.
# usage: tools/gpu_step.sh "<timeout s>|<log>|<cmd>" ...
mkdir -p gpurun_out
for step in "$@"; do
    t="${step%%|*}"; rest="${step#*|}"; log="${rest%%|*}"; cmd="${rest#*|}"
    echo "[step] $cmd -> $log"
    timeout -k 10 "$t" bash -c "$cmd" > "gpurun_out/$log" 2>&1
    rc=$?
    echo "[step] rc=$rc"
    tail -3 "gpurun_out/$log"
    if [ $rc -ge 124 ]; then echo "[step] stopping after rc=$rc"; exit $rc; fi
done
exit 0
