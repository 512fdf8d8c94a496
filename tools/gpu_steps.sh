#!/bin/bash
# Run named GPU steps on the box, each under its own time limit; stop at the first failure.
# Usage (repo root, via gpurun): bash tools/gpu_steps.sh "<name>|<timeout>|<command>" ...
# Each step's output goes to gpurun_out/<name>.log; its tail is echoed.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for spec in "$@"; do
    name="${spec%%|*}"; rest="${spec#*|}"
    tmo="${rest%%|*}"; cmd="${rest#*|}"
    echo "=== $(date +%T) $name ($tmo s): $cmd"
    timeout -k 10 "$tmo" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
    rc=$?
    echo "=== $name rc=$rc"
    tail -n 4 "gpurun_out/$name.log" | cut -c1-1500
    if [ $rc -ne 0 ]; then echo "stopping at $name (rc=$rc)"; exit $rc; fi
done
echo "=== all done"
