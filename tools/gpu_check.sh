#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprof kernel-trace summary.
# Every GPU step runs under its own time limit; a crash/fault/timeout ends the script.
# Usage (from the repo root, via gpurun): bash tools/gpu_check.sh [tests|bench|prof|all] [bench args...]
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
what="${1:-all}"
shift || true

step() {   # step <name> <timeout-seconds> <cmd...>; stops the script on crash / timeout
    local name="$1" tmo="$2"
    shift 2
    echo "=== $name: $*" | tee -a gpurun_out/steps.log
    timeout -k 10 "$tmo" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc" | tee -a gpurun_out/steps.log
    tail -n 30 "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
        echo "stopping: $name ended with rc=$rc" | tee -a gpurun_out/steps.log
        exit $rc
    fi
    return 0
}

if [ "$what" = "tests" ] || [ "$what" = "all" ]; then
    step pytest_gpu 900 python -m pytest tests -m gpu -q -rf
    step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [ "$what" = "bench" ] || [ "$what" = "all" ]; then
    step bench 600 python bench.py "$@"
fi
if [ "$what" = "prof" ] || [ "$what" = "all" ]; then
    export TMPDIR=/tmp
    step rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
        python bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@"
    find gpurun_out/prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/kernel_stats.csv \; 2>/dev/null
    [ -f gpurun_out/kernel_stats.csv ] && cat gpurun_out/kernel_stats.csv | cut -c1-220
fi
exit 0
