#!/bin/bash
# Round-2 GPU call 6: one-triangle kernel with 2 x 2 mirror transposes: sksy tests, C5 bench with
# the one-triangle sketch and with full storage (RBH_SKSY_FULL=1), kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_sksy.py "tests/test_gpu_workloads.py::test_c5_sksy_with_symmetry_check" tests/test_gpu_cpp_dropin.py -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_sksy.log 2>&1; rc=$?
echo "pytest sksy rc=$rc"; tail -n 3 gpurun_out/pytest_sksy.log
[ $rc -eq 0 ] || exit $rc
for v in tri full; do
    if [ $v = full ]; then export RBH_SKSY_FULL=1; fi
    timeout -k 10 300 python -u bench.py --config c5 --no-cpu-baseline > gpurun_out/bench_c5_$v.log 2>&1 || { echo "bench c5 $v failed"; tail gpurun_out/bench_c5_$v.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/bench_c5_$v.log').read().strip().splitlines()[-1]); print('$v', 'step', round(d['ms_per_step'],4), 'kernel', round(d['kernel_ms'],4), 'frac', round(d['roofline']['frac'],4))"
done
unset RBH_SKSY_FULL
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5 -o run --output-format csv -- python3 bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/rocprof_c5.log 2>&1 || { echo "rocprof failed"; tail gpurun_out/rocprof_c5.log; exit 1; }
f=$(find gpurun_out/prof_c5 -name "*kernel_stats.csv" | head -n 1); [ -n "$f" ] && cut -c1-160 "$f" | head -4
echo "=== all done"
