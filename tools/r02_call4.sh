#!/bin/bash
# Round-2 GPU call 4: pool-alias probe (host-side overlap check only), the one-triangle sksy tests,
# C5 bench + kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 ./tools/micro/pool_alias 40 0 > gpurun_out/pool_alias0.log 2>&1; echo "pool_alias keep=0 rc=$?"; tail -n 12 gpurun_out/pool_alias0.log
timeout -k 10 120 ./tools/micro/pool_alias 40 18446744073709551615 > gpurun_out/pool_alias_max.log 2>&1; echo "pool_alias keep=max rc=$?"; tail -n 3 gpurun_out/pool_alias_max.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_sksy.py tests/test_gpu_cpp_dropin.py "tests/test_gpu_workloads.py::test_c5_sksy_with_symmetry_check" -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_sksy.log 2>&1; rc=$?
echo "pytest sksy rc=$rc"; tail -n 15 gpurun_out/pytest_sksy.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config c5 > gpurun_out/bench_c5.log 2>&1 || { echo "bench c5 failed"; tail gpurun_out/bench_c5.log; exit 1; }
tail -n 1 gpurun_out/bench_c5.log | cut -c1-700
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5 -o run --output-format csv -- python3 bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/rocprof_c5.log 2>&1 || { echo "rocprof failed"; tail gpurun_out/rocprof_c5.log; exit 1; }
f=$(find gpurun_out/prof_c5 -name "*kernel_stats.csv" | head -n 1); [ -n "$f" ] && cut -c1-200 "$f" | head -8
echo "=== all done"
