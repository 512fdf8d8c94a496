#!/bin/bash
# Round-2 GPU call 5: pool-growth probe, sksy tests with the rewritten check kernel, C5 bench +
# kernel trace + FETCH/WRITE counters.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 ./tools/micro/pool_grow 0 > gpurun_out/pool_grow0.log 2>&1; echo "pool_grow keep=0 rc=$?"; tail -n 8 gpurun_out/pool_grow0.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_sksy.py "tests/test_gpu_workloads.py::test_c5_sksy_with_symmetry_check" -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_sksy.log 2>&1; rc=$?
echo "pytest sksy rc=$rc"; tail -n 3 gpurun_out/pytest_sksy.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config c5 > gpurun_out/bench_c5.log 2>&1 || { echo "bench c5 failed"; tail gpurun_out/bench_c5.log; exit 1; }
tail -n 1 gpurun_out/bench_c5.log | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5 -o run --output-format csv -- python3 bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/rocprof_c5.log 2>&1 || { echo "rocprof failed"; tail gpurun_out/rocprof_c5.log; exit 1; }
f=$(find gpurun_out/prof_c5 -name "*kernel_stats.csv" | head -n 1); [ -n "$f" ] && cut -c1-160 "$f" | head -5
for pc in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $pc --kernel-trace -d gpurun_out/pmc_c5/$pc -o run --output-format csv -- python3 bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_c5_$pc.log 2>&1 || { echo "pmc $pc failed"; exit 1; }
done
mkdir -p gpurun_out/pmc_c5s && cp -r gpurun_out/pmc_c5/FETCH_SIZE gpurun_out/pmc_c5s/p0 && cp -r gpurun_out/pmc_c5/WRITE_SIZE gpurun_out/pmc_c5s/p1
python3 tools/pmc_summary.py gpurun_out/pmc_c5s > gpurun_out/c5_pmc.json && grep -A3 -E "wide|symcheck" gpurun_out/c5_pmc.json | grep -E "wide|symcheck|hbm_bytes|FETCH|WRITE" | head -12
echo "=== all done"
