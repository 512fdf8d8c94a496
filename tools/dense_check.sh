#!/bin/bash
# Dense check on one GPU box: dense/sksy/workload parity, then the bench line of each config named
# in CONFIGS (default c1 c2).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_dense.py tests/test_gpu_sksy.py tests/test_gpu_workloads.py tests/test_gpu_cpp_dropin.py -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_dense.log 2>&1; rc=$?
echo "pytest dense rc=$rc $(tail -n 1 gpurun_out/pytest_dense.log)"
[ $rc -eq 0 ] || { tail -n 30 gpurun_out/pytest_dense.log; exit $rc; }
for c in ${CONFIGS:-c1 c2}; do
    timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline > gpurun_out/bench_$c.log 2>&1 || { echo "bench $c failed"; tail gpurun_out/bench_$c.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/bench_$c.log').read().strip().splitlines()[-1]); print('$c step', round(d['ms_per_step'],4), 'kernel', round(d['kernel_ms'],4), 'frac', round(d['roofline']['frac'],4))"
done
echo "=== all done"
