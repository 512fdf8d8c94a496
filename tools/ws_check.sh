#!/bin/bash
# Workspace-arena check: the whole GPU suite, the host submit probe, C3 and C1 bench lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest gpu rc=$rc $(tail -n 1 gpurun_out/pytest_gpu.log)"
[ $rc -eq 0 ] || { tail -n 30 gpurun_out/pytest_gpu.log; exit $rc; }
timeout -k 10 200 python -u tools/submit_probe.py 50 || exit 1
for c in c3 c1; do
    timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline > gpurun_out/bench_$c.log 2>&1 || { echo "bench $c failed"; tail gpurun_out/bench_$c.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/bench_$c.log').read().strip().splitlines()[-1]); print('$c step', round(d['ms_per_step'],4), 'kernel', round(d['kernel_ms'],4), 'frac', round(d['roofline']['frac'],4))"
done
echo "=== all done"
