#!/bin/bash
# Round-2 GPU call 13: SASO loader + walkers kernel (section 5b): sparse parity, C3 bench vs the
# lock-step kernel (RBH_SASO_LDR=0), phase timing.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_sparse.py tests/test_gpu_sksp.py tests/test_gpu_spmm.py "tests/test_gpu_workloads.py::test_c3_saso_slices_bitwise" -x -q -rf --timeout 200 --timeout-method thread > gpurun_out/pytest_ldr.log 2>&1; rc=$?
echo "pytest ldr rc=$rc"; tail -n 3 gpurun_out/pytest_ldr.log
[ $rc -eq 0 ] || exit $rc
for v in 1 0; do
    RBH_SASO_LDR=$v timeout -k 10 300 python -u bench.py --config c3 --no-cpu-baseline > gpurun_out/bench_c3_ldr$v.log 2>&1 || { echo "bench c3 ldr$v failed"; tail gpurun_out/bench_c3_ldr$v.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/bench_c3_ldr$v.log').read().strip().splitlines()[-1]); print('ldr$v', 'step', round(d['ms_per_step'],4), 'kernel', round(d['kernel_ms'],4), 'frac', round(d['roofline']['frac'],4))"
done
RBH_LIB_PATH=$PWD/randblas_amd/_var/sdprof.so timeout -k 10 200 python -u tools/saso_prof.py > gpurun_out/sdprof_ldr.log 2>&1 || { echo "prof failed"; tail gpurun_out/sdprof_ldr.log; exit 1; }
tail -n 2 gpurun_out/sdprof_ldr.log
echo "=== all done"
