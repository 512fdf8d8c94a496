#!/bin/bash
# SASO check on one GPU box: sparse parity (all sparse suites), C3 bench,
# phase timing.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_sparse.py tests/test_gpu_sksp.py tests/test_gpu_spmm.py tests/test_gpu_vector.py "tests/test_gpu_workloads.py::test_c3_saso_slices_bitwise" -x -q -rf --timeout 200 --timeout-method thread > gpurun_out/pytest_sparse.log 2>&1; rc=$?
echo "pytest sparse rc=$rc $(tail -n 1 gpurun_out/pytest_sparse.log)"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config c3 --no-cpu-baseline > gpurun_out/bench_c3.log 2>&1 || { echo "bench c3 failed"; tail gpurun_out/bench_c3.log; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/bench_c3.log').read().strip().splitlines()[-1]); print('c3 step', round(d['ms_per_step'],4), 'kernel', round(d['kernel_ms'],4), 'frac', round(d['roofline']['frac'],4))"
RBH_LIB_PATH=$PWD/randblas_amd/_var/sdprof.so timeout -k 10 200 python -u tools/saso_prof.py > gpurun_out/sdprof.log 2>&1 || { echo "prof failed"; tail gpurun_out/sdprof.log; exit 1; }
tail -n 2 gpurun_out/sdprof.log
echo "=== all done"
