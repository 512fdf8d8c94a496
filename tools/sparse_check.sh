#!/bin/bash
# Sparse-data check: sketch_sparse / spmm / SASO parity, then the sketch_sparse timing probe.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_sksp.py tests/test_gpu_spmm.py tests/test_gpu_sparse.py tests/test_gpu_vector.py tests/test_gpu_cpp_dropin.py -x -q -rf --timeout 200 --timeout-method thread > gpurun_out/pytest_sparse.log 2>&1; rc=$?
echo "pytest sparse rc=$rc $(tail -n 1 gpurun_out/pytest_sparse.log)"
[ $rc -eq 0 ] || { tail -n 30 gpurun_out/pytest_sparse.log; exit $rc; }
timeout -k 10 200 python -u tools/sksp_probe.py || exit 1
echo "=== all done"
