#!/bin/bash
# Round-2 GPU call 7: SASO LDS-DMA kernel with a runtime chunk depth / panel ring. Sparse parity
# tests under the default shape (KC 64, 4 panels), then C3 under each shape.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_sparse.py tests/test_gpu_sksp.py tests/test_gpu_spmm.py "tests/test_gpu_workloads.py::test_c3_saso_slices_bitwise" -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_sparse.log 2>&1; rc=$?
echo "pytest sparse rc=$rc"; tail -n 3 gpurun_out/pytest_sparse.log
[ $rc -eq 0 ] || exit $rc
for sh in 64_4 64_2 128_2; do
    export RBH_SASO_KC=${sh%_*} RBH_SASO_NBUF=${sh#*_}
    if [ $sh != 64_4 ]; then
        timeout -k 10 300 python -u -m pytest "tests/test_gpu_workloads.py::test_c3_saso_slices_bitwise" -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_c3_$sh.log 2>&1 || { echo "c3 test $sh failed"; tail gpurun_out/pytest_c3_$sh.log; exit 1; }
    fi
    timeout -k 10 300 python -u bench.py --config c3 --no-cpu-baseline > gpurun_out/bench_c3_$sh.log 2>&1 || { echo "bench c3 $sh failed"; tail gpurun_out/bench_c3_$sh.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/bench_c3_$sh.log').read().strip().splitlines()[-1]); print('$sh', 'step', round(d['ms_per_step'],4), 'kernel', round(d['kernel_ms'],4), 'frac', round(d['roofline']['frac'],4))"
done
echo "=== all done"
