#!/bin/bash
# Round-2 GPU call 15: SASO DMA apply, rotating-loader flag ring (KC 64, 4 panels) vs lock-step
# 128/2: sparse parity under the ring shape, C3 bench and phase timing for both.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
RBH_SASO_KC=64 RBH_SASO_NBUF=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_sparse.py tests/test_gpu_sksp.py tests/test_gpu_spmm.py "tests/test_gpu_workloads.py::test_c3_saso_slices_bitwise" -x -q -rf --timeout 200 --timeout-method thread > gpurun_out/pytest_rot.log 2>&1; rc=$?
echo "pytest rot rc=$rc"; tail -n 2 gpurun_out/pytest_rot.log
[ $rc -eq 0 ] || exit $rc
for sh in 64_4 128_2; do
    export RBH_SASO_KC=${sh%_*} RBH_SASO_NBUF=${sh#*_}
    timeout -k 10 300 python -u bench.py --config c3 --no-cpu-baseline > gpurun_out/bench_c3_$sh.log 2>&1 || { echo "bench c3 $sh failed"; tail gpurun_out/bench_c3_$sh.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/bench_c3_$sh.log').read().strip().splitlines()[-1]); print('$sh', 'step', round(d['ms_per_step'],4), 'kernel', round(d['kernel_ms'],4), 'frac', round(d['roofline']['frac'],4))"
    RBH_LIB_PATH=$PWD/randblas_amd/_var/sdprof.so timeout -k 10 200 python -u tools/saso_prof.py > gpurun_out/sdprof_$sh.log 2>&1 || { echo "prof $sh failed"; tail gpurun_out/sdprof_$sh.log; exit 1; }
    tail -n 1 gpurun_out/sdprof_$sh.log
done
echo "=== all done"
