#!/bin/bash
# Round-2 GPU call 14: SASO DMA apply, record-window wait after the copies (variant late) vs product.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
V=$PWD/randblas_amd/_var
RBH_LIB_PATH=$V/late.so timeout -k 10 300 python -u -m pytest tests/test_gpu_sparse.py "tests/test_gpu_workloads.py::test_c3_saso_slices_bitwise" -x -q -rf --timeout 200 --timeout-method thread > gpurun_out/pytest_late.log 2>&1; rc=$?
echo "pytest late rc=$rc"; tail -n 2 gpurun_out/pytest_late.log
[ $rc -eq 0 ] || exit $rc
for v in product late; do
    lib=$PWD/randblas_amd/librandblas_hip.so; [ $v = product ] || lib=$V/$v.so
    RBH_LIB_PATH=$lib timeout -k 10 300 python -u bench.py --config c3 --no-cpu-baseline > gpurun_out/bench_c3_$v.log 2>&1 || { echo "bench c3 $v failed"; tail gpurun_out/bench_c3_$v.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/bench_c3_$v.log').read().strip().splitlines()[-1]); print('$v', 'step', round(d['ms_per_step'],4), 'kernel', round(d['kernel_ms'],4), 'frac', round(d['roofline']['frac'],4))"
done
for v in sdprof lateprof; do
    RBH_LIB_PATH=$V/$v.so timeout -k 10 200 python -u tools/saso_prof.py > gpurun_out/sdprof_$v.log 2>&1 || { echo "prof $v failed"; tail gpurun_out/sdprof_$v.log; exit 1; }
    echo $v; tail -n 2 gpurun_out/sdprof_$v.log
done
echo "=== all done"
