#!/bin/bash
# Round-2 GPU call 12: SASO DMA apply, lock-step ring with 2/3/4 panels (copies after the walk for
# 3 and 4), product vs one-M0 variant: parity per shape, C3 bench and phase timing.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
V=$PWD/randblas_amd/_var
for sh in 128_2 64_3 64_4; do
    export RBH_SASO_KC=${sh%_*} RBH_SASO_NBUF=${sh#*_}
    for v in product m0; do
        lib=$PWD/randblas_amd/librandblas_hip.so; [ $v = product ] || lib=$V/$v.so
        RBH_LIB_PATH=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_sparse.py "tests/test_gpu_workloads.py::test_c3_saso_slices_bitwise" -x -q -rf --timeout 200 --timeout-method thread > gpurun_out/pytest_${sh}_$v.log 2>&1; rc=$?
        echo "pytest $sh $v rc=$rc $(tail -n 1 gpurun_out/pytest_${sh}_$v.log)"
        [ $rc -eq 0 ] || exit $rc
        RBH_LIB_PATH=$lib timeout -k 10 300 python -u bench.py --config c3 --no-cpu-baseline > gpurun_out/bench_c3_${sh}_$v.log 2>&1 || { echo "bench c3 $sh $v failed"; tail gpurun_out/bench_c3_${sh}_$v.log; exit 1; }
        python3 -c "import json; d=json.loads(open('gpurun_out/bench_c3_${sh}_$v.log').read().strip().splitlines()[-1]); print('$sh $v', 'step', round(d['ms_per_step'],4), 'kernel', round(d['kernel_ms'],4), 'frac', round(d['roofline']['frac'],4))"
    done
    RBH_LIB_PATH=$V/m0prof.so timeout -k 10 200 python -u tools/saso_prof.py > gpurun_out/sdprof_${sh}_m0.log 2>&1 || { echo "prof $sh failed"; tail gpurun_out/sdprof_${sh}_m0.log; exit 1; }
    tail -n 1 gpurun_out/sdprof_${sh}_m0.log
done
echo "=== all done"
