#!/bin/bash
# Round-2 GPU call 17: SASO lock-step apply with an L2 prefetch of panel ch + 2 (variant l2pf):
# parity, C3 kernel time vs product, copies-only ablation, phase timing.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
V=$PWD/randblas_amd/_var
RBH_LIB_PATH=$V/l2pf.so timeout -k 10 300 python -u -m pytest tests/test_gpu_sparse.py "tests/test_gpu_workloads.py::test_c3_saso_slices_bitwise" -x -q -rf --timeout 200 --timeout-method thread > gpurun_out/pytest_l2pf.log 2>&1; rc=$?
echo "pytest l2pf rc=$rc $(tail -n 1 gpurun_out/pytest_l2pf.log)"
[ $rc -eq 0 ] || exit $rc
for v in product l2pf; do
    lib=$PWD/randblas_amd/librandblas_hip.so; [ $v = product ] || lib=$V/$v.so
    for a in 0 1; do
        RBH_SASO_ABLATE=$a RBH_LIB_PATH=$lib timeout -k 10 300 python -u bench.py --config c3 --no-cpu-baseline > gpurun_out/bench_c3_${v}_a$a.log 2>&1 || { echo "bench $v $a failed"; tail gpurun_out/bench_c3_${v}_a$a.log; exit 1; }
        python3 -c "import json; d=json.loads(open('gpurun_out/bench_c3_${v}_a$a.log').read().strip().splitlines()[-1]); print('$v ablate=$a', 'kernel', round(d['kernel_ms'],4), 'step', round(d['ms_per_step'],4))"
    done
done
RBH_LIB_PATH=$V/l2pfprof.so timeout -k 10 200 python -u tools/saso_prof.py > gpurun_out/sdprof_l2pf.log 2>&1 || { echo "prof failed"; tail gpurun_out/sdprof_l2pf.log; exit 1; }
tail -n 1 gpurun_out/sdprof_l2pf.log
echo "=== all done"
