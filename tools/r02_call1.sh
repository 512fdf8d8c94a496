#!/bin/bash
# Round-2 GPU call 1: parity tests (new workload-scale, spmm, drop-in cases), pool-trim stress of the
# C++ client, the f32 GPR-index-mode variants, and a first bench pass. Every GPU step has its own
# time limit; the first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {   # step <log> <timeout> <cmd...>
    local logf="$1" tmo="$2"; shift 2
    echo "=== $(date +%T) $logf"
    timeout -k 10 "$tmo" "$@" > "gpurun_out/$logf" 2>&1
    local rc=$?
    echo "=== $logf rc=$rc"; tail -n 4 "gpurun_out/$logf" | cut -c1-600
    [ $rc -eq 0 ] || { echo "stopping at $logf"; exit $rc; }
}
step pytest_gpu.log 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread
# pool trimming on every sync (the library pool's release threshold 0): the C++ client, 8 runs
g++ -std=c++17 -O2 -I include tests/cpp/test_dropin.cc -L randblas_amd -lrandblas_hip -Wl,-rpath,$PWD/randblas_amd -o /tmp/dropin
for i in 1 2 3 4 5 6 7 8; do
    RBH_POOL_KEEP_BYTES=0 timeout -k 10 120 /tmp/dropin > gpurun_out/dropin_trim_$i.log 2>&1 || { echo "dropin trim run $i failed"; tail -5 gpurun_out/dropin_trim_$i.log; exit 1; }
done
echo "dropin with pool trimming: 8/8 passed"
for v in 0 1 2 3; do
    RBH_SASO_F32_UNIT=1 RBH_LIB_PATH=$PWD/randblas_amd/_var/f32v$v.so DBG_BRIEF=1 DBG_REPS=3 \
        timeout -k 10 200 python -u tools/dbg_f32.py > gpurun_out/f32v$v.log 2>&1 || { echo "f32v$v rc=$?"; exit 1; }
    echo "f32 variant $v: $(grep -c ' 0 differ' gpurun_out/f32v$v.log) clean, $(grep differ gpurun_out/f32v$v.log | grep -vc ' 0 differ') with lost entries"
done
for c in c2 c1 c3 c5; do
    step bench_$c.log 300 python -u bench.py --config $c
done
echo "=== all done"
