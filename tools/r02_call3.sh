#!/bin/bash
# Round-2 GPU call 3: localise the pool-trim failure of the C++ client (workspace modes), then stress
# the f32 GPR-index-mode variants.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
g++ -std=c++17 -O2 -I include tests/cpp/test_dropin.cc -L randblas_amd -lrandblas_hip -Wl,-rpath,$PWD/randblas_amd -o /tmp/dropin || exit 1
for mode in pool legacy sync zero; do
    for rep in 1 2; do
        RBH_WS_MODE=$mode RBH_POOL_KEEP_BYTES=0 timeout -k 10 120 /tmp/dropin > gpurun_out/dropin_$mode$rep.log 2>&1; rc=$?
        echo "keep=0 ws_mode=$mode rep $rep: rc=$rc, $(grep -c FAILED gpurun_out/dropin_$mode$rep.log) failed checks"
        [ $rc -le 1 ] || exit $rc
    done
done
for v in 0 1 3 2; do
    RBH_SASO_F32_UNIT=1 RBH_LIB_PATH=$PWD/randblas_amd/_var/f32v$v.so DBG_BRIEF=1 DBG_REPS=12 \
        timeout -k 10 300 python -u tools/dbg_f32.py > gpurun_out/f32s_v$v.log 2>&1 || { echo "f32v$v rc=$?"; exit 1; }
    echo "f32 variant $v: $(grep -c ' 0 differ' gpurun_out/f32s_v$v.log) clean, $(grep differ gpurun_out/f32s_v$v.log | grep -vc ' 0 differ') with lost entries"
done
echo "=== all done"
