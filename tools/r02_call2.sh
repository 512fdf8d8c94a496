#!/bin/bash
# Round-2 GPU call 2: the pool-trim reproducer, the C++ client under pool trimming (diagnostic
# prints), the f32 GPR-index-mode variants, and a first bench pass.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 180 ./tools/micro/pool_trim 100 > gpurun_out/pool_trim.log 2>&1; rc=$?
echo "pool_trim rc=$rc"; cat gpurun_out/pool_trim.log
[ $rc -le 1 ] || exit $rc
g++ -std=c++17 -O2 -I include tests/cpp/test_dropin.cc -L randblas_amd -lrandblas_hip -Wl,-rpath,$PWD/randblas_amd -o /tmp/dropin || exit 1
RBH_DIAG=1 RBH_POOL_KEEP_BYTES=0 timeout -k 10 120 /tmp/dropin > gpurun_out/dropin_trim.log 2>&1; rc=$?
echo "dropin keep=0 rc=$rc: $(grep -c FAILED gpurun_out/dropin_trim.log) failed checks"; grep diag gpurun_out/dropin_trim.log
[ $rc -le 1 ] || exit $rc
RBH_DIAG=1 timeout -k 10 120 /tmp/dropin > gpurun_out/dropin_keep.log 2>&1; rc=$?
echo "dropin keep=default rc=$rc: $(tail -n 1 gpurun_out/dropin_keep.log)"
[ $rc -le 1 ] || exit $rc
for v in 0 1 2 3; do
    RBH_SASO_F32_UNIT=1 RBH_LIB_PATH=$PWD/randblas_amd/_var/f32v$v.so DBG_BRIEF=1 DBG_REPS=3 \
        timeout -k 10 200 python -u tools/dbg_f32.py > gpurun_out/f32v$v.log 2>&1 || { echo "f32v$v rc=$?"; exit 1; }
    echo "f32 variant $v: $(grep -c ' 0 differ' gpurun_out/f32v$v.log) clean, $(grep differ gpurun_out/f32v$v.log | grep -vc ' 0 differ') with lost entries"
done
for c in c2 c1 c3 c5; do
    timeout -k 10 300 python -u bench.py --config $c > gpurun_out/bench_$c.log 2>&1 || { echo "bench $c rc=$?"; tail -5 gpurun_out/bench_$c.log; exit 1; }
    tail -n 1 gpurun_out/bench_$c.log | cut -c1-400
done
echo "=== all done"
