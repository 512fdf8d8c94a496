#!/bin/bash
# GPR-index-mode stress of saso_unit_kernel (tools/dbg_f32.py): f64 user arrays with +-1 values at the
# shape where the f32 instantiation lost panel rows (d=1000, n=130, m=2048), then f32 (opt-in route).
cd "${GRAFT_REPO_ROOT:-$(pwd)}" && export TMPDIR=/tmp && mkdir -p gpurun_out
DBG_F64_UNIT=1 DBG_BRIEF=1 DBG_REPS=40 timeout -k 10 500 python -u tools/dbg_f32.py > gpurun_out/f64unit.log 2>&1; rc=$?
echo "f64 unit rc=$rc runs=$(grep -c differ gpurun_out/f64unit.log) clean=$(grep -c ' 0 differ' gpurun_out/f64unit.log)"
exit $rc
