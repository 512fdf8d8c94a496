#!/bin/bash
# Index-mode stress of saso_unit_kernel: f32 sampled operators at d=1000, n=130, m=2048, both
# layouts, DBG_REPS repetitions; prints per-run mismatch counts (tools/dbg_f32.py).
cd "${GRAFT_REPO_ROOT:-$(pwd)}" && export TMPDIR=/tmp && mkdir -p gpurun_out
DBG_SAMPLED=1 DBG_F32_ONLY=1 DBG_REPS=${DBG_REPS:-40} timeout -k 10 500 python -u tools/dbg_f32.py > gpurun_out/f32sampled.log 2>&1; rc=$?
echo "f32 sampled unit rc=$rc runs=$(grep -c differ gpurun_out/f32sampled.log) clean=$(grep -c ' 0 differ' gpurun_out/f32sampled.log)"
grep -v ' 0 differ' gpurun_out/f32sampled.log | head -40
exit $rc
