#!/bin/bash
# f32 sampled SASO through saso_unit_kernel (RBH_SASO_F32_UNIT=1) at the shape that lost panel rows
# in round 2 (d=1000, n=130, m=2048, both layouts), DBG_REPS repetitions; prints per-run mismatch counts.
cd "${GRAFT_REPO_ROOT:-$(pwd)}" && export TMPDIR=/tmp && mkdir -p gpurun_out
RBH_SASO_F32_UNIT=1 DBG_SAMPLED=1 DBG_F32_ONLY=1 DBG_REPS=${DBG_REPS:-40} timeout -k 10 500 python -u tools/dbg_f32.py > gpurun_out/f32sampled.log 2>&1; rc=$?
echo "f32 sampled unit rc=$rc runs=$(grep -c differ gpurun_out/f32sampled.log) clean=$(grep -c ' 0 differ' gpurun_out/f32sampled.log)"
grep -v ' 0 differ' gpurun_out/f32sampled.log | head -40
exit $rc
