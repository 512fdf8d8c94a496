#!/bin/bash
# The dense kernels with A's leading dimension padded (L2 set-conflict probe), ws and old kernels.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for pad in ${PADS:-0 32}; do
  for ws in 1 0; do
    echo "=== pad $pad ws $ws"
    RBH_WS=$ws timeout -k 10 200 python -u bench.py --config ${CFG:-c2} --no-cpu-baseline --lda-pad $pad --steps 5 > gpurun_out/pad_${pad}_$ws.log 2>&1 || { tail -5 gpurun_out/pad_${pad}_$ws.log; exit 1; }
    tail -1 gpurun_out/pad_${pad}_$ws.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print("ms", round(d["ms_per_step"],3), "kern", round(d["kernel_ms"],3), "frac", round(d["roofline"]["frac"],4))'
  done
done
