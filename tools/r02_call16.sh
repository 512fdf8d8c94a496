#!/bin/bash
# Round-2 GPU call 16: C3 ablation of the lock-step SASO apply (128/2): 0 full, 1 copies only,
# 2 walk only, 3 neither (kernel time; results are not valid under ablation).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for a in 0 1 2 3; do
    RBH_SASO_ABLATE=$a timeout -k 10 300 python -u bench.py --config c3 --no-cpu-baseline > gpurun_out/abl_$a.log 2>&1 || { echo "ablate $a failed"; tail gpurun_out/abl_$a.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/abl_$a.log').read().strip().splitlines()[-1]); print('ablate=$a', 'kernel_ms', round(d['kernel_ms'],4), 'step_ms', round(d['ms_per_step'],4))"
done
echo "=== all done"
