#!/bin/bash
# C3: cache policy of the SASO panel copies (LDS-DMA buffer loads): product (none) against nt, sc1,
# sc0 sc1 (variants sd_cp1..3, -DSD_CP), same box, three alternations; then the sparse tests of the best.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out/ab
for rep in 1 2 3; do
  for v in product sd_cp1 sd_cp2 sd_cp3; do
    if [ $v = product ]; then lib=""; else lib="$PWD/randblas_amd/_var/$v.so"; fi
    RBH_LIB_PATH="$lib" timeout -k 10 120 python3 bench.py --config c3 --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/ab/c3_$v.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.loads(open('gpurun_out/ab/c3_$v.json').read().strip().splitlines()[-1]); print(json.dumps({'variant': '$v', 'rep': $rep, 'kernel_ms': d['kernel_ms'], 'ms_per_step': d['ms_per_step']}))" >> gpurun_out/ab/c3_cpol.jsonl
  done
done
echo done
