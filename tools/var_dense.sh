#!/bin/bash
# Dense kernel variants (randblas_amd/_var/<name>.so): parity on the C2 shape family, then the C2
# bench kernel time. Usage (via gpurun): VARS="a b" bash tools/var_dense.sh [config]
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
cfg="${1:-c2}"
for v in $VARS; do
  lib="$PWD/randblas_amd/_var/$v.so"
  RBH_LIB_PATH="$lib" timeout -k 10 300 python -m pytest tests/test_gpu_dense.py -k "large_c2_slice or fused or row_shards" -x -q > "gpurun_out/var_$v.test.log" 2>&1
  rc=$?; echo "variant $v tests rc=$rc $(tail -n 1 gpurun_out/var_$v.test.log)"
  if [ $rc -ne 0 ]; then exit $rc; fi
  RBH_LIB_PATH="$lib" timeout -k 10 120 python bench.py --config "$cfg" --no-cpu-baseline --steps 10 --warmup 3 > "gpurun_out/var_$v.json" 2> "gpurun_out/var_$v.err"
  rc=$?
  if [ $rc -ne 0 ]; then echo "variant $v bench rc=$rc"; tail -n 5 "gpurun_out/var_$v.err"; exit $rc; fi
  python3 -c "import json; d=json.loads(open('gpurun_out/var_$v.json').read().strip().splitlines()[-1]); print('variant $v', 'kernel_ms', round(d['kernel_ms'],4), 'step_ms', round(d['ms_per_step'],4), 'frac', round(d['roofline']['frac'],4))"
done
