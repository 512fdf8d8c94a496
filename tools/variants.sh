#!/bin/bash
# Bench (and optionally parity-test) the kernel variants in randblas_amd/_var/*.so on one config.
# Usage (repo root, via gpurun): bash tools/variants.sh <config> [test] ; variant names from $VARS
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
cfg="$1"; dotest="${2:-}"
for v in ${VARS:-$(ls randblas_amd/_var/*.so | xargs -n1 basename | sed 's/\.so$//')}; do
  lib="$PWD/randblas_amd/_var/$v.so"
  if [ "$dotest" = "test" ]; then
    RBH_LIB_PATH="$lib" timeout -k 10 300 python -m pytest tests/test_gpu_sparse.py -x -q > "gpurun_out/var_$v.test.log" 2>&1
    rc=$?; echo "variant $v tests rc=$rc $(tail -n 1 gpurun_out/var_$v.test.log)"
    if [ $rc -gt 1 ]; then exit $rc; fi
  fi
  RBH_LIB_PATH="$lib" timeout -k 10 120 python bench.py --config "$cfg" --no-cpu-baseline --steps 10 --warmup 3 > "gpurun_out/var_$v.json" 2> "gpurun_out/var_$v.err"
  rc=$?
  if [ $rc -ne 0 ]; then echo "variant $v bench rc=$rc"; tail -n 5 "gpurun_out/var_$v.err"; exit $rc; fi
  python3 -c "import json; d=json.load(open('gpurun_out/var_$v.json')); print('variant $v', 'kernel_ms', round(d['kernel_ms'],4), 'step_ms', round(d['ms_per_step'],4), 'frac', round(d['roofline']['frac'],3))"
done
