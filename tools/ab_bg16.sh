#!/bin/bash
# C1 on 16 x 512 tiles (variant bg16: RBH_BG16=1) against the product's 32 x 512, same box, alternating;
# then the variant's parity tests for the split / small-grid / transposed kernels.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out/ab
V="$PWD/randblas_amd/_var/bg16.so"
for rep in 1 2 3; do
  timeout -k 10 120 python3 tools/time_dense.py --dtype f64 --d 128 --m 4096 --n 4096 --reps 50 >> gpurun_out/ab/c1_bg16.jsonl || exit 1
  RBH_LIB_PATH=$V timeout -k 10 120 python3 tools/time_dense.py --dtype f64 --d 128 --m 4096 --n 4096 --reps 50 >> gpurun_out/ab/c1_bg16.jsonl || exit 1
  RBH_LIB_PATH=$V timeout -k 10 120 python3 tools/time_dense.py --dtype f64 --d 128 --m 4096 --n 4096 --reps 50 --layout R >> gpurun_out/ab/c1_bg16.jsonl || exit 1
done
RBH_LIB_PATH=$V timeout -k 10 600 python3 -m pytest tests/test_gpu_dense.py tests/test_gpu_workloads.py -x -q --timeout 120 --timeout-method thread -k "split or c1 or stream or transposed or small" > gpurun_out/ab/bg16_tests.log 2>&1
echo "tests rc=$?"; tail -n 2 gpurun_out/ab/bg16_tests.log
