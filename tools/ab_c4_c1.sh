#!/bin/bash
# A/B of split-K choices (rbh_options.splitk) at C4 per GPU and C1, same box, alternating; then the
# L2-miss bytes (FETCH_SIZE) of C4's GEMM per choice. Usage (repo root, via gpurun): bash tools/ab_c4_c1.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
T="timeout -k 10 120 python3 tools/time_dense.py"
for rep in 1 2 3; do
  for sk in 0 1; do
    $T --dtype f32 --d 256 --m 32768 --n 32768 --splitk $sk --reps 20 >> gpurun_out/ab/c4_split.jsonl || exit 1
  done
  for sk in 0 16 4; do
    $T --dtype f64 --d 128 --m 4096 --n 4096 --splitk $sk --reps 50 >> gpurun_out/ab/c1_split.jsonl || exit 1
  done
  echo "rep $rep done"
done
for sk in 0 1; do
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/ab/pmc_c4_s$sk -o run --output-format csv -- \
      python3 tools/time_dense.py --dtype f32 --d 256 --m 32768 --n 32768 --splitk $sk --reps 3 --warmup 1 \
      > gpurun_out/ab/pmc_c4_s$sk.log 2>&1 || exit 1
  python3 tools/pmc_summary.py gpurun_out/ab/pmc_c4_s$sk > gpurun_out/ab/c4_s${sk}_fetch.json
done
echo "all done"
