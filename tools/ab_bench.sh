#!/bin/bash
# A/B of a variant library against the product one through bench.py configs (RBH_LIB_PATH), same
# box, alternating. Usage (repo root, via gpurun): bash tools/ab_bench.sh <variant> <config> ...
# Appends {"lib": ..., bench line} to gpurun_out/ab/<variant>_bench.jsonl.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
v="$1"; shift
for rep in 1 2; do
  for lib in product "$v"; do
    if [ "$lib" = product ]; then L=randblas_amd/librandblas_hip.so; else L="randblas_amd/_var/$lib.so"; fi
    for c in "$@"; do
      line=$(RBH_LIB_PATH=$L timeout -k 10 200 python3 bench.py --config "$c" --no-cpu-baseline --steps 10 --warmup 3 2>/dev/null | tail -n 1) || exit 1
      echo "{\"lib\": \"$lib\", \"config\": \"$c\", \"line\": $line}" >> "gpurun_out/ab/${v}_bench.jsonl"
    done
  done
  echo "rep $rep done"
done
