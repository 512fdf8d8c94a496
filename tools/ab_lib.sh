#!/bin/bash
# A/B of a variant library against the product one (RBH_LIB_PATH), same box, alternating, through
# tools/time_dense.py. Usage (repo root, via gpurun): bash tools/ab_lib.sh <variant name> "<time_dense args>" ...
# Writes gpurun_out/ab/<variant>.jsonl, one line per run with "lib" set to product / <variant>.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
v="$1"; shift
for rep in 1 2 3; do
  for lib in product "$v"; do
    for args in "$@"; do
      if [ "$lib" = product ]; then L=randblas_amd/librandblas_hip.so; else L="randblas_amd/_var/$lib.so"; fi
      RBH_LIB_PATH=$L timeout -k 10 120 python3 tools/time_dense.py $args --tag "$lib" >> "gpurun_out/ab/$v.jsonl" || exit 1
    done
  done
  echo "rep $rep done"
done
