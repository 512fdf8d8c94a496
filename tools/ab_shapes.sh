#!/bin/bash
# A/B timing of library variants at f32 shapes outside bench.py's configs (tools/time_dense.py):
# one JSON line per (round, variant, shape). Usage: bash tools/ab_shapes.sh "<variants>" [rounds]
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
variants="${1:-prod}"; rounds="${2:-2}"
for r in $(seq 1 "$rounds"); do
 for v in $variants; do
  for sh in "1024 16384 16384" "512 32768 32768" "256 32768 32768"; do
   set -- $sh
   if [ "$v" = prod ]; then lib=""; else lib="$PWD/randblas_amd/_var/$v.so"; fi
   line=$(RBH_LIB_PATH="$lib" timeout -k 10 120 python -u tools/time_dense.py --dtype f32 --d $1 --m $2 --n $3 2>/dev/null | tail -n 1) || exit 1
   echo "$v $line"
  done
 done
done
