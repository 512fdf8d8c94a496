#!/bin/bash
# Build a variant of librandblas_hip.so with extra -D flags into randblas_amd/_var/<name>.so (for
# A/B timing with RBH_LIB_PATH=randblas_amd/_var/<name>.so; the product library is untouched).
# Usage: bash tools/build_variant.sh <name> "<-D flags>"
set -eu
cd "$(dirname "$0")/../randblas_amd/csrc"
name="$1"; flags="$2"
out=../_var/$name; mkdir -p "$out"
for f in capi.cpp fill_dense.hip skge_dense.hip saso.hip sksy.hip shards.hip; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-function -Wno-unused-variable $flags \
      -x hip -c $f -o $out/$f.o 2>&1 | grep -E "error" || true &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../_var/$name.so $out/*.o
echo "built ../_var/$name.so"
