#!/bin/bash
# Build a kernel-variant library randblas_amd/_var/<name>.so: one source of randblas_amd/csrc
# compiled with extra flags, linked with the product objects of the others. Load it with
# RBH_LIB_PATH=randblas_amd/_var/<name>.so. Usage: bash tools/build_var.sh <name> <source> "<-D flags>"
set -eu
cd "$(dirname "$0")/.."
make -s -C randblas_amd/csrc
mkdir -p randblas_amd/_var
o=randblas_amd/_var/$1.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-inline-asm $3 -x hip -c randblas_amd/csrc/$2 -o $o
objs=$(ls randblas_amd/_obj/*.o | grep -v "/$2.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o randblas_amd/_var/$1.so $objs $o
echo built randblas_amd/_var/$1.so
