#!/bin/bash
# Build a SASO kernel variant library randblas_amd/_var/<name>.so: saso.hip compiled with extra
# flags, linked with the product objects. Usage: bash tools/build_saso_var.sh <name> "<-D flags>"
set -eu
cd "$(dirname "$0")/.."
make -s -C randblas_amd/csrc
mkdir -p randblas_amd/_var
o=randblas_amd/_var/saso_$1.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-inline-asm $2 -x hip -c randblas_amd/csrc/saso.hip -o $o
objs=$(ls randblas_amd/_obj/*.o | grep -v saso.hip.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o randblas_amd/_var/$1.so $objs $o
echo built randblas_amd/_var/$1.so
