#!/bin/bash
# Build librandblas_hip.so with extra -D flags for one translation unit into randblas_amd/_var/<name>.so
# (kernel-variant experiments; select at run time with RBH_LIB_PATH).
# Usage: tools/build_variant.sh <name> <source.hip> "<flags>" [replacement-source]
set -e
cd "$(dirname "$0")/../randblas_amd/csrc"
name="$1"; src="$2"; flags="$3"; alt="${4:-$2}"
mkdir -p ../_var
make -s -j16 >/dev/null
objs=""
for o in ../_obj/*.o; do
  b=$(basename "$o" .o)
  if [ "$b" = "$src" ]; then
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC $flags -x hip -c "$alt" -o "../_var/$name.$src.o"
    objs="$objs ../_var/$name.$src.o"
  else
    objs="$objs $o"
  fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "../_var/$name.so" $objs
echo "built randblas_amd/_var/$name.so"
