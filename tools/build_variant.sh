#!/bin/bash
# Build a variant of librandblas_hip.so with extra -D flags into randblas_amd/_var/<name>.so (for
# A/B timing with RBH_LIB_PATH=randblas_amd/_var/<name>.so; the product library is untouched).
# Usage: bash tools/build_variant.sh <name> "<-D flags>"
set -eu
cd "$(dirname "$0")/../randblas_amd/csrc"
name="$1"; flags="$2"
make -s -j8 OBJDIR="../_var/$name" LIB="../_var/$name.so" EXTRA="$flags"
echo "built ../_var/$name.so"
