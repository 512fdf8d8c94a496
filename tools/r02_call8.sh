#!/bin/bash
# Round-2 GPU call 8: phase timing of the SASO DMA apply (C3) under each chunk shape.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for sh in 128_2 64_2 64_4; do
    export RBH_SASO_KC=${sh%_*} RBH_SASO_NBUF=${sh#*_}
    echo "== shape $sh"
    RBH_LIB_PATH=$PWD/randblas_amd/_var/sdprof.so timeout -k 10 200 python -u tools/saso_prof.py > gpurun_out/sdprof_$sh.log 2>&1 || { echo "prof $sh failed"; tail gpurun_out/sdprof_$sh.log; exit 1; }
    tail -n 4 gpurun_out/sdprof_$sh.log
done
echo "=== all done"
