#!/bin/bash
# L2-to-fabric read bytes (FETCH_SIZE x 2, the gfx950 correction) of the dominant kernel per library
# variant, one rocprofv3 --pmc pass each, plus that variant's bench line (bench configs only).
# Usage (repo root, via gpurun): bash tools/fetch_ab.sh <config> "<variants>"   ("prod" = in-tree)
#        bash tools/fetch_ab.sh shape "<variants>" <d> <m> <n> [f32|f64] [splitk]   (tools/time_dense.py)
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
cfg="$1"; variants="$2"
if [ "$cfg" = shape ]; then
  prog=(python3 tools/time_dense.py --d "$3" --m "$4" --n "$5" --dtype "${6:-f32}" --splitk "${7:-0}" --reps 3 --warmup 1)
  tag="shape_$3_$4_$5_${7:-0}"
else
  prog=(python3 bench.py --config "$cfg" --steps 3 --warmup 1 --no-cpu-baseline)
  tag="$cfg"
fi
for v in $variants; do
  if [ "$v" = prod ]; then lib=""; else lib="$PWD/randblas_amd/_var/$v.so"; fi
  out="gpurun_out/fetch_${tag}_$v"; rm -rf "$out"; mkdir -p "$out"
  RBH_LIB_PATH="$lib" timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$out/p0" -o run \
      --output-format csv -- "${prog[@]}" > "$out/log" 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "variant $v pmc rc=$rc"; tail -n 5 "$out/log"; exit $rc; fi
  python3 tools/pmc_summary.py "$out" | python3 -c "
import json, sys
d = json.load(sys.stdin)
for k, v in d.items():
    if ('skge_' in k or 'saso_dma' in k) and 'FETCH_SIZE' in v:
        print('$v', k[:70], 'fetch GB per launch (x2):', round(2 * 1024 * v['FETCH_SIZE'] / 1e9, 3))
"
  if [ "$cfg" = shape ]; then
    RBH_LIB_PATH="$lib" timeout -k 10 120 "${prog[@]}" 2>/dev/null | tail -n 1
  else
    RBH_LIB_PATH="$lib" timeout -k 10 120 python3 bench.py --config "$cfg" --no-cpu-baseline 2>/dev/null | tail -n 1 | \
        python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('$v', 'kernel_ms', round(d['kernel_ms'],4), 'frac', round(d['roofline']['frac'],4))"
  fi
done
