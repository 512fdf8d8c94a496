#!/bin/bash
# A/B timing of library variants: for each round, each variant, each config: one bench line
# (kernel_ms, ms_per_step) into gpurun_out/ab_<tag>.jsonl. Variants: "prod" = the in-tree library,
# otherwise randblas_amd/_var/<name>.so. Usage: bash tools/ab_bench.sh <tag> "<configs>" "<variants>" [rounds]
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
tag="$1"; configs="$2"; variants="$3"; rounds="${4:-2}"
mkdir -p gpurun_out
out="gpurun_out/ab_$tag.jsonl"; : > "$out"
for r in $(seq 1 "$rounds"); do
  for v in $variants; do
    for c in $configs; do
      if [ "$v" = prod ]; then lib=""; else lib="$PWD/randblas_amd/_var/$v.so"; fi
      line=$(RBH_LIB_PATH="$lib" timeout -k 10 200 python -u bench.py --config "$c" --no-cpu-baseline --steps 10 2>/dev/null | tail -n 1)
      rc=$?
      if [ $rc -ne 0 ]; then echo "variant $v config $c failed rc=$rc"; exit $rc; fi
      echo "{\"round\": $r, \"variant\": \"$v\", \"config\": \"$c\", \"line\": $line}" >> "$out"
      python3 -c "import json,sys; d=json.loads(sys.argv[1]); print('$v $c', round(d['kernel_ms'],3), round(d['roofline']['frac'],4))" "$line"
    done
  done
done
