#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, kernel-trace only, no sys/runtime traces) for
# one bench config; tools/pmc_summary.py turns the CSVs into per-kernel averages.
# Usage (repo root, via gpurun): bash tools/pmc.sh <config> [bench args...]
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
cfg="$1"; shift || true
export TMPDIR=/tmp
out="gpurun_out/pmc_$cfg"
mkdir -p "$out"
passes=(
  "FETCH_SIZE"
  "WRITE_SIZE"
  "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY"
  "SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE"
)
i=0
for p in "${passes[@]}"; do
  echo "=== pass $i: $p"
  timeout -k 10 300 rocprofv3 --pmc $p --kernel-trace -d "$out/p$i" -o run --output-format csv -- \
      python bench.py --config "$cfg" --steps 3 --warmup 1 --no-cpu-baseline "$@" > "$out/p$i.log" 2>&1
  rc=$?
  echo "=== pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -n 20 "$out/p$i.log"; exit $rc; fi
  i=$((i+1))
done
python tools/pmc_summary.py "$out" > "$out/summary.json" && cat "$out/summary.json"
