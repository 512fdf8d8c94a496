#!/bin/bash
# GPU tests, then each config's bench line in the default build and with one environment variant
# variant (ALT="ENV=val;ENV2=val2", e.g. ALT="RBH_MATERIALISE=1"). Every step has its own time
# limit; the first failure stops.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {   # run <log> <timeout> <cmd...>
    local logf="$1" tmo="$2"; shift 2
    echo "=== $(date +%T) $logf: $*"
    timeout -k 10 "$tmo" "$@" > "gpurun_out/$logf" 2>&1
    local rc=$?
    echo "=== $logf rc=$rc"
    tail -n 2 "gpurun_out/$logf" | cut -c1-400
    if [ $rc -ne 0 ]; then echo "stopping at $logf (rc=$rc)"; exit $rc; fi
}
summ() { tail -1 "gpurun_out/$1" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print("SUMMARY", sys.argv[1], "ms", round(d["ms_per_step"],3), "kern", round(d["kernel_ms"],3), "frac", round(d["roofline"]["frac"],4), "launches", d["kernel_launches_per_step"])' "$1"; }
if [ -n "${TESTS+x}" ]; then
    run pytest_gpu.log 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread $TESTS
fi
for c in ${CONFIGS:-c2}; do
    run "def_$c.log" 300 python -u bench.py --config "$c" --no-cpu-baseline && summ "def_$c.log"
    i=0
    IFS=';' read -ra alts <<< "${ALT:-}"
    for a in "${alts[@]}"; do
        [ -z "$a" ] && continue
        run "alt${i}_$c.log" 300 env $a python -u bench.py --config "$c" --no-cpu-baseline && summ "alt${i}_$c.log"
        i=$((i+1))
    done
done
echo "=== all done"
