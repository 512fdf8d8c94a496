#!/bin/bash
# Full GPU-box pass for one round: parity tests, smoke, bench of every config, rocprofv3
# kernel-trace stats per config, PMC passes for the configs named in PMC_CONFIGS.
# Each GPU step has its own time limit; any non-zero exit ends the script (nothing retried).
# Usage (repo root, via gpurun): bash tools/round_gpu.sh [tests] [bench] [prof] [pmc]
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
what="${*:-tests bench prof pmc}"
CONFIGS="${CONFIGS:-ns c2 c1 c3 c4 c4full c5 c5p}"
PMC_CONFIGS="${PMC_CONFIGS:-ns c2 c3 c4 c4full c5 c5p c1}"

run() {   # run <log> <timeout> <cmd...>
    local logf="$1" tmo="$2"; shift 2
    echo "=== $(date +%T) $logf: $*"
    timeout -k 10 "$tmo" "$@" > "gpurun_out/$logf" 2>&1
    local rc=$?
    echo "=== $logf rc=$rc"
    tail -n 3 "gpurun_out/$logf" | cut -c1-900
    if [ $rc -ne 0 ]; then echo "stopping at $logf (rc=$rc)"; exit $rc; fi
}

case " $what " in *" tests "*)
    run pytest_gpu.log 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread
    run smoke.log 300 python -u -c "import __graft_entry__ as g; g.smoke()"
;; esac
case " $what " in *" bench "*)
    run bench_all.log 600 python -u bench.py
    for c in $CONFIGS; do run "bench_$c.log" 300 python -u bench.py --config "$c"; done
    run bench_c3pre.log 300 python -u bench.py --config c3 --prefilled
    for c in ${DIST_CONFIGS:-c2 ns c3 c4}; do
        run "bench_${c}_dist1.log" 300 python -u bench.py --config "$c" --dist --no-cpu-baseline
    done
;; esac
case " $what " in *" prof "*)
    # per-launch traces: 20 timed steps after 3 warm-ups, so tools/trace_frac.py recomputes each
    # config's frac from >= 10 steady launches
    for c in $CONFIGS; do
        run "rocprof_$c.log" 300 rocprofv3 --kernel-trace --stats -d "gpurun_out/prof_$c" -o run \
            --output-format csv -- python3 bench.py --config "$c" --steps 20 --warmup 3 --no-cpu-baseline
        f=$(find "gpurun_out/prof_$c" -name "*kernel_stats.csv" | head -n 1)
        [ -n "$f" ] && cp "$f" "gpurun_out/${c}_kernel_stats.csv"
        f=$(find "gpurun_out/prof_$c" -name "*kernel_trace.csv" | head -n 1)
        if [ -n "$f" ]; then
            cp "$f" "gpurun_out/${c}_kernel_trace.csv"
            python3 tools/trace_frac.py "$c" "gpurun_out/${c}_kernel_trace.csv" --warmup 3 --json \
                > "gpurun_out/${c}_trace_frac.json" || true
        fi
    done
;; esac
case " $what " in *" pmc "*)
    for c in $PMC_CONFIGS; do
        out="gpurun_out/pmc_$c"; mkdir -p "$out"; i=0
        for p in "FETCH_SIZE" "WRITE_SIZE" \
                 "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY" \
                 "SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE"; do
            echo "=== pmc $c pass $i: $p"
            timeout -s KILL 120 rocprofv3 --pmc $p --kernel-trace -d "$out/p$i" -o run --output-format csv -- \
                python3 bench.py --config "$c" --steps 3 --warmup 1 --no-cpu-baseline > "$out/p$i.log" 2>&1
            rc=$?
            echo "=== pass rc=$rc"
            if [ $rc -ne 0 ]; then tail -n 20 "$out/p$i.log"; exit $rc; fi
            i=$((i+1))
        done
        python3 tools/pmc_summary.py "$out" > "gpurun_out/${c}_pmc.json"
    done
;; esac
echo "=== all done"
