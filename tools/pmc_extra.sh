cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters.txt 2>&1
timeout -k 10 300 rocprofv3 --pmc TA_BUSY_avr TA_TA_BUSY_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum --kernel-trace -d gpurun_out/pmcx -o run --output-format csv -- python bench.py --config c2 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pmcx.log 2>&1
echo rc=$?
