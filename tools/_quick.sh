cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_sparse.py -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/t_sparse.log 2>&1; rc=$?; tail -3 gpurun_out/t_sparse.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --config c3 --no-cpu-baseline > gpurun_out/b_c3.log 2>&1 || exit $?
python3 -c "import json; d=json.loads(open('gpurun_out/b_c3.log').read().strip().splitlines()[-1]); print('main kernel_ms', d['kernel_ms'], 'step', d['ms_per_step'], 'frac', d['roofline']['frac'])"
out=gpurun_out/pmcx; mkdir -p $out; i=0
for p in "SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE"; do
  timeout -s KILL 90 rocprofv3 --pmc $p --kernel-trace -d $out/p$i -o run --output-format csv -- python3 bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline > $out/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $out/p$i.log; exit 1; }
  i=$((i+1))
done
python3 tools/pmc_summary.py $out > gpurun_out/c3x_pmc.json
