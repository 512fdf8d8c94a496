cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_sparse.py tests/test_gpu_vector.py -x -q -rf --timeout 60 --timeout-method thread > gpurun_out/t_sparse.log 2>&1; rc=$?; grep -E "passed|failed" gpurun_out/t_sparse.log | tail -2; grep -m3 "^FAILED\|Timeout\|test_.*\[" gpurun_out/t_sparse.log | cut -c1-200; [ $rc -ne 0 ] && exit $rc
DBG_BRIEF=1 DBG_REPS=2 timeout -k 10 200 python -u tools/dbg_f32.py > gpurun_out/dbg_cur.log 2>&1 || exit $?
echo "dbg: $(grep -c ' 0 differ' gpurun_out/dbg_cur.log) clean, $(grep differ gpurun_out/dbg_cur.log | grep -vc ' 0 differ') bad"
timeout -k 10 300 python -u bench.py --config c3 --no-cpu-baseline > gpurun_out/b_c3.log 2>&1 || exit $?
python3 -c "import json; d=json.loads(open('gpurun_out/b_c3.log').read().strip().splitlines()[-1]); print('main kernel_ms', d['kernel_ms'], 'step', d['ms_per_step'], 'frac', d['roofline']['frac'])"
RBH_NO_SASO_DMA=1 timeout -k 10 300 python -u bench.py --config c3 --no-cpu-baseline > gpurun_out/b_c3v.log 2>&1 || exit $?
python3 -c "import json; d=json.loads(open('gpurun_out/b_c3v.log').read().strip().splitlines()[-1]); print('no-DMA kernel_ms', d['kernel_ms'], 'step', d['ms_per_step'], 'frac', d['roofline']['frac'])"
[ -d randblas_amd/_var ] && bash tools/variants.sh c3
DBG_SAMPLED=1 timeout -k 10 200 python -u tools/dbg_f32.py > gpurun_out/dbg_s.log 2>&1 || exit $?
echo "dbg sampled: $(grep -c ' 0 differ' gpurun_out/dbg_s.log) clean, $(grep differ gpurun_out/dbg_s.log | grep -vc ' 0 differ') bad"
exit 0
