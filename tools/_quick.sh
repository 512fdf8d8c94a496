cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_sparse.py tests/test_gpu_vector.py -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/t_sparse.log 2>&1; rc=$?; tail -3 gpurun_out/t_sparse.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --config c3 --no-cpu-baseline > gpurun_out/b_c3.log 2>&1 || exit $?
python3 -c "import json; d=json.loads(open('gpurun_out/b_c3.log').read().strip().splitlines()[-1]); print('main kernel_ms', d['kernel_ms'], 'step', d['ms_per_step'], 'frac', d['roofline']['frac'])"
[ -d randblas_amd/_var ] && bash tools/variants.sh c3
exit 0
