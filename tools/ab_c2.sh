cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
for rep in 1 2; do
for v in product oldwide; do
  lib=$PWD/randblas_amd/librandblas_hip.so; [ $v = product ] || lib=$PWD/randblas_amd/_var/$v.so
  RBH_LIB_PATH=$lib timeout -k 10 120 python bench.py --config c2 --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/ab_$v.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/ab_$v.json').read().strip().splitlines()[-1]); print('$v', 'kernel_ms', round(d['kernel_ms'],4))"
done
done
