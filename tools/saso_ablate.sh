cd $GRAFT_REPO_ROOT
for ab in 0 1 2 3; do
  RBH_SASO_ABLATE=$ab timeout -k 10 120 python bench.py --config c3 --no-cpu-baseline --steps 5 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('ablate=$ab', 'kernel_ms', round(d['kernel_ms'],3), 'step_ms', round(d['ms_per_step'],3))"
done
