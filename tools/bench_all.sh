cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for c in c2 ns c3 c4 c5; do
  timeout -k 10 300 python bench.py --config $c > gpurun_out/bench_$c.log 2>&1
  rc=$?; echo "$c rc=$rc"; tail -1 gpurun_out/bench_$c.log | cut -c1-600
  if [ $rc -ne 0 ]; then exit $rc; fi
done
