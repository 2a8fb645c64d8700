#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 900 python -u -m pytest tests -v -m gpu -x -p no:cacheprovider --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $O/gpu_tests.log | head -20; exit $rc; }
for c in c2 c3; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-dropin --no-episode > $O/bench_$c.json 2> $O/bench_$c.err || { echo "bench $c rc=$?"; tail $O/bench_$c.err; exit 1; }
done
echo done
