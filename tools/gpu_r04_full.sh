#!/bin/bash
# Round-4 full check: GPU tests, the default bench line (C2 + episode leg + CPU baseline),
# C3/C4/C5 lines, a kernel-trace summary of C2 and C3.  Stops at the first failing step.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 700 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -1 $O/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/gpu_tests.log | head -20; exit $rc; }
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo "bench default rc=$?"; tail $O/bench_default.err; exit 1; }
tail -c 600 $O/bench_default.json; echo
for c in c3 c4 c5; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-dropin --no-episode > $O/bench_$c.json 2> $O/bench_$c.err || { echo "bench $c rc=$?"; tail $O/bench_$c.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/bench_$c.json').read().strip().splitlines()[-1]);print('$c',d['value'],d['ms_per_step'],d['roofline'])"
done
cd /tmp && export TMPDIR=/tmp
for c in c2 c3; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$c -o run --output-format csv -- python $R/bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline --no-dropin --no-episode > $R/gpurun_out/prof_$c.log 2>&1 || { echo "prof $c rc=$?"; exit 1; }
done
echo done
