#!/bin/bash
# Round-end measurement: GPU tests, smoke, bench lines C2 (with CPU baseline) and C3-C5,
# rocprofv3 kernel-trace summaries of C2, C3 and C5.  Stops at the first failing step.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x -p no:cacheprovider --timeout 120 --timeout-method thread > $O/parity.log 2>&1 || { echo "parity rc=$?"; tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for c in c2 c3 c4 c5; do
  extra=""; [ $c != c2 ] && extra="--no-cpu-baseline"
  timeout -k 10 300 python bench.py --config $c $extra > $O/bench_$c.json 2> $O/bench_$c.err || { echo "bench $c rc=$?"; tail $O/bench_$c.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/bench_$c.json').read().strip().splitlines()[-1]);print('$c',d['value'],d['ms_per_step'],d['roofline']['kernel'],d['roofline']['frac'])"
done
cd /tmp && export TMPDIR=/tmp
for c in c2 c3 c5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$c -o run --output-format csv -- python $R/bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline > $O/prof_$c.log 2>&1 || { echo "prof $c rc=$?"; exit 1; }
done
echo done
