#!/bin/bash
# Full GPU check: every GPU test, smoke(), then a short rocprofv3 kernel trace of
# the C2 and C3 benches (no drop-in leg, no CPU baseline: the trace is the
# library's kernels of warmup + timed steps only).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x -p no:cacheprovider --timeout 150 --timeout-method thread > $O/full_parity.log 2>&1 || { echo "parity rc=$?"; tail -30 $O/full_parity.log; exit 1; }
tail -1 $O/full_parity.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
cd /tmp && export TMPDIR=/tmp
for c in ${PCONF:-c2 c3}; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_$c -o run --output-format csv -- python $R/bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline --no-dropin > $O/prof_$c.log 2>&1 || { echo "prof $c rc=$?"; tail $O/prof_$c.log; exit 1; }
  echo "prof $c ok"
done
