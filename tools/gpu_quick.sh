#!/bin/bash
# Quick GPU check: full GPU test suite, then short benches of the given configs
# (tools/gpu_quick.sh c2 c3 ...); stops at the first failing step.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x -p no:cacheprovider --timeout 120 --timeout-method thread > $O/parity.log 2>&1 || { echo "parity rc=$?"; tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for c in "$@"; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --steps 10 > $O/bench_$c.json 2> $O/bench_$c.err || { echo "bench $c rc=$?"; tail $O/bench_$c.err; exit 1; }
  python -c "import json,sys;d=json.loads(open('$O/bench_$c.json').read().strip().splitlines()[-1]);print('$c',d['value'],d['ms_per_step'],d['roofline']['frac'],json.dumps(d['kernels']),json.dumps(d['hbm_kernels']))"
done
