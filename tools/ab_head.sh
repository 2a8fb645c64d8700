#!/bin/bash
# A/B of the tail (head) GEMM tiles (AAA_HEAD_TILE) on the given config, with per-kernel rocprof stats.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
c=${1:-c2}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -m gpu -x -p no:cacheprovider --timeout 120 --timeout-method thread -k "unroll_vs_oracle" > $O/parity.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/parity.log; exit 1; }
for m in 0 2 3 4 5; do
  AAA_HEAD_TILE=$m timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -m gpu -x -p no:cacheprovider --timeout 120 --timeout-method thread -k "unroll_vs_oracle" > $O/parity_$m.log 2>&1 || { echo "tests $m rc=$?"; tail -30 $O/parity_$m.log; exit 1; }
  AAA_HEAD_TILE=$m timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --steps 20 > $O/ab_${c}_h$m.json 2>/dev/null || exit 1
  python -c "import json;d=json.loads(open('$O/ab_${c}_h$m.json').read().strip().splitlines()[-1]);print('$c head=$m',d['value'],d['ms_per_step'])"
done
