#!/bin/bash
# A/B the per-step tile choices: tools/ab_step.sh "FWD:BWD" ... (runtime.hip step_tile ids).
# Runs the tile-variant parity tests first; stops at the first failure.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -x -p no:cacheprovider -k "tile_variants" > $O/parity.log 2>&1; rc=$?; echo "parity rc=$rc"; tail -3 $O/parity.log; [ $rc -eq 0 ] || exit $rc
for pair in "$@"; do
  f=${pair%%:*}; b=${pair##*:}
  AAA_STEP_TILE=$f AAA_BPTT_TILE=$b timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 ${BENCH_ARGS} > $O/ab_${f}_${b}.json 2>/dev/null; rc=$?; [ $rc -eq 0 ] || { echo "bench $pair rc=$rc"; exit $rc; }
  python -c "import json;d=json.load(open('$O/ab_${f}_${b}.json'));print('tiles $pair',d['value'],d['ms_per_step'],json.dumps(d['kernels']))"
done
