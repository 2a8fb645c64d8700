#!/bin/bash
# Parity of the step tile variants, then A/Bs of AAA_STEP_TILE / AAA_BPTT_TILE on the given config.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -m gpu -x -p no:cacheprovider --timeout 120 --timeout-method thread -k "tile_variants" > $O/parity.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
c=${1:-c2}
run() {  # name env...
  local n=$1; shift
  env "$@" timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --steps 20 > $O/ab_${c}_$n.json 2>/dev/null || exit 1
  python -c "import json;d=json.loads(open('$O/ab_${c}_$n.json').read().strip().splitlines()[-1]);k=d['kernels'];print('$c $n',d['value'],[(n[:20],v['avg_us']) for n,v in k.items()])"
}
run default
for t in 25 26; do run fwd$t AAA_STEP_TILE=$t; done
run default2
