#!/bin/bash
# Parity + A/B of the fp32 batched ConvLSTM x-part (AAA_XPART_TILE) and dx (AAA_DX_TILE) GEMM tiles on C2.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
run() {  # name env...
  local n=$1; shift
  env "$@" timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -q -m gpu -x -p no:cacheprovider --timeout 120 --timeout-method thread -k "unroll_vs_oracle" > $O/parity_$n.log 2>&1 || { echo "tests $n rc=$?"; tail -20 $O/parity_$n.log; exit 1; }
  env "$@" timeout -k 10 200 python bench.py --config c2 --no-cpu-baseline --steps 40 > $O/ab_c2_$n.json 2>/dev/null || exit 1
  python -c "import json;d=json.loads(open('$O/ab_c2_$n.json').read().strip().splitlines()[-1]);print('c2 $n',d['value'],d['ms_per_step'])"
}
run default
for t in 1 2 3 4 5; do run x$t AAA_XPART_TILE=$t; done
for t in 1 2 3 4; do run dx$t AAA_DX_TILE=$t; done
run default2
