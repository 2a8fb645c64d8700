#!/bin/bash
# A/B of the ConvLSTM weight-gradient engine (AAA_WGRAD_PIPE, AAA_WGRAD_WGS) on the given config.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
c=${1:-c2}
run() {  # name env...
  local n=$1; shift
  env "$@" timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --steps 20 > $O/ab_${c}_$n.json 2>/dev/null || exit 1
  python -c "import json;d=json.loads(open('$O/ab_${c}_$n.json').read().strip().splitlines()[-1]);k=d['kernels'];print('$c $n',d['value'],[(n[:20],v['avg_us']) for n,v in k.items()])"
}
run default
for p in 1 2 4 5 6; do for w in 256 512; do run pipe${p}_$w AAA_WGRAD_PIPE=$p AAA_WGRAD_WGS=$w; done; done
