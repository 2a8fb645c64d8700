#!/bin/bash
# Parity + A/B of the bf16 fused forward-step tile (AAA_FUSED_TILE) on the given configs.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
for t in 9 12 13 14 15 16; do
  AAA_FUSED_TILE=$t timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -q -m gpu -x -p no:cacheprovider --timeout 120 --timeout-method thread -k "fused_x_part_both_ways" > $O/parity_f$t.log 2>&1 || { echo "tests $t rc=$?"; tail -30 $O/parity_f$t.log; exit 1; }
done
echo parity ok
for c in "$@"; do for t in 9 12 13 14 15 16; do
  AAA_FUSED_TILE=$t timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --steps 10 > $O/ab_${c}_f$t.json 2>/dev/null || exit 1
  python -c "import json;d=json.loads(open('$O/ab_${c}_f$t.json').read().strip().splitlines()[-1]);k=d['kernels'];print('$c ftile=$t',d['value'],[(n[:20],v['avg_us']) for n,v in k.items()])"
done; done
