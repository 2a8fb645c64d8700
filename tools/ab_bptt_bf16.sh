#!/bin/bash
# Parity of the step tile variants, then an A/B of the bf16 BPTT tile (AAA_BPTT_TILE 7, 8, 19-24) on the given configs.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -m gpu -x -p no:cacheprovider --timeout 120 --timeout-method thread -k "tile_variants" > $O/parity.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for c in "$@"; do for t in 7 8 22 23 24; do
  AAA_BPTT_TILE=$t timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --steps 10 > $O/ab_${c}_b$t.json 2>/dev/null || exit 1
  python -c "import json;d=json.loads(open('$O/ab_${c}_b$t.json').read().strip().splitlines()[-1]);k=d['kernels'];print('$c bptt=$t',d['value'],[(n[:20],v['avg_us']) for n,v in k.items()])"
done; done
