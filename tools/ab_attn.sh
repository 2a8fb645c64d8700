#!/bin/bash
# A/B of the attention-forward readout knobs (AAA_ATTN_PRE, AAA_ATTN_SLICES) on the given configs.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest tests -q -m gpu -x -p no:cacheprovider --timeout 120 --timeout-method thread -k "attn or parity" > $O/parity.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for c in "$@"; do for v in "1 11" "1 8" "1 5" "0 11" "0 8" "0 5"; do set -- $v
  AAA_ATTN_PRE=$1 AAA_ATTN_SLICES=$2 timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --steps 10 > $O/ab_${c}_$1_$2.json 2>/dev/null || exit 1
  python -c "import json;d=json.loads(open('$O/ab_${c}_$1_$2.json').read().strip().splitlines()[-1]);h=d['hbm_kernels'];print('$c pre=$1 sl=$2',d['value'],[(k[:25],v['avg_us'],v['frac']) for k,v in h.items()])"
done; done
