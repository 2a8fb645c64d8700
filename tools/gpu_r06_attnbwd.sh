#!/bin/bash
# Round 6: the attention backward's dA pass on the MFMA (attn_mfma.h k_attn_bwd_mfma, bf16 O): full -m gpu suite
# with it on (default), then C3 / C5 / C4 A/B AAA_ATTN_BWD_MFMA=0 (the VALU kernel) vs 1, twice each.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06attnbwd; mkdir -p $O; cd $R; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
run() {  # name config env...
  local n=$1 c=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-dropin --no-episode > $O/$n.json 2> $O/$n.err || { echo "bench $n rc=$?"; tail -3 $O/$n.err; exit 1; }
  python -c "
import json;d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]);k=d['hbm_kernels']
print('$n',d['value'],d['ms_per_step'],{n[:20]:(v['avg_us'],v['frac']) for n,v in k.items()})"
}
for c in c3 c5 c4; do
  for m in 0 1 0 1; do run ${c}_bm$m $c AAA_ATTN_BWD_MFMA=$m; done
done
echo done
