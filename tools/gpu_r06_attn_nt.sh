#!/bin/bash
# Round 6: the MFMA attention forward with the O rows loaded non-temporal (AAA_ATTN_NT=1) vs default, C3 / C5.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06attnnt; mkdir -p $O; cd $R; export TMPDIR=/tmp
run() {  # name config env...
  local n=$1 c=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-dropin --no-episode > $O/$n.json 2> $O/$n.err || { echo "bench $n rc=$?"; tail -3 $O/$n.err; exit 1; }
  python -c "
import json;d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]);k=d['hbm_kernels']
print('$n',d['value'],d['ms_per_step'],{n[:20]:(v['avg_us'],v['frac']) for n,v in k.items()})"
}
for c in c3 c5; do
  for m in 0 1 0 1; do run ${c}_nt$m $c AAA_ATTN_NT=$m; done
done
echo done
