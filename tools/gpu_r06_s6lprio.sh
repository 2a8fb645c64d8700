#!/bin/bash
# Round 6: s_setprio over the fp32 weight gradient's MFMA cluster (gemm_kernel_s6l, 2 waves per SIMD):
# AAA_S6L_PRIO 0 / 1 at C2, same box, three runs each.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06s6lp; mkdir -p $O; cd $R; export TMPDIR=/tmp
run() {  # name env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python bench.py --config c2 --no-cpu-baseline --no-dropin --no-episode > $O/$n.json 2> $O/$n.err || { echo "bench $n rc=$?"; tail -3 $O/$n.err; exit 1; }
  python -c "
import json;d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]);k=d['kernels']
print('$n',d['value'],d['ms_per_step'],{n[:14]:round(v.get('ms',v.get('avg_us',0)/1e3),4) for n,v in k.items() if 'weight-grad' in n or 'vision bwd' in n})"
}
for i in 1 2 3; do run p0_$i AAA_S6L_PRIO=0; run p1_$i AAA_S6L_PRIO=1; done
echo done
