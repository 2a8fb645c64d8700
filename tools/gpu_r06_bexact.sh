#!/bin/bash
# Round 6: conv1 with the uint8 frames' RGBx operand exact in bf16 (three of the six split products; fp32 path),
# A/B in the ablation build (AAA_CONV1_BEXACT=0 / 1) at C2, then the full -m gpu suite on the product build.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06bx; mkdir -p $O; cd $R; export TMPDIR=/tmp
ABL=$R/towards-interpretable-reinforcement-learning-using-attention-augmented-agents-replication_amd/libaaa_ablation.so
run() {  # name config env...
  local n=$1 c=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-dropin --no-episode > $O/$n.json 2> $O/$n.err || { echo "bench $n rc=$?"; tail -3 $O/$n.err; exit 1; }
  python -c "
import json;d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]);k=d['kernels']
print('$n',d['value'],d['ms_per_step'],{n[:16]:round(v.get('ms',v.get('avg_us',0)/1e3),4) for n,v in k.items() if 'vision' in n})"
}
for m in 0 1 0 1; do run c2_bx$m c2 AAA_LIB=$ABL AAA_CONV1_BEXACT=$m; done
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
echo done
