#!/bin/bash
# Round 6: the backward's side stream (HEAD weight gradients beside the dgrad chain; the layered vision
# backward beside the ConvLSTM weight gradient) -- AAA_SIDE=1 vs 0, same build and box, C2..C5, then
# the full -m gpu suite with it on.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06side; mkdir -p $O; cd $R; export TMPDIR=/tmp
run() {  # name config env...
  local n=$1 c=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-dropin --no-episode > $O/$n.json 2> $O/$n.err || { echo "bench $n rc=$?"; tail -3 $O/$n.err; exit 1; }
  python -c "
import json;d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]);k=d['kernels']
print('$n',d['value'],d['ms_per_step'],{n[:14]:round(v.get('ms',v.get('avg_us',0)/1e3),4) for n,v in k.items() if 'tail' in n or 'vision bwd' in n})"
}
for c in c2 c3 c5 c4; do
  run ${c}_s0 $c AAA_SIDE=0
  run ${c}_s1 $c AAA_SIDE=1
  run ${c}_s0b $c AAA_SIDE=0
  run ${c}_s1b $c AAA_SIDE=1
done
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
echo done
