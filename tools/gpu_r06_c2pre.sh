#!/bin/bash
# Round 6: fp32 conv2 forward with its weights pre-split at packing (k_Wp2s planes, GRows3B) vs the HEAD library
# (tools/ablibs/libaaa_head.so), C2, two runs each; then the full -m gpu suite on the new build.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06c2pre; mkdir -p $O; cd $R; export TMPDIR=/tmp
run() {  # name config env...
  local n=$1 c=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-dropin --no-episode > $O/$n.json 2> $O/$n.err || { echo "bench $n rc=$?"; tail -3 $O/$n.err; exit 1; }
  python -c "
import json;d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]);k=d['kernels']
print('$n',d['value'],d['ms_per_step'],{n[:16]:round(v.get('ms',v.get('avg_us',0)/1e3),4) for n,v in k.items() if 'vision' in n or 'pack' in n})"
}
for m in 0 1 0 1; do
  if [ $m = 0 ]; then run c2_head$m c2 AAA_LIB=$R/tools/ablibs/libaaa_head.so; else run c2_new$m c2; fi
done
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
echo done
