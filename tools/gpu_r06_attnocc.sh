#!/bin/bash
# Round 6: the MFMA attention forward without the per-frame-query logits code in the constant-query kernel
# (a separate instantiation) and, for nq 4, five waves per SIMD (94 VGPRs): HEAD library (tools/ablibs/
# libaaa_head.so) vs the new build, C3 / C4, two runs each; then the full -m gpu suite on the new build.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06attnocc; mkdir -p $O; cd $R; export TMPDIR=/tmp
run() {  # name config env...
  local n=$1 c=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-dropin --no-episode > $O/$n.json 2> $O/$n.err || { echo "bench $n rc=$?"; tail -3 $O/$n.err; exit 1; }
  python -c "
import json;d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]);k=d['hbm_kernels']
print('$n',d['value'],d['ms_per_step'],{n[:20]:(v['avg_us'],v['frac']) for n,v in k.items()})"
}
for c in c3 c4; do
  run ${c}_head_a $c AAA_LIB=$R/tools/ablibs/libaaa_head.so
  run ${c}_new_a $c
  run ${c}_head_b $c AAA_LIB=$R/tools/ablibs/libaaa_head.so
  run ${c}_new_b $c
done
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
echo done
