#!/bin/bash
# Round 6: the fp32 weight gradient (gemm_kernel_s6l) with its FD-2 fetch unconditional
# (AAA_S6L_FETCHALL=1: the compiler keeps tile kt+2 in flight) vs guarded (=0), and the bf16 ring's
# s_setprio around its MFMA cluster (AAA_RA_PRIO=1 vs 0); same box.  Then the parity tests.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06s6l; mkdir -p $O; cd $R; export TMPDIR=/tmp
run() {  # name config env...
  local n=$1 c=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-dropin --no-episode > $O/$n.json 2> $O/$n.err || { echo "bench $n rc=$?"; tail -3 $O/$n.err; exit 1; }
  python -c "
import json;d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]);k=d['kernels']
print('$n',d['value'],d['ms_per_step'],{n[:14]:round(v.get('ms',v.get('avg_us',0)/1e3),4) for n,v in k.items() if 'weight-grad' in n or 'vision bwd' in n})"
}
for i in 1 2; do
  run c2_f0_$i c2 AAA_S6L_FETCHALL=0
  run c2_f1_$i c2 AAA_S6L_FETCHALL=1
done
for i in 1 2; do
  run c3_p0_$i c3 AAA_RA_PRIO=0
  run c3_p1_$i c3 AAA_RA_PRIO=1
done
AAA_S6L_FETCHALL=1 AAA_RA_PRIO=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_f32_frames.py tests/test_gpu_components.py > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
echo done
