#!/bin/bash
# Round 6: k_vision_fwd with the phase-paired RGBx image (conflict-free conv1 B reads) vs the HEAD library
# (tools/ablibs/libaaa_head.so), C3 / C4, two runs each; an LDS-counter pass of C3 on each build; the full -m gpu suite.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06visxim; mkdir -p $O; cd $R; export TMPDIR=/tmp
HEAD=$R/tools/ablibs/libaaa_head.so
run() {  # name config env...
  local n=$1 c=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-dropin --no-episode > $O/$n.json 2> $O/$n.err || { echo "bench $n rc=$?"; tail -3 $O/$n.err; exit 1; }
  python -c "
import json;d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]);k=d['kernels']
print('$n',d['value'],d['ms_per_step'],{n[:14]:round(v.get('ms',v.get('avg_us',0)/1e3),4) for n,v in k.items() if 'vision' in n})"
}
for c in c3 c4; do
  run ${c}_head_a $c AAA_LIB=$HEAD
  run ${c}_new_a $c
  run ${c}_head_b $c AAA_LIB=$HEAD
  run ${c}_new_b $c
done
cd /tmp
for b in head new; do
  if [ $b = head ]; then export AAA_LIB=$HEAD; else unset AAA_LIB; fi
  timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $O/pmc_$b -o p -- python $R/bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline --no-dropin --no-episode > $O/pmc_$b.log 2>&1 || { echo "pmc $b rc=$?"; exit 1; }
done
unset AAA_LIB
cd $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
echo done
