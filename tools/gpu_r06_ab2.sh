#!/bin/bash
# Round 6: branch-free BPTT epilogue loads (frames / pairs / band) + the bf16 forward's in-loop x-image
# DMA from inline asm -- same-box A/B against the round's starting build (tools/ablibs/libaaa_base.so)
# at C3, C4, C5, then the full -m gpu suite on the new build.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06ab2; mkdir -p $O; cd $R; export TMPDIR=/tmp
B=$R/tools/ablibs/libaaa_base.so
run() {  # name config env...
  local n=$1 c=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-dropin --no-episode > $O/$n.json 2> $O/$n.err || { echo "bench $n rc=$?"; tail -3 $O/$n.err; exit 1; }
  python -c "
import json;d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]);k=d['kernels']
print('$n',d['value'],d['ms_per_step'],'fwd',k['ConvLSTM forward step']['avg_us'],'bptt',k['ConvLSTM BPTT step']['avg_us'])"
}
for c in c3 c4 c5; do
  run ${c}_base $c AAA_LIB=$B
  run ${c}_new $c
  run ${c}_base2 $c AAA_LIB=$B
  run ${c}_new2 $c
done
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
echo done
