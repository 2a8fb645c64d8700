#!/bin/bash
# A/B two library builds on one GPU box (boxes differ by up to ~10 %, so only
# same-box numbers compare): tools/ab_lib.sh <lib_a.so> <lib_b.so> ...
# Each arm: bench.py --steps 20 (no CPU baseline) with AAA_LIB=<lib>; BENCH_ARGS adds flags.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
i=0
for lib in "$@"; do
  i=$((i+1))
  AAA_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 ${BENCH_ARGS} > $O/ablib_$i.json 2>/dev/null; rc=$?; [ $rc -eq 0 ] || { echo "bench [$lib] rc=$rc"; exit $rc; }
  python -c "import json;d=json.load(open('$O/ablib_$i.json'));print('[$lib]',d['value'],d['ms_per_step'],json.dumps(d['kernels']))"
done
