#!/bin/bash
# A/B runtime env knobs on the bench: tools/ab_env.sh "AAA_X=1 AAA_Y=2" "AAA_X=0" ...
# Each arm: bench.py --steps 20 (no CPU baseline); with PROF=1 also a rocprofv3 kernel summary per arm.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
i=0
for spec in "$@"; do
  i=$((i+1))
  env $spec timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 ${BENCH_ARGS} > $O/abenv_$i.json 2>/dev/null; rc=$?; [ $rc -eq 0 ] || { echo "bench [$spec] rc=$rc"; exit $rc; }
  python -c "import json;d=json.load(open('$O/abenv_$i.json'));print('[$spec]',d['value'],d['ms_per_step'],json.dumps(d['kernels']))"
  if [ "$PROF" = "1" ]; then
    rm -rf $O/abprof_$i
    (cd /tmp && export TMPDIR=/tmp $spec && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/abprof_$i -o run --output-format csv -- python $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline ${BENCH_ARGS} > $O/abprof_$i.log 2>&1) || { echo "prof [$spec] failed"; exit 1; }
  fi
done
