#!/bin/bash
# rocprofv3 kernel trace of short benches (PCONF configs; no drop-in leg, no CPU
# baseline) into gpurun_out/prof_<config>/; summarise with tools/prof_iter.py.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for c in ${PCONF:-c3}; do
  rm -rf $O/prof_$c
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_$c -o run --output-format csv -- python $R/bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline --no-dropin > $O/prof_$c.log 2>&1 || { echo "prof $c rc=$?"; tail $O/prof_$c.log; exit 1; }
  echo "prof $c ok"
done
