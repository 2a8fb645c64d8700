#!/bin/bash
# rocprofv3 kernel-trace summary of a short bench run per config: tools/prof_cfg.sh c3 c5 ...
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for c in "$@"; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_$c -o run --output-format csv -- python $R/bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline > $O/prof_$c.log 2>&1 || { echo "prof $c rc=$?"; exit 1; }
  echo "prof $c ok"
done
