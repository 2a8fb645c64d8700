#!/bin/bash
# Round 6 baseline at HEAD: C2..C5 bench lines and rocprofv3 kernel traces of C3..C5.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06base; mkdir -p $O; cd $R
for c in c2 c3 c4 c5; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-episode > $O/${c}_bench.json 2> $O/${c}_bench.err || { echo "$c rc=$?"; exit 1; }
  echo "bench $c ok"
done
cd /tmp && export TMPDIR=/tmp
for c in c3 c4 c5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$c -o run --output-format csv -- python $R/bench.py --config $c --no-cpu-baseline --no-dropin --no-episode > $O/${c}_prof.json 2> $O/${c}_prof.err || { echo "prof $c rc=$?"; exit 1; }
  echo "prof $c ok"
done
for c in c2 c3 c4 c5; do python -c "
import json;d=json.loads(open('$O/${c}_bench.json').read().strip().splitlines()[-1])
print('$c', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'], d.get('job_roofline',{}).get('frac'))"; done
echo done
