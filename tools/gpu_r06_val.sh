#!/bin/bash
# Round 6: validation of HEAD -- the full -m gpu suite, then the C2..C5 bench lines (C2 the driver's default
# line with its cpu_baseline / drop-in / episode legs).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06val; mkdir -p $O; cd $R; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > $O/c2_bench.json 2> $O/c2_bench.err || { echo "c2 rc=$?"; tail -5 $O/c2_bench.err; exit 1; }
for c in c3 c4 c5; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > $O/${c}_bench.json 2> $O/${c}_bench.err || { echo "$c rc=$?"; tail -5 $O/${c}_bench.err; exit 1; }
done
for c in c2 c3 c4 c5; do python -c "
import json;d=json.loads(open('$O/${c}_bench.json').read().strip().splitlines()[-1])
print('$c', d['value'], d['ms_per_step'], d['roofline']['kernel'][:40], d['roofline']['frac'], d.get('job_roofline',{}).get('frac'), d.get('episode',{}).get('episode_frames_per_s'))"; done
echo done
