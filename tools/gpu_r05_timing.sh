#!/bin/bash
# Round-5 timing reconciliation: the bench's HIP-event
# kernel times against a rocprofv3 kernel trace of the SAME process, at the
# bench's own steps / warm-up, plus the plain (unprofiled) lines beside them.
# usage: tools/gpu_r05_timing.sh [configs...]   -> gpurun_out/r05t/
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r05t; mkdir -p $O
BA="--no-cpu-baseline --no-dropin --no-episode"
for c in "${@:-c2}"; do
  cd $R
  timeout -k 10 200 python bench.py --config $c $BA --timed-steps 20 > $O/${c}_plain20.json 2> $O/${c}_plain20.err || { echo "plain20 $c rc=$?"; exit 1; }
  timeout -k 10 200 python bench.py --config $c $BA --timed-steps 1 > $O/${c}_plain1.json 2> $O/${c}_plain1.err || { echo "plain1 $c rc=$?"; exit 1; }
  cd /tmp && export TMPDIR=/tmp
  for k in 20 1; do
    timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_${c}_$k -o run --output-format csv -- python $R/bench.py --config $c $BA --timed-steps $k > $O/${c}_prof$k.json 2> $O/${c}_prof$k.err || { echo "prof $c $k rc=$?"; exit 1; }
    python $R/tools/trace_vs_events.py $O/prof_${c}_$k/run_kernel_trace.csv $O/${c}_prof$k.json $k > $O/${c}_cmp$k.json || exit 1
  done
  for f in $O/${c}_plain20.json $O/${c}_plain1.json $O/${c}_prof20.json $O/${c}_prof1.json; do
    python -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$f',d['value'],d['ms_per_step'],{k:v.get('avg_us') for k,v in d['kernels'].items() if 'avg_us' in v})"
  done
  python -c "
import json
for k in (20, 1):
    d = json.load(open('$O/${c}_cmp%d.json' % k))
    for n, e in d['classes'].items():
        print(k, n, e['event_avg_us'], e['trace_avg_us_timed'], e['ratio_trace_over_event'], e['launches_in_trace'])
"
done
echo done
