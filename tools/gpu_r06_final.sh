#!/bin/bash
# Round 6 end-of-round measurements at HEAD: smoke(), the full -m gpu suite, the default bench line (C2 + drop-in +
# episode + CPU baseline), the C3 / C4 / C5 lines, and a kernel trace of the default C2 line at the bench's own
# steps checked against its event timings (tools/trace_vs_events.py).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${FINAL_DIR:-r06final}; mkdir -p $O; cd $R; export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > $O/c2_bench.json 2> $O/c2_bench.err || { echo "c2 rc=$?"; tail -5 $O/c2_bench.err; exit 1; }
for c in c3 c4 c5; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-episode > $O/${c}_bench.json 2> $O/${c}_bench.err || { echo "$c rc=$?"; tail -5 $O/${c}_bench.err; exit 1; }
done
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o run --output-format csv -- python $R/bench.py --no-cpu-baseline --no-dropin --no-episode > $O/c2_prof.json 2> $O/c2_prof.err || { echo "prof rc=$?"; exit 1; }
python $R/tools/trace_vs_events.py $O/prof_c2/run_kernel_trace.csv $O/c2_prof.json 1 > $O/c2_cmp.json || exit 1
for c in c2 c3 c4 c5; do python -c "
import json;d=json.loads(open('$O/${c}_bench.json').read().strip().splitlines()[-1])
print('$c', d['value'], d['ms_per_step'], d['roofline']['kernel'][:40], d['roofline']['frac'], d['roofline'].get('traffic'), d.get('job_roofline',{}).get('frac'), (d.get('episode') or {}).get('episode_frames_per_s'))"; done
echo done
