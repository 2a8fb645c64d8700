#!/bin/bash
# Round 6: the fused vision backward after the reduce rewrite -- tests, C3/C4 A/B (forced on at C4), kernel traces.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06vb2; mkdir -p $O; cd $R; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_vision_bwd.py > $O/tests.log 2>&1; rc=$?
tail -12 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for c in c3 c4; do for v in 0 1 0 1; do
  AAA_VBWD_MINF=0 AAA_VIS_BWD_FRAMES=$v timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-dropin --no-episode > $O/${c}_$v.json 2> $O/${c}_$v.err || { echo "bench $c rc=$?"; tail $O/${c}_$v.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/${c}_$v.json').read().strip().splitlines()[-1]);print('$c vbf=$v',d['value'],d['ms_per_step'],[(n[:24],v.get('avg_us',v.get('ms'))) for n,v in d['kernels'].items() if 'vision' in n])"
done; done
for c in c3 c4; do
  AAA_VBWD_MINF=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$c -o run -- python bench.py --config $c --steps 10 --no-cpu-baseline --no-dropin --no-episode > $O/prof_$c.log 2>&1 || { echo "prof $c failed"; tail $O/prof_$c.log; exit 1; }
done
find $O -name "*kernel_stats.csv" | while read f; do echo $f; grep -i "vbwd\|vision" $f | cut -c1-200; done
echo done
