#!/bin/bash
# Round 6 (session 2): HEAD validation -- full -m gpu suite, then C2..C5 bench lines with the
# frame-resident vision backward on and off (same box), then C3/C5 kernel traces.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06head; mkdir -p $O; cd $R; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > $O/tests.log 2>&1; rc=$?
tail -6 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for c in c2 c3 c4 c5; do for v in 1 0; do
  AAA_VIS_BWD_FRAMES=$v timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-dropin --no-episode > $O/${c}_vb$v.json 2> $O/${c}_vb$v.err || { echo "bench $c rc=$?"; tail $O/${c}_vb$v.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/${c}_vb$v.json').read().strip().splitlines()[-1]);print('$c vbf=$v',d['value'],d['ms_per_step'],[(n[:28],v.get('ms')) for n,v in d['kernels'].items() if 'vision' in n])"
done; done
echo done
