#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06vb1; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_vision_bwd.py > $O/tests.log 2>&1; rc=$?
tail -15 $O/tests.log; [ $rc -eq 0 ] || exit $rc
P=towards-interpretable-reinforcement-learning-using-attention-augmented-agents-replication_amd/libaaa.so
for c in c3 c4; do for v in 0 1 0 1; do
  AAA_VIS_BWD_FRAMES=$v timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-dropin --no-episode > $O/${c}_$v.json 2> $O/${c}_$v.err || { echo "bench $c rc=$?"; tail $O/${c}_$v.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/${c}_$v.json').read().strip().splitlines()[-1]);print('$c vbf=$v',d['value'],d['ms_per_step'],[(n[:24],v.get('avg_us',v.get('ms'))) for n,v in d['kernels'].items() if 'vision' in n])"
done; done
echo done
