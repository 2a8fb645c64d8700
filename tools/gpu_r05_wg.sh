#!/bin/bash
# Round 5: split-at-commit fp32 ConvLSTM weight gradient -- parity + same-box C2 A/B.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r05wg; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity.py -k "wgrad_split6 or c2_full or split6_accuracy or c1_against or f32_frames" \
  > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/tests.log | head -20; exit $rc; }
BA="--no-cpu-baseline --no-dropin --no-episode"
for i in 1 2; do
  for t in 4 6; do
    AAA_WGRAD_S6_TILE=$t timeout -k 10 200 python bench.py $BA > $O/t${t}_$i.json 2> $O/t${t}_$i.err || { echo "t$t rc=$?"; tail $O/t${t}_$i.err; exit 1; }
  done
done
for f in $O/t*.json; do python -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$f',d['value'],d['ms_per_step'],{k:v.get('avg_us') for k,v in d['kernels'].items() if 'avg_us' in v})"; done
