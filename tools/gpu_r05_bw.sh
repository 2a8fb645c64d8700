#!/bin/bash
# Round 5: pre-split fp32 frame-group BPTT -- parity + same-box C2 A/B.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r05bw; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_f32_frames.py tests/test_gpu_parity.py -k "f32_frames or c2_full or split6_accuracy or c1_against or per_step_forward or state_grad or carried" \
  > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/tests.log | head -20; exit $rc; }
BA="--no-cpu-baseline --no-dropin --no-episode"
for i in 1 2; do
  timeout -k 10 200 python bench.py $BA > $O/ps_$i.json 2> $O/ps_$i.err || { echo "ps rc=$?"; tail $O/ps_$i.err; exit 1; }
  AAA_F32_PRESPLIT=1 timeout -k 10 200 python bench.py $BA > $O/old_$i.json 2> $O/old_$i.err || { echo "old rc=$?"; exit 1; }
done
for f in $O/ps_*.json $O/old_*.json; do python -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$f',d['value'],d['ms_per_step'],{k:v.get('avg_us') for k,v in d['kernels'].items() if 'avg_us' in v})"; done
