#!/bin/bash
# A/B the per-step tile choice (0 = 64x64, 1 = 32x64 + in-WG split-K), parity first.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -x -p no:cacheprovider > $O/parity.log 2>&1; rc=$?; echo "parity rc=$rc"; [ $rc -le 1 ] || exit $rc
for v in 0 3; do
  AAA_STEP_TILE=$v AAA_BPTT_TILE=$((v==0?2:3)) timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > $O/ab_$v.json 2>/dev/null; rc=$?; [ $rc -eq 0 ] || { echo "bench $v rc=$rc"; exit $rc; }
  python -c "import json;d=json.load(open('$O/ab_$v.json'));print('tile',$v,d['value'],d['ms_per_step'],json.dumps(d['kernels']))"
done
