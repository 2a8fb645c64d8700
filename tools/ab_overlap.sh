#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -x -p no:cacheprovider > $O/parity.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -1 $O/parity.log; [ $rc -le 1 ] || exit $rc
for cfg in "AAA_OVERLAP=0 AAA_CHUNK=20" "AAA_OVERLAP=1 AAA_CHUNK=4" "AAA_OVERLAP=1 AAA_CHUNK=4 AAA_AUX_WIDE=1" "AAA_OVERLAP=1 AAA_CHUNK=10" "AAA_OVERLAP=1 AAA_CHUNK=7"; do
  env $cfg timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > $O/ab.json 2>/dev/null; rc=$?; [ $rc -eq 0 ] || { echo "bench $cfg rc=$rc"; exit $rc; }
  python -c "import json;d=json.load(open('$O/ab.json'));print('$cfg',d['value'],d['ms_per_step'],json.dumps(d['kernels']))"
done
