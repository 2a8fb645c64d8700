#!/bin/bash
# Round-5 A/B: the fp32 vision forward's conv1 / conv2 on split-at-commit tiles (AAA_VIS_F32_S6L=1,
# ablation build) against the split6 LDS-DMA rings: parity pass, bench arms, kernel traces.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
P=towards-interpretable-reinforcement-learning-using-attention-augmented-agents-replication_amd; A=$P/libaaa_ablation.so
AAA_LIB=$R/$A AAA_VIS_F32_S6L=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t_vf.log 2>&1 || { echo "parity rc=$?"; tail -30 gpurun_out/t_vf.log; exit 1; }
tail -1 gpurun_out/t_vf.log
SKIP_TESTS=1 tools/gpu_ab.sh "$A@AAA_VIS_F32_S6L=0 $A@AAA_VIS_F32_S6L=1 $A@AAA_VIS_F32_S6L=0 $A@AAA_VIS_F32_S6L=1" c2 > gpurun_out/ab_vf.txt 2>&1 || { echo "ab failed"; tail -5 gpurun_out/ab_vf.txt; exit 1; }
for f in gpurun_out/ab_c2_*.json; do python -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$f',d['value'],d['ms_per_step'],[(n[:14],v.get('ms')) for n,v in d['kernels'].items() if 'vision' in n])"; done
cd /tmp && export TMPDIR=/tmp
for c in 0 1; do
  AAA_LIB=$R/$A AAA_VIS_F32_S6L=$c timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_vf$c -o run --output-format csv -- python $R/bench.py --no-cpu-baseline --no-dropin --no-episode --steps 10 > /dev/null 2>&1 || { echo "prof $c failed"; exit 1; }
done
echo profiled
