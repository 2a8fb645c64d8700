#!/bin/bash
# Round-5 A/B: split-at-commit (GemmCfgS6L) tiles for the fp32 conv1 / conv2 weight gradients at C2
# (ablation build; AAA_CONV1_WGRAD_S6L / AAA_CONV2_WGRAD_S6L = 0 product, 1..3 tile variants),
# a parity pass with variant 1, and a kernel trace of 0 and 1.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
P=towards-interpretable-reinforcement-learning-using-attention-augmented-agents-replication_amd; A=$P/libaaa_ablation.so
AAA_LIB=$R/$A AAA_CONV1_WGRAD_S6L=1 AAA_CONV2_WGRAD_S6L=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t_cw.log 2>&1 || { echo "parity rc=$?"; tail -30 gpurun_out/t_cw.log; exit 1; }
tail -1 gpurun_out/t_cw.log
arms=""
for c in 0 1 2 3 0 1; do arms="$arms $A@AAA_CONV1_WGRAD_S6L=$c,AAA_CONV2_WGRAD_S6L=$c"; done
SKIP_TESTS=1 tools/gpu_ab.sh "$arms" c2 > gpurun_out/ab_cw.txt 2>&1 || { echo "ab failed"; tail -5 gpurun_out/ab_cw.txt; exit 1; }
for f in gpurun_out/ab_c2_*.json; do python -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$f',d['value'],d['ms_per_step'],[(n[:12],v.get('ms')) for n,v in d['kernels'].items() if 'vision bwd' in n])"; done
cd /tmp && export TMPDIR=/tmp
for c in 0 1; do
  AAA_LIB=$R/$A AAA_CONV1_WGRAD_S6L=$c AAA_CONV2_WGRAD_S6L=$c timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_cw$c -o run --output-format csv -- python $R/bench.py --no-cpu-baseline --no-dropin --no-episode --steps 10 > /dev/null 2>&1 || { echo "prof $c failed"; exit 1; }
done
echo profiled
