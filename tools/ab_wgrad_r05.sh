#!/bin/bash
# Round-5 A/B of the split-at-commit fp32 weight-gradient tiles at C2 (ablation build):
# 6 = 256x256 (1792 columns for 1728: the last column tile 3/4 used), 7 = 256x192 (9 tiles, none padded).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/ab_wgrad_r05; mkdir -p $O; cd $R
run() { local tag=$1; shift; env AAA_LIB=$R/towards-interpretable-reinforcement-learning-using-attention-augmented-agents-replication_amd/libaaa_ablation.so "$@" timeout -k 10 150 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-dropin --no-episode > $O/$tag.json 2> $O/$tag.err || { echo "$tag failed"; tail -5 $O/$tag.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]);k=d['kernels']['ConvLSTM weight-gradient GEMM'];print('$tag', d['value'], d['ms_per_step'], k['avg_us'], k.get('frac'), k['variant'])"; }
run t6 AAA_WGRAD_S6_TILE=6
run t7 AAA_WGRAD_S6_TILE=7
run t7s28 AAA_WGRAD_S6_TILE=7 AAA_WGRAD_SPLIT=28
run t7s18 AAA_WGRAD_S6_TILE=7 AAA_WGRAD_SPLIT=18
run t6b AAA_WGRAD_S6_TILE=6
run t7b AAA_WGRAD_S6_TILE=7
