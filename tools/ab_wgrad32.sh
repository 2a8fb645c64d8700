#!/bin/bash
# A/B of the fp32 ConvLSTM weight-gradient variants at C2 (bench.py kernel table).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/ab_wgrad32; mkdir -p $O; cd $R
run() { local tag=$1; shift; env "$@" timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-dropin --no-episode > $O/$tag.json 2> $O/$tag.err || { echo "$tag failed"; exit 1; }
  python -c "import json;d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]);k=d['kernels']['ConvLSTM weight-gradient GEMM'];print('$tag', d['ms_per_step'], k['avg_us'], k['variant'])"; }
run default A=0
run tile192 AAA_WGRAD_TILE=1
run split6 AAA_WGRAD_SPLIT=6
run split12 AAA_WGRAD_SPLIT=12
run split18 AAA_WGRAD_SPLIT=18
run pipe1 AAA_WGRAD_PIPE=1
run pipe5 AAA_WGRAD_PIPE=5
run pipe6 AAA_WGRAD_PIPE=6
run pipe6w512 AAA_WGRAD_PIPE=6 AAA_WGRAD_WGS=512
run default2 A=0
