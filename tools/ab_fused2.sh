#!/bin/bash
# A/B of the bf16 fused forward-step tile (AAA_FUSED_TILE) on C3/C4/C5: bench lines
# without the CPU baseline; prints value, ms/step and the forward step's average.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/ab_fused2; mkdir -p $O; cd $R
for c in ${CONFIGS:-c3 c4 c5}; do
  for t in ${TILES:-9 13 14 15 16}; do
    AAA_FUSED_TILE=$t timeout -k 10 200 python bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline > $O/${c}_$t.json 2> $O/${c}_$t.err || { echo "$c tile $t rc=$?"; tail -3 $O/${c}_$t.err; exit 1; }
    python -c "import json;d=json.loads(open('$O/${c}_$t.json').read().strip().splitlines()[-1]);k=d['kernels']['ConvLSTM forward step'];print('$c','tile',$t,d['value'],d['ms_per_step'],k['avg_us'],k['frac'])"
  done
done
