#!/bin/bash
# Round-5 A/B of the attention backward's dA pass: 2 positions per lane (default) vs 1 (round 4),
# same box, ablation build, C2 / C3 / C5 bench kernel table.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/ab_attn_r05; mkdir -p $O; cd $R
L=$R/towards-interpretable-reinforcement-learning-using-attention-augmented-agents-replication_amd/libaaa_ablation.so
for c in ${@:-c2 c3 c5}; do
  for ppl in 1 2 1 2; do
    env AAA_LIB=$L AAA_ATTN_BWD_PPL=$ppl timeout -k 10 200 python bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline --no-dropin --no-episode > $O/${c}_$ppl.json 2> $O/${c}_$ppl.err || { echo "$c ppl=$ppl failed"; tail -5 $O/${c}_$ppl.err; exit 1; }
    python -c "import json;d=json.loads(open('$O/${c}_$ppl.json').read().strip().splitlines()[-1]);print('$c ppl=$ppl', d['value'], d['ms_per_step'], [(n,v['avg_us'],v.get('frac')) for n,v in d.get('hbm_kernels',{}).items() if 'ttention' in n or 'attn' in n])"
  done
done
