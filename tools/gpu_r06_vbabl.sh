#!/bin/bash
# Round 6: where the frame-resident vision backward spends its time (ablation build), and the C2 halo ring A/B.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06vbabl; mkdir -p $O; cd $R
A=$R/towards-interpretable-reinforcement-learning-using-attention-augmented-agents-replication_amd/libaaa_ablation.so
for v in 0 1 2 4 8 7 0; do
  AAA_LIB=$A AAA_VBWD_ABL=$v timeout -k 10 300 python bench.py --config c3 --steps 10 --no-cpu-baseline --no-dropin --no-episode > $O/c3_$v.json 2> $O/c3_$v.err || { echo "bench abl $v rc=$?"; tail $O/c3_$v.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/c3_$v.json').read().strip().splitlines()[-1]);print('c3 abl=$v',d['value'],[(n[:24],v.get('ms')) for n,v in d['kernels'].items() if 'vision bwd' in n])"
done
for nb in 3 2 3 2; do
  AAA_LIB=$A AAA_DGRAD2_NBUF=$nb timeout -k 10 300 python bench.py --config c2 --steps 10 --no-cpu-baseline --no-dropin --no-episode > $O/c2_nb$nb.json 2> $O/c2_nb$nb.err || { echo "bench c2 nb $nb rc=$?"; tail $O/c2_nb$nb.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/c2_nb$nb.json').read().strip().splitlines()[-1]);print('c2 nbuf=$nb',d['value'],[(n[:24],v.get('ms')) for n,v in d['kernels'].items() if 'vision bwd' in n])"
done
echo done
