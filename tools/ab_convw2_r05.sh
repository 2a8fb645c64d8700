#!/bin/bash
# Round-5 A/B: fp32 conv2 weight gradient on one 64x512 split-at-commit tile (AAA_CONV2_WGRAD_S6L=4).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
P=towards-interpretable-reinforcement-learning-using-attention-augmented-agents-replication_amd; A=$P/libaaa_ablation.so
cd /tmp && export TMPDIR=/tmp
for c in 0 4; do
  AAA_LIB=$R/$A AAA_CONV2_WGRAD_S6L=$c timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c2w$c -o run --output-format csv -- python $R/bench.py --no-cpu-baseline --no-dropin --no-episode --steps 10 > $R/gpurun_out/c2w$c.json 2>/dev/null || { echo "prof $c failed"; exit 1; }
  python -c "
import csv
rows=list(csv.DictReader(open('$R/gpurun_out/prof_c2w$c/run_kernel_stats.csv')))
for r in rows:
    if 'LdIm2colTB<float, float, 512' in r['Name'] or ('LdRowsTB<float, float, 64' in r['Name']): print('$c', r['Name'][:90], r['Calls'], round(float(r['AverageNs'])/1e3,1))
"
done
