#!/bin/bash
# Round 5: split-K depth of the split-at-commit wgrad (C2 A/B, same box).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r05wg; mkdir -p $O; cd $R
BA="--no-cpu-baseline --no-dropin --no-episode"
for i in 1 2; do
  for n in 36 18 27 54; do
    AAA_WGRAD_SPLIT=$n timeout -k 10 200 python bench.py $BA > $O/n${n}_$i.json 2> $O/n${n}_$i.err || { echo "n$n rc=$?"; tail $O/n${n}_$i.err; exit 1; }
  done
done
for f in $O/n*.json; do python -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$f',d['value'],d['ms_per_step'],d['kernels']['ConvLSTM weight-gradient GEMM']['avg_us'])"; done
