#!/bin/bash
# Round 6: is the bf16 BPTT epilogue bound by HBM bursts (every frame's epilogue at once)?  C3 on the
# ablation build: start stagger of half the frames (AAA_REC_STAGGER_BWD us), and the epilogue
# ablations (AAA_RECB_ABL 32 = no dZ stores, 64 = no epilogue loads, 2 = neither).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06stag; mkdir -p $O; cd $R
A=$R/towards-interpretable-reinforcement-learning-using-attention-augmented-agents-replication_amd/libaaa_ablation.so
run() {  # name, env...
  local n=$1; shift
  env AAA_LIB=$A "$@" timeout -k 10 300 python bench.py --config c3 --steps 10 --no-cpu-baseline --no-dropin --no-episode > $O/$n.json 2> $O/$n.err || { echo "bench $n rc=$?"; tail -3 $O/$n.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]);k=d['kernels']['ConvLSTM BPTT step'];print('$n',d['value'],k['avg_us'])"
}
run base
run stag15 AAA_REC_STAGGER_BWD=15
run stag30 AAA_REC_STAGGER_BWD=30
run stag45 AAA_REC_STAGGER_BWD=45
run abl32 AAA_RECB_ABL=32
run abl64 AAA_RECB_ABL=64
run abl2 AAA_RECB_ABL=2
run base2
run stag30b AAA_REC_STAGGER_BWD=30
echo done
