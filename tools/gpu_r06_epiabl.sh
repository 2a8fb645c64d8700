#!/bin/bash
# Round 6: which of the bf16 BPTT epilogue's inputs costs what (C3, ablation build):
# AAA_RECB_ABL 128 = no c_{s-1} loads, 256 = no gate loads, 512 = no dO loads, 64 = none of them;
# AAA_BW_RING=1 = the LDS-DMA epilogue ring.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06epi; mkdir -p $O; cd $R
A=$R/towards-interpretable-reinforcement-learning-using-attention-augmented-agents-replication_amd/libaaa_ablation.so
run() {  # name, env...
  local n=$1; shift
  env AAA_LIB=$A "$@" timeout -k 10 300 python bench.py --config c3 --steps 10 --no-cpu-baseline --no-dropin --no-episode > $O/$n.json 2> $O/$n.err || { echo "bench $n rc=$?"; tail -3 $O/$n.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]);k=d['kernels']['ConvLSTM BPTT step'];print('$n',d['value'],k['avg_us'])"
}
run base
run no_c AAA_RECB_ABL=128
run no_gates AAA_RECB_ABL=256
run no_dO AAA_RECB_ABL=512
run no_loads AAA_RECB_ABL=64
run ring AAA_BW_RING=1
run base2
echo done
