#!/bin/bash
# LDS bank conflicts of the single-workgroup bf16 BPTT (C3: frames; C4: bwd_pairs) with and without the row-padded
# images (recur_bwd.h kBwIBP; AAA_BW_ROWPAD): one --pmc pass per arm, summarised by tools/pmcsum.py
C=${1:-c3}; K=${2:-bwd_frames}
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/rowpad_$C; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in 0 1; do
  AAA_BW_ROWPAD=$v timeout -s KILL 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS --output-format csv -d $O/p$v -o p$v -- python $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-dropin --no-episode --config $C > $O/p$v.log 2>&1 || { echo "rc=$? v=$v"; exit 1; }
  python $R/tools/pmcsum.py $O/p$v $K > $O/sum$v.txt
  cat $O/sum$v.txt
done
