#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/abperm; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in 0 1; do
  AAA_REC_PERM=$v timeout -k 10 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS --output-format csv -d $O -o p$v -- python $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-dropin --config c3 > $O/p$v.log 2>&1 || { echo "rc=$? v=$v"; exit 1; }
done
echo done
