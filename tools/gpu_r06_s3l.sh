#!/bin/bash
# Round 6: the bf16 path's 64x64 tail GEMMs split at their LDS commit (GemmCfgS3L on gemm_kernel_s6l) vs split per
# fragment read, in the ablation build (AAA_TAIL_S3L=1 / 0), C3 / C4 / C5, two runs each; then the full -m gpu
# suite on the ablation build with it on.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06s3l; mkdir -p $O; cd $R; export TMPDIR=/tmp
ABL=$R/towards-interpretable-reinforcement-learning-using-attention-augmented-agents-replication_amd/libaaa_ablation.so
run() {  # name config env...
  local n=$1 c=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-dropin --no-episode > $O/$n.json 2> $O/$n.err || { echo "bench $n rc=$?"; tail -3 $O/$n.err; exit 1; }
  python -c "
import json;d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]);k=d['kernels']
print('$n',d['value'],d['ms_per_step'],{n[:12]:round(v.get('ms',v.get('avg_us',0)/1e3),4) for n,v in k.items() if 'tail' in n})"
}
for c in c3 c4 c5; do
  run ${c}_s0a $c AAA_LIB=$ABL AAA_TAIL_S3L=0
  run ${c}_s1a $c AAA_LIB=$ABL AAA_TAIL_S3L=1
  run ${c}_s0b $c AAA_LIB=$ABL AAA_TAIL_S3L=0
  run ${c}_s1b $c AAA_LIB=$ABL AAA_TAIL_S3L=1
done
AAA_LIB=$ABL AAA_TAIL_S3L=1 timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
echo done
