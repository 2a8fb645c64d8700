#!/bin/bash
# A/B of the frame-resident forward's diagnostic ablations (AAA_REC_ABL bits:
# 1 no A loads, 2 no epilogue stores, 4 no MFMA, 8 no B reads) at C3.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
for a in ${ABLS:-0 1 2 3 4 8 12}; do
  AAA_REC_ABL=$a timeout -k 10 200 python bench.py --config ${CFG:-c3} --no-cpu-baseline --no-dropin --steps 5 --warmup 2 > $O/abl_$a.json 2> $O/abl_$a.err || { echo "abl $a rc=$?"; tail -3 $O/abl_$a.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/abl_$a.json').read().strip().splitlines()[-1]);k=d['kernels']['ConvLSTM forward step'];print('abl=$a',k['avg_us'],k['frac'])"
done
