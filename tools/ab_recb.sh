#!/bin/bash
# A/B of the frame-resident BPTT's diagnostic ablations (AAA_RECB_ABL bits:
# 1 no A loads, 2 no epilogue HBM traffic, 4 no MFMA, 8 no chunk-3 DMA) at C3.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
for a in ${ABLS:-0 1 2 3 4 6 8}; do
  AAA_RECB_ABL=$a timeout -k 10 200 python bench.py --config ${CFG:-c3} --no-cpu-baseline --no-dropin --steps 5 --warmup 2 > $O/ablb_$a.json 2> $O/ablb_$a.err || { echo "abl $a rc=$?"; tail -3 $O/ablb_$a.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/ablb_$a.json').read().strip().splitlines()[-1]);k=d['kernels']['ConvLSTM BPTT step'];print('abl=$a',k['avg_us'],k['frac'])"
done
