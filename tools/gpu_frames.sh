#!/bin/bash
# Frame-resident recurrence check: bf16 parity tests, then C3/C4 benches with the
# frame-resident kernels forced to MODES (d = the library's default choice; 0 = per-step).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -q -m gpu -x -p no:cacheprovider --timeout 120 --timeout-method thread -k "bf16 or frame_resident" > $O/frames_parity.log 2>&1 || { echo "parity rc=$?"; tail -30 $O/frames_parity.log; exit 1; }
tail -1 $O/frames_parity.log
for c in ${CONFIGS:-c3 c4}; do
  for v in ${MODES:-1 0}; do
    if [ "$v" = d ]; then unset AAA_FRAMES_FWD AAA_FRAMES_BWD; else export AAA_FRAMES_FWD=$v AAA_FRAMES_BWD=$v; fi
    timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-dropin --steps 10 > $O/fb_${c}_$v.json 2> $O/fb_${c}_$v.err || { echo "bench $c $v rc=$?"; tail $O/fb_${c}_$v.err; exit 1; }
    python -c "import json;d=json.loads(open('$O/fb_${c}_$v.json').read().strip().splitlines()[-1]);print('$c frames=$v',d['value'],d['ms_per_step'],json.dumps(d['kernels']))"
  done
done
