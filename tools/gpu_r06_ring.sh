#!/bin/bash
# Round 6: the bf16 BPTT's LDS-DMA epilogue ring (AAA_BW_RING=1) -- full -m gpu suite with it forced on,
# then same-box C3 A/B (ring off / on, alternating) and a kernel trace of each.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06ring; mkdir -p $O; cd $R; export TMPDIR=/tmp
AAA_BW_RING=1 timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > $O/tests.log 2>&1; rc=$?
tail -4 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1 0 1; do
  AAA_BW_RING=$v timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline --no-dropin --no-episode > $O/c3_r$v.json 2> $O/c3_r$v.err || { echo "bench rc=$?"; tail $O/c3_r$v.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/c3_r$v.json').read().strip().splitlines()[-1]);k=d['kernels']['ConvLSTM BPTT step'];print('c3 ring=$v',d['value'],d['ms_per_step'],k['avg_us'],k['frac'])"
done
echo done
