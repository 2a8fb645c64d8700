#!/bin/bash
# PMC passes over tools/ubench/wino (one counter group per rocprofv3 run).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/pmcw; rm -rf $O; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
run() { local name=$1; shift; timeout -k 10 120 rocprofv3 --pmc "$@" --output-format csv -d $O -o $name -- $R/tools/ubench/wino 32 > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
run p1 FETCH_SIZE
run p2 TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE
run p3 TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY
cd $R && python tools/pmcsum.py $O > $O/summary.txt && echo ok
