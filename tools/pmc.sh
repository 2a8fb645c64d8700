#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, --pmc never combined with
# trace domains) over a short bench; summarise with tools/pmcsum.py.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/pmc; rm -rf $O; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
run() { local name=$1; shift; timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d $O -o $name -- python $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
run p1 SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES
run p2 GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE
run p3 FETCH_SIZE
run p4 WRITE_SIZE
cd $R && python tools/pmcsum.py $O gemm > $O/summary.txt && head -60 $O/summary.txt
