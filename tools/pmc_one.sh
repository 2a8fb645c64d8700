#!/bin/bash
# One PMC pass of tools/pmc.sh for one bench config, into gpurun_out/pmc_<config>/
# (for configs whose profiled process crashes in rocprofv3's teardown after the
# counters are written: one pass per gpurun call).  usage: pmc_one.sh c4 p3
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/pmc_$1; mkdir -p $O
case $2 in
  p1) C="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES" ;;
  p2) C="GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE" ;;
  p3) C="FETCH_SIZE" ;;
  p4) C="WRITE_SIZE" ;;
  *) echo "unknown pass $2"; exit 2 ;;
esac
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d $O -o $2 -- python $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-dropin --config $1 > $O/$2.log 2>&1
rc=$?; echo "$1 $2 rc=$rc"; grep -c "tool finalization" $O/$2.log; exit $rc
