#!/bin/bash
# PMC passes (one counter group per rocprofv3 run) + a kernel-trace summary of
# the bench main line only (no drop-in / episode legs) for each config given.
# usage: tools/pmc_cfg_r04.sh c2 [c3 ...]   -> gpurun_out/pmc_<c>/, gpurun_out/prof_<c>/
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd /tmp && export TMPDIR=/tmp
BA="--steps 2 --warmup 1 --no-cpu-baseline --no-dropin --no-episode"
for c in "$@"; do
  O=$R/gpurun_out/pmc_$c; rm -rf $O; mkdir -p $O
  run() { local name=$1; shift; timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $O -o $name -- python $R/bench.py --config $c $BA > $O/$name.log 2>&1; local rc=$?; echo "$c $name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
  run p1 SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES
  run p2 GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE
  run p3 FETCH_SIZE
  run p4 WRITE_SIZE
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$c -o run --output-format csv -- python $R/bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline --no-dropin --no-episode > $R/gpurun_out/prof_$c.log 2>&1 || { echo "prof $c rc=$?"; exit 1; }
  echo "prof $c ok"
done
