#!/bin/bash
# PMC passes (tools/pmc.sh) for each bench config given, then the per-class HBM
# traffic / MFMA utilisation JSON bench.py reads (profiles/rNN/pmc_traffic_<c>.json).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; cd $R
for c in "$@"; do
  BENCH_ARGS="--config $c --no-dropin" bash tools/pmc.sh > $O/pmc_$c.txt 2>&1 || { echo "pmc $c failed"; tail -5 $O/pmc_$c.txt; exit 1; }
  python tools/pmc_traffic.py gpurun_out/pmc $O/pmc_traffic_$c.json > /dev/null && python tools/pmcsum.py gpurun_out/pmc > $O/pmc_summary_$c.txt
  echo "pmc $c ok"
done
