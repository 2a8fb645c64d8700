#!/bin/bash
# Round 6: PMC passes (FETCH/WRITE_SIZE, SQ counters) and kernel-trace summaries of the bench main line at HEAD,
# C2..C5 (tools/pmc_cfg_r04.sh) -> gpurun_out/pmc_<c>/, gpurun_out/prof_<c>/.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
bash tools/pmc_cfg_r04.sh "$@"
