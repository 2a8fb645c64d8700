#!/bin/bash
# Round 5: the whole GPU suite (no -x: every failure listed), kink / C5 reports kept.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r05tests; mkdir -p $O; cd $R
rm -f gpurun_out/kink_report.jsonl
timeout -k 10 1000 python -u -m pytest tests -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -3 $O/gpu_tests.log; grep -E "^FAILED|^ERROR" $O/gpu_tests.log | head -30
cp gpurun_out/kink_report.jsonl gpurun_out/c5_raw_grads.json $O/ 2>/dev/null
exit $rc
