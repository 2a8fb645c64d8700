#!/bin/bash
# Round 6: the tests this round added or tightened.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06tests; mkdir -p $O; cd $R
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_bench_dp.py tests/test_gpu_share.py tests/test_gpu_coresidency.py \
  "tests/test_gpu_episode.py::test_long_actor_chain_episode_matches_oracle" \
  tests/test_gpu_dp.py tests/test_gpu_parity.py tests/test_gpu_stateful.py > $O/tests.log 2>&1
rc=$?; tail -5 $O/tests.log; cp gpurun_out/kink_report.jsonl $O/ 2>/dev/null; exit $rc
