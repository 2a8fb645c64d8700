#!/bin/bash
# Round 6: the ablation build (make ablation) -- the measured-slower variants' tests, then the full -m gpu suite
# on that build (its product paths must match the product library's).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06abl; mkdir -p $O; cd $R
ABL=$R/towards-interpretable-reinforcement-learning-using-attention-augmented-agents-replication_amd/libaaa_ablation.so
AAA_LIB=$ABL timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -v -m gpu -p no:cacheprovider --timeout 300 \
  --timeout-method thread -k "dx_split6_tiles or wgrad_split6_tiles or xp_chunks" > $O/abl_tests.log 2>&1; rc=$?
tail -2 $O/abl_tests.log; [ $rc -eq 0 ] || exit $rc
AAA_LIB=$ABL timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > $O/abl_full.log 2>&1; rc=$?
tail -2 $O/abl_full.log; [ $rc -eq 0 ] || exit $rc
echo done
