#!/bin/bash
# Round 5: the tests of the measured-slower variants on the A/B build (make ablation):
# dx / wgrad split6 tiles, the Xp chunk buffer -- the product library skips them.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r05abl; mkdir -p $O; cd $R
AAA_LIB=$R/towards-interpretable-reinforcement-learning-using-attention-augmented-agents-replication_amd/libaaa_ablation.so \
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -v -m gpu -p no:cacheprovider --timeout 300 \
  --timeout-method thread -k "dx_split6_tiles or wgrad_split6_tiles or xp_chunks" > $O/abl_tests.log 2>&1; rc=$?
tail -3 $O/abl_tests.log; grep -E "^FAILED|^ERROR" $O/abl_tests.log | head -30
exit $rc
