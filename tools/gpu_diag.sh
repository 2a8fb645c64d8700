#!/bin/bash
# GPU test suite, the BPTT/forward phase-stamp harness (tools/ubench/bwband, built
# beforehand with EXTRA="-DAAA_STAMPS -DAAA_ABLATION"), then same-box A/Bs:
#   tools/gpu_diag.sh "<arm> <arm> ..." c4 c2 ...    (arms as in tools/gpu_ab.sh)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
LIBS=$1; shift
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x -p no:cacheprovider --timeout 120 --timeout-method thread > $O/parity.log 2>&1 || { echo "parity rc=$?"; tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
timeout -k 10 180 tools/ubench/bwband > $O/bwband.txt 2>&1 || { echo "bwband rc=$?"; tail -20 $O/bwband.txt; exit 1; }
cat $O/bwband.txt
SKIP_TESTS=1 bash tools/gpu_ab.sh "$LIBS" "$@"
