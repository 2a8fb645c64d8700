#!/bin/bash
# Round 3: the rocprofv3 --pmc exit SIGSEGV seen with the paired (cooperative)
# kernels.  plain vs cooperative launch of a trivial kernel, no libaaa.so loaded.
# The cooperative run goes LAST: if it faults in exit(), nothing else follows.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/coop; mkdir -p $O
B=$R/tools/ubench/coop_exit
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 $B coop > $O/bare_coop.log 2>&1; echo "bare coop rc=$?" | tee -a $O/rc.txt
timeout -k 10 60 rocprofv3 --pmc SQ_WAVES --output-format csv -d $O -o plain -- $B plain > $O/plain.log 2>&1
rc=$?; echo "pmc plain rc=$rc" | tee -a $O/rc.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 60 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o kt_coop -- $B coop > $O/kt_coop.log 2>&1
rc=$?; echo "kernel-trace coop rc=$rc" | tee -a $O/rc.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 60 rocprofv3 --pmc SQ_WAVES --output-format csv -d $O -o coop -- $B coop > $O/coop.log 2>&1
rc=$?; echo "pmc coop rc=$rc" | tee -a $O/rc.txt; exit 0
