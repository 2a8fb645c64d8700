#!/bin/bash
# One GPU session: parity tests, smoke, bench (c2), rocprofv3 kernel trace.
# Stops at the first step that crashes/hangs (exit status > 1).
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc" >&3; if [ $rc -gt 1 ]; then echo "abort after $name" >&3; exit $rc; fi; }
exec 3>&1
step parity timeout -k 10 700 python -m pytest tests -q -m gpu -x -p no:cacheprovider > $O/parity.log 2>&1
step smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
step bench timeout -k 10 400 python bench.py ${BENCH_ARGS} > $O/bench.json 2> $O/bench.err
cd /tmp && export TMPDIR=/tmp
step prof timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline ${BENCH_ARGS} > $O/prof.log 2>&1
