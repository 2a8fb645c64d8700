#!/bin/bash
# Round 6: smoke() and the full -m gpu suite on the committed product library (no benches).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06check; mkdir -p $O; cd $R; export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; exit $rc
