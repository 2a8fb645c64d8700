#!/bin/bash
# Round 6 same-box A/B: the listed tests on the product library, then each config on the
# base library (tools/ablibs/libaaa_base.so: HEAD of the round's start) and the product one.
#   tools/gpu_r06_ab.sh <out dir name> "<pytest targets or empty>" "<arm lib@ENV=v ...>" c2 c3 ...
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/$1; mkdir -p $O; cd $R; shift
TESTS=$1; shift; ARMS=$1; shift
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu $TESTS > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
  tail -1 $O/tests.log
fi
for c in "$@"; do
  i=0
  for arm in $ARMS; do
    i=$((i+1)); lib=${arm%%@*}; envs=""
    [ "$arm" != "$lib" ] && envs=$(echo "${arm#*@}" | tr ',' ' ')
    env $envs AAA_LIB=$R/$lib timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-dropin --no-episode > $O/${c}_$i.json 2> $O/${c}_$i.err || { echo "bench $c $arm rc=$?"; tail $O/${c}_$i.err; exit 1; }
    python -c "import json;d=json.loads(open('$O/${c}_$i.json').read().strip().splitlines()[-1]);print('$c [$arm]',d['value'],d['ms_per_step'],[(n[:22],v.get('avg_us',v.get('ms'))) for n,v in d['kernels'].items()][:3])"
  done
done
echo done
