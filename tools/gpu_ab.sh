#!/bin/bash
# GPU test suite, then a same-box A/B of library builds on the given configs:
#   tools/gpu_ab.sh "<lib_a> <lib_b>@VAR=v,VAR2=w ..." c3 c4 ...   (stops at the first failing step)
# an arm "<lib>@VAR=v,..." runs that library with those environment variables
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
LIBS=$1; shift
# TESTS_LAST=1: the A/B first, then the suite (a failing test then costs no measurement)
run_tests() {
  timeout -k 10 600 python -u -m pytest tests -q -m gpu -x -p no:cacheprovider --timeout 120 --timeout-method thread > $O/parity.log 2>&1 || { echo "parity rc=$?"; tail -30 $O/parity.log; exit 1; }
  tail -1 $O/parity.log
}
[ -z "$SKIP_TESTS" ] && [ -z "$TESTS_LAST" ] && run_tests
for c in "$@"; do
  i=0
  for arm in $LIBS; do
    i=$((i+1)); lib=${arm%%@*}; envs=""
    [ "$arm" != "$lib" ] && envs=$(echo "${arm#*@}" | tr ',' ' ')
    env $envs AAA_LIB=$R/$lib timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-dropin --no-episode --steps 10 > $O/ab_${c}_$i.json 2> $O/ab_${c}_$i.err || { echo "bench $c [$lib] rc=$?"; tail $O/ab_${c}_$i.err; exit 1; }
    python -c "import json;d=json.loads(open('$O/ab_${c}_$i.json').read().strip().splitlines()[-1]);print('$c [$arm]',d['value'],d['ms_per_step'],[(n[:22],v.get('avg_us',v.get('ms')),v.get('frac')) for n,v in d['kernels'].items()],[(n[:18],v['avg_us']) for n,v in d['hbm_kernels'].items()])"
  done
done
[ -n "$TESTS_LAST" ] && run_tests
exit 0
