#!/bin/bash
# Bench lines for the given configs (first one with the CPU baseline), then a
# rocprofv3 kernel-trace summary of the first config; stops at the first failure.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
first=$1
for c in "$@"; do
  extra=""; [ "$c" != "$first" ] && extra="--no-cpu-baseline"
  timeout -k 10 300 python bench.py --config $c $extra > $O/bench_$c.json 2> $O/bench_$c.err || { echo "bench $c rc=$?"; tail $O/bench_$c.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/bench_$c.json').read().strip().splitlines()[-1]);print('$c',d['value'],d['ms_per_step'],d['roofline']['frac'],d['roofline']['avg_launch_us'],json.dumps(d['hbm_kernels']))"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$first -o run --output-format csv -- python $R/bench.py --config $first --steps 5 --warmup 2 --no-cpu-baseline > $O/prof_$first.log 2>&1 || { echo "prof rc=$?"; exit 1; }
echo done
