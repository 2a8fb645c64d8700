#!/bin/bash
# Actor chain check: actor GPU tests, the actor latency bench, and a rocprofv3
# kernel trace of the 84x84 bench; stops at the first failing step.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_actor.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > $O/actor_tests.log 2>&1 || { echo "tests rc=$?"; tail -40 $O/actor_tests.log; exit 1; }
tail -2 $O/actor_tests.log
timeout -k 10 300 python tools/bench_actor.py --steps 200 --cpu-steps 10 > $O/actor_bench.jsonl 2> $O/actor_bench.err || { echo "bench rc=$?"; tail $O/actor_bench.err; exit 1; }
cat $O/actor_bench.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_actor -o run --output-format csv -- python $R/tools/bench_actor.py --steps 50 --sizes 84x84 --cpu-steps 2 > $O/prof_actor.log 2>&1 || { echo "prof rc=$?"; exit 1; }
echo done
