#!/bin/bash
# Round 6: branch-free (buffer, out-of-range-zero) epilogue loads in the single-workgroup bf16 BPTT --
# C3 same-box A/B against the previous build (tools/ablibs/libaaa_base.so), then the bf16 GPU tests.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06bwl; mkdir -p $O; cd $R; export TMPDIR=/tmp
B=$R/tools/ablibs/libaaa_base.so
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python bench.py --config ${CFG:-c3} --no-cpu-baseline --no-dropin --no-episode > $O/$n.json 2> $O/$n.err || { echo "bench $n rc=$?"; tail -3 $O/$n.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]);k=d['kernels']['ConvLSTM BPTT step'];print('$n',d['value'],d['ms_per_step'],k['avg_us'],k['frac'])"
}
run base AAA_LIB=$B
run new
run base2 AAA_LIB=$B
run new2
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_band.py tests/test_gpu_episode.py > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
echo done
