#!/bin/bash
# Episode-leg tile A/B (GPU box): each arm = space-separated AAA_* settings
# ("-" = defaults); per arm the fused episode leg 3x and one rocprofv3 kernel
# trace -> gpurun_out/ep_ab/<n>/.  Stops at the first failing step.
#   tools/gpu_episode_ab.sh "-" "AAA_FUSED_TILE=4 AAA_BPTT_TILE=16" ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=$PWD
mkdir -p gpurun_out/ep_ab
export TMPDIR=/tmp
n=0
for arm in "$@"; do
  n=$((n + 1))
  a=()
  [ "$arm" != "-" ] && read -r -a a <<< "$arm"
  echo "== arm $n: $arm" | tee -a gpurun_out/ep_ab/log
  env "${a[@]}" timeout -k 10 180 python -u "$R/tools/episode_trace.py" --fused-only --reps 3 \
      >> gpurun_out/ep_ab/log 2>&1 || { echo "arm $n failed"; exit 1; }
  (cd /tmp && env "${a[@]}" timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/ep_ab/$n" -o run \
      --output-format csv -- python "$R/tools/episode_trace.py" --fused-only > "$R/gpurun_out/ep_ab/$n.log" 2>&1) \
      || { echo "arm $n trace failed"; exit 1; }
done
echo ok
