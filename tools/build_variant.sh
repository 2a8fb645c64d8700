#!/bin/bash
# Build an A/B variant of libaaa.so with extra compile flags into tools/ablibs/libaaa_<name>.so
# (not the product library; tools/gpu_ab.sh runs it through AAA_LIB).
#   tools/build_variant.sh <name> "<extra flags>"
set -e
R=$(cd $(dirname $0)/.. && pwd); C=$R/towards-interpretable-reinforcement-learning-using-attention-augmented-agents-replication_amd/csrc
B=/tmp/aaa_build_$1; mkdir -p $B $R/tools/ablibs
SRCS="runtime.hip rt_core.hip rt_forward.hip rt_backward.hip rt_components.hip misc.hip optim.hip loss.hip actor.hip"
for s in $SRCS; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -munsafe-fp-atomics -I$R/include -Wall -Wno-unused-function $2 -c $C/$s -o $B/${s%.hip}.o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $R/tools/ablibs/libaaa_$1.so $B/*.o
echo "built tools/ablibs/libaaa_$1.so"
