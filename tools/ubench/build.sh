#!/bin/bash
# Build the diagnostic microbenchmarks (gfx950).  Output binaries stay in this directory.
D=$(cd $(dirname $0) && pwd); C=$D/../../towards-interpretable-reinforcement-learning-using-attention-augmented-agents-replication_amd/csrc
for s in "$@"; do /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -munsafe-fp-atomics -I$D/../../include -I$C $EXTRA -o $D/${s%.hip} $D/$s || exit 1; done
