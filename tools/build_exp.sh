#!/bin/bash
# Build experiment variants of one source (default the bf16x3 fused kernel; SRC=anr_lgemm for
# another) into animatable_nerf_amd/exp/<name>.so (same C-ABI; load with ANR_LIB_PATH).
# usage: [SRC=anr_x] tools/build_exp.sh name "-DFLAG ..." [name "flags"]...
set -e
cd "$(dirname "$0")/.."
mkdir -p animatable_nerf_amd/exp /tmp/anr_exp
SRC=${SRC:-anr_mlp_b16}
OTHERS=$(ls animatable_nerf_amd/csrc/*.o | grep -v $SRC.o)
pids=()
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  ( /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wall -Wno-unused-function -Iinclude $flags \
      -c animatable_nerf_amd/csrc/$SRC.hip -o /tmp/anr_exp/$name.o && \
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o animatable_nerf_amd/exp/$name.so /tmp/anr_exp/$name.o $OTHERS ) &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
ls -la animatable_nerf_amd/exp/
