#!/bin/bash
# builds tools/microbench/tgemm_<name> for each "name flags" pair (row GEMM experiment variants)
set -e
cd "$(dirname "$0")/../.."
C=animatable_nerf_amd/csrc
pids=()
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -Iinclude $flags tools/microbench/tgemm_bench.hip $C/anr_tgemm.hip $C/anr_gemm.hip -o tools/microbench/tgemm_$name &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
