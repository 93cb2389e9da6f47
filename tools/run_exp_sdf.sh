#!/bin/bash
# time bench.py --mode sdf with each experiment library: tools/run_exp_sdf.sh name...
cd "$(dirname "$0")/.."
for n in "$@"; do
  if [ "$n" = base ]; then lib=""; else lib=animatable_nerf_amd/exp/$n.so; fi
  ANR_LIB_PATH=$lib timeout -k 10 120 python bench.py --mode sdf --no-cpu --steps 3 --warmup 1 > gpurun_out/exp_sdf_$n.log 2>&1 || exit 1
  echo "$n $(tail -n 1 gpurun_out/exp_sdf_$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
done
