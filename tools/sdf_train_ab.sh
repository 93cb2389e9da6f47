#!/bin/bash
# same-box A/B of the sdf_pdf training step: round-3 tree (6439bd0) vs HEAD, alternating
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
for i in 1 2; do
  (cd ab/r3tree && timeout -k 10 300 python bench.py --mode sdf-train --steps 20 --warmup 5 --no-cpu) > gpurun_out/r5h_ab_r3_$i.log 2>&1 || exit 1
  tail -1 gpurun_out/r5h_ab_r3_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('r3', d['ms_per_step'])"
  timeout -k 10 300 python bench.py --mode sdf-train --steps 20 --warmup 5 --no-cpu > gpurun_out/r5h_ab_head_$i.log 2>&1 || exit 1
  tail -1 gpurun_out/r5h_ab_head_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('head', d['ms_per_step'])"
done
