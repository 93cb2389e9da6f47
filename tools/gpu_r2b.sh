# render parity (both precisions) + headline bench timing after a fused-kernel change
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-r2b}
timeout -k 10 400 python -u -m pytest tests/test_gpu_render.py -x -q --timeout 180 --timeout-method thread > gpurun_out/${T}_render_tests.log 2>&1 || { tail -40 gpurun_out/${T}_render_tests.log; exit 1; }
tail -1 gpurun_out/${T}_render_tests.log
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/${T}_bench.log 2>&1 || { tail -20 gpurun_out/${T}_bench.log; exit 1; }
tail -n 1 gpurun_out/${T}_bench.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"], d["roofline"]["frac"], d["roofline"]["achieved_credited"], d.get("fp32_exact"))'
