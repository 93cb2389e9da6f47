# same-box A/B of the bf16x6 fragment prefetch (ab/lib_pf0.so: ANR_X6_PF off) + render/mesh tests
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
B="python bench.py --render-precision bf16x6 --no-cpu --no-exact --no-torch-baseline --no-host-render --steps 10 --warmup 2"
timeout -k 10 300 $B > gpurun_out/abx_pf1.log 2>&1 || exit 1
ANR_LIB_PATH=$PWD/ab/lib_pf0.so timeout -k 10 300 $B > gpurun_out/abx_pf0.log 2>&1 || exit 1
timeout -k 10 300 $B > gpurun_out/abx_pf1b.log 2>&1 || exit 1
for f in abx_pf1 abx_pf0 abx_pf1b; do echo $f $(tail -1 gpurun_out/$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['roofline']['kernel_ms'])"); done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/abx_gpu_tests.log 2>&1 || { tail -30 gpurun_out/abx_gpu_tests.log; exit 1; }
tail -1 gpurun_out/abx_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/abx_smoke.log 2>&1 || { tail -20 gpurun_out/abx_smoke.log; exit 1; }
tail -3 gpurun_out/abx_smoke.log
