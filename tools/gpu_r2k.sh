# final-tree validation: full GPU suite, smoke, headline bench + kernel stats, train / sdf / anim / mesh benches
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/r2k_gpu_tests.log 2>&1 || { tail -30 gpurun_out/r2k_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r2k_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2k_smoke.log 2>&1 || { tail -20 gpurun_out/r2k_smoke.log; exit 1; }
tail -2 gpurun_out/r2k_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/r2k_bench.log 2>&1 || exit 1
tail -n 1 gpurun_out/r2k_bench.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["frac"], d["roofline"]["traffic"], d["cpu_baseline"]["value"])'
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2k_prof -o run --output-format csv -- python bench.py --no-cpu --steps 3 --warmup 1 > gpurun_out/r2k_prof.log 2>&1 && echo PROF_OK
timeout -k 10 300 python bench.py --mode sdf > gpurun_out/r2k_bench_sdf.log 2>&1 && tail -n 1 gpurun_out/r2k_bench_sdf.log | cut -c1-260
timeout -k 10 300 python bench.py --mode train > gpurun_out/r2k_bench_train.log 2>&1 && tail -n 1 gpurun_out/r2k_bench_train.log | cut -c1-260
timeout -k 10 300 python bench.py --mode anim > gpurun_out/r2k_bench_anim.log 2>&1 && tail -n 1 gpurun_out/r2k_bench_anim.log | cut -c1-200
timeout -k 10 300 python bench.py --mode mesh > gpurun_out/r2k_bench_mesh.log 2>&1 && tail -n 1 gpurun_out/r2k_bench_mesh.log | cut -c1-200
