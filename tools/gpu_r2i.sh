# round-end style validation: full GPU suite, smoke, headline bench, rocprof kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/r2i_gpu_tests.log 2>&1 || { tail -30 gpurun_out/r2i_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r2i_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2i_smoke.log 2>&1 || { tail -20 gpurun_out/r2i_smoke.log; exit 1; }
tail -2 gpurun_out/r2i_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/r2i_bench.log 2>&1 || exit 1
tail -n 1 gpurun_out/r2i_bench.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["frac"], d["cpu_baseline"]["value"])'
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2i_prof -o run --output-format csv -- python bench.py --no-cpu --steps 3 --warmup 1 > gpurun_out/r2i_prof.log 2>&1 && echo PROF_OK
timeout -k 10 300 python bench.py --mode train > gpurun_out/r2i_bench_train.log 2>&1 && tail -n 1 gpurun_out/r2i_bench_train.log | cut -c1-300
timeout -k 10 300 python bench.py --mode sdf > gpurun_out/r2i_bench_sdf.log 2>&1 && tail -n 1 gpurun_out/r2i_bench_sdf.log | cut -c1-300
timeout -k 10 300 python bench.py --mode train --precision fp32 > gpurun_out/r2i_bench_train_fp32.log 2>&1 && tail -n 1 gpurun_out/r2i_bench_train_fp32.log | cut -c1-300
timeout -k 10 300 python bench.py --mode anim > gpurun_out/r2i_bench_anim.log 2>&1 && tail -n 1 gpurun_out/r2i_bench_anim.log | cut -c1-200
timeout -k 10 300 python bench.py --mode mesh > gpurun_out/r2i_bench_mesh.log 2>&1 && tail -n 1 gpurun_out/r2i_bench_mesh.log | cut -c1-200
B="python bench.py --steps 1 --warmup 0 --no-cpu --no-exact"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_f -o f --output-format csv -- $B > gpurun_out/pmc_f.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_w -o w --output-format csv -- $B > gpurun_out/pmc_w.log 2>&1 && echo PMC_OK
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2i_sdf_prof -o run --output-format csv -- python bench.py --mode sdf --no-cpu --steps 2 --warmup 1 > gpurun_out/r2i_sdf_prof.log 2>&1 && echo SDF_PROF_OK
